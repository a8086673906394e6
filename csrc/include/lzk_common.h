// Common device helpers for the lazzaro_amd HIP kernels (gfx950 / CDNA4 only).
//
// Everything here is written for the CDNA4 execution model: 64-lane waves,
// MFMA matrix cores (v_mfma_f32_32x32x16_bf16), 160 KiB LDS per CU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef u16 u16x4 __attribute__((ext_vector_type(4)));

#define LZK_WAVE 64
#define LZK_NEG_INF (-__builtin_huge_valf())

#define LZK_EXPORT extern "C" __attribute__((visibility("default")))

// Debug builds (-DLZK_DEBUG=1, `python -m lazzaro_amd._build --debug`, loaded
// with LZK_DEBUG=1): LZK_DCHECK(cond) in index-driven kernels records the
// first violated condition (line number) in a per-file device word, prints it
// once, and skips the offending thread's work instead of faulting the GPU.
// Use only where an early return cannot strand a barrier. Release builds
// compile it away. LZK_DEBUG_STATE(name) defines the word and an exported
// `lzk_<name>_debug_errors()` that returns and clears it.
#if defined(LZK_DEBUG) && LZK_DEBUG
#define LZK_DCHECK(cond)                                                                              \
  do {                                                                                                \
    if (!(cond)) {                                                                                    \
      if (atomicCAS(&g_lzk_dbg_err, 0, __LINE__) == 0)                                                \
        printf("LZK_DCHECK failed: %s (%s:%d) block %d thread %d\n", #cond, __FILE__, __LINE__,       \
               (int)blockIdx.x, (int)threadIdx.x);                                                    \
      return;                                                                                         \
    }                                                                                                 \
  } while (0)
#define LZK_DEBUG_STATE(name)                                                                         \
  static __device__ int g_lzk_dbg_err = 0;                                                            \
  LZK_EXPORT int lzk_##name##_debug_errors() {                                                        \
    int v = 0, z = 0;                                                                                 \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_lzk_dbg_err), sizeof(int)) != hipSuccess) return -1;     \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lzk_dbg_err), &z, sizeof(int));                              \
    return v;                                                                                         \
  }
#else
#define LZK_DCHECK(cond) do { } while (0)
#define LZK_DEBUG_STATE(name) \
  LZK_EXPORT int lzk_##name##_debug_errors() { return 0; }
#endif

// bf16 <-> f32 by bit manipulation (round-to-nearest-even on the way down).
__device__ __forceinline__ float bf16_to_f32(u16 v) {
  return __uint_as_float(((unsigned)v) << 16);
}
__device__ __forceinline__ u16 f32_to_bf16(float f) {
  // gfx950 has a native round-to-nearest-even packed conversion
  // (v_cvt_pk_bf16_f32): one instruction per two values instead of the
  // 6-op integer rounding sequence
  return __builtin_bit_cast(u16, (__bf16)f);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// (score, idx) total order used by every top-k path in the framework:
// higher score first; equal scores -> smaller index first.
__device__ __forceinline__ bool better(float s1, int i1, float s2, int i2) {
  return (s1 > s2) || (s1 == s2 && (unsigned)i1 < (unsigned)i2);
}

// Bijective XCD-aware remap of a 1-D block id (MI355X: 8 XCDs, blocks are dealt
// round-robin). Consecutive logical ids land on the same XCD so neighbouring
// tiles share that XCD's L2. Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int NX = 8;
  if (nwg < NX) return bid;
  int q = nwg / NX, r = nwg % NX;
  int x = bid % NX, o = bid / NX;
  int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + o;
}

static inline int lzk_ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
