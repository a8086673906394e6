// Shared 128x128x64 bf16 MFMA tile machinery (gfx950).
//
// Both operands are K-contiguous row-major matrices ("A rows" and "B rows"):
//   C[a][b] = sum_k A[a][k] * B[b][k]
// 256 threads = 4 waves in a 2x2 arrangement, each wave owns a 64x64 sub-tile
// as 2x2 blocks of v_mfma_f32_32x32x16_bf16. A rows land on the MFMA M axis
// (accumulator registers), B rows on N (lanes): lane l of block (ra, cb) holds
//   C[a = wrow*64 + ra*32 + (r&3) + 8*(r>>2) + 4*(l>>5)][b = wcol*64 + cb*32 + (l&31)]
// in accumulator register r.
//
// Staging: register double-buffering (global_load_dwordx4 issued before the
// MFMAs of the current K-step, ds_write_b128 to the other LDS buffer after),
// XOR-swizzled 128-B LDS rows so each 16-lane group of ds_read_b128 is
// conflict-free. One __syncthreads() per K-step.
#pragma once
#include "lzk_common.h"

namespace lzk {

constexpr int TB = 128;   // rows of A and of B per tile
constexpr int TK = 64;    // K per stage
constexpr int TNT = 256;  // threads
constexpr int TELEMS = TB * TK;

__device__ __forceinline__ int swz(int row, int kc) {
  return row * TK + ((kc ^ ((row >> 1) & 7)) << 3);
}

struct TileStager {
  const u16* asrc[4];
  const u16* bsrc[4];
  int soff[4];
  u16x8 ra[4], rb[4];

  // rows beyond the matrix are clamped (their results are masked by callers)
  __device__ __forceinline__ void setup(const u16* A, long lda, int a0, int na,
                                        const u16* B, long ldb, int b0, int nb, int tid) {
    const int srow = tid >> 3, skc = tid & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int r = srow + 32 * i;
      int ar = min(a0 + r, na - 1);
      int br = min(b0 + r, nb - 1);
      asrc[i] = A + (long)ar * lda + skc * 8;
      bsrc[i] = B + (long)br * ldb + skc * 8;
      soff[i] = swz(r, skc);
    }
  }
  __device__ __forceinline__ void load(int ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = *reinterpret_cast<const u16x8*>(asrc[i] + ks * TK);
      rb[i] = *reinterpret_cast<const u16x8*>(bsrc[i] + ks * TK);
    }
  }
  __device__ __forceinline__ void store(u16* smem, int buf) {
    u16* as = smem + buf * 2 * TELEMS;
    u16* bs = as + TELEMS;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<u16x8*>(as + soff[i]) = ra[i];
      *reinterpret_cast<u16x8*>(bs + soff[i]) = rb[i];
    }
  }
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

// LDS-DMA staging (global_load_lds_dwordx4): each wave-instruction writes one
// contiguous 1 KiB piece = 8 tile rows of 128 B, so the XOR swizzle moves to
// the per-lane SOURCE address (lane l fills physical chunk l&7 of row l>>3 with
// logical chunk (l&7) ^ ((row>>1)&7)); the MFMA-side read applies the same
// involution (swz). No staging VGPRs, no ds_write pass.
struct GldsStager {
  const u16* asrc[4];
  const u16* bsrc[4];
  int piece[4];  // element offset of the wave's 1 KiB pieces inside a tile

  __device__ __forceinline__ void setup(const u16* A, long lda, int a0, int na,
                                        const u16* B, long ldb, int b0, int nb, int tid) {
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = wave * 4 + i;  // 16 pieces per 128-row tile
      const int row = 8 * c + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      asrc[i] = A + (long)min(a0 + row, na - 1) * lda + kc * 8;
      bsrc[i] = B + (long)min(b0 + row, nb - 1) * ldb + kc * 8;
      piece[i] = c * 512;
    }
  }
  __device__ __forceinline__ void issue(u16* smem, int buf, int ks) {
    u16* as = smem + buf * 2 * TELEMS;
    u16* bs = as + TELEMS;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(asrc[i] + ks * TK), (lds_void_t*)(as + piece[i]), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(bsrc[i] + ks * TK), (lds_void_t*)(bs + piece[i]), 16, 0, 0);
    }
  }
};

__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void tile_zero(f32x16 (&acc)[2][2]) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
}

// MFMAs of one 64-deep K-step from LDS buffer `buf`.
__device__ __forceinline__ void tile_mma(const u16* smem, int buf, int wrow, int wcol, int lane,
                                         f32x16 (&acc)[2][2]) {
  const u16* as = smem + buf * 2 * TELEMS;
  const u16* bs = as + TELEMS;
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int s = 0; s < TK / 16; ++s) {
    bf16x8 af[2], bf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      af[i] = *reinterpret_cast<const bf16x8*>(as + swz(wrow * 64 + i * 32 + l32, 2 * s + h));
      bf[i] = *reinterpret_cast<const bf16x8*>(bs + swz(wcol * 64 + i * 32 + l32, 2 * s + h));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
  }
}

// Full K loop with LDS-DMA staging: issue tile k+1's DMA, MFMA on tile k,
// drain + one barrier per K-step (the barrier both publishes tile k+1 and
// frees buffer k for the DMA issued at the top of the next step).
__device__ __forceinline__ void tile_gemm_glds(u16* smem, const u16* A, long lda, int a0, int na,
                                               const u16* B, long ldb, int b0, int nb, int K,
                                               f32x16 (&acc)[2][2]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wrow = wave >> 1, wcol = wave & 1;
  GldsStager st;
  st.setup(A, lda, a0, na, B, ldb, b0, nb, tid);
  tile_zero(acc);
  const int KS = K / TK;
  st.issue(smem, 0, 0);
  vm_drain();
  __syncthreads();
  for (int ks = 0; ks < KS; ++ks) {
    if (ks + 1 < KS) st.issue(smem, (ks + 1) & 1, ks + 1);
    __builtin_amdgcn_s_setprio(1);
    tile_mma(smem, ks & 1, wrow, wcol, lane, acc);
    __builtin_amdgcn_s_setprio(0);
    vm_drain();
    __syncthreads();
  }
}

// Full K loop for one tile: C = A[a0:a0+128] . B[b0:b0+128]^T over K.
__device__ __forceinline__ void tile_gemm(u16* smem, const u16* A, long lda, int a0, int na,
                                          const u16* B, long ldb, int b0, int nb, int K,
                                          f32x16 (&acc)[2][2]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wrow = wave >> 1, wcol = wave & 1;
  TileStager st;
  st.setup(A, lda, a0, na, B, ldb, b0, nb, tid);
  tile_zero(acc);
  const int KS = K / TK;
  st.load(0);
  st.store(smem, 0);
  __syncthreads();
  for (int ks = 0; ks < KS; ++ks) {
    const bool nxt = ks + 1 < KS;
    if (nxt) st.load(ks + 1);
    tile_mma(smem, ks & 1, wrow, wcol, lane, acc);
    if (nxt) st.store(smem, (ks + 1) & 1);
    __syncthreads();
  }
}

}  // namespace lzk
