// Narrow-batch int8 candidate scan of the store search (reference
// src/lazzaro/core/vector_store.py:132-140 search_nodes):
// the interactive search_memories turn and small serving batches (< 128
// queries), where the scan is bound by the int8 rows' HBM bytes, not by the
// MFMA. Same contract as the persistent candidate kernel of search256.hip
// (block-private (query, row, score, lists) records, gathered, re-scored,
// certified and selected by the caller, ops/search.py flat_topk_i8):
//
//   score(q, r) = alpha * qs[q] * (rs[r] * <q8[q], x8[r]>) + bias[r]
//
// (A wide 256 x 256-tile variant of this file was an opt-in experiment in
// round 4 -- faster raw, slower with a real candidate threshold -- and was
// removed in round 5; wide batches take search256.hip's template.)
#include "lzk_common.h"

LZK_DEBUG_STATE(scan8)

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;
typedef __attribute__((address_space(3))) int lds_int;

constexpr int NT = 512;
constexpr int SLOT = 16384;                 // bytes: 128 rows x 128 B (one half-tile of one K-tile)
constexpr int RING = 8 * SLOT;              // 2 K-tile buffers x {A0, A1, B0, B1}
// epilogue operands per tile parity: thr | bias | rs | qs | thr2 | row label | query label | quad stats
// (quad stats: 64 x {max row scale, max bias} of the tile's 4-row quads)
constexpr int NARR = 8;
constexpr int EPI_BYTES = 2 * NARR * 256 * 4;
// candidate records are staged in LDS per wave and written to the wave's
// global region in batches: a global store in the epilogue would join the
// vmcnt the K loop counts its operand DMAs with, so the next counted wait
// would stall on the store's write-back (PMC: 6x the wait cycles)
constexpr int LREC = 120;                   // staged records per wave (16 B each)
constexpr int REC_OFF = RING + EPI_BYTES;
constexpr int LDS_TOTAL = REC_OFF + 8 * LREC * 16;

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Record staging in LDS through inline asm: the compiler treats any ds_write
// to the dynamic LDS array as possibly aliasing the in-flight LDS-DMA
// operand loads and puts an s_waitcnt vmcnt(0) in front of it (draining the
// K loop's prefetch); the staging slots never overlap the DMA destinations,
// so these writes / reads wait only on lgkmcnt, which they count in.
__device__ __forceinline__ void lds_write16(const void* p, int4 v) {
  const unsigned a = (unsigned)(size_t)(lds_void_t*)p;
  const i32x4 w = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(w) : "memory");
}
__device__ __forceinline__ int4 lds_read16(const void* p) {
  const unsigned a = (unsigned)(size_t)(lds_void_t*)p;
  i32x4 w;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(a) : "memory");
  return make_int4(w[0], w[1], w[2], w[3]);
}

struct Recs {
  int4* buf;  // [grid * 8][cap]: one region per wave
  int cap;    // records per wave region
  int* cnt;   // [grid * 8]
};

// tile -> (row base, query base)
struct TileGeo {
  int r0, q0;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const signed char* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

int g_n_cu = 0;
int cu_count() {
  if (g_n_cu <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_n_cu <= 0)
      g_n_cu = 256;
  }
  return g_n_cu;
}


// ------------------------------------------------------------------ narrow batches
// Q < 128 queries (the interactive search_memories turn, small serving
// batches): the scan is bound by the int8 rows' HBM bytes (7.7 GB at 10M x
// 768), not by the MFMA, so there is no 256-wide query tile and no LDS row
// staging. Each wave streams 16-row blocks straight into registers (the A
// fragments of v_mfma_i32_16x16x64_i8: lane l holds row l & 15, 16 bytes at
// 64 kk + 16 (l >> 4)), double-buffered across blocks, and multiplies them by
// NQT 16-query tiles held once per block in LDS (row stride Dp + 16 bytes:
// the 16 query rows of a ds_read_b128 lane group fall on 16 distinct 16-B
// bank slots). Scores past the threshold go to the per-wave record regions
// of the wide kernel (same format, gathered / re-scored / selected the same
// way).
constexpr int NW_WAVES = 8;
constexpr int NW_MAXK = 16;  // Dp <= 1024 bytes = 16 k-chunks of 64

// KKT: the fragment arrays' length (12 = the 768-byte rows of bge-base /
// d = 768 exactly, 16 = any Dp <= 1024); with 12 and one query tile the
// kernel fits 128 VGPRs, so both blocks of a CU are resident at once (twice
// the row bytes in flight of the 16-chunk build, which held 160 VGPRs).
template <bool HAS_BIAS, int NQT, int KKT>
__global__ __launch_bounds__(NW_WAVES * 64, (NQT == 1 && KKT <= 12) ? 2 : 1) void scan8_narrow_kernel(
    const signed char* __restrict__ X, long ldx, int nrows, const signed char* __restrict__ Qm, long ldq, int nq,
    int KK, const float* __restrict__ bias, const float* __restrict__ rs, const float* __restrict__ qs, float alpha,
    const float* __restrict__ thr, Recs rec) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, lq = lane >> 4;
  const int Dp = KK * 64;
  const int qld = Dp + 16;  // LDS bytes per query row
  // stage the block's queries (rows past nq are zero)
  for (int c = threadIdx.x; c < NQT * 16 * (Dp / 16); c += NW_WAVES * 64) {
    const int q = c / (Dp / 16), off = (c % (Dp / 16)) * 16;
    i32x4 v = {0, 0, 0, 0};
    if (q < nq) v = *reinterpret_cast<const i32x4*>(Qm + (long)q * ldq + off);
    *reinterpret_cast<i32x4*>(smem + q * qld + off) = v;
  }
  float th[NQT], al[NQT];
#pragma unroll
  for (int t = 0; t < NQT; ++t) {
    const int q = t * 16 + l16;
    th[t] = q < nq ? thr[q] : __builtin_huge_valf();
    al[t] = q < nq ? alpha * qs[q] : 0.f;
  }
  __syncthreads();

  const int capw = rec.cap;
  int4* wbuf = rec.buf + (long)(blockIdx.x * NW_WAVES + wave) * capw;
  int wpos = 0;
  const int nblk = (nrows + 15) / 16;
  const int stride = gridDim.x * NW_WAVES;
  int blk = blockIdx.x * NW_WAVES + wave;

  // two named fragment buffers (a runtime index into one array would put
  // it in scratch memory)
  i32x4 fa[KKT], fb[KKT];
  auto load = [&](i32x4 (&a)[KKT], int b) {
    const int r = min(b * 16 + l16, nrows - 1);
    const signed char* src = X + (long)r * ldx + lq * 16;
#pragma unroll
    for (int kk = 0; kk < KKT; ++kk)
      if (kk < KK) a[kk] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(src + kk * 64));
  };
  auto body = [&](const i32x4 (&a)[KKT], int b) {
    i32x4 acc[NQT];
#pragma unroll
    for (int t = 0; t < NQT; ++t) acc[t] = (i32x4){0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < KKT; ++kk) {
      if (kk < KK) {
#pragma unroll
        for (int t = 0; t < NQT; ++t) {
          const i32x4 bq = *reinterpret_cast<const i32x4*>(smem + (t * 16 + l16) * qld + kk * 64 + lq * 16);
          acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[kk], bq, acc[t], 0, 0, 0);
        }
      }
    }
    // acc[t][e]: row b*16 + 4*lq + e, query t*16 + l16
    const int rbase = b * 16 + 4 * lq;
    f32x4 rsv, bv = {0.f, 0.f, 0.f, 0.f};
    if (rbase + 3 < nrows) {
      rsv = *reinterpret_cast<const f32x4*>(rs + rbase);
      if (HAS_BIAS) bv = *reinterpret_cast<const f32x4*>(bias + rbase);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = min(rbase + e, nrows - 1);
        rsv[e] = rs[r];
        if (HAS_BIAS) bv[e] = bias[r];
      }
    }
#pragma unroll
    for (int t = 0; t < NQT; ++t) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = rbase + e;
        const float sc = al[t] * ((float)acc[t][e] * rsv[e]) + bv[e];
        const bool take = r < nrows && sc >= th[t] && sc != LZK_NEG_INF;
        const unsigned long long ball = __ballot(take);
        if (ball) {
          const int pos = wpos + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(ball >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((unsigned)ball, 0u));
          if (take && pos < capw) wbuf[pos] = make_int4(t * 16 + l16, r, __float_as_int(sc), 1);
          wpos += __builtin_popcountll(ball);
        }
      }
    }
  };
  if (blk < nblk) load(fa, blk);
  while (blk < nblk) {  // two blocks per trip: the next block loads while this one computes
    const int b1 = blk + stride;
    if (b1 < nblk) load(fb, b1);
    body(fa, blk);
    if (b1 >= nblk) break;
    const int b2 = b1 + stride;
    if (b2 < nblk) load(fa, b2);
    body(fb, b1);
    blk = b2;
  }
  if (lane == 0) rec.cnt[blockIdx.x * NW_WAVES + wave] = wpos;
}

}  // namespace

// Narrow-batch int8 scan (nq < 128): grid (blocks) for a shape; the record
// regions are grid * 8 (one per wave): (query, row, score, lists) records gathered
// by lzk_cand_gather over grid * 8 regions.
LZK_EXPORT int lzk_scan8_narrow_grid(int nrows) {
  const int nblk16 = (nrows + 15) / 16;
  const int want = cu_count() * 2;
  const int need = (nblk16 + NW_WAVES - 1) / NW_WAVES;
  return need < want ? (need > 0 ? need : 1) : want;
}

LZK_EXPORT int lzk_scan8_narrow(const void* X8, long ldx, int nrows, const void* Q8, long ldq, int nq, int D_bytes,
                                const float* bias, const float* rscale, const float* qscale, float alpha,
                                const float* thr, void* blk_buf, int blk_cap, int* blk_cnt, void* stream) {
  if (D_bytes % 64 != 0 || D_bytes <= 0 || D_bytes > 64 * NW_MAXK || (ldx | ldq) % 16 != 0 || nq <= 0 ||
      nq > 128 || nrows <= 0 || !rscale || !qscale || !thr || !blk_buf || blk_cap <= 0 || !blk_cnt ||
      !(alpha > 0.f))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int grid = lzk_scan8_narrow_grid(nrows);
  const Recs rec{(int4*)blk_buf, blk_cap, blk_cnt};
  const int nqt = (nq + 15) / 16;
  const size_t lds = (size_t)nqt * 16 * (D_bytes + 16);
  const signed char* x = (const signed char*)X8;
  const signed char* q = (const signed char*)Q8;
  const int KK = D_bytes / 64;
#define LZK_NW3(B, T, KT)                                                                                       \
  do {                                                                                                          \
    (void)hipFuncSetAttribute((const void*)scan8_narrow_kernel<B, T, KT>,                                       \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                           \
    hipLaunchKernelGGL((scan8_narrow_kernel<B, T, KT>), dim3(grid), dim3(NW_WAVES * 64), lds, st, x, ldx, nrows, \
                       q, ldq, nq, KK, bias, rscale, qscale, alpha, thr, rec);                                  \
  } while (0)
#define LZK_NW(B, T)              \
  do {                            \
    if (KK == 12)                 \
      LZK_NW3(B, T, 12);          \
    else                          \
      LZK_NW3(B, T, NW_MAXK);     \
  } while (0)
#define LZK_NWT(B)                    \
  do {                                \
    switch (nqt) {                    \
      case 1: LZK_NW(B, 1); break;    \
      case 2: LZK_NW(B, 2); break;    \
      case 3: LZK_NW(B, 3); break;    \
      case 4: LZK_NW(B, 4); break;    \
      case 5: LZK_NW(B, 5); break;    \
      case 6: LZK_NW(B, 6); break;    \
      case 7: LZK_NW(B, 7); break;    \
      default: LZK_NW(B, 8); break;   \
    }                                 \
  } while (0)
  if (bias) LZK_NWT(true);
  else LZK_NWT(false);
#undef LZK_NWT
#undef LZK_NW
#undef LZK_NW3
  return (int)hipGetLastError();
}
