// IVF-PQ scan (BASELINE config 5: an index that fills the
// 288 GB of HBM per GPU). LanceDB can build IVF-PQ but the reference never does
// (vector_store.py:55 only builds a scalar index); this is the MI355X design:
//
//   * inverted lists: PQ codes of one list are contiguous [rows][M] uint8
//     (CSR offsets), ids kept alongside;
//   * inner-product metric with PQ on coarse residuals, so the lookup table
//     LUT[j][c] = <q_j, codebook_j[c]> depends on the query only (one LUT per
//     query, reused by all nprobe lists) and score = <q, centroid> + sum_j LUT;
//   * one workgroup per (query, probed list): the query's fp32 LUT (M x 256,
//     64 KiB at M = 64) is staged once in LDS, each thread scores whole code
//     rows (16-byte code loads, LDS gathers) into a register top-K, then the
//     256 per-thread lists are reduced by wave argmax rounds + one 4-way merge;
//   * partial lists go through the shared topk_merge kernel (search.hip).
#include "lzk_common.h"

namespace {

// Sum of the LUT entries of one PQ code row (M bytes, 16-byte loads; M = 8
// with one 8-byte load).
template <int M>
__device__ __forceinline__ float pq_score(const unsigned char* __restrict__ c, const float* __restrict__ slut,
                                          float s) {
  static_assert(M % 16 == 0 || M == 8, "M: 8 or a multiple of 16");
  if constexpr (M == 8) {
    const uint2 v = *reinterpret_cast<const uint2*>(c);
    const unsigned w[2] = {v.x, v.y};
#pragma unroll
    for (int u = 0; u < 8; ++u) s += slut[u * 256 + ((w[u >> 2] >> (8 * (u & 3))) & 0xff)];
  } else {
#pragma unroll
    for (int j0 = 0; j0 < M; j0 += 16) {
      const uint4 v = *reinterpret_cast<const uint4*>(c + j0);
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int u = 0; u < 16; ++u) s += slut[(j0 + u) * 256 + ((w[u >> 2] >> (8 * (u & 3))) & 0xff)];
    }
  }
  return s;
}

template <int K>
struct LaneTopK {
  float s[K];
  int i[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < K; ++j) { s[j] = LZK_NEG_INF; i[j] = -1; }
  }
  __device__ __forceinline__ void push(float v, int r) {  // r increases per thread
    if (v > s[K - 1]) {
#pragma unroll
      for (int j = K - 1; j > 0; --j) {
        bool up = v > s[j - 1], here = v > s[j];
        float ns = up ? s[j - 1] : (here ? v : s[j]);
        int ni = up ? i[j - 1] : (here ? r : i[j]);
        s[j] = ns; i[j] = ni;
      }
      if (v > s[0]) { s[0] = v; i[0] = r; }
    }
  }
};

template <int K, int M>
__global__ __launch_bounds__(256) void ivfpq_scan_kernel(const unsigned char* __restrict__ codes,
                                                         const long* __restrict__ list_off,
                                                         const int* __restrict__ probes,
                                                         const float* __restrict__ coarse,
                                                         const float* __restrict__ lut, int nprobe,
                                                         float* __restrict__ out_s, int* __restrict__ out_i) {
  extern __shared__ __attribute__((aligned(16))) float slut[];  // [M][256]
  __shared__ float ws[4 * K];
  __shared__ int wi[4 * K];
  const int qp = blockIdx.x;  // query * nprobe + p
  const int q = qp / nprobe;
  const int list = probes[qp];
  const float base = coarse[qp];
  const float* L = lut + (long)q * M * 256;
  for (int t = threadIdx.x * 4; t < M * 256; t += 256 * 4)
    *reinterpret_cast<f32x4*>(slut + t) = *reinterpret_cast<const f32x4*>(L + t);
  __syncthreads();
  LaneTopK<K> top;
  top.init();
  const long r0 = (list >= 0) ? list_off[list] : 0, r1 = (list >= 0) ? list_off[list + 1] : 0;
  for (long r = r0 + threadIdx.x; r < r1; r += 256) {
    const unsigned char* c = codes + r * M;
    const float s = pq_score<M>(c, slut, base);
    top.push(s, (int)r);
  }
  // wave-level K rounds of argmax over the 64 lane lists
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int j = 0; j < K; ++j) {
    float hs = top.s[0];
    int hi = top.i[0] < 0 ? 0x7fffffff : top.i[0];
    float bs = hs;
    int bi = hi;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      float s2 = __shfl_xor(bs, o, 64);
      int i2 = __shfl_xor(bi, o, 64);
      if (better(s2, i2, bs, bi)) { bs = s2; bi = i2; }
    }
    if (lane == 0) { ws[wv * K + j] = bs; wi[wv * K + j] = bi; }
    if (hi == bi && hs == bs && bi != 0x7fffffff) {
#pragma unroll
      for (int t = 0; t < K - 1; ++t) { top.s[t] = top.s[t + 1]; top.i[t] = top.i[t + 1]; }
      top.s[K - 1] = LZK_NEG_INF; top.i[K - 1] = -1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int p[4] = {0, 0, 0, 0};
    for (int j = 0; j < K; ++j) {
      int w = -1;
      float bsv = LZK_NEG_INF;
      int biv = 0x7fffffff;
      for (int a = 0; a < 4; ++a) {
        if (p[a] >= K) continue;
        float s = ws[a * K + p[a]];
        int i = wi[a * K + p[a]];
        if (w < 0 || better(s, i, bsv, biv)) { w = a; bsv = s; biv = i; }
      }
      p[w] += 1;
      out_s[(long)qp * K + j] = bsv;
      out_i[(long)qp * K + j] = (biv == 0x7fffffff || bsv == LZK_NEG_INF) ? -1 : biv;
    }
  }
}

// Deep candidates for the exact re-rank (depth >> 16) without a dense score
// buffer: as ivfpq_scan_kernel, but each WAVE emits its own best DEEP_W rows
// (DEEP_W rounds of wave argmax over the lanes' top-16 lists) instead of one
// merged top-K per list, so a (query, list) pair yields 4 * DEEP_W candidates
// -- a list's best ~4 * DEEP_W rows, as clustered data concentrates a query's
// neighbours in few lists (a list can hold thousands of one cluster's rows, so
// the depth is 4 x 128). out[(qp * 4 + wave) * DEEP_W + j]; rows -1 = none.
constexpr int DEEP_W = 128;
template <int M>
__global__ __launch_bounds__(256) void ivfpq_scan_deep_kernel(const unsigned char* __restrict__ codes,
                                                              const long* __restrict__ list_off,
                                                              const int* __restrict__ probes,
                                                              const float* __restrict__ coarse,
                                                              const float* __restrict__ lut, int nprobe,
                                                              float* __restrict__ out_s, int* __restrict__ out_i) {
  extern __shared__ __attribute__((aligned(16))) float slut[];  // [M][256]
  const int qp = blockIdx.x;
  const int q = qp / nprobe;
  const int list = probes[qp];
  const float base = coarse[qp];
  const float* L = lut + (long)q * M * 256;
  for (int t = threadIdx.x * 4; t < M * 256; t += 256 * 4)
    *reinterpret_cast<f32x4*>(slut + t) = *reinterpret_cast<const f32x4*>(L + t);
  __syncthreads();
  LaneTopK<16> top;
  top.init();
  const long r0 = (list >= 0) ? list_off[list] : 0, r1 = (list >= 0) ? list_off[list + 1] : 0;
  for (long r = r0 + threadIdx.x; r < r1; r += 256) {
    const unsigned char* c = codes + r * M;
    const float s = pq_score<M>(c, slut, base);
    top.push(s, (int)r);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long o = ((long)qp * 4 + wv) * DEEP_W;
  for (int j = 0; j < DEEP_W; ++j) {
    const float hs = top.s[0];
    const int hi = top.i[0] < 0 ? 0x7fffffff : top.i[0];
    float bs = hs;
    int bi = hi;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float s2 = __shfl_xor(bs, off, 64);
      const int i2 = __shfl_xor(bi, off, 64);
      if (better(s2, i2, bs, bi)) { bs = s2; bi = i2; }
    }
    if (lane == 0) {
      const bool none = bi == 0x7fffffff || bs == LZK_NEG_INF;
      out_s[o + j] = none ? LZK_NEG_INF : bs;
      out_i[o + j] = none ? -1 : bi;
    }
    if (hi == bi && hs == bs && bi != 0x7fffffff) {
#pragma unroll
      for (int t = 0; t < 15; ++t) { top.s[t] = top.s[t + 1]; top.i[t] = top.i[t + 1]; }
      top.s[15] = LZK_NEG_INF; top.i[15] = -1;
    }
  }
}

// Threshold pass of the deep candidate search: every row of a probed list
// whose PQ score reaches the query's threshold thr[q] is appended to the
// query's list (score, code row). thr[q] is the R-th best PQ score of the
// first pass's per-list pools -- a lower bound of the true R-th best over the
// probed lists -- so the appended set holds the exact PQ top-R however the
// query's neighbours concentrate in one list (the per-list pools cap at
// 4 x DEEP_W). Appends are wave-aggregated (ballot + one atomicAdd per wave
// per step); cnt[q] keeps counting past cap so the caller sees an overflow.
template <int M>
__global__ __launch_bounds__(256) void ivfpq_scan_thresh_kernel(const unsigned char* __restrict__ codes,
                                                                const long* __restrict__ list_off,
                                                                const int* __restrict__ probes,
                                                                const float* __restrict__ coarse,
                                                                const float* __restrict__ lut,
                                                                const float* __restrict__ thr, int nprobe, int cap,
                                                                int* __restrict__ cnt, float* __restrict__ out_s,
                                                                int* __restrict__ out_i) {
  extern __shared__ __attribute__((aligned(16))) float slut[];  // [M][256]
  const int qp = blockIdx.x;
  const int q = qp / nprobe;
  const int list = probes[qp];
  const float base = coarse[qp];
  const float t = thr[q];
  const float* L = lut + (long)q * M * 256;
  for (int i = threadIdx.x * 4; i < M * 256; i += 256 * 4)
    *reinterpret_cast<f32x4*>(slut + i) = *reinterpret_cast<const f32x4*>(L + i);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long r0 = (list >= 0) ? list_off[list] : 0, r1 = (list >= 0) ? list_off[list + 1] : 0;
  for (long rb = r0; rb < r1; rb += 256) {  // uniform trip count: every lane reaches the ballot
    const long r = rb + threadIdx.x;
    float s = LZK_NEG_INF;
    if (r < r1) {
      const unsigned char* c = codes + r * M;
      s = pq_score<M>(c, slut, base);
    }
    const bool take = r < r1 && s >= t;
    const unsigned long long m = __ballot(take);
    if (m == 0ull) continue;
    const int leader = __ffsll((long long)m) - 1;
    int pos0 = 0;
    if (lane == leader) pos0 = atomicAdd(cnt + q, __popcll(m));
    pos0 = __shfl(pos0, leader, 64);
    if (take) {
      const int pos = pos0 + __popcll(m & ((1ull << lane) - 1ull));
      if (pos < cap) {
        out_s[(long)q * cap + pos] = s;
        out_i[(long)q * cap + pos] = (int)r;
      }
    }
  }
}

// Exact re-rank of a deep candidate list (IVF-PQ candidates, BASELINE config 5):
// score = <q, v_row> over the kept copy -- FMT 1: fp8 e4m3, FMT 2: int8, each
// with a per-row scale (D + 4 B/vector), or FMT 0: bf16 -- then the top-k by
// (score desc, row asc). int8 with a per-row absmax scale is ~3x finer than
// e4m3 on embedding-like rows (a uniform grid vs 3 mantissa bits): on
// clustered 1024-d data the fp8 copy alone caps recall@10 near 0.85-0.92. One
// 256-thread block per query: the query is staged once in LDS as fp32; 16 lanes
// score one row (16-B loads, 256 contiguous bytes per group and step), so a
// wave has 4 rows and a block 16 rows in flight per step; scores go to LDS and
// wave 0 selects (lane-local top-K, then k rounds of wave argmax). Replaces a
// gather + fp32 dequantise + batched GEMM + sort chain of library kernels.
template <int K>
struct RerankTopK {
  float s[K];
  int i[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < K; ++j) { s[j] = LZK_NEG_INF; i[j] = 0x7fffffff; }
  }
  __device__ __forceinline__ void push(float v, int r) {
    if (!better(v, r, s[K - 1], i[K - 1])) return;
#pragma unroll
    for (int j = K - 1; j > 0; --j) {
      const bool up = better(v, r, s[j - 1], i[j - 1]);
      const bool here = better(v, r, s[j], i[j]);
      const float ns = up ? s[j - 1] : (here ? v : s[j]);
      const int ni = up ? i[j - 1] : (here ? r : i[j]);
      s[j] = ns; i[j] = ni;
    }
    if (better(v, r, s[0], i[0])) { s[0] = v; i[0] = r; }
  }
};

template <int FMT, int K>
__global__ __launch_bounds__(256) void rerank_kernel(const unsigned char* __restrict__ V, long ldv,
                                                     const float* __restrict__ vscale, const long* __restrict__ rows,
                                                     int R, const float* __restrict__ Q, int D, int kout,
                                                     float* __restrict__ os, long* __restrict__ oi) {
  extern __shared__ __attribute__((aligned(16))) float rsm[];  // [D] query | [R] scores
  float* qs = rsm;
  float* sc = rsm + D;
  const int q = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  for (int d = threadIdx.x; d < D; d += 256) qs[d] = Q[(long)q * D + d];
  __syncthreads();
  const long* rq = rows + (long)q * R;
  const int row_bytes = FMT ? D : 2 * D;  // multiple of 256 (checked by the launcher)
  const int steps = row_bytes / 256;
  for (int c0 = wave * 4; c0 < R; c0 += 16) {
    const int c = c0 + g;
    const long r = c < R ? rq[c] : -1;
    float a = 0.f;
    if (r >= 0) {
      const unsigned char* v = V + r * ldv;
      for (int j = 0; j < steps; ++j) {
        const int b = j * 256 + l16 * 16;
        const uint4 w = *reinterpret_cast<const uint4*>(v + b);
        const unsigned u[4] = {w.x, w.y, w.z, w.w};
        if constexpr (FMT == 1) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)u[t], false);
            const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)u[t], true);
            const float* qq = qs + b + 4 * t;
            a = fmaf(lo[0], qq[0], fmaf(lo[1], qq[1], fmaf(hi[0], qq[2], fmaf(hi[1], qq[3], a))));
          }
        } else if constexpr (FMT == 2) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int w = (int)u[t];
            const float* qq = qs + b + 4 * t;
            a = fmaf((float)((w << 24) >> 24), qq[0], fmaf((float)((w << 16) >> 24), qq[1],
                fmaf((float)((w << 8) >> 24), qq[2], fmaf((float)(w >> 24), qq[3], a))));
          }
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const float* qq = qs + b / 2 + 2 * t;
            a = fmaf(__uint_as_float(u[t] << 16), qq[0], fmaf(__uint_as_float(u[t] & 0xffff0000u), qq[1], a));
          }
        }
      }
    }
    a += __shfl_xor(a, 8, 64);
    a += __shfl_xor(a, 4, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 1, 64);
    if (l16 == 0 && c < R) sc[c] = r >= 0 ? (FMT ? a * vscale[r] : a) : LZK_NEG_INF;
  }
  __syncthreads();
  if (wave != 0) return;
  RerankTopK<K> top;
  top.init();
  for (int c = lane; c < R; c += 64) {
    const long r = rq[c];
    if (r >= 0) top.push(sc[c], (int)r);
  }
  for (int j = 0; j < kout; ++j) {
    const float hs = top.s[0];
    const int hi = top.i[0];
    float bs = hs;
    int bi = hi;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float s2 = __shfl_xor(bs, o, 64);
      const int i2 = __shfl_xor(bi, o, 64);
      if (better(s2, i2, bs, bi)) { bs = s2; bi = i2; }
    }
    if (lane == 0) {
      const bool none = bi == 0x7fffffff || bs == LZK_NEG_INF;
      os[(long)q * kout + j] = none ? LZK_NEG_INF : bs;
      oi[(long)q * kout + j] = none ? -1 : (long)bi;
    }
    if (hi == bi && hs == bs && bi != 0x7fffffff) {
#pragma unroll
      for (int t = 0; t < K - 1; ++t) { top.s[t] = top.s[t + 1]; top.i[t] = top.i[t + 1]; }
      top.s[K - 1] = LZK_NEG_INF; top.i[K - 1] = 0x7fffffff;
    }
  }
}

template <int K>
hipError_t launch_scan(int M, const unsigned char* codes, const long* off, const int* probes, const float* coarse,
                       const float* lut, int nq, int nprobe, float* os, int* oi, hipStream_t st) {
  dim3 grid(nq * nprobe), block(256);
  size_t lds = (size_t)M * 256 * sizeof(float);
#define GO(MM)                                                                                                      \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)ivfpq_scan_kernel<K, MM>, hipFuncAttributeMaxDynamicSharedMemorySize,   \
                              (int)lds);                                                                            \
    hipLaunchKernelGGL((ivfpq_scan_kernel<K, MM>), grid, block, lds, st, codes, off, probes, coarse, lut, nprobe,  \
                       os, oi);                                                                                     \
  } while (0)
  switch (M) {
    case 8: GO(8); break;
    case 16: GO(16); break;
    case 32: GO(32); break;
    case 48: GO(48); break;
    case 64: GO(64); break;
    case 96: GO(96); break;
    case 128: GO(128); break;
    default: return hipErrorInvalidValue;
  }
#undef GO
  return hipGetLastError();
}

}  // namespace

// deep candidates: [nq, nprobe, 4 * DEEP_W] (score, code row; -1 = empty)
LZK_EXPORT int lzk_ivfpq_scan_deep(const void* codes, const long* list_off, const int* probes, const float* coarse,
                                   const float* lut, int nq, int nprobe, int M, float* os, int* oi, void* stream) {
  if (nq <= 0 || nprobe <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)nq * nprobe), block(256);
  size_t lds = (size_t)M * 256 * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  const unsigned char* c = (const unsigned char*)codes;
#define GO(MM)                                                                                                      \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)ivfpq_scan_deep_kernel<MM>,                                              \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                                \
    hipLaunchKernelGGL((ivfpq_scan_deep_kernel<MM>), grid, block, lds, st, c, list_off, probes, coarse, lut,       \
                       nprobe, os, oi);                                                                             \
  } while (0)
  switch (M) {
    case 8: GO(8); break;
    case 16: GO(16); break;
    case 32: GO(32); break;
    case 48: GO(48); break;
    case 64: GO(64); break;
    case 96: GO(96); break;
    case 128: GO(128); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef GO
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_ivfpq_deep_width() { return 4 * DEEP_W; }

// threshold pass: cnt [nq] zeroed by the caller; out [nq, cap]
LZK_EXPORT int lzk_ivfpq_scan_thresh(const void* codes, const long* list_off, const int* probes, const float* coarse,
                                     const float* lut, const float* thr, int nq, int nprobe, int M, int cap, int* cnt,
                                     float* os, int* oi, void* stream) {
  if (nq <= 0 || nprobe <= 0 || cap <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)nq * nprobe), block(256);
  size_t lds = (size_t)M * 256 * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  const unsigned char* c = (const unsigned char*)codes;
#define GO(MM)                                                                                                      \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)ivfpq_scan_thresh_kernel<MM>,                                            \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                                \
    hipLaunchKernelGGL((ivfpq_scan_thresh_kernel<MM>), grid, block, lds, st, c, list_off, probes, coarse, lut, thr, \
                       nprobe, cap, cnt, os, oi);                                                                   \
  } while (0)
  switch (M) {
    case 8: GO(8); break;
    case 16: GO(16); break;
    case 32: GO(32); break;
    case 48: GO(48); break;
    case 64: GO(64); break;
    case 96: GO(96); break;
    case 128: GO(128); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef GO
  return (int)hipGetLastError();
}

// partial lists: [nq, nprobe, kslot] (rows index the code array; -1 = empty)
LZK_EXPORT int lzk_ivfpq_scan(const void* codes, const long* list_off, const int* probes, const float* coarse,
                              const float* lut, int nq, int nprobe, int M, int kslot, float* os, int* oi,
                              void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const unsigned char* c = (const unsigned char*)codes;
  hipError_t e;
  switch (kslot) {
    case 1: e = launch_scan<1>(M, c, list_off, probes, coarse, lut, nq, nprobe, os, oi, st); break;
    case 4: e = launch_scan<4>(M, c, list_off, probes, coarse, lut, nq, nprobe, os, oi, st); break;
    case 10: e = launch_scan<10>(M, c, list_off, probes, coarse, lut, nq, nprobe, os, oi, st); break;
    case 16: e = launch_scan<16>(M, c, list_off, probes, coarse, lut, nq, nprobe, os, oi, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)e;
}

// Re-rank: V rows of ldv bytes (fmt 1 fp8 / 2 int8: D bytes + vscale[row];
// fmt 0 bf16: 2D bytes), rows [nq, R] int64 (-1 = empty), Q [nq, D] fp32 ->
// top-kout per query.
LZK_EXPORT int lzk_rerank(const void* V, long ldv, int fmt, const float* vscale, const long* rows, int nq, int R,
                          const float* Q, int D, int kslot, int kout, float* os, long* oi, void* stream) {
  const int row_bytes = fmt ? D : 2 * D;
  if (fmt < 0 || fmt > 2) return (int)hipErrorInvalidValue;
  if (nq <= 0 || R <= 0 || row_bytes % 256 != 0 || (ldv & 15) || kout > kslot || (fmt && !vscale))
    return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(D + R) * sizeof(float);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const unsigned char* v = (const unsigned char*)V;
#define RR(F, KK)                                                                                                   \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)rerank_kernel<F, KK>, hipFuncAttributeMaxDynamicSharedMemorySize,       \
                              (int)lds);                                                                            \
    hipLaunchKernelGGL((rerank_kernel<F, KK>), dim3(nq), dim3(256), lds, st, v, ldv, vscale, rows, R, Q, D, kout,  \
                       os, oi);                                                                                     \
  } while (0)
#define RK(KK) do { if (fmt == 1) RR(1, KK); else if (fmt == 2) RR(2, KK); else RR(0, KK); } while (0)
  switch (kslot) {
    case 1: RK(1); break;
    case 4: RK(4); break;
    case 10: RK(10); break;
    case 16: RK(16); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef RK
#undef RR
  return (int)hipGetLastError();
}
