// Multi-tenant batched search: every query scans only ITS tenant's rows
// (SURVEY.md §2.4 K3 "tenant segments"; reference vector_store.py:137 filters
// `user_id = '...'` inside LanceDB and the orchestrator serves one tenant at a
// time, memory_system.py:1474-1486).
//
// A batch of queries from many tenants is one launch: query q reads the
// segment described by (xptr[q], nrows[q]) -- a tenant arena or a slice of a
// shared arena, any mix -- so thousands of small tenants cost one grid, not
// thousands of launches. Per-tenant segments are small (10^2..10^5 rows), so
// the scan is HBM-bound GEMV work, not MFMA work: one workgroup per query,
// 8 lanes per row reading 16-B pieces (each 8-lane group streams one full
// 128-B line), fp32 accumulate, 3 xor-shuffles per row, per-lane top-K,
// wave argmax merge, 4-way LDS merge. Works on bf16 rows or on the arenas'
// exact fp32 copies (then no re-rank is needed).
//
//   score = alpha * <q, x_r> * scale[r] + bias[r] + qbias[q]
// covers ip (alpha 1), L2 (alpha 2, bias -|x|^2, qbias -|q|^2), cosine
// (scale 1/|x|) and tombstones (bias -inf).
#include "lzk_common.h"

namespace {

template <int K>
struct TopK {
  float s[K];
  int i[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < K; ++j) { s[j] = LZK_NEG_INF; i[j] = 0x7fffffff; }
  }
  __device__ __forceinline__ void push(float v, int r) {  // r increasing per lane
    if (!(v > s[K - 1])) return;
#pragma unroll
    for (int j = K - 1; j > 0; --j) {
      const bool up = v > s[j - 1], here = v > s[j];
      const float ns = up ? s[j - 1] : (here ? v : s[j]);
      const int ni = up ? i[j - 1] : (here ? r : i[j]);
      s[j] = ns; i[j] = ni;
    }
    if (v > s[0]) { s[0] = v; i[0] = r; }
  }
};

template <typename T>
struct Piece;
template <>
struct Piece<u16> {  // 16 B = 8 bf16
  static constexpr int E = 8;
  __device__ __forceinline__ static float dot(const u16* p, const float* q) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(p);
    float a = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) a = fmaf(bf16_to_f32(v[e]), q[e], a);
    return a;
  }
};
template <>
struct Piece<float> {  // 16 B = 4 fp32
  static constexpr int E = 4;
  __device__ __forceinline__ static float dot(const float* p, const float* q) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p);
    return fmaf(v[0], q[0], fmaf(v[1], q[1], fmaf(v[2], q[2], v[3] * q[3])));
  }
};

constexpr int SEG_MAXD = 2048;

template <int K, typename T>
__global__ __launch_bounds__(256) void segment_topk_kernel(
    const unsigned long long* __restrict__ xptr, const int* __restrict__ nrows, long ld,
    const unsigned long long* __restrict__ bptr, const unsigned long long* __restrict__ sptr,
    const T* __restrict__ Q, long ldq, int D, float alpha, const float* __restrict__ qbias, int kout,
    float* __restrict__ os, long* __restrict__ oi) {
  constexpr int E = Piece<T>::E;
  __shared__ __attribute__((aligned(16))) float qs[SEG_MAXD];
  __shared__ float ws[4 * K];
  __shared__ int wi[4 * K];
  const int q = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int part = lane & 7, sub = lane >> 3;
  for (int c = threadIdx.x; c < D; c += 256) {
    if constexpr (sizeof(T) == 2) qs[c] = bf16_to_f32(Q[(long)q * ldq + c]);
    else qs[c] = Q[(long)q * ldq + c];
  }
  __syncthreads();
  const T* X = reinterpret_cast<const T*>(xptr[q]);
  const float* B = bptr ? reinterpret_cast<const float*>(bptr[q]) : nullptr;
  const float* Sc = sptr ? reinterpret_cast<const float*>(sptr[q]) : nullptr;
  const int n = nrows[q];
  const float qb = qbias ? qbias[q] : 0.f;
  TopK<K> top;
  top.init();
  for (int r = wave * 8 + sub; r < n; r += 32) {
    const T* xr = X + (long)r * ld;
    float a = 0.f;
#pragma unroll 4
    for (int c = part * E; c < D; c += 8 * E) a += Piece<T>::dot(xr + c, qs + c);
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (part == 0) {
      float s = alpha * a;
      if (Sc) s *= Sc[r];
      if (B) s += B[r];
      top.push(s + qb, r);
    }
  }
  // K rounds of wave argmax over the lane lists, then a 4-way merge
  for (int j = 0; j < K; ++j) {
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
    if (lane == 0) { ws[wave * K + j] = bs; wi[wave * K + j] = bi; }
    if (hi == bi && hs == bs && bi != 0x7fffffff) {
#pragma unroll
      for (int t = 0; t < K - 1; ++t) { top.s[t] = top.s[t + 1]; top.i[t] = top.i[t + 1]; }
      top.s[K - 1] = LZK_NEG_INF; top.i[K - 1] = 0x7fffffff;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int p[4] = {0, 0, 0, 0};
    for (int j = 0; j < kout; ++j) {
      int w = -1;
      float bsv = LZK_NEG_INF;
      int biv = 0x7fffffff;
      for (int a = 0; a < 4; ++a) {
        if (p[a] >= K) continue;
        const float s = ws[a * K + p[a]];
        const int i = wi[a * K + p[a]];
        if (w < 0 || better(s, i, bsv, biv)) { w = a; bsv = s; biv = i; }
      }
      p[w] += 1;
      const bool none = biv == 0x7fffffff || bsv == LZK_NEG_INF;
      os[(long)q * kout + j] = none ? LZK_NEG_INF : bsv;
      oi[(long)q * kout + j] = none ? -1 : (long)biv;
    }
  }
}

template <typename T>
int launch_segment(int kslot, const unsigned long long* xptr, const int* nrows, long ld,
                   const unsigned long long* bptr, const unsigned long long* sptr, const void* Q, long ldq,
                   int nq, int D, float alpha, const float* qbias, int kout, float* os, long* oi, hipStream_t st) {
  const T* q = reinterpret_cast<const T*>(Q);
#define LZK_SEG(KK)                                                                                             \
  hipLaunchKernelGGL((segment_topk_kernel<KK, T>), dim3(nq), dim3(256), 0, st, xptr, nrows, ld, bptr, sptr, q, \
                     ldq, D, alpha, qbias, kout, os, oi)
  switch (kslot) {
    case 1: LZK_SEG(1); break;
    case 2: LZK_SEG(2); break;
    case 4: LZK_SEG(4); break;
    case 8: LZK_SEG(8); break;
    case 10: LZK_SEG(10); break;
    case 16: LZK_SEG(16); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef LZK_SEG
  return (int)hipGetLastError();
}

}  // namespace

// xptr/bptr/sptr: device arrays of nq addresses (bptr/sptr may be null, or
// hold 0 for "none" per query is NOT supported: pass null for the whole batch).
// dtype: 0 = bf16 rows + bf16 queries, 1 = fp32 rows + fp32 queries. Row
// pointers must be 16-B aligned and ld a multiple of 8 (bf16) / 4 (fp32)
// elements; D a multiple of 64 (bf16) / 32 (fp32), D <= 2048.
LZK_EXPORT int lzk_segment_topk(const unsigned long long* xptr, const int* nrows, long ld,
                                const unsigned long long* bptr, const unsigned long long* sptr, const void* Q,
                                long ldq, int nq, int D, int dtype, float alpha, const float* qbias, int kslot,
                                int kout, float* os, long* oi, void* stream) {
  if (nq <= 0) return 0;
  if (D <= 0 || D > SEG_MAXD || kout > kslot) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0) {
    if (D % 64 != 0 || ld % 8 != 0) return (int)hipErrorInvalidValue;
    return launch_segment<u16>(kslot, xptr, nrows, ld, bptr, sptr, Q, ldq, nq, D, alpha, qbias, kout, os, oi, st);
  }
  if (D % 32 != 0 || ld % 4 != 0) return (int)hipErrorInvalidValue;
  return launch_segment<float>(kslot, xptr, nrows, ld, bptr, sptr, Q, ldq, nq, D, alpha, qbias, kout, os, oi, st);
}
