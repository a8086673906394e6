// Global (cross-tenant) search over the small tenants of a rank in ONE MFMA
// pass (every query against every resident tenant; the
// reference serves one tenant per MemorySystem, memory_system.py:1430-1439
// lists them and :1460-1472 searches one).
//
// Each small tenant keeps its own column allocations (TenantGraph), so the
// rank's rows are not one matrix. A host-built TILE TABLE turns them into
// one: tile t = up to 256 consecutive rows of one tenant, described by the
// address of its first bf16 row, of its first store-bias entry and its row
// count. The candidate pass is the 256x256 bf16 MFMA pipeline of
// lzk_g256.h over (tile, 256-query block) pairs -- a tenant of 800 rows is 4
// tiles, so padding costs < 1/4 of a tile per tenant -- with the sampled
// threshold of search256.hip: a query keeps every row whose bf16 score
// clears a lower bound of its k-th best (the exact top-k of a strided 1/64
// sample of the table's rows, gathered by mt_sample_kernel). The candidate id
// is tile * 256 + row-in-tile; cand_select_kernel picks each query's best
// candidates, and mt_rerank_kernel re-scores them exactly in fp32 from the
// tenants' stored vectors (the store search's own re-rank, tenant.hip
// store_rerank_kernel), resolves (tenant slot, row) through the tile table and
// drops rows that are not live nodes.
#include "lzk_g256.h"

namespace {

using namespace g256;

constexpr int MT_NODE = 1;  // TenantGraph kind of a live node

// score = alpha * <q, x> + bias[row]; rows past the tile's count are empty.
__global__ __launch_bounds__(NT, 1) void mt_cand_kernel(const long* __restrict__ t_x, const long* __restrict__ t_b,
                                                        const int* __restrict__ t_n, long ldx,
                                                        const u16* __restrict__ Qm, long ldq, int nq, int D,
                                                        float alpha, const float* __restrict__ thr, int n_qt, int cap,
                                                        int* __restrict__ cnt, float* __restrict__ cs,
                                                        int* __restrict__ ci) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = logical / n_qt, qt = logical % n_qt;
  const int q0 = qt * BN;
  const u16* X = reinterpret_cast<const u16*>(t_x[tile]);
  const float* bias = reinterpret_cast<const float*>(t_b[tile]);
  const int nrows = t_n[tile];

  Stager st;
  st.setup(X, ldx, 0, nrows, Qm, ldq, q0, nq);
  f32x4 acc[8][4];
  mainloop(smem, st, D / BK, acc);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  int qq[4];
  float th[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = q0 + wc * 64 + j * 16 + (lane & 15);
    qq[j] = q;
    th[j] = (q < nq) ? thr[q] : __builtin_huge_valf();
  }
  const int vbase = tile * BM;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rb = wr * 128 + i * 16 + 4 * (lane >> 4);
    float bv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[e] = bias[min(rb + e, nrows - 1)];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s[4];
      float m = LZK_NEG_INF;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[e] = (rb + e < nrows) ? alpha * acc[i][j][e] + bv[e] : LZK_NEG_INF;
        m = fmaxf(m, s[e]);
      }
      if (m >= th[j]) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (s[e] >= th[j] && s[e] != LZK_NEG_INF) {
            const int pos = atomicAdd(cnt + qq[j], 1);
            if (pos < cap) {
              cs[(long)qq[j] * cap + pos] = s[e];
              ci[(long)qq[j] * cap + pos] = vbase + rb + e;
            }
          }
        }
      }
    }
  }
}

// Sample row s = (tile s_tile[s], row s_row[s]) -> contiguous bf16 rows + bias.
__global__ __launch_bounds__(128) void mt_sample_kernel(const long* __restrict__ t_x, const long* __restrict__ t_b,
                                                        const int* __restrict__ s_tile, const int* __restrict__ s_row,
                                                        long ldx, int Dp, u16* __restrict__ out,
                                                        float* __restrict__ outb) {
  const int s = blockIdx.x;
  const int t = s_tile[s], r = s_row[s];
  const u16* src = reinterpret_cast<const u16*>(t_x[t]) + (long)r * ldx;
  u16* dst = out + (long)s * Dp;
  for (int c = threadIdx.x * 8; c < Dp; c += 128 * 8)
    *reinterpret_cast<u16x8*>(dst + c) = *reinterpret_cast<const u16x8*>(src + c);
  if (threadIdx.x == 0) outb[s] = reinterpret_cast<const float*>(t_b[t])[r];
}

// Exact fp32 re-rank of each query's C candidate ids (tile * 256 + row in
// tile, -1 = none): score = 2<q,x> + bias[row] - |q|^2 (L2, metric 0) or
// <q,x> + bias[row] (ip, metric 1) from the tenant's fp32 rows; top-k by
// (score desc, key asc), key = slot << 32 | row; then rows that are not live
// nodes become (-inf, -1), as the per-tenant path filters its results. One
// wave per query, 4 lanes per candidate (store_rerank_kernel's layout).
__global__ __launch_bounds__(256) void mt_rerank_kernel(const float* __restrict__ Q, long ldq, int D,
                                                        const long* __restrict__ cand, int C, int M, int k,
                                                        const int* __restrict__ t_slot, const int* __restrict__ t_row0,
                                                        const long* __restrict__ p_e32, const long* __restrict__ p_bias,
                                                        const long* __restrict__ p_kind, int metric,
                                                        float* __restrict__ os, long* __restrict__ okey) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= M) return;
  const float* qr = Q + (long)q * ldq;
  float qq = 0.f;
  for (int d = lane; d < D; d += 64) qq = fmaf(qr[d], qr[d], qq);
  qq = wave_sum(qq);
  const int part = lane & 3, cl = lane >> 2;
  float my_s = LZK_NEG_INF;
  long my_k = -1;
  const bool vec = (D % 16) == 0 && (ldq % 4) == 0;
  for (int c0 = 0; c0 < C; c0 += 16) {
    const int c = c0 + cl;
    const long v = c < C ? cand[(long)q * C + c] : -1;
    float acc = 0.f;
    int slot = -1, row = -1;
    if (v >= 0) {
      const int t = (int)(v >> 8);
      slot = t_slot[t];
      row = t_row0[t] + (int)(v & 255);
      const float* xr = reinterpret_cast<const float*>(p_e32[slot]) + (long)row * D;
      if (vec) {
        for (int d = part * 4; d < D; d += 16) {
          const float4 xv = *reinterpret_cast<const float4*>(xr + d);
          const float4 qv = *reinterpret_cast<const float4*>(qr + d);
          acc = fmaf(qv.x, xv.x, acc);
          acc = fmaf(qv.y, xv.y, acc);
          acc = fmaf(qv.z, xv.z, acc);
          acc = fmaf(qv.w, xv.w, acc);
        }
      } else {
        for (int d = part; d < D; d += 4) acc = fmaf(qr[d], xr[d], acc);
      }
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    float sc = LZK_NEG_INF;
    long key = -1;
    if (v >= 0) {
      const float b = reinterpret_cast<const float*>(p_bias[slot])[row];
      sc = metric == 0 ? 2.f * acc + b - qq : acc + b;
      key = ((long)slot << 32) | (long)row;
    }
    const int src = 4 * ((lane - c0) & 15);
    const float s2 = __shfl(sc, src, 64);
    const long k2 = __shfl(key, src, 64);
    if (lane >= c0 && lane < c0 + 16 && lane < C) { my_s = s2; my_k = k2; }
  }
  const bool live = lane < C && my_k >= 0 && my_s != LZK_NEG_INF;
  int rank = 0;
  for (int o = 0; o < C; ++o) {
    const float s2 = __shfl(my_s, o, 64);
    const long k2 = __shfl(my_k, o, 64);
    const bool l2 = k2 >= 0 && s2 != LZK_NEG_INF;
    if (l2 && o != lane && (s2 > my_s || (s2 == my_s && k2 < my_k))) ++rank;
  }
  const int nlive = __popcll(__ballot(live));
  if (live && rank < k) {
    const int slot = (int)(my_k >> 32), row = (int)(my_k & 0xFFFFFFFF);
    const bool node = reinterpret_cast<const unsigned char*>(p_kind[slot])[row] == MT_NODE;
    os[(long)q * k + rank] = node ? my_s : LZK_NEG_INF;
    okey[(long)q * k + rank] = node ? my_k : -1;
  }
  for (int j = nlive + lane; j < k; j += 64) {
    os[(long)q * k + j] = LZK_NEG_INF;
    okey[(long)q * k + j] = -1;
  }
}

}  // namespace

// Candidate pass over a tile table (t_x / t_b: int64 addresses of each tile's
// first bf16 row / bias entry, t_n: its row count 1..256; row stride ldx
// elements for every tile). cnt [nq] zeroed by the caller; cs / ci [nq, cap].
LZK_EXPORT int lzk_mt_cand(const long* t_x, const long* t_b, const int* t_n, int n_tiles, long ldx, const void* Qm,
                           long ldq, int nq, int D, float alpha, const float* thr, int cap, int* cnt, float* cs,
                           int* ci, void* stream) {
  if (D % BK != 0 || nq <= 0 || n_tiles <= 0 || cap <= 0 || ldx < D || ldq < D) return (int)hipErrorInvalidValue;
  if ((long)n_tiles * BM > 0x7fffffffL) return (int)hipErrorInvalidValue;  // candidate ids are int32
  const int n_qt = (nq + BN - 1) / BN;
  const long nblk = (long)n_tiles * n_qt;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  (void)hipFuncSetAttribute((const void*)mt_cand_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
  hipLaunchKernelGGL(mt_cand_kernel, dim3((unsigned)nblk), dim3(NT), LDS_BYTES, st, t_x, t_b, t_n, ldx,
                     (const u16*)Qm, ldq, nq, D, alpha, thr, n_qt, cap, cnt, cs, ci);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_mt_sample(const long* t_x, const long* t_b, const int* s_tile, const int* s_row, int ns, long ldx,
                             int Dp, void* out, float* outb, void* stream) {
  if (ns <= 0 || Dp % 8 != 0 || ldx < Dp) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mt_sample_kernel, dim3((unsigned)ns), dim3(128), 0, (hipStream_t)stream, t_x, t_b, s_tile, s_row,
                     ldx, Dp, (u16*)out, outb);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_mt_rerank(const float* Q, long ldq, int D, const long* cand, int C, int M, int k, const int* t_slot,
                             const int* t_row0, const long* p_e32, const long* p_bias, const long* p_kind, int metric,
                             float* os, long* okey, void* stream) {
  if (C <= 0 || C > 64 || k <= 0 || k > C || M <= 0 || ldq < D) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mt_rerank_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, (hipStream_t)stream, Q, ldq, D,
                     cand, C, M, k, t_slot, t_row0, p_e32, p_bias, p_kind, metric, os, okey);
  return (int)hipGetLastError();
}
