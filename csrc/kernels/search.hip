// Flat (exhaustive) similarity top-k over an HBM-resident vector arena.
//
// Replaces the reference's LanceDB flat kNN (`LanceDBStore.search_nodes`,
// reference src/lazzaro/core/vector_store.py:132-140) and every Python cosine
// loop that ranks candidates (memory_system.py:464-472 super-node scoring,
// :719-733 dedupe, :816-836 / :853-889 linking). See SURVEY.md §2.4 K1-K6.
//
// Design (CDNA4-first, not a translation):
//   * S = X · Qᵀ as an MFMA GEMM (v_mfma_f32_32x32x16_bf16), database rows on
//     the MFMA M axis and queries on N, so each lane's accumulator column is ONE
//     query: top-k selection is lane-local, no cross-lane traffic per tile.
//   * 128 rows x 128 queries per workgroup tile, BK = 64, two LDS buffers with
//     register staging (issue next tile's global loads before the MFMAs, write
//     them to the other buffer after), one barrier per K-step.
//   * LDS images are XOR-swizzled by (row>>1)&7 so every 16-lane group of a
//     ds_read_b128 hits 16 distinct 16-B slots (conflict-free).
//   * Workgroups are persistent over a row chunk; the qblocks of one chunk get
//     consecutive XCD-remapped ids so they stream the same X rows through one L2.
//   * Fused epilogue: score = alpha*dot + bias[row] (L2 / tombstones), optional
//     per-row label filter (tenant / shard), running per-lane top-K kept in
//     registers (threshold compare fast path, insertion rarely taken).
//   * Two-stage: per-(query, chunk) partial top-K, then topk_merge.
#include "lzk_tile.h"

#include <cstdlib>

namespace {

constexpr int BM = 128;       // database rows per tile
constexpr int BN = 128;       // queries per tile
constexpr int BK = 64;        // K per stage
constexpr int NT = 256;       // threads per workgroup (4 waves, 2x2)
constexpr int TILE_ELEMS = BM * BK;  // per operand per stage (bf16 elements)

__device__ __forceinline__ int swz_off(int row, int kc) {
  // element offset of 16-byte chunk kc (0..7) of tile row `row`
  return row * BK + ((kc ^ ((row >> 1) & 7)) << 3);
}

template <int K>
struct TopK {
  float s[K];
  int i[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < K; ++j) { s[j] = LZK_NEG_INF; i[j] = -1; }
  }
  // rows are offered in increasing index order per lane, so a strict compare
  // keeps the smaller index among equal scores.
  __device__ __forceinline__ void push(float v, int r) {
    if (v > s[K - 1]) {
#pragma unroll
      for (int j = K - 1; j > 0; --j) {
        bool up = v > s[j - 1];
        bool here = v > s[j];
        float ns = up ? s[j - 1] : (here ? v : s[j]);
        int ni = up ? i[j - 1] : (here ? r : i[j]);
        s[j] = ns; i[j] = ni;
      }
      if (v > s[0]) { s[0] = v; i[0] = r; }
    }
  }
};

template <int K, bool HAS_BIAS, bool HAS_LABEL, bool GLDS>
__global__ __launch_bounds__(NT, 2) void flat_topk_kernel(
    const u16* __restrict__ X, long ldx, int nrows,
    const u16* __restrict__ Qm, long ldq, int nq,
    const float* __restrict__ bias, const int* __restrict__ row_label,
    const int* __restrict__ q_label, float alpha, int D,
    int rows_per_chunk, int n_chunks, int n_qblocks,
    float* __restrict__ out_s, int* __restrict__ out_i, const int* __restrict__ q_active) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wrow = wave >> 1, wcol = wave & 1;
  const int h = lane >> 5, l32 = lane & 31;

  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = logical / n_qblocks;
  const int qb = logical % n_qblocks;
  if (chunk >= n_chunks) return;
  const int q0 = qb * BN;
  if (q_active) {  // masked re-run: skip query tiles with no active query (block-uniform exit)
    int any = 0;
    for (int t = tid; t < BN; t += NT) any |= (q0 + t < nq) && q_active[q0 + t];
    if (!__syncthreads_or(any)) return;
  }
  const int row_lo = chunk * rows_per_chunk;
  const int row_hi = min(nrows, row_lo + rows_per_chunk);
  const int ntiles = (row_hi > row_lo) ? (row_hi - row_lo + BM - 1) / BM : 0;
  const int KSTEPS = D / BK;
  const int T = ntiles * KSTEPS;

  // per-lane query labels (two query columns per lane)
  int qlab[2] = {-1, -1};
  if (HAS_LABEL) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      int q = q0 + wcol * 64 + cb * 32 + l32;
      qlab[cb] = (q < nq) ? q_label[q] : -1;
    }
  }

  TopK<K> top[2];
  top[0].init(); top[1].init();

  // ---- staging addresses: thread loads 4 chunks of X and 4 of Q per stage ----
  const int srow = tid >> 3;   // 0..31, +32*i
  const int skc = tid & 7;
  const u16* xsrc[4];
  const u16* qsrc[4];
  int soff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r = srow + 32 * i;
    int q = min(q0 + r, nq - 1);
    qsrc[i] = Qm + (long)q * ldq + skc * 8;
    soff[i] = swz_off(r, skc);
  }
  auto set_xsrc = [&](int rt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int r = row_lo + rt * BM + srow + 32 * i;
      r = min(r, nrows - 1);
      xsrc[i] = X + (long)r * ldx + skc * 8;
    }
  };

  // LDS-DMA variant: per-lane pre-swizzled sources, wave-uniform 1 KiB pieces
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const u16* gx[4];
  const u16* gq[4];
  int gpiece[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = wave_u * 4 + i;
    const int row = 8 * c + (lane >> 3);
    const int kc = (lane & 7) ^ ((row >> 1) & 7);
    gq[i] = Qm + (long)min(q0 + row, nq - 1) * ldq + kc * 8;
    gx[i] = X;
    gpiece[i] = c * 512;
  }
  auto set_gx = [&](int rt_) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 8 * (wave_u * 4 + i) + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      gx[i] = X + (long)min(row_lo + rt_ * BM + row, nrows - 1) * ldx + kc * 8;
    }
  };
  float* ebias_g = reinterpret_cast<float*>(smem + 4 * TILE_ELEMS);
  int* elab_g = reinterpret_cast<int*>(ebias_g + 2 * BM);
  auto gissue = [&](int buf, int ks_, int rt_) {
    u16* xs = smem + buf * 2 * TILE_ELEMS;
    u16* qs = xs + TILE_ELEMS;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_global_load_lds((lzk::gbl_void_t*)(gx[i] + ks_ * BK), (lzk::lds_void_t*)(xs + gpiece[i]), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((lzk::gbl_void_t*)(gq[i] + ks_ * BK), (lzk::lds_void_t*)(qs + gpiece[i]), 16, 0, 0);
    }
    if ((HAS_BIAS || HAS_LABEL) && ks_ == 0 && wave_u == 0) {
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int r = min(row_lo + rt_ * BM + h2 * 64 + lane, nrows - 1);
        if (HAS_BIAS)
          __builtin_amdgcn_global_load_lds((lzk::gbl_void_t*)(bias + r), (lzk::lds_void_t*)(ebias_g + (rt_ & 1) * BM + h2 * 64), 4, 0, 0);
        if (HAS_LABEL)
          __builtin_amdgcn_global_load_lds((lzk::gbl_void_t*)(row_label + r), (lzk::lds_void_t*)(elab_g + (rt_ & 1) * BM + h2 * 64), 4, 0, 0);
      }
    }
  };

  u16x8 rx[4], rq[4];
  float rbias = 0.f;
  int rlab = 0;
  // per-row epilogue operands (bias, label) for a row tile live in a small
  // double-buffered LDS area indexed by row-tile parity.
  float* ebias = reinterpret_cast<float*>(smem + 4 * TILE_ELEMS);
  int* elab = reinterpret_cast<int*>(ebias + 2 * BM);
  auto gload = [&](int ks, int rt_) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rx[i] = *reinterpret_cast<const u16x8*>(xsrc[i] + ks * BK);
      rq[i] = *reinterpret_cast<const u16x8*>(qsrc[i] + ks * BK);
    }
    if ((HAS_BIAS || HAS_LABEL) && ks == 0 && tid < BM) {
      int r = min(row_lo + rt_ * BM + tid, nrows - 1);
      if (HAS_BIAS) rbias = bias[r];
      if (HAS_LABEL) rlab = row_label[r];
    }
  };
  auto swrite = [&](int buf, int ks, int rt_) {
    u16* xs = smem + buf * 2 * TILE_ELEMS;
    u16* qs = xs + TILE_ELEMS;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<u16x8*>(xs + soff[i]) = rx[i];
      *reinterpret_cast<u16x8*>(qs + soff[i]) = rq[i];
    }
    if ((HAS_BIAS || HAS_LABEL) && ks == 0 && tid < BM) {
      if (HAS_BIAS) ebias[(rt_ & 1) * BM + tid] = rbias;
      if (HAS_LABEL) elab[(rt_ & 1) * BM + tid] = rlab;
    }
  };

  f32x16 acc[2][2];

  if (T > 0) {
    if (GLDS) {
      set_gx(0);
      gissue(0, 0, 0);
      lzk::vm_drain();
    } else {
      set_xsrc(0);
      gload(0, 0);
      swrite(0, 0, 0);
    }
  }
  __syncthreads();

  int rt = 0, ks = 0;
  for (int t = 0; t < T; ++t) {
    const bool has_next = (t + 1 < T);
    const int nks = (ks + 1 == KSTEPS) ? 0 : ks + 1;
    const int nrt = (ks + 1 == KSTEPS) ? rt + 1 : rt;
    if (has_next) {
      if (GLDS) {
        if (nks == 0) set_gx(nrt);
        gissue((t + 1) & 1, nks, nrt);
      } else {
        if (nks == 0) set_xsrc(nrt);
        gload(nks, nrt);
      }
    }
    if (ks == 0) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
    }
    // ---- MFMA over this K-step ----
    if (GLDS) __builtin_amdgcn_s_setprio(1);
    {
      const u16* xs = smem + (t & 1) * 2 * TILE_ELEMS;
      const u16* qs = xs + TILE_ELEMS;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          int r = wrow * 64 + rb * 32 + l32;
          af[rb] = *reinterpret_cast<const bf16x8*>(xs + swz_off(r, 2 * s + h));
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          int r = wcol * 64 + cb * 32 + l32;
          bfr[cb] = *reinterpret_cast<const bf16x8*>(qs + swz_off(r, 2 * s + h));
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[rb], bfr[cb], acc[rb][cb], 0, 0, 0);
      }
    }
    if (GLDS) __builtin_amdgcn_s_setprio(0);
    // ---- fused top-k epilogue at the end of a row tile ----
    if (ks == KSTEPS - 1) {
      const int lrow0 = wrow * 64 + 4 * h;
      const int tile0 = row_lo + rt * BM + lrow0;
      const float* eb = ebias + (rt & 1) * BM + lrow0;
      const int* el = elab + (rt & 1) * BM + lrow0;
      const bool full_tile = row_lo + (rt + 1) * BM <= row_hi;  // wave-uniform
      auto score = [&](int rb, int cb, int e) -> float {
        float x = alpha * acc[rb][cb][e];
        if (HAS_BIAS) x += eb[rb * 32 + 8 * (e >> 2) + (e & 3)];
        bool ok = true;
        if (!full_tile) ok = tile0 + rb * 32 + (e & 3) + 8 * (e >> 2) < row_hi;
        if (HAS_LABEL) ok = ok && (qlab[cb] < 0 || el[rb * 32 + 8 * (e >> 2) + (e & 3)] == qlab[cb]);
        return ok ? x : LZK_NEG_INF;
      };
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          // pre-filter: block max vs the lane's current k-th score; the
          // per-score insertion path below is rare after warm-up
          float m = LZK_NEG_INF;
#pragma unroll
          for (int e = 0; e < 16; ++e) m = fmaxf(m, score(rb, cb, e));
          if (m > top[cb].s[K - 1]) {
#pragma unroll
            for (int e = 0; e < 16; ++e)
              top[cb].push(score(rb, cb, e), tile0 + rb * 32 + (e & 3) + 8 * (e >> 2));
          }
        }
      }
    }
    if (GLDS) {
      lzk::vm_drain();
    } else if (has_next) {
      swrite((t + 1) & 1, nks, nrt);
    }
    __syncthreads();
    ks = nks; rt = nrt;
  }

  // ---- merge the 4 per-query lane lists (2 row-waves x 2 half-waves) ----
  float* ms = reinterpret_cast<float*>(smem);
  int* mi = reinterpret_cast<int*>(smem) + BN * 4 * K;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    int ql = wcol * 64 + cb * 32 + l32;
    int li = wrow * 2 + h;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      ms[(ql * 4 + li) * K + j] = top[cb].s[j];
      mi[(ql * 4 + li) * K + j] = top[cb].i[j];
    }
  }
  __syncthreads();
  if (tid < BN) {
    const int ql = tid;
    const int q = q0 + ql;
    if (q < nq) {
      int p0 = 0, p1 = 0, p2 = 0, p3 = 0;
      const float* bs = ms + ql * 4 * K;
      const int* bi = mi + ql * 4 * K;
      long obase = ((long)q * n_chunks + chunk) * K;
      for (int j = 0; j < K; ++j) {
        float bsv = LZK_NEG_INF; int biv = -1; int w = -1;
        if (p0 < K) { float s = bs[0 * K + p0]; int i = bi[0 * K + p0]; if (w < 0 || better(s, i, bsv, biv)) { bsv = s; biv = i; w = 0; } }
        if (p1 < K) { float s = bs[1 * K + p1]; int i = bi[1 * K + p1]; if (w < 0 || better(s, i, bsv, biv)) { bsv = s; biv = i; w = 1; } }
        if (p2 < K) { float s = bs[2 * K + p2]; int i = bi[2 * K + p2]; if (w < 0 || better(s, i, bsv, biv)) { bsv = s; biv = i; w = 2; } }
        if (p3 < K) { float s = bs[3 * K + p3]; int i = bi[3 * K + p3]; if (w < 0 || better(s, i, bsv, biv)) { bsv = s; biv = i; w = 3; } }
        p0 += (w == 0); p1 += (w == 1); p2 += (w == 2); p3 += (w == 3);
        out_s[obase + j] = bsv;
        out_i[obase + j] = (bsv == LZK_NEG_INF) ? -1 : biv;
      }
    }
  }
}

// Merge per-(query, chunk) partial lists into the final top-k. One wave per
// query: lane-local candidate lists, then k rounds of a wave-wide argmax.
template <int K>
__global__ __launch_bounds__(256) void topk_merge_kernel(
    const float* __restrict__ ps, const int* __restrict__ pi, int ncand, int nq,
    int kout, long idx_offset, float* __restrict__ os, long* __restrict__ oi, const int* __restrict__ q_active) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  if (q_active && !q_active[q]) return;
  TopK<K> top;
  top.init();
  const float* s = ps + (long)q * ncand;
  const int* ix = pi + (long)q * ncand;
  for (int c = lane; c < ncand; c += 64) {
    float v = s[c];
    int r = ix[c];
    if (r < 0) continue;
    // lists arrive in arbitrary index order: insert with the full (score, idx) order
    if (better(v, r, top.s[K - 1], top.i[K - 1] < 0 ? 0x7fffffff : top.i[K - 1])) {
#pragma unroll
      for (int j = K - 1; j > 0; --j) {
        int ij1 = top.i[j - 1] < 0 ? 0x7fffffff : top.i[j - 1];
        int ij = top.i[j] < 0 ? 0x7fffffff : top.i[j];
        bool up = better(v, r, top.s[j - 1], ij1);
        bool here = better(v, r, top.s[j], ij);
        float ns = up ? top.s[j - 1] : (here ? v : top.s[j]);
        int ni = up ? top.i[j - 1] : (here ? r : top.i[j]);
        top.s[j] = ns; top.i[j] = ni;
      }
      int i0 = top.i[0] < 0 ? 0x7fffffff : top.i[0];
      if (better(v, r, top.s[0], i0)) { top.s[0] = v; top.i[0] = r; }
    }
  }
  for (int j = 0; j < kout; ++j) {
    float hs = top.s[0];
    int hi = top.i[0] < 0 ? 0x7fffffff : top.i[0];
    float bs = hs; int bi = hi;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      float s2 = __shfl_xor(bs, o, 64);
      int i2 = __shfl_xor(bi, o, 64);
      if (better(s2, i2, bs, bi)) { bs = s2; bi = i2; }
    }
    if (lane == 0) {
      os[(long)q * kout + j] = bs;
      oi[(long)q * kout + j] = (bi == 0x7fffffff || bs == LZK_NEG_INF) ? -1 : (long)bi + idx_offset;
    }
    if (hi == bi && hs == bs && bi != 0x7fffffff) {
#pragma unroll
      for (int t = 0; t < K - 1; ++t) { top.s[t] = top.s[t + 1]; top.i[t] = top.i[t + 1]; }
      top.s[K - 1] = LZK_NEG_INF; top.i[K - 1] = -1;
    }
  }
}

// K2 across ranks: merge the all-gathered candidate lists [nq, ncand] whose
// ids are GLOBAL 64-bit keys (row offset + local row, or tenant<<32 | row)
// into the exact top-kout by (score desc, id asc); id < 0 marks an empty slot.
// One wave per query; every lane keeps a sorted K-list of its strided share,
// then kout rounds of a wave-wide (score, id) argmax pop the global order.
// Replaces two full argsorts of [nq, world*k] (parallel/sharded.py merge_topk).
__device__ __forceinline__ bool better64(float a, long ia, float b, long ib) {
  return a > b || (a == b && ia < ib);
}

template <int K>
__global__ __launch_bounds__(256) void topk_merge64_kernel(
    const float* __restrict__ ps, const long* __restrict__ pi, int ncand, int nq,
    int kout, float* __restrict__ os, long* __restrict__ oi) {
  constexpr long NONE = 0x7fffffffffffffffL;
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;  // whole wave exits together (q is wave-uniform)
  float ts[K];
  long ti[K];
#pragma unroll
  for (int j = 0; j < K; ++j) { ts[j] = LZK_NEG_INF; ti[j] = NONE; }
  const float* s = ps + (long)q * ncand;
  const long* ix = pi + (long)q * ncand;
  for (int c = lane; c < ncand; c += 64) {
    float v = s[c];
    long r = ix[c];
    if (r < 0) continue;
    if (better64(v, r, ts[K - 1], ti[K - 1])) {
#pragma unroll
      for (int j = K - 1; j > 0; --j) {
        bool up = better64(v, r, ts[j - 1], ti[j - 1]);
        bool here = better64(v, r, ts[j], ti[j]);
        float ns = up ? ts[j - 1] : (here ? v : ts[j]);
        long ni = up ? ti[j - 1] : (here ? r : ti[j]);
        ts[j] = ns; ti[j] = ni;
      }
      if (better64(v, r, ts[0], ti[0])) { ts[0] = v; ti[0] = r; }
    }
  }
  for (int j = 0; j < kout; ++j) {
    float hs = ts[0];
    long hi = ti[0];
    float bs = hs; long bi = hi;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      float s2 = __shfl_xor(bs, o, 64);
      long i2 = __shfl_xor(bi, o, 64);
      if (better64(s2, i2, bs, bi)) { bs = s2; bi = i2; }
    }
    if (lane == 0) {
      os[(long)q * kout + j] = bs;
      oi[(long)q * kout + j] = (bi == NONE) ? -1 : bi;
    }
    // ids are unique per query, so exactly one lane owns the winner
    if (hi == bi && hs == bs && bi != NONE) {
#pragma unroll
      for (int t = 0; t < K - 1; ++t) { ts[t] = ts[t + 1]; ti[t] = ti[t + 1]; }
      ts[K - 1] = LZK_NEG_INF; ti[K - 1] = NONE;
    }
  }
}

int g_search_staging = -1;  // 1 = LDS-DMA (default), 0 = register staging (LZK_STAGING=reg)

int search_staging() {
  if (g_search_staging < 0) g_search_staging = 1;
  return g_search_staging;
}

template <int K>
hipError_t launch_flat(const u16* X, long ldx, int nrows, const u16* Qm, long ldq, int nq,
                       const float* bias, const int* row_label, const int* q_label,
                       float alpha, int D, int n_chunks, float* ps, int* pi,
                       hipStream_t st, const int* q_active) {
  int n_qblocks = (nq + BN - 1) / BN;
  int rows_per_chunk = ((nrows + n_chunks - 1) / n_chunks + BM - 1) / BM * BM;
  n_chunks = (nrows + rows_per_chunk - 1) / rows_per_chunk;
  if (n_chunks < 1) n_chunks = 1;
  size_t lds = (size_t)2 * 2 * TILE_ELEMS * sizeof(u16) + 2 * BM * 8;
  size_t lds_merge = (size_t)BN * 4 * K * 8;
  if (lds_merge > lds) lds = lds_merge;
  dim3 grid(n_qblocks * n_chunks);
#define LZK_GO(B, L, G) do { \
  (void)hipFuncSetAttribute((const void*)flat_topk_kernel<K, B, L, G>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
  hipLaunchKernelGGL((flat_topk_kernel<K, B, L, G>), grid, dim3(NT), lds, st, X, ldx, nrows, Qm, ldq, nq, \
                     bias, row_label, q_label, alpha, D, rows_per_chunk, n_chunks, n_qblocks, ps, pi, q_active); } while (0)
  if (search_staging() == 1) {
    if (bias && row_label) LZK_GO(true, true, true);
    else if (bias) LZK_GO(true, false, true);
    else if (row_label) LZK_GO(false, true, true);
    else LZK_GO(false, false, true);
  } else {
    if (bias && row_label) LZK_GO(true, true, false);
    else if (bias) LZK_GO(true, false, false);
    else if (row_label) LZK_GO(false, true, false);
    else LZK_GO(false, false, false);
  }
#undef LZK_GO
  return hipGetLastError();
}

}  // namespace

LZK_EXPORT void lzk_set_search_staging(int glds) { g_search_staging = glds; }

// Number of row chunks the partial buffers must be sized for.
LZK_EXPORT int lzk_flat_topk_chunks(int nrows, int nq, int target_wgs) {
  int n_qblocks = (nq + BN - 1) / BN;
  int n_chunks = (target_wgs + n_qblocks - 1) / n_qblocks;
  int max_chunks = (nrows + BM - 1) / BM;
  if (n_chunks > max_chunks) n_chunks = max_chunks;
  if (n_chunks < 1) n_chunks = 1;
  int rows_per_chunk = ((nrows + n_chunks - 1) / n_chunks + BM - 1) / BM * BM;
  return (nrows + rows_per_chunk - 1) / rows_per_chunk;
}

LZK_EXPORT int lzk_flat_topk_kslot(int k) {
  if (k <= 1) return 1;
  if (k <= 2) return 2;
  if (k <= 4) return 4;
  if (k <= 8) return 8;
  if (k <= 10) return 10;
  if (k <= 16) return 16;
  return -1;
}

// Partial pass: ps/pi are [nq, n_chunks, kslot]. q_active (optional): only
// query tiles holding an active query are computed (the rest of ps/pi is
// left untouched) -- the device-side fallback of the candidate path.
static int flat_partial(const void* X, long ldx, int nrows, const void* Qm, long ldq, int nq, const float* bias,
                        const int* row_label, const int* q_label, float alpha, int D, int kslot, int n_chunks,
                        float* ps, int* pi, void* stream, const int* q_active) {
  if (D % BK != 0 || nq <= 0 || nrows <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  const u16* q = (const u16*)Qm;
#define LZK_KS(KK) return launch_flat<KK>(x, ldx, nrows, q, ldq, nq, bias, row_label, q_label, alpha, D, n_chunks, ps, pi, st, q_active)
  switch (kslot) {
    case 1: LZK_KS(1);
    case 2: LZK_KS(2);
    case 4: LZK_KS(4);
    case 8: LZK_KS(8);
    case 10: LZK_KS(10);
    case 16: LZK_KS(16);
    default: return (int)hipErrorInvalidValue;
  }
#undef LZK_KS
}

LZK_EXPORT int lzk_flat_topk_partial(const void* X, long ldx, int nrows, const void* Qm, long ldq,
                                     int nq, const float* bias, const int* row_label,
                                     const int* q_label, float alpha, int D, int kslot,
                                     int n_chunks, float* ps, int* pi, void* stream) {
  return flat_partial(X, ldx, nrows, Qm, ldq, nq, bias, row_label, q_label, alpha, D, kslot, n_chunks, ps, pi,
                      stream, nullptr);
}

LZK_EXPORT int lzk_flat_topk_partial_masked(const void* X, long ldx, int nrows, const void* Qm, long ldq, int nq,
                                            const float* bias, const int* row_label, const int* q_label,
                                            float alpha, int D, int kslot, int n_chunks, float* ps, int* pi,
                                            const int* q_active, void* stream) {
  return flat_partial(X, ldx, nrows, Qm, ldq, nq, bias, row_label, q_label, alpha, D, kslot, n_chunks, ps, pi,
                      stream, q_active);
}

static int topk_merge(const float* ps, const int* pi, int ncand, int nq, int kslot, int kout, long idx_offset,
                      float* os, long* oi, void* stream, const int* q_active) {
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((nq + 3) / 4), block(256);
  if (kout > kslot) return (int)hipErrorInvalidValue;
#define LZK_M(KK) hipLaunchKernelGGL(topk_merge_kernel<KK>, grid, block, 0, st, ps, pi, ncand, nq, kout, idx_offset, os, oi, q_active)
  switch (kslot) {
    case 1: LZK_M(1); break;
    case 2: LZK_M(2); break;
    case 4: LZK_M(4); break;
    case 8: LZK_M(8); break;
    case 10: LZK_M(10); break;
    case 16: LZK_M(16); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef LZK_M
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_topk_merge(const float* ps, const int* pi, int ncand, int nq, int kslot,
                              int kout, long idx_offset, float* os, long* oi, void* stream) {
  return topk_merge(ps, pi, ncand, nq, kslot, kout, idx_offset, os, oi, stream, nullptr);
}

// Cross-rank merge of all-gathered candidates with 64-bit global ids:
// ps/pi [nq, ncand] -> os/oi [nq, kout], kout <= 32. Each lane's list holds
// the best K of its share, so kout <= K keeps the result exact.
LZK_EXPORT int lzk_topk_merge64(const float* ps, const long* pi, int ncand, int nq, int kout, float* os, long* oi,
                                void* stream) {
  if (nq <= 0) return 0;
  if (kout < 1 || ncand < 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((nq + 3) / 4), block(256);
#define LZK_M64(KK) hipLaunchKernelGGL(topk_merge64_kernel<KK>, grid, block, 0, st, ps, pi, ncand, nq, kout, os, oi)
  if (kout <= 4) LZK_M64(4);
  else if (kout <= 10) LZK_M64(10);
  else if (kout <= 16) LZK_M64(16);
  else if (kout <= 32) LZK_M64(32);
  else return (int)hipErrorInvalidValue;
#undef LZK_M64
  return (int)hipGetLastError();
}

// Merge only the active queries' rows of os/oi (others untouched).
LZK_EXPORT int lzk_topk_merge_masked(const float* ps, const int* pi, int ncand, int nq, int kslot, int kout,
                                     long idx_offset, float* os, long* oi, const int* q_active, void* stream) {
  return topk_merge(ps, pi, ncand, nq, kslot, kout, idx_offset, os, oi, stream, q_active);
}
