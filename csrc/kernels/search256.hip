// Flat top-k, large-batch path: threshold-filtered candidate generation on the
// 256x256 8-wave MFMA pipeline (lzk_g256.h), then an exact per-query select.
//
// Same contract as flat_topk_kernel in search.hip (reference
// src/lazzaro/core/vector_store.py:132-140 search_nodes):
// score = alpha * <x, q> + bias[row], rows with a different label than the
// query's (label >= 0) excluded, results ordered by (score desc, row asc).
//
// Why a different algorithm at Q >= 256 and N in the millions: a per-lane
// running top-K costs 2K registers per query column and an insertion network
// per tile, which caps the tile at 128x128 with 4 waves. Here the top-K state
// is replaced by ONE number per query, a lower bound `thr[q]` of its k-th best
// score, taken from an exact top-k over a strided 1/S sample of the rows (the
// k-th best of a subset never exceeds the k-th best of the whole). Every
// score >= thr[q] is appended to the query's candidate list (expected ~k*S
// of N rows); the epilogue is one compare per score, so the 256x256 tile can
// spend its registers on MFMA accumulators. A query whose list overflows its
// capacity is flagged and recomputed by the caller with the per-lane kernel.
#include "lzk_g256.h"

#include <cstdlib>
#include <cfloat>
#include <map>
#include <mutex>

LZK_DEBUG_STATE(search256)

namespace {

using namespace g256;

// Diagnostic stamps (OPT bit 8, never in a default build's path): wave 0
// lane 0 of each block records s_memtime around the phases of its first
// kStampTiles tiles into g_stamps[block][tile][4]: before the K loop's
// first wait, after it, after the K loop, after the epilogue.
constexpr int kStampTiles = 32;
__device__ unsigned long long* g_stamps = nullptr;

template <bool HAS_BIAS, bool HAS_LABEL>
__global__ __launch_bounds__(NT, 1) void flat_cand_kernel(
    const u16* __restrict__ X, long ldx, int nrows, const u16* __restrict__ Qm, long ldq, int nq, int D,
    const float* __restrict__ bias, const int* __restrict__ row_label, const int* __restrict__ q_label,
    float alpha, const float* __restrict__ thr, int n_qt, int cap, int* __restrict__ cnt,
    float* __restrict__ cs, int* __restrict__ ci) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = logical / n_qt, qt = logical % n_qt;
  const int r0 = rt * BM, q0 = qt * BN;

  Stager st;
  st.setup(X, ldx, r0, nrows, Qm, ldq, q0, nq);
  f32x4 acc[8][4];
  mainloop(smem, st, D / BK, acc);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  int qq[4], ql[4];
  float th[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = q0 + wc * 64 + j * 16 + (lane & 15);
    qq[j] = q;
    th[j] = (q < nq) ? thr[q] : __builtin_huge_valf();
    ql[j] = (HAS_LABEL && q < nq) ? q_label[q] : -1;
  }
  const bool full = r0 + BM <= nrows;  // wave-uniform
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rb = r0 + wr * 128 + i * 16 + 4 * (lane >> 4);
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    int lv[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = min(rb + e, nrows - 1);
      if (HAS_BIAS) bv[e] = bias[r];
      if (HAS_LABEL) lv[e] = row_label[r];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s[4];
      float m = LZK_NEG_INF;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[e] = alpha * acc[i][j][e] + bv[e];
        bool ok = full || (rb + e < nrows);
        if (HAS_LABEL) ok = ok && (ql[j] < 0 || lv[e] == ql[j]);
        s[e] = ok ? s[e] : LZK_NEG_INF;
        m = fmaxf(m, s[e]);
      }
      if (m >= th[j]) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (s[e] >= th[j] && s[e] != LZK_NEG_INF) {
            const int pos = atomicAdd(cnt + qq[j], 1);
            if (pos < cap) {
              cs[(long)qq[j] * cap + pos] = s[e];
              ci[(long)qq[j] * cap + pos] = rb + e;
            }
          }
        }
      }
    }
  }
}

// Persistent variant: one block per CU walks its XCD's tiles; the next
// tile's prologue DMA (operand half-tiles AND its epilogue operands: bias,
// row labels, thresholds, query labels -> spare LDS, double-buffered by tile
// parity) is issued before this tile's epilogue, so the pipeline fill of
// tile i+1 overlaps the epilogue of tile i and no epilogue global load can
// drain the in-flight DMA.
constexpr int EPI_OFF = 8 * HALF;               // u16 offset of the epilogue area (128 KiB)
constexpr int EPI_ARRAYS = 7;  // thr | bias | row label | query label | thr2 | row scale | query scale (int8)
constexpr int CNT_OFF = EPI_OFF + 2 * EPI_ARRAYS * 256 * 2;  // u16 offset of the block's append counter
constexpr int CAND_P_LDS = LDS_BYTES + 2 * EPI_ARRAYS * 256 * 4 + 16;
typedef __attribute__((address_space(3))) int lds_int;

// Candidate appends go to a block-private region (no returning global
// atomic in the scan): the slot comes from an LDS counter (ds_add_rtn, an
// lgkmcnt wait) and the (query, row, score, list) record is a plain 16-B
// store. A returning global atomic would make the compiler wait vmcnt(0) --
// i.e. for the next tile's in-flight operand DMA -- in the middle of the
// epilogue, and would break the counted vmcnt at the next K loop's start.
// cand_gather_kernel then files the records into the per-query lists. A
// record that does not fit marks its query overflowed (exact fallback).
struct BlkCands {
  int4* buf;  // [grid][cap]
  int cap;
  int* cnt;   // [grid] records written
  // int8 scan (MMA::kInt) only: fp32 row / query scales, staged into the
  // epilogue's slots 5 / 6 with the other per-tile operands
  const float* rs = nullptr;
  const float* qs = nullptr;
};

// DUAL: one GEMM pass serves two searches of the same queries -- list A keeps
// every row with score >= thr[q] (no label filter), list B keeps rows whose
// label equals the query's and score >= thr2[q]. Consolidation needs exactly
// this pair (global dedupe/links + within-shard links, reference
// memory_system.py:719-733 / :816-836 / :853-889) and the scan is MFMA-bound,
// so fusing halves its cost.
// MMA = MmaFp8: the rows / queries are e4m3 bytes passed as u16 pairs (row
// strides and D in u16 units), so one 128-B K-row feeds the block-scaled
// 16x16x128 MFMA at twice the bf16 rate -- same LDS image and schedule.
template <bool HAS_BIAS, bool HAS_LABEL, bool DUAL, int OPT = 0, class MMA = MmaBf16>
__global__ __launch_bounds__(NT, 1) void flat_cand_persistent_kernel(
    const u16* __restrict__ X, long ldx, int nrows, const u16* __restrict__ Qm, long ldq, int nq, int D,
    const float* __restrict__ bias, const int* __restrict__ row_label, const int* __restrict__ q_label,
    float alpha, const float* __restrict__ thr, int n_qt, int n_tiles, int cap, int* __restrict__ cnt,
    float* __restrict__ cs, int* __restrict__ ci, const float* __restrict__ thr2, int* __restrict__ cnt2,
    float* __restrict__ cs2, int* __restrict__ ci2, BlkCands blk) {
  static_assert(!DUAL || HAS_LABEL, "dual search needs labels");
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  float* epi = reinterpret_cast<float*>(smem + EPI_OFF);  // [parity][array][256]
  lds_int* lcnt = (lds_int*)(smem + CNT_OFF);
  if (threadIdx.x == 0) *lcnt = 0;  // ordered before any append by the K loop's barriers
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int KS = D / BK;

  TileWalk walk;
  walk.init(n_tiles);
  int tile = walk.next;
  if (!walk.valid(tile)) {
    if (threadIdx.x == 0) blk.cnt[blockIdx.x] = 0;
    return;
  }

  // 4 wave-level DMAs (64 x 4 B) per array, spread over the 8 waves
  auto stage_epi = [&](int tl, int par) {
    const int r0 = (tl / n_qt) * BM, q0 = (tl % n_qt) * BN;
#pragma unroll
    for (int g = wave; g < 4 * EPI_ARRAYS; g += 8) {
      const int a = g >> 2, c = g & 3;  // wave-uniform
      const bool need = a == 0 || (a == 1 && HAS_BIAS) || ((a == 2 || a == 3) && HAS_LABEL) || (a == 4 && DUAL) ||
                        ((a == 5 || a == 6) && MMA::kInt);
      if (!need) continue;
      const void* src;
      if (a == 0) src = thr + min(q0 + c * 64 + lane, nq - 1);
      else if (a == 1) src = bias + min(r0 + c * 64 + lane, nrows - 1);
      else if (a == 2) src = row_label + min(r0 + c * 64 + lane, nrows - 1);
      else if (a == 3) src = q_label + min(q0 + c * 64 + lane, nq - 1);
      else if (a == 4) src = thr2 + min(q0 + c * 64 + lane, nq - 1);
      else if (a == 5) src = blk.rs + min(r0 + c * 64 + lane, nrows - 1);
      else src = blk.qs + min(q0 + c * 64 + lane, nq - 1);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                       (lds_void_t*)(epi + par * (EPI_ARRAYS * 256) + a * 256 + c * 64), 4, 0, 0);
    }
  };

  // one record per (query, row) with its list mask (bit 0: list A, bit 1:
  // list B): one append site per score keeps the fully unrolled epilogue
  // small -- the kernel's code must stay inside the CU's instruction cache
  auto append = [&](int lists, int q, float v, int r) {
    const int pos = __atomic_fetch_add(lcnt, 1, __ATOMIC_RELAXED);
    if (pos < blk.cap) blk.buf[(long)blockIdx.x * blk.cap + pos] = make_int4(q, r, __float_as_int(v), lists);
  };

  Stager st;
  st.setup(X, ldx, (tile / n_qt) * BM, nrows, Qm, ldq, (tile % n_qt) * BN, nq);
  auto ex0 = [&]() { stage_epi(tile, 0); };
  prologue<decltype(ex0), OPT>(smem, st, KS, ex0);
  // OPT bit 5: cross-tile prefetch (lzk_g256.h NextTile) -- needs an even K-tile count
  const bool can_pre = ((OPT & 32) != 0) && (KS % 2 == 0);
  int par = 0;
  f32x4 acc[8][4];
  int tix = 0;
  auto stamp = [&](int slot) {
    if constexpr ((OPT & 256) != 0) {
      unsigned long long t;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      if (threadIdx.x == 0 && tix < kStampTiles && g_stamps)
        g_stamps[((long)blockIdx.x * kStampTiles + tix) * 4 + slot] = t;
    }
  };
  while (true) {
    const int cur = tile, cpar = par;
    tile += walk.step;
    const bool more = walk.valid(tile);
    const int nr0 = (tile / n_qt) * BM, nc0 = (tile % n_qt) * BN;
    auto exn = [&]() { stage_epi(tile, cpar ^ 1); };
    const NextTile<decltype(exn)> pre{X, ldx, nr0, nrows, Qm, ldq, nc0, nq, &exn, more && can_pre};
    if constexpr ((OPT & 256) != 0) {  // diagnostic: the K loop's first wait, stamped on its own
      stamp(0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      bar();
      stamp(1);
    }
    if constexpr ((OPT & 8) != 0) body2<MMA>(smem, st, KS, acc, !(OPT & 2), pre);
    else body<MMA, (OPT & 3)>(smem, st, KS, acc, pre);
    stamp(2);
    if (more) {
      st.setup(X, ldx, nr0, nrows, Qm, ldq, nc0, nq);
      if (!can_pre) prologue<decltype(exn), OPT>(smem, st, KS, exn);
    }
    if constexpr ((OPT & 4) != 0) {
      // probe only: the GEMM without the candidate epilogue (one max per
      // lane keeps the accumulators live)
      float m = LZK_NEG_INF;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) m = fmaxf(m, acc[i][j][e]);
      if (m > 1e30f) append(1, 0, m, cur);
      if (!more) break;
      par = cpar ^ 1;
      continue;
    }
    // ---- epilogue of `cur` (operands from LDS only) ----
    {
      const int r0 = (cur / n_qt) * BM, q0 = (cur % n_qt) * BN;
      const float* e_thr = epi + cpar * (EPI_ARRAYS * 256);
      const float* e_bias = e_thr + 256;
      const int* e_lab = reinterpret_cast<const int*>(e_thr + 512);
      const int* e_qlab = reinterpret_cast<const int*>(e_thr + 768);
      const float* e_thr2 = e_thr + 1024;
      int qq[4], ql[4];
      float th[4], th2[4], al[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qlo = wc * 64 + j * 16 + (lane & 15);
        qq[j] = q0 + qlo;
        th[j] = (qq[j] < nq) ? e_thr[qlo] : __builtin_huge_valf();
        th2[j] = (DUAL && qq[j] < nq) ? e_thr2[qlo] : __builtin_huge_valf();
        ql[j] = HAS_LABEL ? e_qlab[qlo] : -1;
        // int8 scan: the query's scale (slot 6) joins alpha
        al[j] = MMA::kInt ? alpha * e_thr[6 * 256 + qlo] : alpha;
      }
      if constexpr (MMA::kInt) {
        // int32 sums -> float * the row's scale (slot 5), in place: the
        // rest of the epilogue (column prefilter, per-score test) is the bf16
        // one with alpha = alpha * qscale. Exact: |acc| < 2^24 for D <= 1024.
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        const float* e_rs = e_thr + 5 * 256;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const f32x4 rs = *reinterpret_cast<const f32x4*>(e_rs + wr * 128 + i * 16 + 4 * (lane >> 4));
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const i32x4 v = __builtin_bit_cast(i32x4, acc[i][j]);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[i][j][e] = (float)v[e] * rs[e];
          }
        }
      }
      const bool full = r0 + BM <= nrows;
      // (int8: a prefilter on the raw int32 sums, bounded by the wave's
      // largest / smallest row scale and converting only surviving columns,
      // measured 9.8 vs 8.9 ms per headline store search -- the looser bound
      // lets more waves into the per-score path, which then also pays the
      // conversion: profiles/r6/serving/i8_int_prefilter_ab/)
      // OPT bit 4: column prefilter. For alpha > 0 every score of query
      // column j is <= alpha * max_i acc[i][j] + max(bias over the wave's
      // rows), so a column whose bound is below its threshold (the common
      // case: ~k*S/N of the scores pass) skips the per-score pass -- ~70
      // VALU per tile instead of ~320. Labels only remove rows, and list B's
      // threshold is covered by min(th, th2), so the bound is conservative.
      float bmax = 0.f;
      if constexpr ((OPT & 16) != 0 && HAS_BIAS)
        bmax = wave_max(fmaxf(e_bias[wr * 128 + lane], e_bias[wr * 128 + 64 + lane]));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr ((OPT & 16) != 0) {
          float mx = acc[0][j][0];
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) mx = fmaxf(mx, acc[i][j][e]);
          const float tmin = DUAL ? fminf(th[j], th2[j]) : th[j];
          // slack of a few ulp: the per-score path may contract alpha*acc+bias differently
          // (tmin = +inf -> NaN -> skipped; tmin = -inf -> kept)
          if (al[j] > 0.f && !(al[j] * mx + bmax >= tmin - 1e-6f * fabsf(tmin))) continue;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int rl = wr * 128 + i * 16 + 4 * (lane >> 4);
          const int rb = r0 + rl;
          f32x4 bv = {0.f, 0.f, 0.f, 0.f};
          if (HAS_BIAS) bv = *reinterpret_cast<const f32x4*>(e_bias + rl);
          float sc[4];
          float m = LZK_NEG_INF;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sc[e] = al[j] * acc[i][j][e] + bv[e];
            const bool in = full || (rb + e < nrows);
            if (!in) sc[e] = LZK_NEG_INF;
            if constexpr (HAS_LABEL && !DUAL) {  // single search: the label filters list A
              if (ql[j] >= 0 && e_lab[rl + e] != ql[j]) sc[e] = LZK_NEG_INF;
            }
            m = fmaxf(m, sc[e]);
          }
          // dual: list B's label test only where a score clears its (low)
          // threshold -- the unlabelled max bounds the labelled one
          const float tlo = DUAL ? fminf(th[j], th2[j]) : th[j];
          if (m >= tlo) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              int lists = (sc[e] >= th[j]) ? 1 : 0;
              if (DUAL && sc[e] >= th2[j] && (ql[j] < 0 || e_lab[rl + e] == ql[j])) lists |= 2;
              if (lists && sc[e] != LZK_NEG_INF) append(lists, qq[j], sc[e], rb + e);
            }
          }
        }
      }
    }
    stamp(3);
    ++tix;
    if (!more) break;
    par = cpar ^ 1;
  }
  bar();  // every wave's appends done
  if (threadIdx.x == 0) blk.cnt[blockIdx.x] = *lcnt;  // > cap: records were dropped
}

// Files the block-private candidate records into the per-query lists read by
// cand_select_kernel (cnt zeroed by the caller before the scan). A block that
// dropped records (count > bcap: pathological score distributions) marks
// every query overflowed, so the select's exact fallback recomputes them all.
__global__ __launch_bounds__(256) void cand_gather_kernel(const int4* __restrict__ buf, int bcap,
                                                          const int* __restrict__ bcnt, int cap, int nq,
                                                          int* __restrict__ cnt, float* __restrict__ cs,
                                                          int* __restrict__ ci, int* __restrict__ cnt2,
                                                          float* __restrict__ cs2, int* __restrict__ ci2) {
  const int b = blockIdx.y;
  const int n0 = bcnt[b];
  if (n0 > bcap) {
    for (int q = blockIdx.x * 256 + threadIdx.x; q < nq; q += gridDim.x * 256) {
      atomicOr(cnt + q, 0x40000000);  // idempotent across blocks: the count stays positive
      if (cnt2) atomicOr(cnt2 + q, 0x40000000);
    }
  }
  const int n = min(n0, bcap);
  if (nq < 64) {
    // narrow batches: every record of a wave mostly files into the same one
    // or few lists, so one atomic per (wave, query) with the lanes' slots from
    // mbcnt -- per-lane atomics on the single count of a one-query search
    // serialise (~30 us for its ~10k records)
    const int lane = threadIdx.x & 63;
    for (int e0 = blockIdx.x * 256 + (threadIdx.x & ~63); e0 < n; e0 += gridDim.x * 256) {
      const int e = e0 + lane;
      int4 v = make_int4(-1, 0, 0, 0);
      if (e < n) v = buf[(long)b * bcap + e];
      const bool ok = (unsigned)v.x < (unsigned)nq;
#pragma unroll
      for (int list = 0; list < 2; ++list) {
        int* cn = list ? cnt2 : cnt;
        if (!cn) continue;
        bool want = ok && (v.w & (1 << list));
        unsigned long long todo = __ballot(want);
        while (todo) {
          const int lead = __builtin_ctzll(todo);
          const int ql = __shfl(v.x, lead, 64);
          const unsigned long long grp = __ballot(want && v.x == ql);
          int base = 0;
          if (lane == lead) base = atomicAdd(cn + ql, __popcll(grp)) & 0x3fffffff;
          base = __shfl(base, lead, 64);
          if (want && v.x == ql) {
            const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(grp >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((unsigned)grp, 0u));
            if (pos < cap) {
              (list ? cs2 : cs)[(long)ql * cap + pos] = __int_as_float(v.z);
              (list ? ci2 : ci)[(long)ql * cap + pos] = v.y;
            }
            want = false;
          }
          todo &= ~grp;
        }
      }
    }
    return;
  }
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int4 v = buf[(long)b * bcap + e];
    if ((unsigned)v.x >= (unsigned)nq) continue;  // (a +inf score of a padding query column)
    // positions come from the count's low 30 bits: another block may have set
    // the overflow flag (bit 30) already, and the entries [0, min(count, cap))
    // must all be written -- cand_select / cand_rescore read exactly those
    if (v.w & 1) {
      const int pos = atomicAdd(cnt + v.x, 1) & 0x3fffffff;
      if (pos < cap) {
        cs[(long)v.x * cap + pos] = __int_as_float(v.z);
        ci[(long)v.x * cap + pos] = v.y;
      }
    }
    if (v.w & 2) {
      const int pos = atomicAdd(cnt2 + v.x, 1) & 0x3fffffff;
      if (pos < cap) {
        cs2[(long)v.x * cap + pos] = __int_as_float(v.z);
        ci2[(long)v.x * cap + pos] = v.y;
      }
    }
  }
}

int g_cand_persist = -1;
// Schedule of the persistent candidate kernel (OPT bits): bit 3 = two-phase
// main loop (body2), bit 4 = column prefilter in the epilogue. Interleaved A/B
// on one MI355X, 10M x 768 x 1024 queries
// (profiles/ab_search_sched_r1.json): four-phase 13.73 ms, +body2 13.09,
// +prefilter 13.38, both 12.80 ms (-6.8 %); cross-tile prefetch (bit 5) was
// 8 % slower and stays an A/B knob only.
constexpr int kCandOpt = 24;
// The dual kernel's list-B threshold comes from a 1/S sample of one shard's
// rows, so it is low and the column prefilter rarely skips
// (profiles/ab_dual_r1.json) 0: 16.27 ms, body2: 15.65, +prefilter 15.90.
constexpr int kDualOpt = 8;
int g_dual_opt = -1;  // A/B override of kCandOpt for the dual kernel (lzk_set_dual_opt)
int g_i8_opt = -1;  // A/B override of kCandOpt for the int8 scan (lzk_set_i8_opt; probes only)
int g_g256_opt = 0;  // A/B override of kCandOpt for the plain (no bias / label) variant; 100 = OPT 0
int g_dev_cu = 0;  // the device's CU count (read once)
// grid_cap() budget of the CALLING thread (lzk_set_cu_budget): the grid a
// launch uses and the record buffers its caller sized from lzk_cand_grid*
// come from the same thread's budget, so a budget set by another thread (a
// prefetched consolidation scan beside a search) cannot resize a launch
// between the sizing call and the launch.
thread_local int g_cu_budget = 0;
int n_cu() {
  if (g_dev_cu <= 0) {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    g_dev_cu = c;
  }
  return (g_cu_budget > 0 && g_cu_budget < g_dev_cu) ? g_cu_budget : g_dev_cu;
}

template <int K>
struct TopK {
  float s[K];
  int i[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < K; ++j) { s[j] = LZK_NEG_INF; i[j] = 0x7fffffff; }
  }
  __device__ __forceinline__ void push(float v, int r) {  // arbitrary index order
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

// One wave per query: lane-local top-K over the candidate list, then K
// rounds of wave argmax. ovf[q] = 1 when the list overflowed its capacity, or
// (need != null) when it holds fewer than need[q] entries: a speculative
// threshold above the query's true k-th score -- both recomputed exactly by
// the caller's masked fallback.
template <int K>
__global__ __launch_bounds__(256) void cand_select_kernel(const int* __restrict__ cnt, const float* __restrict__ cs,
                                                          const int* __restrict__ ci, int cap, int nq, int kout,
                                                          long idx_offset, float* __restrict__ os,
                                                          long* __restrict__ oi, int* __restrict__ ovf,
                                                          const int* __restrict__ need) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  const int c = cnt[q];
  if (lane == 0) ovf[q] = (c > cap || (need && c < need[q])) ? 1 : 0;
  // bit 30: a block dropped records (cand_gather_kernel) -- only the first
  // (c & 0x3fffffff) entries were written; ovf is set either way
  const int n = min(c & 0x3fffffff, cap);
  TopK<K> top;
  top.init();
  const float* s = cs + (long)q * cap;
  const int* ix = ci + (long)q * cap;
  for (int p = lane; p < n; p += 64) top.push(s[p], ix[p]);
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
      oi[(long)q * kout + j] = none ? -1 : (long)bi + idx_offset;
    }
    if (hi == bi && hs == bs && bi != 0x7fffffff) {
#pragma unroll
      for (int t = 0; t < K - 1; ++t) { top.s[t] = top.s[t + 1]; top.i[t] = top.i[t + 1]; }
      top.s[K - 1] = LZK_NEG_INF; top.i[K - 1] = 0x7fffffff;
    }
  }
}

// The same selection with a whole block per query (narrow batches: one
// wave walking a list of thousands of entries with a dependent load per
// entry was ~50 us of the single-query search): the list is read 16 entries
// per thread at a time (loads issued before any push: a 16k-entry list in
// one round trip); each wave takes its own kout best by shuffles alone into
// LDS, then wave 0 selects the block's kout of those 16 x kout -- one
// barrier instead of two per round.
template <int K>
__global__ __launch_bounds__(1024) void cand_select_block_kernel(const int* __restrict__ cnt,
                                                                 const float* __restrict__ cs,
                                                                 const int* __restrict__ ci, int cap, int nq,
                                                                 int kout, long idx_offset, float* __restrict__ os,
                                                                 long* __restrict__ oi, int* __restrict__ ovf,
                                                                 const int* __restrict__ need) {
  __shared__ float ls[16 * K];
  __shared__ int li[16 * K];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x;
  const int c = cnt[q];
  if (threadIdx.x == 0) ovf[q] = (c > cap || (need && c < need[q])) ? 1 : 0;
  const int n = min(c & 0x3fffffff, cap);
  TopK<K> top;
  top.init();
  const float* s = cs + (long)q * cap;
  const int* ix = ci + (long)q * cap;
  constexpr int U = 16;
  for (int p0 = 0; p0 < n; p0 += 1024 * U) {
    float sv[U];
    int iv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * 1024 + (int)threadIdx.x;
      sv[u] = p < n ? s[p] : LZK_NEG_INF;
      iv[u] = p < n ? ix[p] : 0x7fffffff;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (p0 + u * 1024 + (int)threadIdx.x < n) top.push(sv[u], iv[u]);
  }
  // stage 1: the wave's kout best (wave argmax rounds, no barrier)
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
    if (lane == 0) { ls[wave * K + j] = bs; li[wave * K + j] = bi; }
    if (hi == bi && hs == bs && bi != 0x7fffffff) {
#pragma unroll
      for (int t = 0; t < K - 1; ++t) { top.s[t] = top.s[t + 1]; top.i[t] = top.i[t + 1]; }
      top.s[K - 1] = LZK_NEG_INF; top.i[K - 1] = 0x7fffffff;
    }
  }
  __syncthreads();
  if (wave != 0) return;
  // stage 2: wave 0 over the 16 x kout wave winners
  TopK<K> t2;
  t2.init();
  for (int p = lane; p < 16 * kout; p += 64) t2.push(ls[(p / kout) * K + p % kout], li[(p / kout) * K + p % kout]);
  for (int j = 0; j < kout; ++j) {
    const float hs = t2.s[0];
    const int hi = t2.i[0];
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
      oi[(long)q * kout + j] = none ? -1 : (long)bi + idx_offset;
    }
    if (hi == bi && hs == bs && bi != 0x7fffffff) {
#pragma unroll
      for (int t = 0; t < K - 1; ++t) { t2.s[t] = t2.s[t + 1]; t2.i[t] = t2.i[t + 1]; }
      t2.s[K - 1] = LZK_NEG_INF; t2.i[K - 1] = 0x7fffffff;
    }
  }
}

// Exact top-1 (argmax) per query on the 256x256 pipeline: the k-means assign
// step (every buffer row against a few thousand
// centroids). With k = 1 the per-query state is one (score, row) pair, so the
// epilogue folds each lane's 32 accumulators, then the 4 row groups of a wave
// by shuffles, and merges across row tiles with one 64-bit atomicMax per
// (query, wave row) on a packed key: order-preserving score bits high,
// (~row) low -> max score, smallest row on ties. Blocks of one query tile
// are adjacent (row tile = fastest index), so a query tile is read from HBM
// once and the small centroid matrix stays in L2.
__device__ __forceinline__ unsigned long long top1_pack(float s, int r) {
  unsigned u = __float_as_uint(s);
  const unsigned key = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)key << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)r);
}

__global__ __launch_bounds__(NT, 1) void flat_top1_kernel(const u16* __restrict__ X, long ldx, int nrows,
                                                          const u16* __restrict__ Qm, long ldq, int nq, int D,
                                                          int n_rt, unsigned long long* __restrict__ best) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = logical % n_rt, qt = logical / n_rt;
  const int r0 = rt * BM, q0 = qt * BN;
  Stager st;
  st.setup(X, ldx, r0, nrows, Qm, ldq, q0, nq);
  f32x4 acc[8][4];
  mainloop(smem, st, D / BK, acc);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float m = LZK_NEG_INF;
    int mr = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rb = r0 + wr * 128 + i * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // rows ascend within a lane: strict > keeps the smaller row
        const float v = acc[i][j][e];
        if (rb + e < nrows && v > m) { m = v; mr = rb + e; }
      }
    }
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float om = __shfl_xor(m, off);
      const int orr = __shfl_xor(mr, off);
      if (om > m || (om == m && orr < mr)) { m = om; mr = orr; }
    }
    const int q = q0 + wc * 64 + j * 16 + (lane & 15);
    if ((lane >> 4) == 0 && q < nq && mr < nrows) atomicMax(best + q, top1_pack(m, mr));
  }
}

// Grouped top-1 (the two-level k-means assign in ONE launch): query group g
// (the data rows whose nearest topic is g, given as row indices `qidx` into
// Xq -- no gather of the rows) is scored only against its own centroid range
// (centroids sorted by topic). Each block is one (centroid tile, query tile)
// of one group, from a host-built table {c0, nc, p0, np}: centroid rows
// [c0, c0 + min(256, nc)) x query positions [p0, p0 + min(256, np)).
// Result per query position: packed (score, sorted centroid index), merged
// with the same 64-bit atomicMax as flat_top1_kernel, so ties go to the
// smaller centroid index -- identical to one flat_top1 per group.
__global__ __launch_bounds__(NT, 1) void flat_top1_grouped_kernel(const u16* __restrict__ C, long ldc,
                                                                  const u16* __restrict__ Xq, long ldx,
                                                                  const int* __restrict__ qidx,
                                                                  const int4* __restrict__ blocks, int D,
                                                                  unsigned long long* __restrict__ best) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int4 bd = blocks[xcd_remap(blockIdx.x, gridDim.x)];
  const int c0 = bd.x, nc = bd.y, p0 = bd.z, np = bd.w;
  Stager st;
  st.setup(C + (long)c0 * ldc, ldc, 0, nc, Xq, ldx, 0, 1);
  {  // query operand: the indexed data rows (clamped to the tile's last query)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 8 * (wave * 2 + i) + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      LZK_DCHECK(qidx[p0 + min(row, np - 1)] >= 0);
      st.src[2][i] = Xq + (long)qidx[p0 + min(row, np - 1)] * ldx + kc * 8;
      st.src[3][i] = Xq + (long)qidx[p0 + min(128 + row, np - 1)] * ldx + kc * 8;
    }
  }
  f32x4 acc[8][4];
  mainloop(smem, st, D / BK, acc);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float m = LZK_NEG_INF;
    int mr = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rb = wr * 128 + i * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = acc[i][j][e];
        if (rb + e < nc && v > m) { m = v; mr = rb + e; }
      }
    }
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float om = __shfl_xor(m, off);
      const int orr = __shfl_xor(mr, off);
      if (om > m || (om == m && orr < mr)) { m = om; mr = orr; }
    }
    const int q = wc * 64 + j * 16 + (lane & 15);
    if ((lane >> 4) == 0 && q < np && mr < nc) atomicMax(best + p0 + q, top1_pack(m, c0 + mr));
  }
}

__global__ __launch_bounds__(256) void top1_decode_kernel(const unsigned long long* __restrict__ best, int nq,
                                                          float* __restrict__ score, int* __restrict__ row) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const unsigned long long b = best[q];
  if (b == 0ull) { score[q] = LZK_NEG_INF; row[q] = -1; return; }
  const unsigned key = (unsigned)(b >> 32);
  const unsigned u = (key & 0x80000000u) ? (key & 0x7fffffffu) : ~key;
  score[q] = __uint_as_float(u);
  row[q] = (int)(0xFFFFFFFFu - (unsigned)(b & 0xFFFFFFFFull));
}

// Exact re-score of the candidate lists of a low-precision (fp8 / int8) scan:
// the list entry (q, row) gets alpha * <Q[q], X[row]> + bias[row] (fp32
// accumulate) from the bf16 rows (F32 false: the same scores as the bf16 path)
// or -- a lean tenant that keeps no bf16 copy -- from the fp32 rows and fp32
// queries (F32 true). One 256-thread block per query, 4 waves take alternate
// 64-entry windows of the list and re-score the window's kept entries one by
// one; lane c reads the c-th 4-element chunk of a row (8 B bf16 / 16 B fp32).
// cut (optional, [nq]): entries whose scan score is below cut[q] cannot reach
// the query's top-k (the caller's error bound) and become -inf without a row
// read.
template <bool F32>
__device__ __forceinline__ void load4(const void* p, long off, float (&v)[4]) {
  if constexpr (F32) {
    const float4 u = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + off);
    v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const u16*>(p) + off);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  }
}

template <bool F32>
__global__ __launch_bounds__(256) void cand_rescore_kernel(const void* __restrict__ X, long ldx,
                                                           const void* __restrict__ Qm, long ldq, int D,
                                                           const float* __restrict__ bias, float alpha,
                                                           const int* __restrict__ cnt, int cap,
                                                           float* __restrict__ cs, const int* __restrict__ ci,
                                                           const float* __restrict__ cut, float floor,
                                                           const float* __restrict__ tau, int k_need,
                                                           int need_val, int* __restrict__ need,
                                                           int* __restrict__ hitc, int* __restrict__ done) {
  __shared__ int s_hits;
  const int q = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // gridDim.y blocks share a query's list (narrow batches): block y takes
  // the 256-entry groups y, y + gridDim.y, ...; the certificate's hit count
  // is summed over them (hitc / done: per-query counters zeroed by the
  // launcher) and the query's last block writes need[q]
  const int split = gridDim.y;
  if (threadIdx.x == 0) s_hits = 0;
  __syncthreads();
  const float tq = tau ? tau[q] : LZK_NEG_INF;
  int hits = 0;
  const int n = min(cnt[q] & 0x3fffffff, cap);
  const int chunks = D >> 2;  // 4 elements per chunk
  constexpr int MAXC = 8;     // D <= 64 * 4 * MAXC = 2048
  float qv[MAXC][4];
#pragma unroll
  for (int t = 0; t < MAXC; ++t) {
    const int c = lane + 64 * t;
    if (c < chunks) load4<F32>(Qm, (long)q * ldq + 4 * c, qv[t]);
  }
  const float cq = cut ? cut[q] : LZK_NEG_INF;
  for (int base = blockIdx.y * 256 + wave * 64; base < n; base += 256 * split) {
    const long li = (long)q * cap + base + lane;
    bool keep = base + lane < n;
    if (keep && cut) {
      keep = cs[li] >= cq;
      if (!keep) cs[li] = LZK_NEG_INF;
    }
    unsigned long long live = __ballot(keep);
    while (live) {
    const int jj = __builtin_ctzll(live);
    live &= live - 1;
    const long idx = (long)q * cap + base + jj;
    const int r = ci[idx];
    LZK_DCHECK(r >= 0);
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < MAXC; ++t) {
      const int c = lane + 64 * t;
      if (c < chunks) {
        float xv[4];
        load4<F32>(X, (long)r * ldx + 4 * c, xv);
        acc = fmaf(qv[t][0], xv[0], acc);
        acc = fmaf(qv[t][1], xv[1], acc);
        acc = fmaf(qv[t][2], xv[2], acc);
        acc = fmaf(qv[t][3], xv[3], acc);
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    const float sc = alpha * acc + (bias ? bias[r] : 0.f);
    if (lane == 0) cs[idx] = sc >= floor ? sc : LZK_NEG_INF;  // below the caller's floor: dropped
    hits += (sc >= floor && sc >= tq) ? 1 : 0;  // wave-uniform (sc is the reduced sum)
    }
  }
  // per-query certificate of the low-precision scans: the list is kept only
  // when k_need re-scored entries reach tau -- the scan threshold plus the
  // worst-case error bound, above which no unlisted row can score -- else
  // need_val sends the query to the exact fallback
  if (need) {
    if (lane == 0 && hits) atomicAdd(&s_hits, hits);
    __syncthreads();
    // tau = -inf: every row that can matter is in the list (the caller's
    // threshold already sits a worst-case margin below its floor)
    if (threadIdx.x == 0) {
      int tot = s_hits;
      bool last = true;
      if (split > 1) {
        atomicAdd(&hitc[q], s_hits);
        __threadfence();
        last = atomicAdd(&done[q], 1) == split - 1;
        if (last) tot = atomicAdd(&hitc[q], 0);
      }
      if (last) need[q] = (tot >= k_need || tq == LZK_NEG_INF) ? 0 : need_val;
    }
  }
}

// cand_rescore_kernel for narrow batches (split over gridDim.y blocks per
// query): 16 lanes per entry, so a wave re-scores up to 4 live entries per
// row-read latency instead of one; the query staged once per block in LDS.
// Same outputs and certificate counters as the wave-per-entry kernel.
template <bool F32>
__global__ __launch_bounds__(256) void cand_rescore4_kernel(const void* __restrict__ X, long ldx,
                                                            const void* __restrict__ Qm, long ldq, int D,
                                                            const float* __restrict__ bias, float alpha,
                                                            const int* __restrict__ cnt, int cap,
                                                            float* __restrict__ cs, const int* __restrict__ ci,
                                                            const float* __restrict__ cut, float floor,
                                                            const float* __restrict__ tau, int k_need, int need_val,
                                                            int* __restrict__ need, int* __restrict__ hitc,
                                                            int* __restrict__ done) {
  __shared__ float qs_l[2048];
  __shared__ int s_hits;
  const int q = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int part = lane & 15, g = lane >> 4;
  const int split = gridDim.y;
  if (threadIdx.x == 0) s_hits = 0;
  for (int c = threadIdx.x; c < (D >> 2); c += 256) {
    float v[4];
    load4<F32>(Qm, (long)q * ldq + 4 * c, v);
    qs_l[4 * c] = v[0]; qs_l[4 * c + 1] = v[1]; qs_l[4 * c + 2] = v[2]; qs_l[4 * c + 3] = v[3];
  }
  __syncthreads();
  const float tq = tau ? tau[q] : LZK_NEG_INF;
  int hits = 0;
  const int n = min(cnt[q] & 0x3fffffff, cap);
  const int chunks = D >> 2;
  const float cq = cut ? cut[q] : LZK_NEG_INF;
  for (int base = blockIdx.y * 256 + wave * 64; base < n; base += 256 * split) {
    const long li0 = (long)q * cap + base + lane;
    bool keep = base + lane < n;
    if (keep && cut) {
      keep = cs[li0] >= cq;
      if (!keep) cs[li0] = LZK_NEG_INF;
    }
    unsigned long long live = __ballot(keep);
    while (live) {
      // the next (up to) 4 live entries: lane group g takes the g-th
      int jj = -1;
      unsigned long long m = live;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int b = m ? __builtin_ctzll(m) : -1;
        if (t == g) jj = b;
        if (m) m &= m - 1;
      }
      live = m;
      float acc = 0.f;
      int r = -1;
      if (jj >= 0) {
        r = ci[(long)q * cap + base + jj];
        for (int c = part; c < chunks; c += 16) {
          float xv[4];
          load4<F32>(X, (long)r * ldx + 4 * c, xv);
          acc = fmaf(qs_l[4 * c], xv[0], acc);
          acc = fmaf(qs_l[4 * c + 1], xv[1], acc);
          acc = fmaf(qs_l[4 * c + 2], xv[2], acc);
          acc = fmaf(qs_l[4 * c + 3], xv[3], acc);
        }
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) acc += __shfl_xor(acc, o, 64);
      bool hit = false;
      if (jj >= 0) {
        const float sc = alpha * acc + (bias ? bias[r] : 0.f);
        if (part == 0) cs[(long)q * cap + base + jj] = sc >= floor ? sc : LZK_NEG_INF;
        hit = part == 0 && sc >= floor && sc >= tq;
      }
      hits += __popcll(__ballot(hit));  // wave-uniform
    }
  }
  if (need) {
    if (lane == 0 && hits) atomicAdd(&s_hits, hits);
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = s_hits;
      bool last = true;
      if (split > 1) {
        atomicAdd(&hitc[q], s_hits);
        __threadfence();
        last = atomicAdd(&done[q], 1) == split - 1;
        if (last) tot = atomicAdd(&hitc[q], 0);
      }
      if (last) need[q] = (tot >= k_need || tq == LZK_NEG_INF) ? 0 : need_val;
    }
  }
}

// Re-score cut of a low-precision candidate list (ops.search
// _rescore_above_cut), one wave per query: the k best list entries by scan
// score (rows [q, 0..k) of cand_select's output, -1 = empty) are scored
// exactly -- alpha <Q[q], X[row]> + bias[row] from the bf16 rows (F32 false)
// or the fp32 rows / queries (F32 true, lean tenants) -- and their minimum L
// (-inf unless all k are real rows with finite scores) gives
//   cut[q] = L - margin[q] - (2e-4 |alpha| + 1e-6 (1 + |L|))
// (the slack covers this kernel's fp32 accumulation order against the
// re-score kernel's), raised to floor - margin[q] when has_floor. A row of the
// true top-k has a scan score >= L - margin, so entries below the cut cannot
// reach the top-k. Replaces a gather + batched GEMM (einsum) + where/min
// chain of ~10 ATen launches with one.
template <bool F32>
__global__ __launch_bounds__(256) void cand_cut_kernel(const void* __restrict__ X, long ldx, long nrows,
                                                       const void* __restrict__ Qm, long ldq, int D, int nq,
                                                       const float* __restrict__ bias, float alpha,
                                                       const long* __restrict__ rows, int ldr, int k,
                                                       const float* __restrict__ margin, float floor, int has_floor,
                                                       float* __restrict__ cut) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  const int chunks = D >> 2;
  constexpr int MAXC = 8;  // D <= 2048
  float qv[MAXC][4];
#pragma unroll
  for (int t = 0; t < MAXC; ++t) {
    const int c = lane + 64 * t;
    if (c < chunks) load4<F32>(Qm, (long)q * ldq + 4 * c, qv[t]);
  }
  float lo = __builtin_inff();
  for (int j = 0; j < k; ++j) {
    const long r = rows[(long)q * ldr + j];  // wave-uniform
    if (r < 0 || r >= nrows) { lo = LZK_NEG_INF; break; }
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < MAXC; ++t) {
      const int c = lane + 64 * t;
      if (c < chunks) {
        float xv[4];
        load4<F32>(X, r * ldx + 4 * c, xv);
        acc = fmaf(qv[t][0], xv[0], acc);
        acc = fmaf(qv[t][1], xv[1], acc);
        acc = fmaf(qv[t][2], xv[2], acc);
        acc = fmaf(qv[t][3], xv[3], acc);
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    const float sc = alpha * acc + (bias ? bias[r] : 0.f);
    if (!(sc > LZK_NEG_INF && sc < __builtin_inff())) { lo = LZK_NEG_INF; break; }  // -inf, +inf or nan
    lo = fminf(lo, sc);
  }
  if (lane != 0) return;
  const float m = margin[q];
  float c = lo - m - (2e-4f * fabsf(alpha) + 1e-6f * (1.f + fabsf(lo)));
  if (has_floor) c = fmaxf(c, floor - m);  // (fmaxf: a nan c takes the floor)
  if (c != c) c = LZK_NEG_INF;
  cut[q] = c;
}

// cand_cut_kernel for narrow batches: a 1024-thread block per query, wave j
// scores row j (k <= 16) -- the k exact scores in one row-read latency
// instead of k dependent ones (~32 us for one query).
template <bool F32>
__global__ __launch_bounds__(1024) void cand_cut_block_kernel(const void* __restrict__ X, long ldx, long nrows,
                                                              const void* __restrict__ Qm, long ldq, int D, int nq,
                                                              const float* __restrict__ bias, float alpha,
                                                              const long* __restrict__ rows, int ldr, int k,
                                                              const float* __restrict__ margin, float floor,
                                                              int has_floor, float* __restrict__ cut) {
  __shared__ float sc_w[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x;
  const int chunks = D >> 2;
  constexpr int MAXC = 8;  // D <= 2048
  if (wave < k) {
    const long r = rows[(long)q * ldr + wave];  // wave-uniform
    float sc = LZK_NEG_INF;
    if (r >= 0 && r < nrows) {
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < MAXC; ++t) {
        const int c = lane + 64 * t;
        if (c < chunks) {
          float qv[4], xv[4];
          load4<F32>(Qm, (long)q * ldq + 4 * c, qv);
          load4<F32>(X, r * ldx + 4 * c, xv);
          acc = fmaf(qv[0], xv[0], acc);
          acc = fmaf(qv[1], xv[1], acc);
          acc = fmaf(qv[2], xv[2], acc);
          acc = fmaf(qv[3], xv[3], acc);
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
      sc = alpha * acc + (bias ? bias[r] : 0.f);
      if (!(sc > LZK_NEG_INF && sc < __builtin_inff())) sc = LZK_NEG_INF;  // -inf, +inf or nan
    }
    if (lane == 0) sc_w[wave] = sc;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  float lo = __builtin_inff();
  for (int j = 0; j < k; ++j) lo = fminf(lo, sc_w[j]);
  const float m = margin[q];
  float c = lo - m - (2e-4f * fabsf(alpha) + 1e-6f * (1.f + fabsf(lo)));
  if (has_floor) c = fmaxf(c, floor - m);
  if (c != c) c = LZK_NEG_INF;
  cut[q] = c;
}

// Query side of the int8 store search in one launch per batch (one block
// per query): symmetric per-row int8 of the bf16 query (s = max|q| / 127,
// q8 = rint(q / s) clamped to +-127, s = 0 for a zero row -- ops.search
// quantize_i8_rows) and BOTH error margins of TenantGraph._i8_query, with
// eta = q8 s - q and floor = smax / 2 * sum|eta|:
//   statistical (margin):  |alpha| (z sqrt(sum eta^2 mu2 + sum q^2 smax^2 / 12) + floor),
//     mu2 the rows' per-dimension mean square (sumsq / nsq) -- sets the scan
//     threshold (how many candidates are kept);
//   worst case (margin_rig): |alpha| (|eta| xn + smax / 2 sum|q| + floor
//     + d 2^-23 xn |q|) (1 + 1e-5) + 1e-6 -- a bound on |int8 score - bf16
//     score| for EVERY row of norm <= xn (the last term covers the fp32
//     accumulation of the exact re-score), used for the re-score cut and the
//     per-query certificate, so results never depend on the statistical one.
// A batch of one query was ~25 torch launches of a few elements each.
__global__ __launch_bounds__(256) void i8_query_kernel(const u16* __restrict__ q16, long ldq, int Dp, int d,
                                                       const double* __restrict__ sumsq, double inv_nsq,
                                                       const float* __restrict__ smax_p, float alpha_abs, float z,
                                                       float xn, signed char* __restrict__ q8, long ld8,
                                                       float* __restrict__ qs, float* __restrict__ margin,
                                                       float* __restrict__ margin_rig) {
  constexpr int NS = 5;
  __shared__ float s_f[4];
  __shared__ double s_d[NS][4];
  const int q = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const u16* row = q16 + (long)q * ldq;
  float am = 0.f;
  for (int c = t; c < Dp; c += 256) am = fmaxf(am, fabsf(bf16_to_f32(row[c])));
  for (int o = 32; o >= 1; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
  if (lane == 0) s_f[w] = am;
  __syncthreads();
  am = fmaxf(fmaxf(s_f[0], s_f[1]), fmaxf(s_f[2], s_f[3]));
  const float sc = am > 0.f ? am * (1.f / 127.f) : 0.f;  // torch: amax / 127.0 = amax * (1/127) (scalar divisor)
  const float den = am > 0.f ? sc : 1.f;
  double a_eta = 0.0, v1 = 0.0, q2 = 0.0, q1 = 0.0, e2 = 0.0;
  for (int c = t; c < Dp; c += 256) {
    const float x = bf16_to_f32(row[c]);
    const float qq = fminf(fmaxf(rintf(x / den), -127.f), 127.f);
    q8[(long)q * ld8 + c] = (signed char)qq;
    const float eta = __fsub_rn(__fmul_rn(qq, sc), x);
    a_eta += fabs((double)eta);
    q2 += (double)x * (double)x;
    q1 += fabs((double)x);
    if (c < d) {
      const double e = (double)eta * (double)eta;
      e2 += e;
      v1 += e * (double)(float)(sumsq[c] * inv_nsq);
    }
  }
  double vals[NS] = {a_eta, v1, q2, q1, e2};
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    double v = vals[k];
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_d[k][w] = v;
  }
  __syncthreads();
  if (t == 0) {
    double r[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) r[k] = s_d[k][0] + s_d[k][1] + s_d[k][2] + s_d[k][3];
    const double smax = (double)smax_p[0];
    const double fl = 0.5 * smax * r[0];
    qs[q] = sc;
    margin[q] = (float)(alpha_abs * (z * sqrt(r[1] + r[2] * (smax * smax / 12.0)) + fl));
    if (margin_rig) {
      const double acc = (double)d * 0x1p-23 * (double)xn * sqrt(r[2]);
      margin_rig[q] = (float)(alpha_abs * (sqrt(r[4]) * xn + 0.5 * smax * r[3] + fl + acc) * (1.0 + 1e-5) + 1e-6);
    }
  }
}

}  // namespace

// Exact argmax of Q @ X.T per query (no bias/labels). ws: [nq] u64 scratch.
// score fp32 [nq], row int32 [nq] (-1 when nrows == 0).
LZK_EXPORT int lzk_flat_top1(const void* X, long ldx, int nrows, const void* Qm, long ldq, int nq, int D, void* ws,
                             float* score, int* row, void* stream) {
  if (D % BK != 0 || nq <= 0 || nrows <= 0) return (int)hipErrorInvalidValue;
  const int n_rt = (nrows + BM - 1) / BM, n_qt = (nq + BN - 1) / BN;
  const long nblk = (long)n_rt * n_qt;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  unsigned long long* best = (unsigned long long*)ws;
  hipError_t e = hipMemsetAsync(best, 0, (size_t)nq * 8, st);
  if (e != hipSuccess) return (int)e;
  (void)hipFuncSetAttribute((const void*)flat_top1_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
  hipLaunchKernelGGL(flat_top1_kernel, dim3((unsigned)nblk), dim3(NT), LDS_BYTES, st, (const u16*)X, ldx, nrows,
                     (const u16*)Qm, ldq, nq, D, n_rt, best);
  hipLaunchKernelGGL(top1_decode_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, best, nq, score, row);
  return (int)hipGetLastError();
}

// Grouped argmax (two-level k-means assign): blocks [nblk] int4 {c0, nc, p0,
// np} built by the caller (every nc, np >= 1; c0 + nc <= centroid rows;
// p0 + np <= npos; qidx[0, npos) valid rows of Xq). ws: [npos] u64 scratch.
// score fp32 / pos int32 [npos]: best sorted-centroid index per query position.
LZK_EXPORT int lzk_flat_top1_grouped(const void* C, long ldc, const void* Xq, long ldx, const int* qidx, int npos,
                                     const void* blocks, int nblk, int D, void* ws, float* score, int* row,
                                     void* stream) {
  if (D % BK != 0 || npos <= 0 || nblk <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  unsigned long long* best = (unsigned long long*)ws;
  hipError_t e = hipMemsetAsync(best, 0, (size_t)npos * 8, st);
  if (e != hipSuccess) return (int)e;
  (void)hipFuncSetAttribute((const void*)flat_top1_grouped_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            LDS_BYTES);
  hipLaunchKernelGGL(flat_top1_grouped_kernel, dim3((unsigned)nblk), dim3(NT), LDS_BYTES, st, (const u16*)C, ldc,
                     (const u16*)Xq, ldx, qidx, (const int4*)blocks, D, best);
  hipLaunchKernelGGL(top1_decode_kernel, dim3((unsigned)((npos + 255) / 256)), dim3(256), 0, st, best, npos, score,
                     row);
  return (int)hipGetLastError();
}

LZK_EXPORT void lzk_set_cand_persist(int p) { g_cand_persist = p; }
// CU budget of the persistent scans' grids (one block per CU): a search
// launched on a CU-masked stream sizes its grid to the CUs it may use; <= 0
// restores the device's CU count.
LZK_EXPORT void lzk_set_cu_budget(int n) { g_cu_budget = n > 0 ? n : 0; }
LZK_EXPORT void lzk_set_g256_opt(int o) { g_g256_opt = o; }
LZK_EXPORT void lzk_set_dual_opt(int o) { g_dual_opt = o; }
LZK_EXPORT void lzk_set_i8_opt(int o) { g_i8_opt = o; }
LZK_EXPORT int lzk_set_stamp_buffer(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p));
}
LZK_EXPORT int lzk_stamp_tiles() { return kStampTiles; }

// Candidate pass. cnt [nq] must be zeroed by the caller (same stream);
// cs/ci are [nq, cap].
LZK_EXPORT int lzk_flat_cand(const void* X, long ldx, int nrows, const void* Qm, long ldq, int nq, int D,
                             const float* bias, const int* row_label, const int* q_label, float alpha,
                             const float* thr, int cap, int* cnt, float* cs, int* ci, void* blk_buf, int blk_cap,
                             int* blk_cnt, void* stream) {
  if (D % BK != 0 || nq <= 0 || nrows <= 0 || cap <= 0) return (int)hipErrorInvalidValue;
  const BlkCands blk{(int4*)blk_buf, blk_cap, blk_cnt};
  if (row_label && !q_label) return (int)hipErrorInvalidValue;
  const int n_rt = (nrows + BM - 1) / BM, n_qt = (nq + BN - 1) / BN;
  const long nblk = (long)n_rt * n_qt;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  const u16* q = (const u16*)Qm;
  if (g_cand_persist < 0) g_cand_persist = 1;
  const int ncu = n_cu();
  if (g_cand_persist && nblk >= ncu) {
    if (!blk_buf || blk_cap <= 0 || !blk_cnt) return (int)hipErrorInvalidValue;  // lzk_cand_grid() > 0: records needed
    const int grid = ncu;
#define LZK_GP(B, L)                                                                                                \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)flat_cand_persistent_kernel<B, L, false, kCandOpt>,                                \
                              hipFuncAttributeMaxDynamicSharedMemorySize, CAND_P_LDS);                              \
    hipLaunchKernelGGL((flat_cand_persistent_kernel<B, L, false, kCandOpt>), dim3(grid), dim3(NT), CAND_P_LDS, st, x, ldx,    \
                       nrows, q, ldq, nq, D, bias, row_label, q_label, alpha, thr, n_qt, (int)nblk, cap, cnt, cs,   \
                       ci, (const float*)nullptr, (int*)nullptr, (float*)nullptr, (int*)nullptr, blk);               \
  } while (0)
    if (bias && row_label) LZK_GP(true, true);
    else if (bias) LZK_GP(true, false);
    else if (row_label) LZK_GP(false, true);
    else if (g_g256_opt > 0) {
#define LZK_GX(O)                                                                                                   \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)flat_cand_persistent_kernel<false, false, false, O>,                     \
                              hipFuncAttributeMaxDynamicSharedMemorySize, CAND_P_LDS);                              \
    hipLaunchKernelGGL((flat_cand_persistent_kernel<false, false, false, O>), dim3(grid), dim3(NT), CAND_P_LDS, st, \
                       x, ldx, nrows, q, ldq, nq, D, bias, row_label, q_label, alpha, thr, n_qt, (int)nblk, cap,    \
                       cnt, cs, ci, (const float*)nullptr, (int*)nullptr, (float*)nullptr, (int*)nullptr, blk);     \
  } while (0)
      switch (g_g256_opt) {
        case 1: LZK_GX(1); break;
        case 2: LZK_GX(2); break;
        case 4: LZK_GX(4); break;
        case 8: LZK_GX(8); break;
        case 16: LZK_GX(16); break;
        case 24: LZK_GX(24); break;
        case 26: LZK_GX(26); break;
        case 280: LZK_GX(280); break;
        case 312: LZK_GX(312); break;
        case 32: LZK_GX(32); break;
        case 36: LZK_GX(36); break;
        case 40: LZK_GX(40); break;
        case 48: LZK_GX(48); break;
        case 56: LZK_GX(56); break;
        case 100: LZK_GX(0); break;
        default: LZK_GX(kCandOpt); break;
      }
#undef LZK_GX
    } else LZK_GP(false, false);
#undef LZK_GP
    return (int)hipGetLastError();
  }
#define LZK_GO(B, L)                                                                                              \
  do {                                                                                                            \
    (void)hipFuncSetAttribute((const void*)flat_cand_kernel<B, L>, hipFuncAttributeMaxDynamicSharedMemorySize,   \
                              LDS_BYTES);                                                                         \
    hipLaunchKernelGGL((flat_cand_kernel<B, L>), dim3((unsigned)nblk), dim3(NT), LDS_BYTES, st, x, ldx, nrows, q, \
                       ldq, nq, D, bias, row_label, q_label, alpha, thr, n_qt, cap, cnt, cs, ci);                 \
  } while (0)
  if (bias && row_label) LZK_GO(true, true);
  else if (bias) LZK_GO(true, false);
  else if (row_label) LZK_GO(false, true);
  else LZK_GO(false, false);
#undef LZK_GO
  return (int)hipGetLastError();
}

// Dual candidate pass (one GEMM, two lists): list A unfiltered (thr), list B
// label-filtered (thr2). row_label / q_label required. Counts zeroed by caller.
LZK_EXPORT int lzk_flat_cand_dual(const void* X, long ldx, int nrows, const void* Qm, long ldq, int nq, int D,
                                  const float* bias, const int* row_label, const int* q_label, float alpha,
                                  const float* thr, const float* thr2, int cap, int* cnt, float* cs, int* ci,
                                  int* cnt2, float* cs2, int* ci2, void* blk_buf, int blk_cap, int* blk_cnt,
                                  void* stream) {
  const BlkCands blk{(int4*)blk_buf, blk_cap, blk_cnt};
  if (!blk_buf || blk_cap <= 0 || !blk_cnt) return (int)hipErrorInvalidValue;
  if (D % BK != 0 || nq <= 0 || nrows <= 0 || cap <= 0 || !row_label || !q_label) return (int)hipErrorInvalidValue;
  const int n_rt = (nrows + BM - 1) / BM, n_qt = (nq + BN - 1) / BN;
  const long nblk = (long)n_rt * n_qt;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  const int ncu = n_cu();
  const int grid = (int)(nblk < ncu ? nblk : ncu);
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  const u16* q = (const u16*)Qm;
#define LZK_GDO(B, O)                                                                                              \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)flat_cand_persistent_kernel<B, true, true, O>,                           \
                              hipFuncAttributeMaxDynamicSharedMemorySize, CAND_P_LDS);                              \
    hipLaunchKernelGGL((flat_cand_persistent_kernel<B, true, true, O>), dim3(grid), dim3(NT), CAND_P_LDS, st, x,    \
                       ldx, nrows, q, ldq, nq, D, bias, row_label, q_label, alpha, thr, n_qt, (int)nblk, cap, cnt,  \
                       cs, ci, thr2, cnt2, cs2, ci2, blk);                                                          \
  } while (0)
#define LZK_GD(B)                              \
  do {                                         \
    switch (g_dual_opt) {                      \
      case 0: LZK_GDO(B, 0); break;            \
      case 8: LZK_GDO(B, 8); break;            \
      case 16: LZK_GDO(B, 16); break;          \
      default: LZK_GDO(B, kDualOpt); break;    \
    }                                          \
  } while (0)
  if (bias) LZK_GD(true);
  else LZK_GD(false);
#undef LZK_GD
#undef LZK_GDO
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_cand_select(const int* cnt, const float* cs, const int* ci, int cap, int nq, int kslot, int kout,
                               long idx_offset, float* os, long* oi, int* ovf, const int* need, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((nq + 3) / 4), block(256);
  if (kout > kslot) return (int)hipErrorInvalidValue;
  // narrow batches: a block per query (cand_select_block_kernel)
  const bool blk = nq < 64;
#define LZK_SEL(KK)                                                                                                   \
  do {                                                                                                                \
    if (blk)                                                                                                          \
      hipLaunchKernelGGL(cand_select_block_kernel<KK>, dim3((unsigned)nq), dim3(1024), 0, st, cnt, cs, ci, cap, nq,   \
                         kout, idx_offset, os, oi, ovf, need);                                                        \
    else                                                                                                              \
      hipLaunchKernelGGL(cand_select_kernel<KK>, grid, block, 0, st, cnt, cs, ci, cap, nq, kout, idx_offset, os, oi,  \
                         ovf, need);                                                                                  \
  } while (0)
  switch (kslot) {
    case 1: LZK_SEL(1); break;
    case 2: LZK_SEL(2); break;
    case 4: LZK_SEL(4); break;
    case 8: LZK_SEL(8); break;
    case 10: LZK_SEL(10); break;
    case 16: LZK_SEL(16); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef LZK_SEL
  return (int)hipGetLastError();
}

// Records of the last candidate pass -> per-query lists (grid = the pass's grid).
LZK_EXPORT int lzk_cand_gather(const void* blk_buf, int blk_cap, const int* blk_cnt, int grid, int cap, int nq,
                               int* cnt, float* cs, int* ci, int* cnt2, float* cs2, int* ci2, void* stream) {
  if (grid <= 0 || blk_cap <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(cand_gather_kernel, dim3(4, grid), dim3(256), 0, (hipStream_t)stream, (const int4*)blk_buf,
                     blk_cap, blk_cnt, cap, nq, cnt, cs, ci, cnt2, cs2, ci2);
  return (int)hipGetLastError();
}

// Grid of the persistent candidate pass for a shape (the gather's grid); 0
// when lzk_flat_cand would take the non-persistent kernel (global appends).
LZK_EXPORT int lzk_cand_grid(int nrows, int nq, int dual) {
  const int ncu = n_cu();
  if (g_cand_persist < 0) g_cand_persist = 1;
  const long nblk = (long)((nrows + BM - 1) / BM) * ((nq + BN - 1) / BN);
  if (dual) return (int)(nblk < ncu ? nblk : ncu);
  return (g_cand_persist && nblk >= ncu) ? ncu : 0;
}

// fp8 candidate pass (rows / queries: e4m3 bytes, row strides in bytes,
// D_bytes % 128 == 0): score = alpha * <q8, x8> + bias[row] >= thr[q] is
// appended to the block-private records (persistent grid = one block per CU).
// Re-score the gathered lists exactly with lzk_cand_rescore before selecting.
LZK_EXPORT int lzk_flat_cand_f8(const void* X8, long ldx_bytes, int nrows, const void* Q8, long ldq_bytes, int nq,
                                int D_bytes, const float* bias, float alpha, const float* thr, int cap, int* cnt,
                                float* cs, int* ci, void* blk_buf, int blk_cap, int* blk_cnt, void* stream) {
  if (D_bytes % 128 != 0 || (ldx_bytes | ldq_bytes) % 16 != 0 || nq <= 0 || nrows <= 0 || cap <= 0)
    return (int)hipErrorInvalidValue;
  if (!blk_buf || blk_cap <= 0 || !blk_cnt) return (int)hipErrorInvalidValue;
  const BlkCands blk{(int4*)blk_buf, blk_cap, blk_cnt};
  const int n_rt = (nrows + BM - 1) / BM, n_qt = (nq + BN - 1) / BN;
  const long nblk = (long)n_rt * n_qt;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  const int ncu = n_cu();
  const int grid = (int)(nblk < ncu ? nblk : ncu);
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X8;
  const u16* q = (const u16*)Q8;
#define LZK_GF(B)                                                                                                   \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)flat_cand_persistent_kernel<B, false, false, kCandOpt, MmaFp8>,          \
                              hipFuncAttributeMaxDynamicSharedMemorySize, CAND_P_LDS);                              \
    hipLaunchKernelGGL((flat_cand_persistent_kernel<B, false, false, kCandOpt, MmaFp8>), dim3(grid), dim3(NT),     \
                       CAND_P_LDS, st, x, ldx_bytes / 2, nrows, q, ldq_bytes / 2, nq, D_bytes / 2, bias,            \
                       (const int*)nullptr, (const int*)nullptr, alpha, thr, n_qt, (int)nblk, cap, cnt, cs, ci,      \
                       (const float*)nullptr, (int*)nullptr, (float*)nullptr, (int*)nullptr, blk);                  \
  } while (0)
  if (bias) LZK_GF(true);
  else LZK_GF(false);
#undef LZK_GF
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_cand_grid_f8(int nrows, int nq) {
  const int ncu = n_cu();
  const long nblk = (long)((nrows + BM - 1) / BM) * ((nq + BN - 1) / BN);
  return (int)(nblk < ncu ? nblk : ncu);
}

// Blocks per query of the re-score: one for wide batches; a narrow batch
// (the interactive turn: ONE query, a list of hundreds to thousands of
// entries above the cut) spreads each list over up to 64 blocks -- one block
// re-scoring a list row by row was 330 us of a 2.2 ms single-query search.
// The certificate's per-query counters live in a per-(device, stream) scratch
// zeroed on the stream before each split launch.
namespace {
constexpr int RESCORE_SPLIT_MAX = 64;
int rescore_split(int nq) {
  if (nq >= 64) return 1;
  int s = 256 / nq;
  return s < 1 ? 1 : (s > RESCORE_SPLIT_MAX ? RESCORE_SPLIT_MAX : s);
}
// one scratch per (device, stream): two streams re-scoring at once (a
// serving search beside a consolidation scan on its side stream) never share
// counters; within a stream the memset and the launch are stream-ordered
struct RsScratch {
  int* p = nullptr;
  int cap = 0;
};
std::mutex g_rs_mu;
std::map<std::pair<int, hipStream_t>, RsScratch> g_rs;
int* rescore_counters(int nq, hipStream_t st) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_rs_mu);
  RsScratch& s = g_rs[{dev, st}];
  if (s.cap < 2 * nq) {
    if (s.p) (void)hipFree(s.p);  // synchronous: no launch still reads it
    s.p = nullptr;
    const int cap = 2 * (nq > 4096 ? nq : 4096);
    if (hipMalloc(&s.p, (size_t)cap * sizeof(int)) != hipSuccess) {
      s.cap = 0;
      return nullptr;
    }
    s.cap = cap;
  }
  if (hipMemsetAsync(s.p, 0, (size_t)2 * nq * sizeof(int), st) != hipSuccess) return nullptr;
  return s.p;
}

template <bool F32>
int launch_rescore(const void* X, long ldx, const void* Q, long ldq, int nq, int D, const float* bias, float alpha,
                   const int* cnt, int cap, float* cs, const int* ci, const float* cut, float floor, const float* tau,
                   int k_need, int need_val, int* need, hipStream_t st) {
  int split = rescore_split(nq);
  int* ctr = nullptr;
  if (split > 1 && need) {
    ctr = rescore_counters(nq, st);
    if (!ctr) split = 1;
  }
  if (split > 1)  // narrow: 4 entries per wave per row read
    hipLaunchKernelGGL(cand_rescore4_kernel<F32>, dim3((unsigned)nq, (unsigned)split), dim3(256), 0, st, X, ldx, Q,
                       ldq, D, bias, alpha, cnt, cap, cs, ci, cut, floor, tau, k_need, need_val, need, ctr,
                       ctr ? ctr + nq : nullptr);
  else
    hipLaunchKernelGGL(cand_rescore_kernel<F32>, dim3((unsigned)nq, 1u), dim3(256), 0, st, X, ldx, Q, ldq, D, bias,
                       alpha, cnt, cap, cs, ci, cut, floor, tau, k_need, need_val, need, ctr, ctr ? ctr + nq : nullptr);
  return (int)hipGetLastError();
}
}  // namespace

// Exact bf16 re-score of candidate lists in place (see cand_rescore_kernel).
LZK_EXPORT int lzk_cand_rescore(const void* X16, long ldx, const void* Q16, long ldq, int nq, int D, const float* bias,
                                float alpha, const int* cnt, int cap, float* cs, const int* ci, const float* cut,
                                float floor, const float* tau, int k_need, int need_val, int* need, void* stream) {
  if (D % 4 != 0 || D > 2048 || nq <= 0) return (int)hipErrorInvalidValue;
  return launch_rescore<false>(X16, ldx, Q16, ldq, nq, D, bias, alpha, cnt, cap, cs, ci, cut, floor, tau, k_need,
                               need_val, need, (hipStream_t)stream);
}

// The same from fp32 rows (X32 [*, ldx] fp32, 16-B aligned rows) and fp32
// queries (Q32 [nq, ldq]): lean tenants without a bf16 copy. D % 4 == 0.
LZK_EXPORT int lzk_cand_rescore32(const float* X32, long ldx, const float* Q32, long ldq, int nq, int D,
                                  const float* bias, float alpha, const int* cnt, int cap, float* cs, const int* ci,
                                  const float* cut, float floor, const float* tau, int k_need, int need_val,
                                  int* need, void* stream) {
  if (D % 4 != 0 || D > 2048 || nq <= 0 || ldx % 4 != 0 || ldq % 4 != 0) return (int)hipErrorInvalidValue;
  return launch_rescore<true>(X32, ldx, Q32, ldq, nq, D, bias, alpha, cnt, cap, cs, ci, cut, floor, tau, k_need,
                              need_val, need, (hipStream_t)stream);
}

// Per-query thresholds of a low-precision store search in ONE launch (ops.
// search flat_topk_i8; it replaced ~12 elementwise ATen launches, ~55 us of a
// single-query search): from the sample's column ``col`` of ``ts``
//   tau  = t - 2e-4 (1 + |t|), nan -> -inf, +-inf -> +-FLT_MAX (torch
//          nan_to_num(nan=-inf): the sample's accumulation-order slack)
//   thr  = tau - margin (margin null: tau)                -- the scan threshold
//   cert = thr + margin_rig, + 1e-6 (1 + |.|), nan / -inf -> -inf, +inf ->
//          FLT_MAX (ops.search _cert_tau without a floor) -- the certificate
// and the per-query list counts zeroed. Rounded op by op like the torch chain.
__global__ __launch_bounds__(256) void thr_prep_kernel(const float* __restrict__ ts, long ldts, int col,
                                                       const float* __restrict__ margin,
                                                       const float* __restrict__ margin_rig, int nq,
                                                       float* __restrict__ thr, float* __restrict__ cert,
                                                       int* __restrict__ cnt) {
#pragma clang fp contract(off)
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  float t = ts[(long)q * ldts + col];
  const float sl = 1.0f + fabsf(t);
  t = t - 2e-4f * sl;
  if (t != t) t = LZK_NEG_INF;
  else if (t == LZK_NEG_INF) t = -FLT_MAX;
  else if (t == __builtin_inff()) t = FLT_MAX;
  const float th = margin ? t - margin[q] : t;
  thr[q] = th;
  if (cert) {
    float c = margin_rig ? th + margin_rig[q] : th;
    const float cs = 1.0f + fabsf(c);
    c = c + 1e-6f * cs;
    if (c != c) c = LZK_NEG_INF;
    else if (c == __builtin_inff()) c = FLT_MAX;
    cert[q] = c;
  }
  if (cnt) cnt[q] = 0;
}

LZK_EXPORT int lzk_thr_prep(const float* ts, long ldts, int col, const float* margin, const float* margin_rig, int nq,
                            float* thr, float* cert, int* cnt, void* stream) {
  if (nq <= 0 || col < 0 || col >= ldts || !ts || !thr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(thr_prep_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ts, ldts,
                     col, margin, margin_rig, nq, thr, cert, cnt);
  return (int)hipGetLastError();
}

// The re-score cut of a low-precision candidate list (cand_cut_kernel);
// f32 = 1: X / Q are fp32 (lean tenants), else bf16. rows: cand_select's
// int64 output [nq, ldr], the first k columns read.
LZK_EXPORT int lzk_cand_cut(const void* X, long ldx, long nrows, const void* Q, long ldq, int D, int nq, int f32,
                            const float* bias, float alpha, const long* rows, int ldr, int k, const float* margin,
                            float floor, int has_floor, float* cut, void* stream) {
  if (D % 4 != 0 || D > 2048 || nq <= 0 || k <= 0 || k > ldr || !margin) return (int)hipErrorInvalidValue;
  if (f32 && (ldx % 4 != 0 || ldq % 4 != 0)) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((nq + 3) / 4)), block(256);
  if (nq < 64 && k <= 16) {  // narrow: a block per query, a wave per row
    if (f32)
      hipLaunchKernelGGL(cand_cut_block_kernel<true>, dim3((unsigned)nq), dim3(1024), 0, (hipStream_t)stream, X, ldx,
                         nrows, Q, ldq, D, nq, bias, alpha, rows, ldr, k, margin, floor, has_floor, cut);
    else
      hipLaunchKernelGGL(cand_cut_block_kernel<false>, dim3((unsigned)nq), dim3(1024), 0, (hipStream_t)stream, X,
                         ldx, nrows, Q, ldq, D, nq, bias, alpha, rows, ldr, k, margin, floor, has_floor, cut);
    return (int)hipGetLastError();
  }
  if (f32)
    hipLaunchKernelGGL(cand_cut_kernel<true>, grid, block, 0, (hipStream_t)stream, X, ldx, nrows, Q, ldq, D, nq,
                       bias, alpha, rows, ldr, k, margin, floor, has_floor, cut);
  else
    hipLaunchKernelGGL(cand_cut_kernel<false>, grid, block, 0, (hipStream_t)stream, X, ldx, nrows, Q, ldq, D, nq,
                       bias, alpha, rows, ldr, k, margin, floor, has_floor, cut);
  return (int)hipGetLastError();
}

// int8 candidate pass (rows / queries: int8 bytes, row strides in bytes,
// D_bytes % 128 == 0, D_bytes <= 1024 so the int32 sums stay exact in fp32):
// score = alpha * qscale[q] * (<q8, x8> * rscale[row]) + bias[row] >= thr[q]
// goes to the block-private records (persistent grid). rscale / qscale > 0.
LZK_EXPORT int lzk_flat_cand_i8(const void* X8, long ldx_bytes, int nrows, const void* Q8, long ldq_bytes, int nq,
                                int D_bytes, const float* bias, const float* rscale, const float* qscale, float alpha,
                                const float* thr, int cap, int* cnt, float* cs, int* ci, void* blk_buf, int blk_cap,
                                int* blk_cnt, void* stream) {
  if (D_bytes % 128 != 0 || D_bytes > 1024 || (ldx_bytes | ldq_bytes) % 16 != 0 || nq <= 0 || nrows <= 0 ||
      cap <= 0 || !rscale || !qscale || !(alpha > 0.f))
    return (int)hipErrorInvalidValue;
  if (!blk_buf || blk_cap <= 0 || !blk_cnt) return (int)hipErrorInvalidValue;
  const BlkCands blk{(int4*)blk_buf, blk_cap, blk_cnt, rscale, qscale};
  const int n_rt = (nrows + BM - 1) / BM, n_qt = (nq + BN - 1) / BN;
  const long nblk = (long)n_rt * n_qt;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  const int ncu = n_cu();
  const int grid = (int)(nblk < ncu ? nblk : ncu);
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X8;
  const u16* q = (const u16*)Q8;
  const int* rs = nullptr;  // no labels
  const int* qs = nullptr;
#define LZK_GIO(B, O)                                                                                               \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)flat_cand_persistent_kernel<B, false, false, O, MmaI8>,                  \
                              hipFuncAttributeMaxDynamicSharedMemorySize, CAND_P_LDS);                              \
    hipLaunchKernelGGL((flat_cand_persistent_kernel<B, false, false, O, MmaI8>), dim3(grid), dim3(NT), CAND_P_LDS, \
                       st, x, ldx_bytes / 2, nrows, q, ldq_bytes / 2, nq, D_bytes / 2, bias, rs, qs, alpha, thr,    \
                       n_qt, (int)nblk, cap, cnt, cs, ci, (const float*)nullptr, (int*)nullptr, (float*)nullptr,    \
                       (int*)nullptr, blk);                                                                         \
  } while (0)
  // (a cross-tile prefetch variant, OPT bit 5, measured 11.0 vs 10.0 ms per
  // store search on 10M x 768 x 1024 -- bench/ab_i8_search.py -- and spills)
  // g_i8_opt (probe A/B only, lzk_set_i8_opt): 28 = the GEMM without the
  // candidate epilogue (OPT bit 2), 8 = no column prefilter
#define LZK_GIS(B)                              \
  do {                                          \
    switch (g_i8_opt) {                         \
      case 28: LZK_GIO(B, 28); break;           \
      case 8: LZK_GIO(B, 8); break;             \
      default: LZK_GIO(B, kCandOpt); break;     \
    }                                           \
  } while (0)
  if (bias) LZK_GIS(true);
  else LZK_GIS(false);
#undef LZK_GIS
#undef LZK_GIO
  return (int)hipGetLastError();
}

// int8 dual candidate pass (rows / queries int8 bytes with fp32 scales, see
// lzk_flat_cand_i8; labels as lzk_flat_cand_dual): list A unfiltered (thr),
// list B label-filtered (thr2), scores alpha * qscale * <q8, x8> * rscale + bias.
LZK_EXPORT int lzk_flat_cand_dual_i8(const void* X8, long ldx_bytes, int nrows, const void* Q8, long ldq_bytes,
                                     int nq, int D_bytes, const float* bias, const float* rscale,
                                     const float* qscale, const int* row_label, const int* q_label, float alpha,
                                     const float* thr, const float* thr2, int cap, int* cnt, float* cs, int* ci,
                                     int* cnt2, float* cs2, int* ci2, void* blk_buf, int blk_cap, int* blk_cnt,
                                     void* stream) {
  if (D_bytes % 128 != 0 || D_bytes > 1024 || (ldx_bytes | ldq_bytes) % 16 != 0 || nq <= 0 || nrows <= 0 ||
      cap <= 0 || !rscale || !qscale || !row_label || !q_label || !(alpha > 0.f))
    return (int)hipErrorInvalidValue;
  if (!blk_buf || blk_cap <= 0 || !blk_cnt) return (int)hipErrorInvalidValue;
  const BlkCands blk{(int4*)blk_buf, blk_cap, blk_cnt, rscale, qscale};
  const int n_rt = (nrows + BM - 1) / BM, n_qt = (nq + BN - 1) / BN;
  const long nblk = (long)n_rt * n_qt;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  const int ncu = n_cu();
  const int grid = (int)(nblk < ncu ? nblk : ncu);
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X8;
  const u16* q = (const u16*)Q8;
#define LZK_GDI(B)                                                                                                  \
  do {                                                                                                              \
    (void)hipFuncSetAttribute((const void*)flat_cand_persistent_kernel<B, true, true, kCandOpt, MmaI8>,             \
                              hipFuncAttributeMaxDynamicSharedMemorySize, CAND_P_LDS);                              \
    hipLaunchKernelGGL((flat_cand_persistent_kernel<B, true, true, kCandOpt, MmaI8>), dim3(grid), dim3(NT),        \
                       CAND_P_LDS, st, x, ldx_bytes / 2, nrows, q, ldq_bytes / 2, nq, D_bytes / 2, bias, row_label, \
                       q_label, alpha, thr, n_qt, (int)nblk, cap, cnt, cs, ci, thr2, cnt2, cs2, ci2, blk);          \
  } while (0)
  if (bias) LZK_GDI(true);
  else LZK_GDI(false);
#undef LZK_GDI
  return (int)hipGetLastError();
}

// int8 query + error margin of the store search (i8_query_kernel).
LZK_EXPORT int lzk_i8_query(const void* q16, long ldq, int nq, int Dp, int d, const double* sumsq, double inv_nsq,
                            const float* smax, float alpha_abs, float z, float xn, void* q8, long ld8, float* qs,
                            float* margin, float* margin_rig, void* stream) {
  if (nq <= 0) return 0;
  if (Dp <= 0 || d > Dp || !sumsq || !smax) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(i8_query_kernel, dim3((unsigned)nq), dim3(256), 0, (hipStream_t)stream, (const u16*)q16, ldq, Dp,
                     d, sumsq, inv_nsq, smax, alpha_abs, z, xn, (signed char*)q8, ld8, qs, margin, margin_rig);
  return (int)hipGetLastError();
}
