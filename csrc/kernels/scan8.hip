// int8 candidate scan for the store search and the consolidation dual search
// (reference src/lazzaro/core/vector_store.py:132-140 search_nodes, and the
// dedupe / link searches of memory_system.py:719-733, 816-836, 853-889;
// SURVEY.md §2.4 K1/K5/K6). Same contract as the persistent candidate kernel
// of search256.hip (block-private (query, row, score, lists) records, gathered
// and selected by the caller), written for the int8 shape:
//
//   score(q, r) = alpha * qs[q] * (rs[r] * <q8[q], x8[r]>) + bias[r]
//
// with v_mfma_i32_16x16x64_i8 on a 256 x 256 tile (8 waves as 2 x 4, 128 x 64
// per wave, acc = 8 x 4 int32x4 = 128 VGPRs). What changes against the shared
// 256^2 template at int8 (K = 768 bytes is only 6 K-tiles of 128 B, so the
// per-tile fixed costs decide the rate):
//
//  * One continuous K-tile stream across the block's tiles. The operands are
//    staged with buffer_load ... lds through per-tile SGPR descriptors (the
//    per-lane part is a tile-invariant 32-bit offset: 4 VGPRs in all), so the
//    next tile's first K-tiles are issued during the current tile's last ones
//    and the pipeline never drains at a tile boundary. Rows past the end are
//    cut by the descriptor's record count (and masked in the epilogue).
//  * The first K-tile of a tile feeds the MFMAs a literal zero accumulator,
//    so nothing re-initialises the 128 accumulator registers.
//  * The epilogue bounds the scores before converting them: per lane and
//    16-row block i, the max of its 4 int32 sums times the largest row scale
//    of those 4 rows (+ their largest bias) bounds all 4 scores (one
//    {scale, bias} pair per 4-row quad, staged with the tile's other epilogue
//    operands); a query column whose 8 block bounds all miss its threshold is
//    skipped, and only a block whose bound clears it converts its sums. (A
//    bound over the 128-row group's largest scale instead was ~35 % loose on
//    unit rows: 98 % of the columns and half the blocks went through the
//    per-score path at a store-search threshold.) It sits between two
//    MFMA phases of the staggered wave groups, so one group's epilogue runs
//    beside the other group's MFMAs on every SIMD.
//
// Schedule per K-tile g (buffer g & 1; group 1 = waves 4-7 one barrier behind):
//   P0: ds_read A rows 0-127 of the wave's half, B cols 0-31; issue B(g+1)
//       [+ the next tile's epilogue operands] | lgkm0, bar | 32 MFMA | bar
//   P1: ds_read B cols 32-63; issue A(g+2); vmcnt(A(g+2))  | lgkm0, bar | 32 MFMA | bar
// Every ds_read is retired (lgkmcnt 0) before the barrier that ends its
// interval, so a slot may be re-staged in the very next interval (WAR); a
// K-tile is waited for (vmcnt) one interval before any wave reads it (RAW).
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

// 16 MFMAs of one output quadrant (rows mq*64 .., cols nq*32 ..), two K
// halves s = 0, 1 of the 128-B K-row; FIRST: the s = 0 MFMA starts from 0.
template <int MQ, int NQ, bool FIRST>
__device__ __forceinline__ void quad(i32x4 (&acc)[8][4], const i32x4 (&a)[4][2], const i32x4 (&b)[2][2]) {
  const i32x4 z = {0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        i32x4& c = acc[MQ * 4 + mb][NQ * 2 + nb];
        c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mb][s], b[nb][s], (FIRST && s == 0) ? z : c, 0, 0, 0);
      }
}

template <bool V>
struct BoolTag {
  static constexpr bool value = V;
};

template <bool HAS_BIAS, bool DUAL>
__global__ __launch_bounds__(NT, 1) void scan8_kernel(
    const signed char* __restrict__ X, long ldx, int nrows, const signed char* __restrict__ Qm, long ldq, int nq,
    int KS, const float* __restrict__ bias, const float* __restrict__ rs, const float* __restrict__ qs,
    const float* __restrict__ grp, int ngrp, const int* __restrict__ row_label, const int* __restrict__ q_label,
    float alpha, const float* __restrict__ thr, const float* __restrict__ thr2, int n_qt, int n_tiles, Recs rec) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* epi = reinterpret_cast<float*>(smem + RING);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int l16 = lane & 15, lq = lane >> 4;

  // persistent walk: the blocks of one XCD take consecutive tiles of that
  // XCD's contiguous share (the 4 query tiles of a row tile run side by side
  // and share it in the XCD's L2)
  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid % 8, slot_in = bid / 8;
  const int nb_x = (G - xcd + 7) / 8;
  const int per = (n_tiles + 7) / 8;
  const int lo = min(xcd * per, n_tiles);
  const int t_end = min(lo + per, n_tiles);
  int cur = lo + slot_in;
  if (cur >= t_end) {
    if (lane == 0) rec.cnt[bid * 8 + wave] = 0;
    return;
  }
  const int step = nb_x;

  // tile-invariant per-lane staging offsets: piece c = 2 * wave + i covers
  // rows 8c .. 8c+7 of a half-tile; the 16-B chunk is XOR-swizzled on the
  // SOURCE address (the LDS image is lane-linear), undone by the reads. The
  // half-tile's row offset is part of the VGPR offset (index [h]): the buffer
  // range check covers the VGPR offset only -- not the SGPR offset, which
  // carries just the K-tile's byte offset (< one row) -- so rows past the
  // tile's last valid row read as zero instead of past the operand.
  int voA[2][2], voB[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = wave * 2 + i;
      const int row = 8 * c + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      voA[h][i] = (int)((128 * h + row) * ldx) + kc * 16;
      voB[h][i] = (int)((128 * h + row) * ldq) + kc * 16;
    }
  // per-lane read bases inside a slot: row l16 of a 16-row block, chunk
  // (4s + lq) ^ ((l16 >> 1) & 7); the block's row offset is an immediate
  int rb[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) rb[s] = l16 * 128 + (((4 * s + lq) ^ ((l16 >> 1) & 7)) << 4);

  auto geo = [&](int t) {
    TileGeo g;
    g.r0 = (t / n_qt) * 256;
    g.q0 = (t % n_qt) * 256;
    return g;
  };
  // H: 0/1 = A rows 0-127 / 128-255, 2/3 = B cols 0-127 / 128-255
  auto issue = [&](int t, int kt, int buf, int H) {
    const TileGeo g = geo(t);
    const bool isA = H < 2;
    const long ld = isA ? ldx : ldq;
    const int n_left = isA ? min(256, nrows - g.r0) : min(256, nq - g.q0);
    const signed char* base = isA ? X + (long)g.r0 * ldx : Qm + (long)g.q0 * ldq;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(base, (long)n_left * ld);
    const int soff = kt * 128;
    unsigned char* sl = smem + (buf * 4 + H) * SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(sl + (wave * 2 + i) * 1024), 16,
                                               isA ? voA[H & 1][i] : voB[H & 1][i], soff, 0, 0);
  };
  // epilogue operands of tile t -> parity p: 4 wave-level DMAs (64 x 4 B)
  // per array, spread over the 8 waves
  auto stage_epi = [&](int t, int p) {
    const TileGeo g = geo(t);
#pragma unroll
    for (int k = wave; k < 4 * NARR; k += 8) {
      const int a = k >> 2, c = k & 3;  // wave-uniform
      const bool need = a == 0 || (a == 1 && HAS_BIAS) || a == 2 || a == 3 || (DUAL && (a == 4 || a == 5 || a == 6)) ||
                        (a == 7 && c < 2);
      if (!need) continue;
      const void* src;
      if (a == 0) src = thr + min(g.q0 + c * 64 + lane, nq - 1);
      else if (a == 1) src = bias + min(g.r0 + c * 64 + lane, nrows - 1);
      else if (a == 2) src = rs + min(g.r0 + c * 64 + lane, nrows - 1);
      else if (a == 3) src = qs + min(g.q0 + c * 64 + lane, nq - 1);
      else if (a == 4) src = thr2 + min(g.q0 + c * 64 + lane, nq - 1);
      else if (a == 5) src = row_label + min(g.r0 + c * 64 + lane, nrows - 1);
      else if (a == 6) src = q_label + min(g.q0 + c * 64 + lane, nq - 1);
      else src = grp + min(2 * (g.r0 >> 2) + c * 64 + lane, 2 * ngrp - 1);  // {rs4, b4} of the tile's 64 quads
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(epi + (p * NARR + a) * 256 + c * 64), 4, 0, 0);
    }
  };

  // Candidate appends: each wave owns 1/8 of the block's record region and
  // keeps its fill count in a scalar register (ballot + mbcnt), so appending
  // needs no atomic -- an LDS atomic would make the compiler drain the
  // in-flight operand DMA (vmcnt(0)) before it.
  const int capw = rec.cap;
  int4* wbuf = rec.buf + (long)(bid * 8 + wave) * capw;
  int4* lrec = reinterpret_cast<int4*>(smem + REC_OFF) + wave * LREC;
  int wpos = 0;  // records of this wave written to its global region (wave-uniform)
  int lpos = 0;  // records staged in its LDS slots (wave-uniform)
  auto flush = [&]() {  // staged records -> the global region, one 16-B store per lane
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the staged writes landed
    if (lane < lpos) {
      const int4 v = lds_read16(lrec + lane);
      if (wpos + lane < capw) wbuf[wpos + lane] = v;
    }
    if (lpos > 64 && lane < lpos - 64) {
      const int4 v = lds_read16(lrec + 64 + lane);
      if (wpos + 64 + lane < capw) wbuf[wpos + 64 + lane] = v;
    }
    wpos += lpos;
    lpos = 0;
  };
  auto append = [&](bool take, int lists, int q, float v, int r) {
    const unsigned long long ball = __ballot(take);
    if (ball == 0ull) return;
    const int nb = __builtin_popcountll(ball);
    if (lpos + nb > LREC) flush();
    const int pos = lpos + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(ball >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((unsigned)ball, 0u));
    if (take) lds_write16(lrec + pos, make_int4(q, r, __float_as_int(v), lists));
    lpos += nb;
  };

  // ---- prologue: K-tile 0 of the first tile + its epilogue operands (buffer
  // 0), then A of K-tile 1 (buffer 1); KS >= 2 (host-checked)
  issue(cur, 0, 0, 0);
  issue(cur, 0, 0, 1);
  issue(cur, 0, 0, 2);
  issue(cur, 0, 0, 3);
  stage_epi(cur, 0);
  issue(cur, 1, 1, 0);
  issue(cur, 1, 1, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  bar();
  if (wr == 1) bar();  // stagger: group 1 runs one barrier interval behind

  i32x4 acc[8][4];
  i32x4 a0[4][2], a1[4][2], b[2][2];
  int tix = 0;  // tile sequence number (epilogue parity)
  int gpar = 0; // buffer of the current K-tile

  // one K-tile: two phases (see the header)
  auto ktile = [&](auto first_tag, int kt, int nxt, bool has_nxt) {
    constexpr bool FIRST = decltype(first_tag)::value;
    const unsigned char* As = smem + (gpar * 4 + wr) * SLOT;
    const unsigned char* Bs = smem + (gpar * 4 + 2 + (wc >> 1)) * SLOT;
    const int bcol = (wc & 1) * 64;
    // ---- P0 ----
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) a0[mb][s] = *reinterpret_cast<const i32x4*>(As + rb[s] + (mb * 16) * 128);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) b[nb][s] = *reinterpret_cast<const i32x4*>(Bs + rb[s] + (bcol + nb * 16) * 128);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) a1[mb][s] = *reinterpret_cast<const i32x4*>(As + rb[s] + (64 + mb * 16) * 128);
    }
    if (kt + 1 < KS) {
      issue(cur, kt + 1, gpar ^ 1, 2);
      issue(cur, kt + 1, gpar ^ 1, 3);
    } else if (has_nxt) {
      issue(nxt, 0, gpar ^ 1, 2);
      issue(nxt, 0, gpar ^ 1, 3);
      stage_epi(nxt, (tix + 1) & 1);
    }
    lgkm0();
    bar();
    __builtin_amdgcn_s_setprio(1);
    quad<0, 0, FIRST>(acc, a0, b);
    quad<1, 0, FIRST>(acc, a1, b);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- P1 ----
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        b[nb][s] = *reinterpret_cast<const i32x4*>(Bs + rb[s] + (bcol + 32 + nb * 16) * 128);
    bool issued = true;
    if (kt + 2 < KS) {
      issue(cur, kt + 2, gpar, 0);
      issue(cur, kt + 2, gpar, 1);
    } else if (has_nxt) {
      issue(nxt, kt + 2 - KS, gpar, 0);
      issue(nxt, kt + 2 - KS, gpar, 1);
    } else {
      issued = false;
    }
    if (issued) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lgkm0();
    bar();
    __builtin_amdgcn_s_setprio(1);
    quad<1, 1, FIRST>(acc, a1, b);
    quad<0, 1, FIRST>(acc, a0, b);
    __builtin_amdgcn_s_setprio(0);
    bar();
    gpar ^= 1;
  };

  while (true) {
    const int nxt = cur + step;
    const bool has_nxt = nxt < t_end;
    ktile(BoolTag<true>{}, 0, nxt, has_nxt);
    for (int kt = 1; kt < KS; ++kt) ktile(BoolTag<false>{}, kt, nxt, has_nxt);

    // ---- epilogue of `cur` (operands from LDS only) ----
    {
      const TileGeo g = geo(cur);
      const float* E = epi + (tix & 1) * (NARR * 256);
      const float2* S4 = reinterpret_cast<const float2*>(E + 7 * 256) + wr * 32 + lq;  // quad (i, lq) at [4 i]
      const bool full = g.r0 + 256 <= nrows;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qlo = wc * 64 + j * 16 + l16;
        const int q = g.q0 + qlo;
        const float th = q < nq ? E[qlo] : __builtin_huge_valf();
        const float th2 = (DUAL && q < nq) ? E[4 * 256 + qlo] : __builtin_huge_valf();
        const float tlo = DUAL ? fminf(th, th2) : th;
        const float tcut = tlo - 1e-6f * fabsf(tlo);  // slack: the per-score path may contract differently
        const float al = alpha * E[3 * 256 + qlo];
        // bit i: the bound of the lane's 4 rows of block i clears tcut --
        // every score there is <= al * max(m, 0) * rs4 + b4 (al >= 0)
        unsigned pm = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const i32x4 v = acc[i][j];
          const int mi = max(max(v[0], v[1]), max(v[2], v[3]));
          const float2 s4 = S4[4 * i];
          const float bnd = (mi > 0 ? al * ((float)mi * s4.x) : 0.f) + s4.y;
          pm |= (bnd >= tcut ? 1u : 0u) << i;
        }
        // the skips are wave-uniform (ballots), so the append counter wpos
        // stays uniform -- a lane that skipped would miss the counts
        if (__ballot(pm != 0u) == 0ull) continue;
        const int qlab = DUAL ? reinterpret_cast<const int*>(E)[6 * 256 + qlo] : -1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (__ballot((pm >> i) & 1u) == 0ull) continue;
          const i32x4 v = acc[i][j];
          const int rl = wr * 128 + i * 16 + 4 * lq;
          const f32x4 rsv = *reinterpret_cast<const f32x4*>(E + 2 * 256 + rl);
          f32x4 bv = {0.f, 0.f, 0.f, 0.f};
          if (HAS_BIAS) bv = *reinterpret_cast<const f32x4*>(E + 256 + rl);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = g.r0 + rl + e;
            const float sc = al * ((float)v[e] * rsv[e]) + bv[e];
            const bool ok = (full || r < nrows) && q < nq && sc != LZK_NEG_INF;
            int lists = (ok && sc >= th) ? 1 : 0;
            if (DUAL && ok && sc >= th2) {
              const int rlab = reinterpret_cast<const int*>(E)[5 * 256 + rl + e];
              if (qlab < 0 || rlab == qlab) lists |= 2;
            }
            append(lists != 0, lists, q, sc, r);
          }
        }
      }
    }
    ++tix;
    if (!has_nxt) break;
    cur = nxt;
  }
  if (wr == 0) bar();  // un-stagger
  flush();
  if (lane == 0) rec.cnt[bid * 8 + wave] = wpos;  // > cap: records were dropped
}

// {max row scale, max bias} of every 4-row quad (the epilogue's bounds).
template <bool HAS_BIAS>
__global__ __launch_bounds__(256) void quad_stats_kernel(const float* __restrict__ rs, const float* __restrict__ bias,
                                                         int nrows, int nquad, float* __restrict__ q4) {
  const int qi = blockIdx.x * 256 + threadIdx.x;
  if (qi >= nquad) return;
  float m = 0.f, bm = HAS_BIAS ? LZK_NEG_INF : 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = qi * 4 + e;
    if (r < nrows) {
      m = fmaxf(m, rs[r]);
      if (HAS_BIAS) bm = fmaxf(bm, bias[r]);
    }
  }
  q4[2 * qi] = m;
  q4[2 * qi + 1] = bm;
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

template <bool HAS_BIAS, int NQT>
__global__ __launch_bounds__(NW_WAVES * 64, 1) void scan8_narrow_kernel(
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
  i32x4 fa[NW_MAXK], fb[NW_MAXK];
  auto load = [&](i32x4 (&a)[NW_MAXK], int b) {
    const int r = min(b * 16 + l16, nrows - 1);
    const signed char* src = X + (long)r * ldx + lq * 16;
#pragma unroll
    for (int kk = 0; kk < NW_MAXK; ++kk)
      if (kk < KK) a[kk] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(src + kk * 64));
  };
  auto body = [&](const i32x4 (&a)[NW_MAXK], int b) {
    i32x4 acc[NQT];
#pragma unroll
    for (int t = 0; t < NQT; ++t) acc[t] = (i32x4){0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < NW_MAXK; ++kk) {
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

// Grid (block-record count) of lzk_scan8 for a shape.
LZK_EXPORT int lzk_scan8_grid(int nrows, int nq) {
  const long nblk = (long)((nrows + 255) / 256) * ((nq + 255) / 256);
  const int n = cu_count();
  return (int)(nblk < n ? nblk : n);
}

// Bytes of the group-stats workspace lzk_scan8 needs.
LZK_EXPORT long lzk_scan8_ws_bytes(int nrows) { return (long)((nrows + 3) / 4) * 8 + 256; }

// int8 candidate scan (single list: thr2/labels null; dual: both lists, see
// lzk_flat_cand_dual). X8 / Q8: int8 rows / queries with byte strides (16-B
// multiples), D_bytes % 128 == 0, 256 <= D_bytes <= 1024; rscale / qscale
// fp32 (>= 0). Records go to blk_buf [grid * 8][blk_cap] (one region per
// wave, grid = lzk_scan8_grid) with counts blk_cnt [grid * 8]; gather them
// with lzk_cand_gather over grid * 8 regions (same record format).
// ws: lzk_scan8_ws_bytes.
LZK_EXPORT int lzk_scan8(const void* X8, long ldx, int nrows, const void* Q8, long ldq, int nq, int D_bytes,
                         const float* bias, const float* rscale, const float* qscale, const int* row_label,
                         const int* q_label, float alpha, const float* thr, const float* thr2, void* ws,
                         void* blk_buf, int blk_cap, int* blk_cnt, void* stream) {
  const bool dual = thr2 != nullptr;
  if (D_bytes % 128 != 0 || D_bytes < 256 || D_bytes > 1024 || (ldx | ldq) % 16 != 0 || nq <= 0 || nrows <= 0 ||
      !rscale || !qscale || !thr || !ws || !blk_buf || blk_cap <= 0 || !blk_cnt || !(alpha > 0.f))
    return (int)hipErrorInvalidValue;
  if (dual && (!row_label || !q_label)) return (int)hipErrorInvalidValue;
  // 32-bit buffer offsets: a 256-row tile of either operand must fit
  if (256L * ldx >= (1L << 31) || 256L * ldq >= (1L << 31)) return (int)hipErrorInvalidValue;
  const int n_rt = (nrows + 255) / 256, n_qt = (nq + 255) / 256;
  const long nblk = (long)n_rt * n_qt;
  if (nblk > 0x7fffffffL) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int ngrp = (nrows + 3) / 4;  // 4-row quads
  float* grp = (float*)ws;
  if (bias)
    hipLaunchKernelGGL(quad_stats_kernel<true>, dim3((ngrp + 255) / 256), dim3(256), 0, st, rscale, bias, nrows, ngrp,
                       grp);
  else
    hipLaunchKernelGGL(quad_stats_kernel<false>, dim3((ngrp + 255) / 256), dim3(256), 0, st, rscale, bias, nrows, ngrp,
                       grp);
  const int grid = lzk_scan8_grid(nrows, nq);
  const Recs rec{(int4*)blk_buf, blk_cap, blk_cnt};
  const signed char* x = (const signed char*)X8;
  const signed char* q = (const signed char*)Q8;
  const int KS = D_bytes / 128;
#define LZK_S8(B, DU)                                                                                              \
  do {                                                                                                             \
    (void)hipFuncSetAttribute((const void*)scan8_kernel<B, DU>, hipFuncAttributeMaxDynamicSharedMemorySize,        \
                              LDS_TOTAL);                                                                          \
    hipLaunchKernelGGL((scan8_kernel<B, DU>), dim3(grid), dim3(NT), LDS_TOTAL, st, x, ldx, nrows, q, ldq, nq, KS,   \
                       bias, rscale, qscale, (const float*)grp, ngrp, row_label, q_label, alpha, thr, thr2, n_qt,  \
                       (int)nblk, rec);                                                                            \
  } while (0)
  if (bias && dual) LZK_S8(true, true);
  else if (bias) LZK_S8(true, false);
  else if (dual) LZK_S8(false, true);
  else LZK_S8(false, false);
#undef LZK_S8
  return (int)hipGetLastError();
}

// Narrow-batch int8 scan (nq < 128): grid (blocks) for a shape; the record
// regions are grid * 8 (one per wave), the same format as lzk_scan8.
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
#define LZK_NW(B, T)                                                                                           \
  do {                                                                                                         \
    (void)hipFuncSetAttribute((const void*)scan8_narrow_kernel<B, T>,                                          \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                          \
    hipLaunchKernelGGL((scan8_narrow_kernel<B, T>), dim3(grid), dim3(NW_WAVES * 64), lds, st, x, ldx, nrows, q, \
                       ldq, nq, KK, bias, rscale, qscale, alpha, thr, rec);                                    \
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
  return (int)hipGetLastError();
}
