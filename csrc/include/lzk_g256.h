// 256x256x64 bf16 MFMA main loop, 8 waves, LDS-DMA staging with a counted
// vmcnt pipeline (gfx950 / CDNA4). Shared by the flat-search candidate kernel
// and the encoder projection GEMMs.
//
//   C[a][b] = sum_k A[a][k] * B[b][k]   (both operands K-contiguous rows)
//
// Geometry
//   * 512 threads = 8 waves as 2 (A halves) x 4 (B quarters); wave (wr, wc)
//     owns C rows [wr*128, +128) x cols [wc*64, +64) as 8 x 4 blocks of
//     v_mfma_f32_16x16x32_bf16 -> acc[8][4] (128 VGPRs).
//   * One K-tile = 4 half-tiles of 128 rows x 64 k (16 KiB each): HA0, HA1
//     (A rows 0-127 / 128-255) and HB0, HB1. Two K-tile buffers = 8 slots =
//     128 KiB of LDS, all in ONE dynamic __shared__ array.
//   * Each half-tile is staged by 16 wave-level global_load_lds_dwordx4 (1 KiB
//     = 8 rows x 128 B each, 2 per wave). The LDS image is lane-linear, so the
//     XOR swizzle (chunk ^= (row>>1)&7) is applied to the per-lane SOURCE
//     address and undone by the ds_read_b128 address; for the 16x16x32 lane
//     map every ds_read_b128 lane group touches 16 distinct 16-B bank slots.
//
// Schedule (per K-tile t, buffer b = t&1; four phases, each phase is
//   [ds_reads + DMA issue] s_barrier [lgkmcnt(0) MFMA x16] s_barrier):
//   p0: read A rows 0-63 of the wave's half + B cols 0-31; issue HA1,HB0 of t+1
//   p1: read A rows 64-127;                                 issue HB1 of t+1
//   p2: read B cols 32-63
//   p3: no reads;                issue HA0 of t+2, then s_waitcnt vmcnt(2)
//   MFMA quadrants: p0 (A0,B0), p1 (A1,B0), p2 (A1,B1), p3 (A0,B1).
// The waves with wr == 1 run one barrier behind (an extra s_barrier before
// the loop, matched by one after it for wr == 0), so on every SIMD one wave's
// MFMA section overlaps its partner's ds_read/issue section.
//
// Hazards, with phases numbered globally (P = 4t + p):
//   RAW  tile t+1 is complete once every wave passed the vmcnt(2) of phase
//        4t+3 (only HA0 of t+2 may remain in flight) and the barrier after it;
//        group 0 reads it after barrier 2P+2, group 1 after 2P+3.
//   WAR  a slot is re-staged >= 2 phases after its last ds_read (A slots:
//        last read p1, re-staged at p3 / next p0; B slots: last read p2,
//        re-staged at next p0 / p1), which orders the DMA after every
//        reader's lgkmcnt(0) for both barrier offsets.
// The vmcnt is never 0 in the steady state: one half-tile stays in flight
// across every K-tile boundary, three more are in flight inside a tile.
#pragma once
#include "lzk_common.h"

namespace g256 {

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BK = 64;
constexpr int NT = 512;
constexpr int HALF = 128 * BK;                   // bf16 elements per half-tile slot
constexpr int LDS_BYTES = 8 * HALF * 2;          // 128 KiB

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ int swz(int row, int kc) { return row * BK + ((kc ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void vm2() { asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); }

struct Stager {
  const u16* src[4][2];  // [slot HA0 HA1 HB0 HB1][piece]
  int dst[2];            // element offset of the wave's pieces inside a slot

  // rows past na / nb are clamped (callers mask their results)
  __device__ __forceinline__ void setup(const u16* A, long lda, int a0, int na, const u16* B, long ldb,
                                        int b0, int nb) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = wave * 2 + i;
      const int row = 8 * c + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      src[0][i] = A + (long)min(a0 + row, na - 1) * lda + kc * 8;
      src[1][i] = A + (long)min(a0 + 128 + row, na - 1) * lda + kc * 8;
      src[2][i] = B + (long)min(b0 + row, nb - 1) * ldb + kc * 8;
      src[3][i] = B + (long)min(b0 + 128 + row, nb - 1) * ldb + kc * 8;
      dst[i] = c * 512;
    }
  }
  template <int H>
  __device__ __forceinline__ void issue(u16* smem, int buf, int ks) const {
    u16* slot = smem + (buf * 4 + H) * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(src[H][i] + ks * BK), (lds_void_t*)(slot + dst[i]), 16, 0, 0);
  }
};

// 16 MFMAs of one quadrant: A frags a[mb][s] (rows mq*64 + mb*16), B frags
// b[nb][s] (cols nq*32 + nb*16).
template <int MQ, int NQ>
__device__ __forceinline__ void quad_mma(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2], const bf16x8 (&b)[2][2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        acc[MQ * 4 + mb][NQ * 2 + nb] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mb][s], b[nb][s], acc[MQ * 4 + mb][NQ * 2 + nb], 0, 0, 0);
}

typedef int i32x8 __attribute__((ext_vector_type(8)));

// MFMA policies: how one quadrant's fragments are consumed. The LDS image and
// the 16-B reads are the same for both: lane group g = lane>>4 reads 16-B
// chunks g and g+4 of each 128-B K-row. bf16 uses them as k-steps s = 0, 1 of
// 16x16x32; fp8 concatenates them into the 32-byte operand of the block-scaled
// 16x16x128 (unit E8M0 scales = plain fp8 GEMM at twice the bf16 rate). Any
// byte->k assignment is valid as long as A and B use the same one; this one
// keeps every ds_read_b128 lane group on 16 distinct bank slots.
struct MmaBf16 {
  static constexpr int KPER = 64;  // K elements per 128-B K-row
  static constexpr bool kInt = false;
  template <int MQ, int NQ>
  __device__ __forceinline__ static void quad(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2], const bf16x8 (&b)[2][2]) {
    quad_mma<MQ, NQ>(acc, a, b);
  }
};

struct MmaFp8 {
  static constexpr int KPER = 128;
  static constexpr bool kInt = false;
  __device__ __forceinline__ static i32x8 cat(const bf16x8& lo, const bf16x8& hi) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 l = __builtin_bit_cast(i32x4, lo), h = __builtin_bit_cast(i32x4, hi);
    return i32x8{l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
  }
  template <int MQ, int NQ>
  __device__ __forceinline__ static void quad(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2], const bf16x8 (&b)[2][2]) {
    i32x8 bb[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) bb[nb] = cat(b[nb][0], b[nb][1]);
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const i32x8 aa = cat(a[mb][0], a[mb][1]);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        acc[MQ * 4 + mb][NQ * 2 + nb] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            aa, bb[nb], acc[MQ * 4 + mb][NQ * 2 + nb], 0, 0, 0, 127, 0, 127);
    }
  }
};

// int8 rows / queries (per-row / per-query scales applied by the caller's
// epilogue): chunks g and g+4 of a 128-B K-row are the 16-byte operands of two
// v_mfma_i32_16x16x64_i8 (same cycles as 16x16x32 bf16 at twice the K: 2x the
// bf16 rate, exact int32 sums). acc holds the int32 accumulators' BIT
// PATTERNS (kInt): the zero-initialised f32x4 is int 0, and an epilogue must
// read them with __builtin_bit_cast, never as floats.
struct MmaI8 {
  static constexpr int KPER = 128;
  static constexpr bool kInt = true;
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  template <int MQ, int NQ>
  __device__ __forceinline__ static void quad(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2], const bf16x8 (&b)[2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          f32x4& c = acc[MQ * 4 + mb][NQ * 2 + nb];
          c = __builtin_bit_cast(f32x4, __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, a[mb][s]),
                                                                            __builtin_bit_cast(i32x4, b[nb][s]),
                                                                            __builtin_bit_cast(i32x4, c), 0, 0, 0));
        }
  }
};

struct NoExtra {
  __device__ __forceinline__ void operator()() const {}
};

// Prologue DMA of one output tile: the four half-tiles of K-tile 0 into
// buffer 0, then `extra()` (small per-tile epilogue operands a caller stages
// into spare LDS), then HA0 of K-tile 1. Every slot must be free (no wave
// still reading it): call it at kernel start or after body() returned.
// Cross-tile prefetch for persistent callers (KS even): the next tile's
// K-tiles 0 and 1 are staged as if they were K-tiles KS and KS+1 of the
// current loop (same buffer parity, same slots, same issue points), so the
// next tile's pipeline fill overlaps this tile's last K-tiles and epilogue
// instead of following them; extra() goes right after the next K-tile 0.
// The loop then returns with exactly the DMAs prologue() would have left in
// flight (next K-tile 1's A half-tile(s), youngest), so the next body starts
// with the same counted wait. Without prefetch (NoPrefetch, or on() false)
// the loop drains to vmcnt(0) and the caller runs prologue(). on() must be
// false when KS is odd (the next K-tile 0 would land in buffer 1).
struct NoPrefetch {
  static constexpr bool kAny = false;
  __device__ __forceinline__ bool on() const { return false; }
  template <int H>
  __device__ __forceinline__ void issue(u16*, int, int) const {}
  __device__ __forceinline__ void extra() const {}
};

// The next tile's operands as wave-uniform scalars: its per-lane source
// addresses are rebuilt at each issue (a few VALU in a read section) instead
// of holding a second Stager's 18 VGPRs through the main loop.
template <class Extra>
struct NextTile {
  static constexpr bool kAny = true;
  const u16* A;
  long lda;
  int a0, na;
  const u16* B;
  long ldb;
  int b0, nb;
  const Extra* ex;
  bool enabled;
  __device__ __forceinline__ bool on() const { return enabled; }
  template <int H>
  __device__ __forceinline__ void issue(u16* smem, int buf, int kt) const {
    Stager s;
    s.setup(A, lda, a0, na, B, ldb, b0, nb);
    s.issue<H>(smem, buf, kt);
  }
  __device__ __forceinline__ void extra() const { (*ex)(); }
};

// K-tile kt of the current tile, or (kt >= KS, prefetch on) K-tile kt-KS of the next.
template <int H, class Pre>
__device__ __forceinline__ void stage(u16* smem, const Stager& st, const Pre& pre, int buf, int kt, int KS) {
  if (kt < KS) st.issue<H>(smem, buf, kt);
  else if (Pre::kAny && pre.on()) pre.template issue<H>(smem, buf, kt - KS);
}

template <class Extra = NoExtra, int OPT = 0>
__device__ __forceinline__ void prologue(u16* smem, const Stager& st, int KS, const Extra& extra = Extra()) {
  st.issue<0>(smem, 0, 0);
  st.issue<1>(smem, 0, 0);
  st.issue<2>(smem, 0, 0);
  st.issue<3>(smem, 0, 0);
  extra();
  if (KS > 1) {
    st.issue<0>(smem, 1, 1);
    if constexpr ((OPT & 8) != 0) st.issue<1>(smem, 1, 1);  // two-phase body: both A halves of tile 1
  }
}

// Two-phase K loop (OPT bit 3): the same 64 MFMAs per wave and K-tile as
// body() below in two 32-MFMA phases, i.e. half the barriers per K-tile.
//   P0: read a0, a1, b(cols 0-31);  issue HB0, HB1 of t+1   | MFMA (A0,B0) (A1,B0)
//   P1: read b(cols 32-63);         issue HA0, HA1 of t+2   | MFMA (A1,B1) (A0,B1)
//       then s_waitcnt vmcnt(4): everything but A(t+2) landed
// Global intervals (group 0 reads in 4t, 4t+2; group 1 one interval later):
//   WAR  A slots of a buffer are last read at 4t+1 (group 1, P0) and
//        re-staged from 4t+2; B slots last read at 4t+3 and re-staged from
//        4t+4 (P0 of t+1 stages B of t+2 into the other buffer).
//   RAW  tile t+1 is waited for by group 0 at 4t+2 and group 1 at 4t+3, and
//        first read at 4t+4 behind the barrier.
template <class Mma, class Pre = NoPrefetch>
__device__ __forceinline__ void body2(u16* smem, const Stager& st, int KS, f32x4 (&acc)[8][4], bool stagger,
                                      const Pre& pre = Pre()) {
  const bool pre_on = Pre::kAny && pre.on();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int aoff[2][4][2], boff[2][2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) aoff[mq][mb][s] = swz(mq * 64 + mb * 16 + l16, 4 * s + lq);
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) boff[nq][nb][s] = swz((wc & 1) * 64 + nq * 32 + nb * 16 + l16, 4 * s + lq);
  }
  if (KS > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else vm0();
  bar();
  if (stagger && wr == 1) bar();

  bf16x8 a0[4][2], a1[4][2], b[2][2];
  for (int t = 0; t < KS; ++t) {
    const int buf = t & 1;
    const u16* As = smem + (buf * 4 + wr) * HALF;
    const u16* Bs = smem + (buf * 4 + 2 + (wc >> 1)) * HALF;
    // ---- P0 ----
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) a0[mb][s] = *reinterpret_cast<const bf16x8*>(As + aoff[0][mb][s]);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) b[nb][s] = *reinterpret_cast<const bf16x8*>(Bs + boff[0][nb][s]);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) a1[mb][s] = *reinterpret_cast<const bf16x8*>(As + aoff[1][mb][s]);
    }
    if (t + 1 < KS || pre_on) {
      stage<2>(smem, st, pre, buf ^ 1, t + 1, KS);
      stage<3>(smem, st, pre, buf ^ 1, t + 1, KS);
      if (t + 1 == KS) pre.extra();
    }
    bar();
    lgkm0();
    __builtin_amdgcn_s_setprio(1);
    Mma::template quad<0, 0>(acc, a0, b);
    Mma::template quad<1, 0>(acc, a1, b);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- P1 ----
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) b[nb][s] = *reinterpret_cast<const bf16x8*>(Bs + boff[1][nb][s]);
    if (t + 2 < KS || pre_on) {
      stage<0>(smem, st, pre, buf, t + 2, KS);
      stage<1>(smem, st, pre, buf, t + 2, KS);
      // t + 2 == KS + 1: this tile's operands all landed at P1 of K-tile KS-2
      if (t + 2 <= KS) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      vm0();
    }
    bar();
    lgkm0();
    __builtin_amdgcn_s_setprio(1);
    Mma::template quad<1, 1>(acc, a1, b);
    Mma::template quad<0, 1>(acc, a0, b);
    __builtin_amdgcn_s_setprio(0);
    bar();
  }
  if (stagger && wr == 0) bar();
}

// K loop after prologue() (K = KS * 64). On return acc[i][j][e] holds
//   C[wr*128 + i*16 + 4*(lane>>4) + e][wc*64 + j*16 + (lane&15)]
// and every wave has passed the final barrier with all of its DMA retired
// (smem may be reused or re-staged).
// OPT (schedule experiments, A/B results in profiles/ab_search_sched_r1.json): bit 0 = no
// s_setprio around the MFMA clusters, bit 1 = no wave-group stagger.
template <class Mma = MmaBf16, int OPT = 0, class Pre = NoPrefetch>
__device__ __forceinline__ void body(u16* smem, const Stager& st, int KS, f32x4 (&acc)[8][4],
                                     const Pre& pre = Pre()) {
  const bool pre_on = Pre::kAny && pre.on();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane LDS read offsets (elements) inside a slot
  int aoff[2][4][2], boff[2][2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) aoff[mq][mb][s] = swz(mq * 64 + mb * 16 + l16, 4 * s + lq);
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) boff[nq][nb][s] = swz((wc & 1) * 64 + nq * 32 + nb * 16 + l16, 4 * s + lq);
  }

  // tile 0 (and anything issued before HA0 of tile 1) complete; at most the
  // 2 youngest DMAs (HA0 of tile 1) in flight
  if (KS > 1) vm2();
  else vm0();
  bar();
  if (!(OPT & 2) && wr == 1) bar();

  bf16x8 a0[4][2], a1[4][2], b[2][2];
  for (int t = 0; t < KS; ++t) {
    const int buf = t & 1;
    const u16* As = smem + (buf * 4 + wr) * HALF;
    const u16* Bs = smem + (buf * 4 + 2 + (wc >> 1)) * HALF;
    const bool nxt = t + 1 < KS;
    // ---- p0 ----
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) a0[mb][s] = *reinterpret_cast<const bf16x8*>(As + aoff[0][mb][s]);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) b[nb][s] = *reinterpret_cast<const bf16x8*>(Bs + boff[0][nb][s]);
    }
    if (nxt || pre_on) {
      stage<1>(smem, st, pre, buf ^ 1, t + 1, KS);
      stage<2>(smem, st, pre, buf ^ 1, t + 1, KS);
    }
    bar();
    lgkm0();
    if constexpr (!(OPT & 1)) __builtin_amdgcn_s_setprio(1);
    Mma::template quad<0, 0>(acc, a0, b);
    if constexpr (!(OPT & 1)) __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- p1 ----
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) a1[mb][s] = *reinterpret_cast<const bf16x8*>(As + aoff[1][mb][s]);
    if (nxt || pre_on) {
      stage<3>(smem, st, pre, buf ^ 1, t + 1, KS);
      if (!nxt) pre.extra();
    }
    bar();
    lgkm0();
    if constexpr (!(OPT & 1)) __builtin_amdgcn_s_setprio(1);
    Mma::template quad<1, 0>(acc, a1, b);
    if constexpr (!(OPT & 1)) __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- p2 ----
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) b[nb][s] = *reinterpret_cast<const bf16x8*>(Bs + boff[1][nb][s]);
    bar();
    lgkm0();
    if constexpr (!(OPT & 1)) __builtin_amdgcn_s_setprio(1);
    Mma::template quad<1, 1>(acc, a1, b);
    if constexpr (!(OPT & 1)) __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- p3 ----
    if (t + 2 < KS || pre_on) {
      stage<0>(smem, st, pre, buf, t + 2, KS);
      if (t + 2 <= KS) vm2();  // t + 2 == KS + 1: this tile's operands all landed at p3 of K-tile KS-2
    } else {
      vm0();
    }
    bar();
    if constexpr (!(OPT & 1)) __builtin_amdgcn_s_setprio(1);
    Mma::template quad<0, 1>(acc, a0, b);
    if constexpr (!(OPT & 1)) __builtin_amdgcn_s_setprio(0);
    bar();
  }
  if (!(OPT & 2) && wr == 0) bar();
}

template <class Mma = MmaBf16>
__device__ __forceinline__ void mainloop(u16* smem, const Stager& st, int KS, f32x4 (&acc)[8][4]) {
  prologue<NoExtra, 8>(smem, st, KS);
  body2<Mma>(smem, st, KS, acc, true);
}

// Persistent tile walk: the blocks resident on one XCD (blocks are dealt to
// the 8 XCDs round-robin) take consecutive tiles of that XCD's contiguous
// share, so concurrently running tiles of an XCD share operand panels in its
// L2. Speed only: every tile is visited exactly once for any grid size.
struct TileWalk {
  int next, end, step;
  __device__ __forceinline__ void init(int n_tiles) {
    const int G = gridDim.x, b = blockIdx.x;
    const int x = b % 8, s = b / 8;
    const int nb = (G - x + 7) / 8;          // blocks on this XCD
    const int per = (n_tiles + 7) / 8;       // tiles per XCD share
    const int lo = min(x * per, n_tiles);
    end = min(lo + per, n_tiles);
    next = lo + s;
    step = nb;
  }
  __device__ __forceinline__ bool valid(int t) const { return t < end; }
};

}  // namespace g256
