// On-device sentence-transformer encoder kernels (BERT family: MiniLM-L6,
// bge-base, e5-large). Replaces the reference's remote embedding calls
// (reference src/lazzaro/core/providers.py:36-57, 101-128, 170-196) with a
// local forward pass; SURVEY.md §2.4 K14.
//
//   gemm_bias_act  Y = act(X W^T + b) (+ R)  -- MFMA 128x128x64 tiles, features on
//                  the MFMA M axis so each lane stores 4 consecutive outputs (8 B)
//   attention      flash-style per (sequence, head, 32-query block): S^T = K Q^T on
//                  MFMA, online softmax lane-local (keys in registers), O^T = V^T P
//                  with the accumulator reused as the B operand (no LDS for P)
//   layernorm      y = LN(x + r) * g + b, one wave per token row
//   embed_ln       word + position + type embedding gather fused with LayerNorm
//   pool_norm      masked mean / CLS pooling + L2 normalisation (+ bf16 copy
//                  padded to the index arena's width)
#include "lzk_g256.h"
#include "lzk_tile.h"

#include <cstdlib>

namespace {

using namespace lzk;

// GELU(x) = x/2 (1 + erf(x/sqrt2)) with erf as an odd degree-17 polynomial
// z P(z^2) (least-squares minimax fit on |z| <= 3, coefficients below), z
// clamped to +-Zc beyond. The polynomial's terms cancel heavily near |z| = 3,
// so its value there depends on the FMA evaluation order at the 1e-5 level;
// the negative tail therefore clamps x itself (x >= -Zc sqrt2): GELU of any
// x below is returned as GELU(-4.24) ~ 1e-5 (true value < 5e-5) instead of
// x * 1e-5 growing with |x|. |error| < 1e-4 over the fp32 range (test:
// tests/kernels/test_kernels_gpu.py::test_gelu_polynomial_extremes), far below
// a bf16 ulp of the output. Only FMAs -- no v_rcp / v_exp, which issue at a
// quarter of the VALU rate (the erf-based epilogue cost the FFN1 tiles ~6 us
// per 256x256 tile at 11k tokens).
#define LZK_GELU_P(X) \
  X(1.128268480e+00f) X(-3.753148913e-01f) X(1.110793427e-01f) X(-2.510286681e-02f) X(4.235429689e-03f) \
  X(-5.110373604e-04f) X(4.106058259e-05f) X(-1.944826636e-06f) X(4.074221138e-08f)
constexpr float kGeluZc = 3.000014066696167f;
constexpr float kGeluXc = 4.2426605f;  // Zc * sqrt(2)
constexpr float kGeluC[9] = {
#define LZK_C(v) v,
    LZK_GELU_P(LZK_C)
#undef LZK_C
};

__device__ __forceinline__ float gelu_erf(float x) {
  const float xc = fmaxf(x, -kGeluXc);
  const float z = fminf(xc * 0.70710678118654752f, kGeluZc);
  const float u = z * z;
  float p = kGeluC[8];
#pragma unroll
  for (int k = 7; k >= 0; --k) p = __builtin_fmaf(p, u, kGeluC[k]);
  const float hx = 0.5f * xc;
  return __builtin_fmaf(hx, p * z, hx);
}

// Two lanes of work per instruction: the clamps are scalar v_max / v_min,
// everything else packed fp32 (v_pk_mul_f32 / v_pk_fma_f32).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const f32x2 xc = {fmaxf(x.x, -kGeluXc), fmaxf(x.y, -kGeluXc)};
  const f32x2 zs = xc * 0.70710678118654752f;
  const f32x2 z = {fminf(zs.x, kGeluZc), fminf(zs.y, kGeluZc)};
  const f32x2 u = z * z;
  f32x2 p = {kGeluC[8], kGeluC[8]};
#pragma unroll
  for (int k = 7; k >= 0; --k) p = __builtin_elementwise_fma(p, u, (f32x2){kGeluC[k], kGeluC[k]});
  const f32x2 hx = 0.5f * xc;
  return __builtin_elementwise_fma(hx, p * z, hx);
}

// ---------------------------------------------------------------- GEMM
template <int ACT, bool RES, bool GLDS>
__global__ __launch_bounds__(TNT, 2) void gemm_bias_act_kernel(
    const u16* __restrict__ X, long ldx, int T, const u16* __restrict__ W, long ldw, int N,
    const float* __restrict__ bias, const u16* __restrict__ R, long ldr, u16* __restrict__ Y,
    long ldy, int K, int n_ft) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tt = logical / n_ft, ft = logical % n_ft;
  const int n0 = ft * TB, t0 = tt * TB;
  f32x16 acc[2][2];
  if (GLDS) tile_gemm_glds(smem, W, ldw, n0, N, X, ldx, t0, T, K, acc);
  else tile_gemm(smem, W, ldw, n0, N, X, ldx, t0, T, K, acc);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wrow = wave >> 1, wcol = wave & 1, h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int t = t0 + wcol * 64 + cb * 32 + l32;
    if (t >= T) continue;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wrow * 64 + rb * 32 + 8 * g + 4 * h;
        if (n >= N) continue;
        f32x4 bv = *reinterpret_cast<const f32x4*>(bias + n);
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = acc[rb][cb][4 * g + u] + bv[u];
        if (ACT == 1) {
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = gelu_erf(v[u]);
        }
        if (RES) {
          u16x4 rv = *reinterpret_cast<const u16x4*>(R + (long)t * ldr + n);
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] += bf16_to_f32(rv[u]);
        }
        u16x4 o;
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = f32_to_bf16(v[u]);
        *reinterpret_cast<u16x4*>(Y + (long)t * ldy + n) = o;
      }
    }
  }
}

// 256x256 tiles on the 8-wave counted-vmcnt pipeline (lzk_g256.h): features
// (W rows) on the A side, tokens on B. Epilogue in two passes through the
// (then idle) LDS: (1) bias + activation in the MFMA layout (lane = token,
// 4 consecutive features), bf16 into a [token][feature] image with 520-B rows
// (conflict-free 8-B writes); (2) one wave per token row streams 512
// contiguous bytes to Y (+ the residual row read the same way), so stores
// and residual loads are whole cache lines instead of 32-B pieces.
constexpr int G256_OUT_LD = g256::BN + 4;  // u16 per LDS output row (520 B)
constexpr int G256_GEMM_LDS = (g256::BM * G256_OUT_LD * 2 > g256::LDS_BYTES) ? g256::BM * G256_OUT_LD * 2
                                                                              : g256::LDS_BYTES;

// One 256x256 output tile `logical` (token tile = logical / n_ft). `plain`
// (wave-uniform): no bias and no residual -- the second K-half of a split-K
// pair (gemm256_split2_kernel).
template <int ACT, bool RES, int BODY>
__device__ __forceinline__ void gemm256_tile(u16* smem, const u16* __restrict__ X, long ldx, int T,
                                             const u16* __restrict__ W, long ldw, int N,
                                             const float* __restrict__ bias, const u16* __restrict__ R, long ldr,
                                             u16* __restrict__ Y, long ldy, int K, int n_ft, int logical,
                                             bool plain) {
  const int tt = logical / n_ft, ft = logical % n_ft;
  const int n0 = ft * g256::BM, t0 = tt * g256::BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  float* sbias = reinterpret_cast<float*>(smem + g256::LDS_BYTES / 2);  // 1 KiB past the staging slots
  g256::Stager st;
  st.setup(W, ldw, n0, N, X, ldx, t0, T);
  const int KS = K / g256::BK;
  // the tile's 256 bias values ride along with the prologue DMA (no global
  // load latency in the epilogue)
  auto stage_bias = [&]() {
    if (wave < 4 && !plain)
      __builtin_amdgcn_global_load_lds((g256::gbl_void_t*)(bias + min(n0 + wave * 64 + lane, N - 1)),
                                       (g256::lds_void_t*)(sbias + wave * 64), 4, 0, 0);
  };
  f32x4 acc[8][4];
  if constexpr (BODY == 1) {  // two-phase main loop (lzk_g256.h body2)
    g256::prologue<decltype(stage_bias), 8>(smem, st, KS, stage_bias);
    g256::body2<g256::MmaBf16>(smem, st, KS, acc, true);
  } else {
    g256::prologue(smem, st, KS, stage_bias);
    g256::body(smem, st, KS, acc);
  }
  if (ACT == 9) {  // measurement probe (act=9): main loop only, epilogue cost = difference
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) z += acc[i][j][0];
    if (z != z) Y[threadIdx.x] = 0;
    return;
  }
  f32x4 bv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    bv[i] = plain ? (f32x4){0.f, 0.f, 0.f, 0.f}
                  : *reinterpret_cast<const f32x4*>(sbias + wr * 128 + i * 16 + 4 * (lane >> 4));
  __syncthreads();  // the output image below overwrites the bias slot
  // pass 1: registers -> LDS image [token][feature] (bias + activation + one
  // v_cvt_pk_bf16_f32 per pair; 520-B rows keep the 8-B writes conflict-free)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int nl = wr * 128 + i * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tl = wc * 64 + j * 16 + (lane & 15);
      u16x4 o;
      f32x2 v0 = {acc[i][j][0] + bv[i][0], acc[i][j][1] + bv[i][1]};
      f32x2 v1 = {acc[i][j][2] + bv[i][2], acc[i][j][3] + bv[i][3]};
      if (ACT == 1) {
        v0 = gelu_erf2(v0);
        v1 = gelu_erf2(v1);
      }
      o[0] = f32_to_bf16(v0.x);
      o[1] = f32_to_bf16(v0.y);
      o[2] = f32_to_bf16(v1.x);
      o[3] = f32_to_bf16(v1.y);
      *reinterpret_cast<u16x4*>(smem + tl * G256_OUT_LD + nl) = o;
    }
  }
  __syncthreads();
  // pass 2: each wave streams 32 token rows, two rows per instruction (lanes
  // 0-31 / 32-63), 8 features = 16 B per lane: whole cache lines out
  const int half = lane >> 5;
  const int nl = (lane & 31) * 8;
  const int n = n0 + nl;
  if (n < N) {
#pragma unroll 4
    for (int rr = 0; rr < g256::BN / 16; ++rr) {
      const int tl = wave * (g256::BN / 8) + 2 * rr + half;
      const int t = t0 + tl;
      if (t >= T) break;
      const u16* src = smem + tl * G256_OUT_LD + nl;
      const u16x4 lo = *reinterpret_cast<const u16x4*>(src);
      const u16x4 hi = *reinterpret_cast<const u16x4*>(src + 4);
      u16x8 o = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (RES && !plain) {
        const u16x8 rv = *reinterpret_cast<const u16x8*>(R + (long)t * ldr + n);
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = f32_to_bf16(bf16_to_f32(o[u]) + bf16_to_f32(rv[u]));
      }
      if (ACT == 10) {  // measurement probe: everything but the global store
        if (o[0] == 0x7fc1 && o[1] == 0x7fc1) Y[t] = 0;
        continue;
      }
      *reinterpret_cast<u16x8*>(Y + (long)t * ldy + n) = o;
    }
  }
}

template <int ACT, bool RES, int BODY = 0>
__global__ __launch_bounds__(g256::NT, 1) void gemm256_bias_act_kernel(
    const u16* __restrict__ X, long ldx, int T, const u16* __restrict__ W, long ldw, int N,
    const float* __restrict__ bias, const u16* __restrict__ R, long ldr, u16* __restrict__ Y,
    long ldy, int K, int n_ft) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  gemm256_tile<ACT, RES, BODY>(smem, X, ldx, T, W, ldw, N, bias, R, ldr, Y, ldy, K, n_ft,
                               xcd_remap(blockIdx.x, gridDim.x), false);
}

// Split-K pair in ONE launch: tiles [0, tiles) form Ya = X[:, :K/2] W[:, :K/2]^T
// + b (+ R), tiles [tiles, 2 tiles) Yb = X[:, K/2:] W[:, K/2:]^T; the consumer
// (LayerNorm with residual) adds Ya + Yb in fp32. For the N = 768 projections
// (O, FFN2 of bge-base) a token batch gives only 3 feature tiles per 256 tokens,
// so e.g. 270 full-K tiles cost 2 rounds on 256 CUs; 540 half-K tiles cost
// 3 half-length rounds (1.5), and FFN2's K = 3072 tiles are the longest of the
// layer.
template <bool RES>
__global__ __launch_bounds__(g256::NT, 1) void gemm256_split2_kernel(
    const u16* __restrict__ X, long ldx, int T, const u16* __restrict__ W, long ldw, int N,
    const float* __restrict__ bias, const u16* __restrict__ R, long ldr, u16* __restrict__ Ya,
    u16* __restrict__ Yb, long ldy, int K, int n_ft) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int half = logical & 1, tile = logical >> 1;
  const int Kh = K / 2;
  gemm256_tile<0, RES, 1>(smem, X + half * Kh, ldx, T, W + half * Kh, ldw, N, bias, R, ldr, half ? Yb : Ya, ldy,
                          Kh, n_ft, tile, half != 0);
}

// Persistent variant: one block per CU walks its XCD's contiguous share of
// the tiles (g256::TileWalk). After a tile's K loop the NEXT tile's prologue
// DMA (first K-tiles + its 256 bias values, parity double-buffered) is issued
// before this tile's epilogue, which then runs from registers -- bias, GELU,
// residual, bf16 -- with 8-B stores straight from the MFMA layout (no LDS
// image, so the staging slots are free for the next tile's DMA). The HBM
// latency of each tile's first K-tiles hides behind the previous epilogue
// instead of every block of a round waiting for it at once, and there is no
// per-tile launch / drain. Residual rows are loaded before the next prologue
// so their wait does not also wait for the DMA.
constexpr int G256P_EPI_OFF = G256_GEMM_LDS;  // bytes; past the output image
constexpr int G256P_LDS = G256P_EPI_OFF + 2 * 256 * 4;

// IMG 1: the one-tile kernel's LDS-image epilogue (coalesced 16-B stores), the
// next tile's prologue issued after it (the image overlays the staging slots).
template <int ACT, bool RES, int IMG>
__global__ __launch_bounds__(g256::NT, 1) void gemm256p_kernel(
    const u16* __restrict__ X, long ldx, int T, const u16* __restrict__ W, long ldw, int N,
    const float* __restrict__ bias, const u16* __restrict__ R, long ldr, u16* __restrict__ Y, long ldy, int K,
    int n_ft, int n_tiles) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  float* epi = reinterpret_cast<float*>(smem + G256P_EPI_OFF / 2);  // [parity][256] bias
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int KS = K / g256::BK;
  g256::TileWalk walk;
  walk.init(n_tiles);
  int tile = walk.next;
  if (!walk.valid(tile)) return;
  auto stage_bias = [&](int tl, int par) {
    const int n0 = (tl % n_ft) * g256::BM;
    if (wave < 4)
      __builtin_amdgcn_global_load_lds((g256::gbl_void_t*)(bias + min(n0 + wave * 64 + lane, N - 1)),
                                       (g256::lds_void_t*)(epi + par * 256 + wave * 64), 4, 0, 0);
  };
  g256::Stager st;
  st.setup(W, ldw, (tile % n_ft) * g256::BM, N, X, ldx, (tile / n_ft) * g256::BN, T);
  auto ex0 = [&]() { stage_bias(tile, 0); };
  g256::prologue<decltype(ex0), 8>(smem, st, KS, ex0);
  int par = 0;
  f32x4 acc[8][4];
  while (true) {
    const int cur = tile, cpar = par;
    tile += walk.step;
    const bool more = walk.valid(tile);
    g256::body2<g256::MmaBf16>(smem, st, KS, acc, true);
    if constexpr (IMG == 1) {
      const int n0 = (cur % n_ft) * g256::BM, t0 = (cur / n_ft) * g256::BN;
      const float* eb = epi + cpar * 256;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int nl = wr * 128 + i * 16 + 4 * (lane >> 4);
        const f32x4 bv = *reinterpret_cast<const f32x4*>(eb + nl);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int tl = wc * 64 + j * 16 + (lane & 15);
          f32x2 v0 = {acc[i][j][0] + bv[0], acc[i][j][1] + bv[1]};
          f32x2 v1 = {acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]};
          if (ACT == 1) {
            v0 = gelu_erf2(v0);
            v1 = gelu_erf2(v1);
          }
          u16x4 o;
          o[0] = f32_to_bf16(v0.x);
          o[1] = f32_to_bf16(v0.y);
          o[2] = f32_to_bf16(v1.x);
          o[3] = f32_to_bf16(v1.y);
          *reinterpret_cast<u16x4*>(smem + tl * G256_OUT_LD + nl) = o;
        }
      }
      __syncthreads();
      const int half = lane >> 5;
      const int nl = (lane & 31) * 8;
      const int n = n0 + nl;
      if (n < N) {
#pragma unroll 4
        for (int rr = 0; rr < g256::BN / 16; ++rr) {
          const int tl = wave * (g256::BN / 8) + 2 * rr + half;
          const int t = t0 + tl;
          if (t >= T) break;
          const u16* src = smem + tl * G256_OUT_LD + nl;
          const u16x4 lo = *reinterpret_cast<const u16x4*>(src);
          const u16x4 hi = *reinterpret_cast<const u16x4*>(src + 4);
          u16x8 o = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          if (RES) {
            const u16x8 rv = *reinterpret_cast<const u16x8*>(R + (long)t * ldr + n);
#pragma unroll
            for (int u = 0; u < 8; ++u) o[u] = f32_to_bf16(bf16_to_f32(o[u]) + bf16_to_f32(rv[u]));
          }
          *reinterpret_cast<u16x8*>(Y + (long)t * ldy + n) = o;
        }
      }
      __syncthreads();  // image reads done before the next prologue's DMA overwrites the slots
      if (!more) break;
      st.setup(W, ldw, (tile % n_ft) * g256::BM, N, X, ldx, (tile / n_ft) * g256::BN, T);
      auto exn = [&]() { stage_bias(tile, cpar ^ 1); };
      g256::prologue<decltype(exn), 8>(smem, st, KS, exn);
      par = cpar ^ 1;
      continue;
    }
    const int n0 = (cur % n_ft) * g256::BM, t0 = (cur / n_ft) * g256::BN;
    const int tb = t0 + wc * 64 + (lane & 15);
    u16x4 rv[8][4];
    if constexpr (RES) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int n = min(n0 + wr * 128 + i * 16 + 4 * (lane >> 4), N - 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int t = min(tb + j * 16, T - 1);
          rv[i][j] = *reinterpret_cast<const u16x4*>(R + (long)t * ldr + n);
        }
      }
    }
    if (more) {
      st.setup(W, ldw, (tile % n_ft) * g256::BM, N, X, ldx, (tile / n_ft) * g256::BN, T);
      auto exn = [&]() { stage_bias(tile, cpar ^ 1); };
      g256::prologue<decltype(exn), 8>(smem, st, KS, exn);
    }
    const float* eb = epi + cpar * 256;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int nl = wr * 128 + i * 16 + 4 * (lane >> 4);
      const int n = n0 + nl;
      const f32x4 bv = *reinterpret_cast<const f32x4*>(eb + nl);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int t = tb + j * 16;
        f32x2 v0 = {acc[i][j][0] + bv[0], acc[i][j][1] + bv[1]};
        f32x2 v1 = {acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]};
        if (ACT == 1) {
          v0 = gelu_erf2(v0);
          v1 = gelu_erf2(v1);
        }
        if constexpr (RES) {
          v0 += (f32x2){bf16_to_f32(rv[i][j][0]), bf16_to_f32(rv[i][j][1])};
          v1 += (f32x2){bf16_to_f32(rv[i][j][2]), bf16_to_f32(rv[i][j][3])};
        }
        u16x4 o;
        o[0] = f32_to_bf16(v0.x);
        o[1] = f32_to_bf16(v0.y);
        o[2] = f32_to_bf16(v1.x);
        o[3] = f32_to_bf16(v1.y);
        if (t < T && n < N) *reinterpret_cast<u16x4*>(Y + (long)t * ldy + n) = o;
      }
    }
    if (!more) break;
    par = cpar ^ 1;
  }
}

// ---------------------------------------------------------------- skinny GEMM
// T <= 64 tokens (the per-turn query embed of chat/search_memories): the
// projection is a weight-streaming GEMV, not an MFMA-bound GEMM. One block per
// 16 output features; its 4 waves split K in quarters, each wave keeps the
// 16 x T tile in registers (v_mfma_f32_16x16x32_bf16, A = W rows and B = token
// rows straight from global memory -- weights are read exactly once, tokens
// are L2-resident), partial sums are reduced through LDS and wave 0 applies
// bias / GELU / residual. Grid = N/16 blocks instead of the 256-wide tiles'
// handful, so a 12-layer forward at batch 1 is bounded by weight bytes.
template <int ACT, bool RES, int NT16>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(const u16* __restrict__ X, long ldx, int T,
                                                          const u16* __restrict__ W, long ldw, int N,
                                                          const float* __restrict__ bias, const u16* __restrict__ R,
                                                          long ldr, u16* __restrict__ Y, long ldy, int K) {
  __shared__ f32x4 part[3][NT16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f0 = blockIdx.x * 16;
  const int kq = K / 4, kb = wave * kq;
  const int fr = min(f0 + (lane & 15), N - 1);
  const u16* wrow = W + (long)fr * ldw + kb + 8 * (lane >> 4);
  const u16* xrow[NT16];
#pragma unroll
  for (int j = 0; j < NT16; ++j) xrow[j] = X + (long)min(16 * j + (lane & 15), T - 1) * ldx + kb + 8 * (lane >> 4);
  f32x4 acc[NT16];
#pragma unroll
  for (int j = 0; j < NT16; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k = 0; k < kq; k += 32) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(wrow + k);
#pragma unroll
    for (int j = 0; j < NT16; ++j) {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(xrow[j] + k);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
    }
  }
  if (wave > 0) {
#pragma unroll
    for (int j = 0; j < NT16; ++j) part[wave - 1][j][lane] = acc[j];
  }
  __syncthreads();
  if (wave != 0) return;
  const int n = f0 + 4 * (lane >> 4);
  if (n >= N) return;
  const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + n);
#pragma unroll
  for (int j = 0; j < NT16; ++j) {
    const int t = 16 * j + (lane & 15);
    f32x4 v = acc[j] + part[0][j][lane] + part[1][j][lane] + part[2][j][lane];
    if (t >= T) continue;
    u16x4 o;
    float r[4] = {0.f, 0.f, 0.f, 0.f};
    if (RES) {
      const u16x4 rv = *reinterpret_cast<const u16x4*>(R + (long)t * ldr + n);
#pragma unroll
      for (int u = 0; u < 4; ++u) r[u] = bf16_to_f32(rv[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float y = v[u] + bv[u];
      if (ACT == 1) y = gelu_erf(y);
      o[u] = f32_to_bf16(y + r[u]);
    }
    *reinterpret_cast<u16x4*>(Y + (long)t * ldy + n) = o;
  }
}

// ---------------------------------------------------------------- fp8 path
// SURVEY.md §2.4 K15 / BASELINE config 5: OCP e4m3 weights (per output
// channel scale) x e4m3 activations (per token scale) on the block-scaled
// 16x16x128 MFMA with unit block scales -- the same 256x256 pipeline and LDS
// image as bf16 (a 128-B K-row holds 128 fp8 instead of 64 bf16), twice the
// MFMA rate; dequantisation, bias, GELU and residual fused in the epilogue.
template <int ACT, bool RES>
__global__ __launch_bounds__(g256::NT, 1) void gemm256_f8_kernel(
    const unsigned char* __restrict__ Xq, long ldx, int T, const float* __restrict__ sx,
    const unsigned char* __restrict__ Wq, long ldw, int N, const float* __restrict__ sw,
    const float* __restrict__ bias, const u16* __restrict__ R, long ldr, u16* __restrict__ Y, long ldy, int K,
    int n_ft) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tt = logical / n_ft, ft = logical % n_ft;
  const int n0 = ft * g256::BM, t0 = tt * g256::BN;
  g256::Stager st;
  st.setup(reinterpret_cast<const u16*>(Wq), ldw / 2, n0, N, reinterpret_cast<const u16*>(Xq), ldx / 2, t0, T);
  f32x4 acc[8][4];
  g256::mainloop<g256::MmaFp8>(smem, st, K / g256::MmaFp8::KPER, acc);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  float tsc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) tsc[j] = sx[min(t0 + wc * 64 + j * 16 + (lane & 15), T - 1)];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int nl = wr * 128 + i * 16 + 4 * (lane >> 4);
    const int n = min(n0 + nl, N - 4);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + n);
    const f32x4 wv = *reinterpret_cast<const f32x4*>(sw + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tl = wc * 64 + j * 16 + (lane & 15);
      u16x4 o;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float v = acc[i][j][u] * wv[u] * tsc[j] + bv[u];
        if (ACT == 1) v = gelu_erf(v);
        o[u] = f32_to_bf16(v);
      }
      *reinterpret_cast<u16x4*>(smem + tl * G256_OUT_LD + nl) = o;
    }
  }
  __syncthreads();
  const int nl = lane * 4;
  const int n = n0 + nl;
  if (n < N) {
#pragma unroll 8
    for (int rr = 0; rr < g256::BN / 8; ++rr) {
      const int tl = wave * (g256::BN / 8) + rr;
      const int t = t0 + tl;
      if (t >= T) break;
      u16x4 o = *reinterpret_cast<const u16x4*>(smem + tl * G256_OUT_LD + nl);
      if (RES) {
        const u16x4 rv = *reinterpret_cast<const u16x4*>(R + (long)t * ldr + n);
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = f32_to_bf16(bf16_to_f32(o[u]) + bf16_to_f32(rv[u]));
      }
      *reinterpret_cast<u16x4*>(Y + (long)t * ldy + n) = o;
    }
  }
}

// bf16 rows -> e4m3 rows + per-row scale (amax / 448), one wave per row.
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const u16* __restrict__ X, long ldx, int rows, int D,
                                                             unsigned char* __restrict__ Q, long ldq,
                                                             float* __restrict__ scale) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const u16* x = X + (long)row * ldx;
  float amax = 0.f;
  for (int c = lane * 8; c < D; c += 512) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(x + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(bf16_to_f32(v[e])));
  }
  amax = wave_max(amax);
  const float sc = amax > 0.f ? amax * (1.f / 448.f) : 1.f;
  const float inv = 1.f / sc;
  unsigned char* q = Q + (long)row * ldq;
  for (int c = lane * 8; c < D; c += 512) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(x + c);
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(v[0]) * inv, bf16_to_f32(v[1]) * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(v[2]) * inv, bf16_to_f32(v[3]) * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(v[4]) * inv, bf16_to_f32(v[5]) * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(v[6]) * inv, bf16_to_f32(v[7]) * inv, hi, true);
    *reinterpret_cast<uint2*>(q + c) = make_uint2((unsigned)lo, (unsigned)hi);
  }
  if (lane == 0) scale[row] = sc;
}

// ---------------------------------------------------------------- attention
// qkv: [B*S, 3*H] rows (q | k | v), head dim HD in {32, 64}. One wave per (b, head, qblock).
template <int HD>
__global__ __launch_bounds__(64) void attention_kernel(
    const u16* __restrict__ qkv, long ldq, const int* __restrict__ lens, int S, int H, int nheads,
    float scale_log2, u16* __restrict__ out, long ldo, const int* __restrict__ cu) {
  constexpr int KSQ = HD / 16;   // k-steps of the S = K Q^T product
  constexpr int NDB = HD / 32;   // 32-row blocks of the output O^T
  __shared__ __attribute__((aligned(16))) u16 vt[HD * 40];  // V^T block: [dim][key], padded rows
  const int lane = threadIdx.x, h = lane >> 5, l32 = lane & 31;
  const int nqb = (S + 31) / 32;
  const int qb = blockIdx.x % nqb;
  const int hd = (blockIdx.x / nqb) % nheads;
  const int b = blockIdx.x / (nqb * nheads);
  const int len = lens[b];
  // padded layout: sequence b owns rows [b*S, b*S + S); packed ("varlen")
  // layout: rows [cu[b], cu[b] + len) only -- padding tokens are never stored
  const long tok0 = cu ? (long)cu[b] : (long)b * S;
  const int Sb = cu ? len : S;
  if (qb * 32 >= Sb) return;  // whole (single-wave) block past the sequence
  const int q = qb * 32 + l32;
  const int qc = min(q, Sb - 1);
  const u16* qrow = qkv + (tok0 + qc) * ldq + hd * HD;
  bf16x8 qf[KSQ];
#pragma unroll
  for (int s = 0; s < KSQ; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qrow + 16 * s + 8 * h);

  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[i][e] = 0.f;
  float m = -1e30f, l = 0.f;
  const int nkb = (len + 31) / 32;
  for (int kb = 0; kb < nkb; ++kb) {
    // S^T block [32 keys x 32 queries]: A = K rows, B = Q rows
    const int key = kb * 32 + l32;
    const u16* krow = qkv + (tok0 + min(key, Sb - 1)) * ldq + H + hd * HD;
    f32x16 st;
#pragma unroll
    for (int e = 0; e < 16; ++e) st[e] = 0.f;
#pragma unroll
    for (int s = 0; s < KSQ; ++s) {
      bf16x8 kf = *reinterpret_cast<const bf16x8*>(krow + 16 * s + 8 * h);
      st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], st, 0, 0, 0);
    }
    // stage V^T for this key block (each lane: one key, HD/2 dims)
    {
      const int vk = lane >> 1, vd0 = (lane & 1) * (HD / 2);
      const u16* vrow = qkv + (tok0 + min(kb * 32 + vk, Sb - 1)) * ldq + 2 * H + hd * HD + vd0;
#pragma unroll
      for (int c = 0; c < HD / 16; ++c) {
        u16x8 v8 = *reinterpret_cast<const u16x8*>(vrow + 8 * c);
#pragma unroll
        for (int j = 0; j < 8; ++j) vt[(vd0 + 8 * c + j) * 40 + vk] = v8[j];
      }
    }
    // masked online softmax over keys (registers + one cross-half shuffle)
    float mx = -1e30f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      int kk = kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      float v = (kk < len) ? st[e] * scale_log2 : -1e30f;
      st[e] = v;
      mx = fmaxf(mx, v);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float corr = exp2f(m - mn);
    float ps = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      float p = exp2f(st[e] - mn);
      st[e] = p;
      ps += p;
    }
    ps += __shfl_xor(ps, 32, 64);
    l = l * corr + ps;
    m = mn;
#pragma unroll
    for (int i = 0; i < NDB; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) o[i][e] *= corr;
    __syncthreads();  // V^T staged (single-wave block: orders the LDS writes)
    // O^T[dim][q] += V^T[dim][key] . P^T[key][q]; P^T is the accumulator `st`
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[j] = (__bf16)st[8 * s + j];
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        const int d = db * 32 + l32;
        const u16* base = vt + d * 40 + 16 * s + 4 * h;
        u16x4 lo = *reinterpret_cast<const u16x4*>(base);
        u16x4 hi = *reinterpret_cast<const u16x4*>(base + 8);
        u16x8 a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bf16x8 af = __builtin_bit_cast(bf16x8, a8);
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, pf, o[db], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (q >= Sb) return;
  const float inv = 1.f / l;
  u16* orow = out + (tok0 + q) * ldo + hd * HD;
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u16x4 w;
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = f32_to_bf16(o[db][4 * g + u] * inv);
      *reinterpret_cast<u16x4*>(orow + db * 32 + 8 * g + 4 * h) = w;
    }
}

// ---------------------------------------------------------------- LayerNorm
// y = LN(x (+ r)) * g + b. One wave per RPW rows, NC chunks of 4 features per
// lane (H <= 256 * NC): gamma/beta are loaded once per wave and reused for its
// RPW rows, and every row's loads are issued before the first reduction so a
// wave has RPW * NC (x2 with the residual) 8-B loads in flight instead of NC.
template <int NC, bool RES, int RPW>
__global__ __launch_bounds__(256) void layernorm_kernel(const u16* __restrict__ X, long ldx,
                                                        const u16* __restrict__ R, long ldr,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ bta, int rows,
                                                        int H, float eps, u16* __restrict__ Y, long ldy) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= rows) return;
  f32x4 gg[NC], bb[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = (lane + 64 * c) * 4;
    if (col < H) {
      gg[c] = *reinterpret_cast<const f32x4*>(g + col);
      bb[c] = *reinterpret_cast<const f32x4*>(bta + col);
    }
  }
  float v[RPW][NC][4];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = min(row0 + rr, rows - 1);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col < H) {
        const u16x4 x = *reinterpret_cast<const u16x4*>(X + (long)row * ldx + col);
        u16x4 r = {0, 0, 0, 0};
        if (RES) r = *reinterpret_cast<const u16x4*>(R + (long)row * ldr + col);
#pragma unroll
        for (int u = 0; u < 4; ++u) v[rr][c][u] = bf16_to_f32(x[u]) + (RES ? bf16_to_f32(r[u]) : 0.f);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) v[rr][c][u] = 0.f;
      }
    }
  }
  const float invH = 1.f / H;
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = row0 + rr;
    if (row >= rows) break;  // wave-uniform
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int u = 0; u < 4; ++u) sum += v[rr][c][u];
    const float mean = wave_sum(sum) * invH;
    float var = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if ((lane + 64 * c) * 4 < H)
#pragma unroll
        for (int u = 0; u < 4; ++u) { const float d = v[rr][c][u] - mean; var += d * d; }
    }
    const float rstd = rsqrtf(wave_sum(var) * invH + eps);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = (lane + 64 * c) * 4;
      if (col < H) {
        u16x4 o;
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = f32_to_bf16((v[rr][c][u] - mean) * rstd * gg[c][u] + bb[c][u]);
        *reinterpret_cast<u16x4*>(Y + (long)row * ldy + col) = o;
      }
    }
  }
}

// Same op for H % 256 == 0 (bge-base 768, e5-large 1024): half a wave per
// row, each lane moving C chunks of 8 features as 16-B loads and stores (H =
// 32 lanes * 8 * C), two rows per wave-instruction, RPW row pairs per wave.
// Q8 (the fp8 encoder): the row is also written as OCP e4m3 with its
// scale, exactly what quant_fp8_rows_kernel makes of the bf16 output (amax of
// the bf16-rounded values / 448) -- the next projection's input without the
// separate quantise pass (one read + one write of the activations per GEMM).
template <int C, bool RES, int RPW, bool Q8 = false>
__global__ __launch_bounds__(256) void layernorm16_kernel(const u16* __restrict__ X, long ldx,
                                                          const u16* __restrict__ R, long ldr,
                                                          const float* __restrict__ g,
                                                          const float* __restrict__ bta, int rows, float eps,
                                                          u16* __restrict__ Y, long ldy,
                                                          unsigned char* __restrict__ Q = nullptr, long ldq = 0,
                                                          float* __restrict__ qscale = nullptr) {
  constexpr int H = C * 256;
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 * RPW;
  if (row0 >= rows) return;
  float v[RPW][C][8];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = min(row0 + 2 * rr + half, rows - 1);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int col = c * 256 + l32 * 8;
      const u16x8 x = *reinterpret_cast<const u16x8*>(X + (long)row * ldx + col);
      u16x8 r = {0, 0, 0, 0, 0, 0, 0, 0};
      if (RES) r = *reinterpret_cast<const u16x8*>(R + (long)row * ldr + col);
#pragma unroll
      for (int u = 0; u < 8; ++u) v[rr][c][u] = bf16_to_f32(x[u]) + (RES ? bf16_to_f32(r[u]) : 0.f);
    }
  }
  constexpr float invH = 1.f / H;
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int u = 0; u < 8; ++u) sum += v[rr][c][u];
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);  // within the half wave
    const float mean = sum * invH;
    float var = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int u = 0; u < 8; ++u) { const float d = v[rr][c][u] - mean; var += d * d; }
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) var += __shfl_xor(var, o, 64);
    const float rstd = rsqrtf(var * invH + eps);
    const int row = row0 + 2 * rr + half;
    u16x8 ov[C];
    float amax = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int col = c * 256 + l32 * 8;
      const f32x4 g0 = *reinterpret_cast<const f32x4*>(g + col), g1 = *reinterpret_cast<const f32x4*>(g + col + 4);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(bta + col), b1 = *reinterpret_cast<const f32x4*>(bta + col + 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ov[c][u] = f32_to_bf16((v[rr][c][u] - mean) * rstd * g0[u] + b0[u]);
        ov[c][u + 4] = f32_to_bf16((v[rr][c][u + 4] - mean) * rstd * g1[u] + b1[u]);
      }
      if (Q8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) amax = fmaxf(amax, fabsf(bf16_to_f32(ov[c][u])));
      }
      if (row < rows) *reinterpret_cast<u16x8*>(Y + (long)row * ldy + col) = ov[c];
    }
    if (Q8) {
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));  // within the half wave
      const float sc = amax > 0.f ? amax * (1.f / 448.f) : 1.f;
      const float inv = 1.f / sc;
      if (row < rows) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const int col = c * 256 + l32 * 8;
          int lo = 0, hi = 0;
          lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(ov[c][0]) * inv, bf16_to_f32(ov[c][1]) * inv, lo, false);
          lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(ov[c][2]) * inv, bf16_to_f32(ov[c][3]) * inv, lo, true);
          hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(ov[c][4]) * inv, bf16_to_f32(ov[c][5]) * inv, hi, false);
          hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(ov[c][6]) * inv, bf16_to_f32(ov[c][7]) * inv, hi, true);
          *reinterpret_cast<uint2*>(Q + (long)row * ldq + col) = make_uint2((unsigned)lo, (unsigned)hi);
        }
        if (l32 == 0) qscale[row] = sc;
      }
    }
  }
}

// embeddings (bf16 tables) + LayerNorm, one wave per token
template <int NC>
__global__ __launch_bounds__(256) void embed_ln_kernel(const int* __restrict__ ids, int T, int S,
                                                       const u16* __restrict__ wemb,
                                                       const u16* __restrict__ pemb,
                                                       const u16* __restrict__ temb,
                                                       const float* __restrict__ g,
                                                       const float* __restrict__ bta, int H, float eps,
                                                       u16* __restrict__ Y, const int* __restrict__ posv) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int id = ids[t];
  const int pos = posv ? posv[t] : t % S;
  float v[NC][4];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    int col = (lane + 64 * c) * 4;
    if (col < H) {
      u16x4 a = *reinterpret_cast<const u16x4*>(wemb + (long)id * H + col);
      u16x4 p = *reinterpret_cast<const u16x4*>(pemb + (long)pos * H + col);
      u16x4 ty = *reinterpret_cast<const u16x4*>(temb + col);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[c][u] = bf16_to_f32(a[u]) + bf16_to_f32(p[u]) + bf16_to_f32(ty[u]);
        sum += v[c][u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[c][u] = 0.f;
    }
  }
  const float mean = wave_sum(sum) / H;
  float var = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    int col = (lane + 64 * c) * 4;
    if (col < H)
#pragma unroll
      for (int u = 0; u < 4; ++u) { float d = v[c][u] - mean; var += d * d; }
  }
  const float rstd = rsqrtf(wave_sum(var) / H + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    int col = (lane + 64 * c) * 4;
    if (col < H) {
      f32x4 gg = *reinterpret_cast<const f32x4*>(g + col);
      f32x4 bb = *reinterpret_cast<const f32x4*>(bta + col);
      u16x4 o;
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = f32_to_bf16((v[c][u] - mean) * rstd * gg[u] + bb[u]);
      *reinterpret_cast<u16x4*>(Y + (long)t * H + col) = o;
    }
  }
}

// pooling (mode 0 = masked mean, 1 = CLS) + L2 normalise; one workgroup per sequence
__global__ __launch_bounds__(256) void pool_norm_kernel(const u16* __restrict__ X, const int* __restrict__ lens,
                                                        int S, int H, int mode, float* __restrict__ out32,
                                                        u16* __restrict__ out16, int ld16,
                                                        const int* __restrict__ cu) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  const int len = max(1, lens[b]);
  const long base = (cu ? (long)cu[b] : (long)b * S) * H;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};  // up to H = 1024 with 256 threads
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    int col = threadIdx.x + 256 * c;
    if (col >= H) continue;
    float s = 0.f;
    if (mode == 1) {
      s = bf16_to_f32(X[base + col]);
    } else {
      for (int t = 0; t < len; ++t) s += bf16_to_f32(X[base + (long)t * H + col]);
      s /= len;
    }
    acc[c] = s;
    ss += s * s;
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.f / fmaxf(sqrtf(tot), 1e-12f);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    int col = threadIdx.x + 256 * c;
    if (col >= H) continue;
    float v = acc[c] * inv;
    if (out32) out32[(long)b * H + col] = v;
    if (out16) out16[(long)b * ld16 + col] = f32_to_bf16(v);
  }
  if (out16)
    for (int col = H + threadIdx.x; col < ld16; col += 256) out16[(long)b * ld16 + col] = 0;
}

}  // namespace

static int g_gemm_staging = -1;  // 1 = LDS-DMA (default), 0 = register staging (lzk_set_staging)
static int g_gemm_tile = -1;     // 256 = 8-wave 256x256 pipeline when the grid fills the chip, 128 = always 128x128
static int g_g256_body = -1;     // 256x256 main loop: 0 = four-phase body, 1 = two-phase body2 (default)

LZK_EXPORT void lzk_set_staging(int glds) { g_gemm_staging = glds; }
LZK_EXPORT void lzk_set_gemm_tile(int t) { g_gemm_tile = t; }
LZK_EXPORT void lzk_set_g256_body(int b) { g_g256_body = b; }
static int g_g256_min_n = -1;  // smallest N routed to the 256x256 pipeline
LZK_EXPORT void lzk_set_g256_min_n(int n) { g_g256_min_n = n; }
static int g_g256_min_tiles = -1;  // smallest grid routed to the 256x256 pipeline
LZK_EXPORT void lzk_set_g256_min_tiles(int n) { g_g256_min_tiles = n; }
static int g_g256_tail = -1;  // largest last-round fill (% of the CUs) split off to the 128x128 kernel (A/B setter)
LZK_EXPORT void lzk_set_g256_tail(int pct) { g_g256_tail = pct; }
static int g_n_cu_enc = 0;
static int g_g256_persist = -1;  // persistent 256x256 GEMM: 1 = register epilogue, 2 = LDS image (A/B setter)
LZK_EXPORT void lzk_set_g256_persist(int p) { g_g256_persist = p; }

LZK_EXPORT int lzk_gemm_bias_act(const void* X, long ldx, int T, const void* W, long ldw, int N,
                                 const float* bias, const void* R, long ldr, void* Y, long ldy, int K,
                                 int act, void* stream) {
  if (g_gemm_staging < 0) g_gemm_staging = 1;
  if (K % TK != 0 || N % 4 != 0 || T <= 0 || N <= 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (T <= 64 && K % 128 == 0 && g_gemm_tile != 128) {
    const u16* x = (const u16*)X;
    const u16* w = (const u16*)W;
    const u16* r = (const u16*)R;
    u16* y = (u16*)Y;
    dim3 grid((N + 15) / 16), block(256);
#define SK(A, RS, NT) hipLaunchKernelGGL((gemm_skinny_kernel<A, RS, NT>), grid, block, 0, st, x, ldx, T, w, ldw, N, bias, r, ldr, y, ldy, K)
#define SKT(NT) do { if (act == 1) { if (r) SK(1, true, NT); else SK(1, false, NT); } \
                     else { if (r) SK(0, true, NT); else SK(0, false, NT); } } while (0)
    if (T <= 16) SKT(1);
    else if (T <= 32) SKT(2);
    else SKT(4);
#undef SKT
#undef SK
    return (int)hipGetLastError();
  }
  // 128x128 launch over token rows [0, Tn) of x / r / y
  auto launch128 = [&](const u16* x, int Tn, const u16* r, u16* y, int tiles, int nft) {
    dim3 grid(tiles), block(TNT);
    const size_t lds = 2 * 2 * TELEMS * sizeof(u16);
    const u16* w = (const u16*)W;
#define GO(A, RS, G) hipLaunchKernelGGL((gemm_bias_act_kernel<A, RS, G>), grid, block, lds, st, x, ldx, Tn, w, ldw, N, bias, r, ldr, y, ldy, K, nft)
    if (g_gemm_staging) {
      if (act == 1) { if (r) GO(1, true, true); else GO(1, false, true); }
      else { if (r) GO(0, true, true); else GO(0, false, true); }
    } else {
      if (act == 1) { if (r) GO(1, true, false); else GO(1, false, false); }
      else { if (r) GO(0, true, false); else GO(0, false, false); }
    }
#undef GO
  };
  if (g_gemm_tile < 0) g_gemm_tile = 256;
  {
    const int n_ft = (N + g256::BM - 1) / g256::BM, n_tt = (T + g256::BN - 1) / g256::BN;
    // measured (profiles/ab_body_r1.json): with the two-phase main loop the
    // 256x256 pipeline beats the 128x128 kernel even on half the chip -- bge-base O / FFN2
    // (N = 768) at 11k tokens: 132 tiles, 24 / 60 us vs 34 / 90 us -- so every grid of at
    // least 64 tiles takes it (from 128: bench forward 5.72 -> 5.13 ms; from 64: the consolidation
    // bench's 7k-token fact halves 21.8 -> 21.1 ms per step)
    if (g_g256_min_n < 0) g_g256_min_n = 768;
    if (g_g256_min_tiles < 0) g_g256_min_tiles = 64;
    const u16* w = (const u16*)W;
    // 256x256 launch over token rows [0, Tn) of x / r / y
    auto launch256 = [&](const u16* x, int Tn, const u16* r, u16* y) {
      const int ntt = (Tn + g256::BN - 1) / g256::BN;
      dim3 grid(n_ft * ntt), block(g256::NT);
      if (g_g256_persist < 0) {
        // off by default (profiles/ab_persist_r1.json): with the LDS-image
        // epilogue (2) the per-GEMM times equal the one-tile kernel's and the whole forward is
        // slower (2 streams 5.14 -> 5.50 ms); 8-B stores straight from the MFMA layout (1) cost
        // ~3.5 us per 256x256 tile more than the coalesced image stores (QKV 93 -> 107 us)
        g_g256_persist = 0;
      }
      if ((g_g256_persist == 1 || g_g256_persist == 2) && (act == 0 || act == 1)) {
        if (g_n_cu_enc <= 0) {
          int dev = 0;
          (void)hipGetDevice(&dev);
          if (hipDeviceGetAttribute(&g_n_cu_enc, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
              g_n_cu_enc <= 0)
            g_n_cu_enc = 256;
        }
        const int tiles = n_ft * ntt;
        dim3 pgrid(tiles < g_n_cu_enc ? tiles : g_n_cu_enc);
#define GP1(A, RS, IM)                                                                                             \
  do {                                                                                                             \
    (void)hipFuncSetAttribute((const void*)gemm256p_kernel<A, RS, IM>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                              G256P_LDS);                                                                          \
    hipLaunchKernelGGL((gemm256p_kernel<A, RS, IM>), pgrid, block, G256P_LDS, st, x, ldx, Tn, w, ldw, N, bias, r,  \
                       ldr, y, ldy, K, n_ft, tiles);                                                               \
  } while (0)
#define GP(A, RS)                                   \
  do {                                              \
    if (g_g256_persist == 2) GP1(A, RS, 1);         \
    else GP1(A, RS, 0);                             \
  } while (0)
        if (act == 1) { if (r) GP(1, true); else GP(1, false); }
        else { if (r) GP(0, true); else GP(0, false); }
#undef GP
#undef GP1
        return;
      }
      if (g_g256_body < 0) {
        g_g256_body = 1;  // body2: 2-4 % faster on the bge-base projections (profiles/ab_body_r1.json)
      }
#define GO1(A, RS, BD)                                                                                        \
  do {                                                                                                        \
    (void)hipFuncSetAttribute((const void*)gemm256_bias_act_kernel<A, RS, BD>,                                \
                              hipFuncAttributeMaxDynamicSharedMemorySize, G256_GEMM_LDS);                     \
    hipLaunchKernelGGL((gemm256_bias_act_kernel<A, RS, BD>), grid, block, G256_GEMM_LDS, st, x, ldx, Tn, w,   \
                       ldw, N, bias, r, ldr, y, ldy, K, n_ft);                                                \
  } while (0)
#define GO(A, RS)                        \
  do {                                   \
    if (g_g256_body == 1) GO1(A, RS, 1); \
    else GO1(A, RS, 0);                  \
  } while (0)
      if (act == 9) GO(9, false);
      else if (act == 10) GO(10, false);
      else if (act == 1) { if (r) GO(1, true); else GO(1, false); }
      else { if (r) GO(0, true); else GO(0, false); }
#undef GO
#undef GO1
    };
    if (g_gemm_tile == 256 && n_ft * n_tt >= g_g256_min_tiles && N >= g_g256_min_n && N % 8 == 0 && ldy % 8 == 0 &&
        (!R || ldr % 8 == 0)) {
      const u16* x = (const u16*)X;
      const u16* r = (const u16*)R;
      u16* y = (u16*)Y;
      // Tile-quantisation tail: a grid of n_cu * q + f tiles costs q + 1 full
      // rounds of 256x256 tiles. When the last round would be at most
      // g_g256_tail % full, the 256x256 kernel takes only the token rows that
      // fill whole rounds and the leftover rows (< 1 round of tiles, usually a
      // few hundred tokens) go to the 128x128 kernel, whose 4x smaller tiles
      // spread them over 4x more CUs (bge-base FFN2 at 22.6k tokens: 267 tiles
      // = 255 + 825 tokens).
      if (g_n_cu_enc <= 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&g_n_cu_enc, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            g_n_cu_enc <= 0)
          g_n_cu_enc = 256;
      }
      if (g_g256_tail < 0) {
        // off by default: in isolation FFN2 at 22.6k tokens gains 132 -> 119 us, but the
        // 128x128 tail kernels run at ~1/4 of the per-CU rate (one small tile per CU) and the
        // whole forward loses (profiles/ab_tail_r1.json: 1 stream 5.54 ->
        // 5.76 ms, 2 streams 4.97 -> 5.11 ms)
        g_g256_tail = 0;
      }
      const int tiles = n_ft * n_tt, P = g_n_cu_enc;
      const int q = tiles / P, f = tiles - q * P;
      const int tt0 = (q * P) / n_ft;  // whole token tiles inside q full rounds
      if (q >= 1 && f > 0 && f * 100 <= g_g256_tail * P && tt0 > 0 && act != 9 && act != 10) {
        const int T0 = tt0 * g256::BN;
        launch256(x, T0, r, y);
        const int T1 = T - T0;
        const int n128 = (N + TB - 1) / TB, t128 = (T1 + TB - 1) / TB;
        launch128(x + (long)T0 * ldx, T1, r ? r + (long)T0 * ldr : nullptr, y + (long)T0 * ldy, n128 * t128, n128);
        return (int)hipGetLastError();
      }
      launch256(x, T, r, y);
      return (int)hipGetLastError();
    }
  }
  const int n_ft = (N + TB - 1) / TB, n_tt = (T + TB - 1) / TB;
  launch128((const u16*)X, T, (const u16*)R, (u16*)Y, n_ft * n_tt, n_ft);
  return (int)hipGetLastError();
}

// Split-K pair (gemm256_split2_kernel): Ya = X[:, :K/2] W[:, :K/2]^T + b (+ R),
// Yb = X[:, K/2:] W[:, K/2:]^T, one launch. K % 128 == 0, N % 8 == 0.
LZK_EXPORT int lzk_gemm_split2(const void* X, long ldx, int T, const void* W, long ldw, int N, const float* bias,
                               const void* R, long ldr, void* Ya, void* Yb, long ldy, int K, void* stream) {
  if (K % (2 * g256::BK) != 0 || N % 8 != 0 || ldy % 8 != 0 || (R && ldr % 8 != 0) || T <= 0 || N <= 0)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int n_ft = (N + g256::BM - 1) / g256::BM, n_tt = (T + g256::BN - 1) / g256::BN;
  dim3 grid(2 * n_ft * n_tt), block(g256::NT);
#define GO(RS)                                                                                                     \
  do {                                                                                                             \
    (void)hipFuncSetAttribute((const void*)gemm256_split2_kernel<RS>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                              G256_GEMM_LDS);                                                                      \
    hipLaunchKernelGGL((gemm256_split2_kernel<RS>), grid, block, G256_GEMM_LDS, st, (const u16*)X, ldx, T,         \
                       (const u16*)W, ldw, N, bias, (const u16*)R, ldr, (u16*)Ya, (u16*)Yb, ldy, K, n_ft);         \
  } while (0)
  if (R) GO(true);
  else GO(false);
#undef GO
  return (int)hipGetLastError();
}

// Y[T, N] = act((Xq * sx) (Wq * sw)^T + b) (+ R); Xq/Wq OCP e4m3 rows
// (ldx/ldw in bytes, even), K % 128 == 0, N % 4 == 0.
LZK_EXPORT int lzk_gemm_f8(const void* Xq, long ldx, int T, const float* sx, const void* Wq, long ldw, int N,
                           const float* sw, const float* bias, const void* R, long ldr, void* Y, long ldy, int K,
                           int act, void* stream) {
  if (K % 128 != 0 || N % 4 != 0 || T <= 0 || N <= 0 || (ldx & 1) || (ldw & 1)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int n_ft = (N + g256::BM - 1) / g256::BM, n_tt = (T + g256::BN - 1) / g256::BN;
  dim3 grid(n_ft * n_tt), block(g256::NT);
  const unsigned char* x = (const unsigned char*)Xq;
  const unsigned char* w = (const unsigned char*)Wq;
  const u16* r = (const u16*)R;
  u16* y = (u16*)Y;
#define GO(A, RS)                                                                                                  \
  do {                                                                                                             \
    (void)hipFuncSetAttribute((const void*)gemm256_f8_kernel<A, RS>, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                              G256_GEMM_LDS);                                                                      \
    hipLaunchKernelGGL((gemm256_f8_kernel<A, RS>), grid, block, G256_GEMM_LDS, st, x, ldx, T, sx, w, ldw, N, sw,   \
                       bias, r, ldr, y, ldy, K, n_ft);                                                             \
  } while (0)
  if (act == 1) { if (r) GO(1, true); else GO(1, false); }
  else { if (r) GO(0, true); else GO(0, false); }
#undef GO
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_quant_fp8_rows(const void* X, long ldx, int rows, int D, void* Q, long ldq, float* scale,
                                  void* stream) {
  if (D % 8 != 0 || rows <= 0) return rows == 0 ? 0 : (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(quant_fp8_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, (const u16*)X,
                     ldx, rows, D, (unsigned char*)Q, ldq, scale);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_attention(const void* qkv, long ldq, const int* lens, int B, int S, int H, int nheads,
                             float scale, void* out, long ldo, const int* cu, void* stream) {
  const int hdim = H / nheads;
  if (H != nheads * hdim || (hdim != 32 && hdim != 64)) return (int)hipErrorInvalidValue;
  const int nqb = (S + 31) / 32;
  dim3 grid(B * nheads * nqb), block(64);
  if (hdim == 64)
    hipLaunchKernelGGL(attention_kernel<64>, grid, block, 0, (hipStream_t)stream, (const u16*)qkv, ldq, lens, S, H,
                       nheads, scale * 1.4426950408889634f, (u16*)out, ldo, cu);
  else
    hipLaunchKernelGGL(attention_kernel<32>, grid, block, 0, (hipStream_t)stream, (const u16*)qkv, ldq, lens, S, H,
                       nheads, scale * 1.4426950408889634f, (u16*)out, ldo, cu);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_layernorm(const void* X, long ldx, const void* R, long ldr, const float* g, const float* b,
                             int rows, int H, float eps, void* Y, long ldy, void* stream) {
  if (H % 4 != 0 || H > 64 * 4 * 4 || rows <= 0) return (int)hipErrorInvalidValue;
  constexpr int RPW = 4;
  dim3 grid((rows + 4 * RPW - 1) / (4 * RPW)), block(256);
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  const u16* r = (const u16*)R;
  u16* y = (u16*)Y;
  const bool v16 = (H == 768 || H == 1024) && ldx % 8 == 0 && ldy % 8 == 0 && (!r || ldr % 8 == 0) &&
                   ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Y) |
                     reinterpret_cast<uintptr_t>(R)) & 15) == 0;
  if (v16) {
    constexpr int RP = 2;  // row pairs per wave -> 16 rows per 256-thread block
    dim3 grid16((rows + 16 - 1) / 16);
#define LN16(C)                                                                                                 \
  do {                                                                                                          \
    if (r) hipLaunchKernelGGL((layernorm16_kernel<C, true, RP>), grid16, block, 0, st, x, ldx, r, ldr, g, b,    \
                              rows, eps, y, ldy);                                                               \
    else hipLaunchKernelGGL((layernorm16_kernel<C, false, RP>), grid16, block, 0, st, x, ldx, r, ldr, g, b,     \
                            rows, eps, y, ldy);                                                                 \
  } while (0)
    if (H == 768) LN16(3);
    else LN16(4);
#undef LN16
    return (int)hipGetLastError();
  }
#define LN(NC)                                                                                                  \
  do {                                                                                                          \
    if (r) hipLaunchKernelGGL((layernorm_kernel<NC, true, RPW>), grid, block, 0, st, x, ldx, r, ldr, g, b, rows, \
                              H, eps, y, ldy);                                                                  \
    else hipLaunchKernelGGL((layernorm_kernel<NC, false, RPW>), grid, block, 0, st, x, ldx, r, ldr, g, b, rows,  \
                            H, eps, y, ldy);                                                                    \
  } while (0)
  if (H <= 256) LN(1);
  else if (H <= 512) LN(2);
  else if (H <= 768) LN(3);
  else LN(4);
#undef LN
  return (int)hipGetLastError();
}

// lzk_layernorm + the row's e4m3 copy and scale (layernorm16_kernel Q8):
// H 768 / 1024, 16-B aligned rows only (else hipErrorInvalidValue: the caller
// quantises separately).
LZK_EXPORT int lzk_layernorm_q8(const void* X, long ldx, const void* R, long ldr, const float* g, const float* b,
                                int rows, int H, float eps, void* Y, long ldy, void* Q, long ldq, float* qscale,
                                void* stream) {
  const bool v16 = (H == 768 || H == 1024) && ldx % 8 == 0 && ldy % 8 == 0 && (!R || ldr % 8 == 0) &&
                   ldq % 8 == 0 && ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Y) |
                                     reinterpret_cast<uintptr_t>(R) | reinterpret_cast<uintptr_t>(Q)) & 15) == 0;
  if (!v16 || rows <= 0 || !Q || !qscale) return (int)hipErrorInvalidValue;
  constexpr int RP = 2;
  dim3 grid16((rows + 16 - 1) / 16), block(256);
  hipStream_t st = (hipStream_t)stream;
  const u16* x = (const u16*)X;
  const u16* r = (const u16*)R;
  u16* y = (u16*)Y;
  unsigned char* q = (unsigned char*)Q;
#define LNQ(C)                                                                                                     \
  do {                                                                                                             \
    if (r) hipLaunchKernelGGL((layernorm16_kernel<C, true, RP, true>), grid16, block, 0, st, x, ldx, r, ldr, g, b, \
                              rows, eps, y, ldy, q, ldq, qscale);                                                  \
    else hipLaunchKernelGGL((layernorm16_kernel<C, false, RP, true>), grid16, block, 0, st, x, ldx, r, ldr, g, b,  \
                            rows, eps, y, ldy, q, ldq, qscale);                                                    \
  } while (0)
  if (H == 768) LNQ(3);
  else LNQ(4);
#undef LNQ
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_embed_ln(const int* ids, int T, int S, const void* wemb, const void* pemb, const void* temb,
                            const float* g, const float* b, int H, float eps, void* Y, const int* pos,
                            void* stream) {
  if (H % 4 != 0 || H > 64 * 4 * 4) return (int)hipErrorInvalidValue;
  dim3 grid((T + 3) / 4), block(256);
  hipLaunchKernelGGL((embed_ln_kernel<4>), grid, block, 0, (hipStream_t)stream, ids, T, S, (const u16*)wemb,
                     (const u16*)pemb, (const u16*)temb, g, b, H, eps, (u16*)Y, pos);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_pool_norm(const void* X, const int* lens, int B, int S, int H, int mode, float* out32,
                             void* out16, int ld16, const int* cu, void* stream) {
  if (H > 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pool_norm_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, (const u16*)X, lens, S, H, mode,
                     out32, (u16*)out16, ld16, cu);
  return (int)hipGetLastError();
}
