// Farthest-first seeding of the k-means hierarchy (the
// reference's hierarchy is one mean super-node per shard,
// memory_system.py:893-933 -- the k-means mode clusters the whole tenant).
//
// Farthest-first is sequential: pick t is the sample row least similar to
// every pick so far, so each step is one pass over the sample (a GEMV against
// the last pick, a running max, an argmin). As torch ops that is a rocBLAS
// GEMV + a max + an ArgMin reduction per pick, thousands of launches from
// Python. Here ONE kernel per step does all three: every block scores its
// rows against the pick (8 lanes per row, 16-B bf16 pieces, fp32 sums),
// updates the rows' best similarity and folds its argmin into the NEXT
// step's 64-bit key with one atomicMin (order-preserving score bits high,
// row low: the smallest score, ties to the smaller row -- torch.argmin's
// first occurrence). The next step decodes its pick from that key on the
// device, and the host loop that enqueues the k steps runs in C++: no host
// sync, no Python per pick.
#include "lzk_common.h"

namespace {

constexpr int FF_THREADS = 256;
constexpr int FF_MAXD = 2048;

__device__ __forceinline__ unsigned long long ff_key(float s, int r) {
  const unsigned u = __float_as_uint(s);
  const unsigned k = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)k << 32) | (unsigned)r;
}

// step t: pick j (row 0 at t = 0, else decoded from keys[t]); best[r] =
// max(best[r], <S_r, S_j>) (= the dot at t = 0); argmin -> keys[t + 1].
__global__ __launch_bounds__(FF_THREADS) void ff_step_kernel(const u16* __restrict__ S, long ld, int m, int D, int t,
                                                             float* __restrict__ best, int* __restrict__ picks,
                                                             unsigned long long* __restrict__ keys) {
  __shared__ __attribute__((aligned(16))) float qv[FF_MAXD];
  __shared__ unsigned long long red[FF_THREADS / 64];
  const int j = t == 0 ? 0 : (int)(keys[t] & 0xFFFFFFFFull);
  if (blockIdx.x == 0 && threadIdx.x == 0) picks[t] = j;
  for (int c = threadIdx.x; c < D; c += FF_THREADS) qv[c] = bf16_to_f32(S[(long)j * ld + c]);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int part = lane & 7, sub = lane >> 3;
  unsigned long long mine = ~0ull;
  const int rows_per_block = (FF_THREADS / 8);  // 32 rows per block-iteration
  for (int r0 = blockIdx.x * rows_per_block; r0 < m; r0 += gridDim.x * rows_per_block) {
    const int r = r0 + wave * 8 + sub;
    float a = 0.f;
    if (r < m) {
      const u16* xr = S + (long)r * ld;
      for (int c = part * 8; c < D; c += 64) {
        const u16x8 v = *reinterpret_cast<const u16x8*>(xr + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) a = fmaf(bf16_to_f32(v[e]), qv[c + e], a);
      }
    }
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (part == 0 && r < m) {
      const float b = t == 0 ? a : fmaxf(best[r], a);
      best[r] = b;
      const unsigned long long k = ff_key(b, r);
      mine = k < mine ? k : mine;
    }
  }
  // block min of the packed keys
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long other = __shfl_xor(mine, o, 64);
    mine = other < mine ? other : mine;
  }
  if (lane == 0) red[wave] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long k = red[0];
    for (int w = 1; w < FF_THREADS / 64; ++w) k = red[w] < k ? red[w] : k;
    if (k != ~0ull) atomicMin(keys + t + 1, k);
  }
}

}  // namespace

// Farthest-first picks over the bf16 sample rows S [m, D] (row stride ld
// elements, D % 8 == 0, D <= 2048, rows 16-B aligned): picks[0] = 0, then
// picks[t] = argmin_r max_{u < t} <S_r, S_picks[u]> for t < k (k <= m).
// ws: (k + 1) * 8 bytes of keys + m * 4 bytes of best similarities.
LZK_EXPORT long lzk_farthest_first_ws(int m, int k) { return (long)(k + 1) * 8 + (long)m * 4 + 64; }

LZK_EXPORT int lzk_farthest_first(const void* S, long ld, int m, int D, int k, int* picks, void* ws, void* stream) {
  if (m <= 0 || k <= 0 || k > m || D <= 0 || D > FF_MAXD || D % 8 != 0 || ld % 8 != 0)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  unsigned long long* keys = (unsigned long long*)ws;
  float* best = (float*)((char*)ws + (((long)(k + 1) * 8 + 63) / 64) * 64);
  hipError_t e = hipMemsetAsync(keys, 0xFF, (size_t)(k + 1) * 8, st);
  if (e != hipSuccess) return (int)e;
  const int rows_per_block = FF_THREADS / 8;
  int grid = (m + rows_per_block - 1) / rows_per_block;
  if (grid > 1024) grid = 1024;
  for (int t = 0; t < k; ++t) {
    hipLaunchKernelGGL(ff_step_kernel, dim3(grid), dim3(FF_THREADS), 0, st, (const u16*)S, ld, m, D, t, best, picks,
                       keys);
  }
  return (int)hipGetLastError();
}
