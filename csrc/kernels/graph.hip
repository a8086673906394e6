// Graph kernels shared by the tenant engine.
// The per-edge / per-node maintenance kernels (decay + prune, eviction
// scoring, neighbour boost, touch) live in tenant.hip, on the TenantGraph
// columns; this file holds the whole-graph algorithms:
//   connected comps   buffer_graph.py:99-120 (recursive DFS)                  (K9)
//   all-pairs merge   memory_system.py:1065-1120 (intended semantics)         (K7)
//   centroids         memory_system.py:916-917 (np.mean) / k-means update     (K8)
// plus the block-count scan used by every stable compaction.
#include "lzk_tile.h"

LZK_DEBUG_STATE(graph)

namespace {

constexpr int NTB = 256;

// Exclusive scan of per-block counts, in place, total in *total: one
// workgroup, 8192 counts per step -- 8 per thread, wave inclusive scan by
// shuffles, the 16 wave totals scanned by wave 0 -- two barriers per step
// (a 20M-edge compaction has 78K block counts: 10 steps).
constexpr int SCAN_PER = 8;
__global__ __launch_bounds__(1024) void scan_kernel(int* __restrict__ cnt, int n, int* __restrict__ total) {
  __shared__ int wsum[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int carry = 0;
  for (int base = 0; base < n; base += 1024 * SCAN_PER) {
    const int i0 = base + threadIdx.x * SCAN_PER;
    int v[SCAN_PER];
    int t = 0;
#pragma unroll
    for (int u = 0; u < SCAN_PER; ++u) {
      v[u] = i0 + u < n ? cnt[i0 + u] : 0;
      t += v[u];
    }
    int x = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    if (wv == 0) {
      int z = lane < 16 ? wsum[lane] : 0;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const int y = __shfl_up(z, o, 64);
        if (lane >= o) z += y;
      }
      if (lane < 16) wsum[lane] = z;
    }
    __syncthreads();
    int ex = carry + (wv ? wsum[wv - 1] : 0) + x - t;
#pragma unroll
    for (int u = 0; u < SCAN_PER; ++u) {
      if (i0 + u < n) cnt[i0 + u] = ex;
      ex += v[u];
    }
    carry += wsum[15];
    __syncthreads();  // wsum is rewritten by the next step
  }
  if (threadIdx.x == 0) *total = carry;
}

// ------------------------------------------------------------------ K9
// Connected components: min-label hooking on roots + pointer jumping.
__device__ __forceinline__ int find_root(const int* __restrict__ p, int x) {
  int y = p[x];
  while (y != x) { x = y; y = p[x]; }
  return x;
}

__global__ __launch_bounds__(NTB) void cc_hook_kernel(const int* __restrict__ src, const int* __restrict__ dst, long ne,
                                                      const float* __restrict__ w, float min_w, int* __restrict__ parent,
                                                      int* __restrict__ changed) {
  const long e = (long)blockIdx.x * NTB + threadIdx.x;
  if (e >= ne) return;
  LZK_DCHECK(src[e] >= 0 && dst[e] >= 0);
  if (w && w[e] < min_w) return;
  int ru = find_root(parent, src[e]);
  int rv = find_root(parent, dst[e]);
  if (ru == rv) return;
  int hi = max(ru, rv), lo = min(ru, rv);
  int old = atomicMin(&parent[hi], lo);
  if (old != lo) *changed = 1;
}

// One-pass lock-free union-find (the iterative hook/compress above needs a
// host-synchronised convergence loop). Every edge unites its endpoints'
// trees by CAS-hooking the larger root under the smaller, retrying from the
// value the CAS returns. Parent pointers only ever move to smaller indices
// and trees only merge, so a stale read (per-XCD L2s are not coherent, L1 is
// never refreshed by other CUs) can only name an older ancestor: two finds
// that agree are in the same tree, and every failed CAS strictly lowers one
// of the two roots, so each edge terminates. Reads and the path-halving
// writes are agent-scope (sc1, L2-served / write-through), so no dirty L2
// line can later overwrite a hook made on another XCD. After the pass (and
// cc_compress_kernel) every row's label is the smallest row of its
// component -- the same contract as the iterative kernels.
template <bool PLAIN>
__device__ __forceinline__ int uf_ld(const int* p, int x) {
  if constexpr (PLAIN) return p[x];
  return __hip_atomic_load(p + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// PLAIN (the default, ops.graph_ops.UF_PLAIN): cached loads. A stale line
// can only name an older ancestor -- a parent only ever moves to an ancestor
// of itself -- so finds still descend strictly, two finds that agree are in
// one tree, and a CAS on a stale root fails and continues from the value it
// returns; the hooks and halving stores stay agent-scope (coherent across
// XCDs). Same labels, 2.8 -> 2.05 ms on 10M rows / 20M random edges.
template <bool PLAIN>
__device__ __forceinline__ int uf_find(int* __restrict__ p, int x) {
  int y = uf_ld<PLAIN>(p, x);
  while (y != x) {
    const int z = uf_ld<PLAIN>(p, y);
    if (z == y) return y;
    __hip_atomic_store(p + x, z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // path halving: z is an ancestor of x
    x = z;
    y = uf_ld<PLAIN>(p, x);
  }
  return x;
}

template <bool PLAIN>
__global__ __launch_bounds__(NTB) void uf_union_kernel(const int* __restrict__ src, const int* __restrict__ dst, long ne,
                                                       const float* __restrict__ w, float min_w,
                                                       int* __restrict__ parent) {
  for (long e = (long)blockIdx.x * NTB + threadIdx.x; e < ne; e += (long)gridDim.x * NTB) {
    if (w && w[e] < min_w) continue;
    int a = src[e], b = dst[e];
    LZK_DCHECK(a >= 0 && b >= 0);
    while (true) {
      a = uf_find<PLAIN>(parent, a);
      b = uf_find<PLAIN>(parent, b);
      if (a == b) break;
      if (a < b) { const int t = a; a = b; b = t; }  // hook the larger root a under b
      const int old = atomicCAS(parent + a, a, b);
      if (old == a) break;
      a = old;  // a was hooked meanwhile: continue from its (smaller) parent
    }
  }
}

// The union pass over one side of an edge selection (incremental components
// across a consolidation batch, TenantGraph.cc_begin): an edge is VOLATILE --
// it may be deleted, or was added, during the batch -- when an endpoint is a
// row >= n0 (inserted since the mark), an endpoint is marked in vmark (a
// batch victim; rows < n0), or its weight is below wthr (the prune may take
// it). sel = 0 unions the stable edges (the batch's base labels, once),
// sel = 1 the volatile ones (on top of a copy of the base labels, at every
// consolidation point).
template <bool PLAIN>
__global__ __launch_bounds__(NTB) void uf_union_sel_kernel(const int* __restrict__ src, const int* __restrict__ dst,
                                                           long ne, const float* __restrict__ w, float wthr,
                                                           const unsigned char* __restrict__ vmark, int n0, int sel,
                                                           int* __restrict__ parent) {
  for (long e = (long)blockIdx.x * NTB + threadIdx.x; e < ne; e += (long)gridDim.x * NTB) {
    int a = src[e], b = dst[e];
    LZK_DCHECK(a >= 0 && b >= 0);
    const bool vol = a >= n0 || b >= n0 || vmark[a] || vmark[b] || (w && w[e] < wthr);
    if (vol != (sel != 0)) continue;
    while (true) {
      a = uf_find<PLAIN>(parent, a);
      b = uf_find<PLAIN>(parent, b);
      if (a == b) break;
      if (a < b) { const int t = a; a = b; b = t; }
      const int old = atomicCAS(parent + a, a, b);
      if (old == a) break;
      a = old;
    }
  }
}

__global__ __launch_bounds__(NTB) void cc_compress_kernel(int* __restrict__ parent, long n) {
  const long i = (long)blockIdx.x * NTB + threadIdx.x;
  if (i >= n) return;
  int r = find_root(parent, (int)i);
  parent[i] = r;
}

// ------------------------------------------------------------------ K7
// All pairs (i < j) with <x_i, x_j> > tau over unit rows: upper-triangular
// 128x128 MFMA tiles, pairs appended through one atomic counter.
__global__ __launch_bounds__(lzk::TNT, 2) void pairs_kernel(const u16* __restrict__ X, long ldx, int n, int D, float tau,
                                                       int ntile, int* __restrict__ count, int max_pairs,
                                                       int2* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  // linear id -> (ti <= tj)
  int id = blockIdx.x, ti = 0;
  while (id >= ntile - ti) { id -= ntile - ti; ++ti; }
  const int tj = ti + id;
  f32x16 acc[2][2];
  lzk::tile_gemm(smem, X, ldx, ti * lzk::TB, n, X, ldx, tj * lzk::TB, n, D, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wrow = wave >> 1, wcol = wave & 1, h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        int a = ti * lzk::TB + wrow * 64 + rb * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        int b = tj * lzk::TB + wcol * 64 + cb * 32 + l32;
        if (a < b && b < n && acc[rb][cb][e] > tau) {
          int o = atomicAdd(count, 1);
          if (o < max_pairs) out[o] = make_int2(a, b);
        }
      }
}

// ------------------------------------------------------------------ K8
// Segmented sums for centroids: one wave per row, f32 atomics into [C, D]
// (rows of one cluster are contiguous in memory for k-means updates after a
// sort, so the atomics mostly hit distinct lines).
__global__ __launch_bounds__(256) void seg_sum_kernel(const u16* __restrict__ X, long ldx, long n, int D,
                                                      const int* __restrict__ label, float* __restrict__ sums,
                                                      int* __restrict__ counts) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const int c = label[r];
  if (c < 0) return;  // negative label = tombstoned row (valid input)
  for (int d = lane * 4; d < D; d += 256) {
    u16x4 v = *reinterpret_cast<const u16x4*>(X + r * ldx + d);
#pragma unroll
    for (int u = 0; u < 4; ++u) atomicAdd(&sums[(long)c * D + d + u], bf16_to_f32(v[u]));
  }
  if (lane == 0) atomicAdd(&counts[c], 1);
}

// Atomic-free segmented sum over label-sorted rows: one workgroup per cluster,
// its 4 waves stride over the cluster's rows (two rows in flight per wave),
// each lane owns 4 consecutive dims of every 256-dim slice in registers; the
// waves meet once in LDS. Reads each row once (1.5 KB contiguous at d=768)
// instead of D fp32 atomics per row onto a few thousand hot addresses.
constexpr int SEG_MAXV = 8;  // D <= 2048
__global__ __launch_bounds__(256) void seg_sum_sorted_kernel(const u16* __restrict__ X, long ldx, int D,
                                                             const long* __restrict__ order,
                                                             const long* __restrict__ off,
                                                             float* __restrict__ sums, int* __restrict__ counts) {
  __shared__ float red[4][SEG_MAXV * 256];
  const int c = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long b = off[c], e = off[c + 1];
  float acc[SEG_MAXV][4];
#pragma unroll
  for (int v = 0; v < SEG_MAXV; ++v)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[v][u] = 0.f;
  long i = b + wave;
  for (; i + 4 < e; i += 8) {
    const u16* r0 = X + order[i] * ldx;
    const u16* r1 = X + order[i + 4] * ldx;
#pragma unroll
    for (int v = 0; v < SEG_MAXV; ++v) {
      const int d = (v * 64 + lane) * 4;
      if (d < D) {
        const u16x4 x0 = *reinterpret_cast<const u16x4*>(r0 + d);
        const u16x4 x1 = *reinterpret_cast<const u16x4*>(r1 + d);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[v][u] += bf16_to_f32(x0[u]) + bf16_to_f32(x1[u]);
      }
    }
  }
  if (i < e) {
    const u16* r0 = X + order[i] * ldx;
#pragma unroll
    for (int v = 0; v < SEG_MAXV; ++v) {
      const int d = (v * 64 + lane) * 4;
      if (d < D) {
        const u16x4 x0 = *reinterpret_cast<const u16x4*>(r0 + d);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[v][u] += bf16_to_f32(x0[u]);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < SEG_MAXV; ++v) {
    const int d = (v * 64 + lane) * 4;
    if (d < D)
#pragma unroll
      for (int u = 0; u < 4; ++u) red[wave][d + u] = acc[v][u];
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += 256)
    sums[(long)c * D + d] = (red[0][d] + red[1][d]) + (red[2][d] + red[3][d]);
  if (threadIdx.x == 0) counts[c] = (int)(e - b);
}

// centroid = sums / count, optionally L2-normalised; written as fp32 and bf16 (padded)
__global__ __launch_bounds__(64) void centroid_kernel(const float* __restrict__ sums, const int* __restrict__ counts,
                                                      int D, int normalize, float* __restrict__ c32,
                                                      u16* __restrict__ c16, int ld16) {
  const int c = blockIdx.x, lane = threadIdx.x;
  const float cnt = (float)max(1, counts[c]);
  float ss = 0.f;
  for (int d = lane; d < D; d += 64) { float v = sums[(long)c * D + d] / cnt; ss += v * v; }
  ss = wave_sum(ss);
  const float inv = (normalize && ss > 0.f) ? rsqrtf(ss) : 1.f;
  for (int d = lane; d < D; d += 64) {
    float v = sums[(long)c * D + d] / cnt * inv;
    if (c32) c32[(long)c * D + d] = v;
    if (c16) c16[(long)c * ld16 + d] = f32_to_bf16(v);
  }
  if (c16)
    for (int d = D + lane; d < ld16; d += 64) c16[(long)c * ld16 + d] = 0;
}

inline dim3 blocks_for(long n, int per = NTB) { return dim3((unsigned)((n + per - 1) / per)); }

}  // namespace

LZK_EXPORT int lzk_scan_blocks(int* cnt, int n, int* total, void* stream) {
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, cnt, n, total);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_cc_hook(const int* src, const int* dst, long ne, const float* w, float min_w, int* parent,
                           int* changed, void* stream) {
  if (ne == 0) return 0;
  hipLaunchKernelGGL(cc_hook_kernel, blocks_for(ne), dim3(NTB), 0, (hipStream_t)stream, src, dst, ne, w, min_w,
                     parent, changed);
  return (int)hipGetLastError();
}

static int uf_union_launch(const int* src, const int* dst, long ne, const float* w, float min_w, int* parent, bool plain,
                           void* stream) {
  if (ne == 0) return 0;
  // grid-stride: enough blocks to fill every CU several times over
  const long nb0 = (ne + NTB - 1) / NTB, nb = nb0 < 256L * 32 ? nb0 : 256L * 32;
  if (plain)
    hipLaunchKernelGGL(uf_union_kernel<true>, dim3((unsigned)nb), dim3(NTB), 0, (hipStream_t)stream, src, dst, ne, w,
                       min_w, parent);
  else
    hipLaunchKernelGGL(uf_union_kernel<false>, dim3((unsigned)nb), dim3(NTB), 0, (hipStream_t)stream, src, dst, ne, w,
                       min_w, parent);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_uf_union(const int* src, const int* dst, long ne, const float* w, float min_w, int* parent,
                            void* stream) {
  return uf_union_launch(src, dst, ne, w, min_w, parent, false, stream);
}

LZK_EXPORT int lzk_uf_union_plain(const int* src, const int* dst, long ne, const float* w, float min_w, int* parent,
                                  void* stream) {
  return uf_union_launch(src, dst, ne, w, min_w, parent, true, stream);
}

LZK_EXPORT int lzk_uf_union_sel(const int* src, const int* dst, long ne, const float* w, float wthr,
                                const unsigned char* vmark, int n0, int sel, int* parent, void* stream) {
  if (ne == 0) return 0;
  const long nb0 = (ne + NTB - 1) / NTB, nb = nb0 < 256L * 32 ? nb0 : 256L * 32;
  hipLaunchKernelGGL(uf_union_sel_kernel<true>, dim3((unsigned)nb), dim3(NTB), 0, (hipStream_t)stream, src, dst, ne,
                     w, wthr, vmark, n0, sel, parent);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_cc_compress(int* parent, long n, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(cc_compress_kernel, blocks_for(n), dim3(NTB), 0, (hipStream_t)stream, parent, n);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_pairs_above(const void* X, long ldx, int n, int D, float tau, int* count, int max_pairs,
                               void* out, void* stream) {
  if (D % lzk::TK != 0 || n <= 0) return (int)hipErrorInvalidValue;
  int nt = (n + lzk::TB - 1) / lzk::TB;
  long ntri = (long)nt * (nt + 1) / 2;
  size_t lds = 2 * 2 * lzk::TELEMS * sizeof(u16);
  hipLaunchKernelGGL(pairs_kernel, dim3((unsigned)ntri), dim3(lzk::TNT), lds, (hipStream_t)stream, (const u16*)X, ldx,
                     n, D, tau, nt, count, max_pairs, (int2*)out);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_seg_sum(const void* X, long ldx, long n, int D, const int* label, float* sums, int* counts,
                           void* stream) {
  if (n == 0) return 0;
  if (D % 4 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(seg_sum_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, (const u16*)X,
                     ldx, n, D, label, sums, counts);
  return (int)hipGetLastError();
}

// order: row indices sorted by label; off: [C+1] segment offsets into order.
// Writes every cluster's sums/counts (no pre-zeroing needed).
LZK_EXPORT int lzk_seg_sum_sorted(const void* X, long ldx, int D, const long* order, const long* off, int C,
                                  float* sums, int* counts, void* stream) {
  if (C == 0) return 0;
  if (D % 4 != 0 || D > SEG_MAXV * 256) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(seg_sum_sorted_kernel, dim3((unsigned)C), dim3(256), 0, (hipStream_t)stream, (const u16*)X, ldx,
                     D, order, off, sums, counts);
  return (int)hipGetLastError();
}

LZK_EXPORT int lzk_centroids(const float* sums, const int* counts, int C, int D, int normalize, float* c32, void* c16,
                             int ld16, void* stream) {
  if (C == 0) return 0;
  hipLaunchKernelGGL(centroid_kernel, dim3(C), dim3(64), 0, (hipStream_t)stream, sums, counts, D, normalize, c32,
                     (u16*)c16, ld16);
  return (int)hipGetLastError();
}
