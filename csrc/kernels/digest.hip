// Component digest of run_consolidation without sorting the graph
// (reference memory_system.py:967-990: components with >= 3 members and mean
// edge weight > 0.3 feed the profile prompt with their first 10 contents).
//
// Input: union-find labels (graph.hip uf_union/cc_compress: label = smallest
// row of the component) over a tenant graph's SoA columns. Output: for every
// qualifying component, its first `take` live shard-node rows in row order,
// tagged with the component's order key (smallest (super ? 0 : shard + 1) *
// n + row over its live nodes -- the reference's BufferGraph.nodes order).
//
// The sort + segmented-scan formulation (engine/tenant_graph.py, CPU path)
// sorts every touched row and every edge by label: ~11 ms at 10M rows / 20M
// edges, almost all of it the sorts. Here every per-component quantity is a
// keyed reduction with two levels of aggregation so that one giant component
// (the usual shape: one component holding most rows) does not serialise
// atomics on one address:
//   wave   lanes with the leader's label reduce by DPP/shuffle, one push per
//          distinct label (a few passes, then per-lane pushes)
//   block  a 1024-slot LDS cache keyed by label absorbs the pushes (LDS
//          atomics); one global atomic per cached label per block at the end
// The first-`take` selection is exact and sort-free: components with <= take
// candidates take all of them (one append pass); larger ones run `take`
// rounds of "smallest eligible row above the last one selected", where only
// the first lane of each label in a wave (the smallest row, lanes are in row
// order) tests the running minimum and issues an atomicMin if it improves it.
#include "lzk_common.h"

LZK_DEBUG_STATE(digest)

namespace {

constexpr int DNT = 256;
constexpr int HS = 1024;  // LDS cache slots per block
constexpr int MATCH_PASSES = 4;
constexpr long long BIGKEY = 1LL << 62;
constexpr int NOROW = 0x7fffffff;

__device__ __forceinline__ int slot_of(int L) { return (int)(((unsigned)L * 2654435761u) >> 22); }  // 10 bits

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ long long wave_min_ll(long long v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const long long u = __shfl_xor(v, o, 64);
    v = u < v ? u : v;
  }
  return v;
}

// Claim (or find) the LDS slot of label L; false when another label holds it.
__device__ __forceinline__ bool lds_claim(int* keys, int s, int L) {
  int k = __hip_atomic_load(keys + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (k == L) return true;
  if (k != -1) return false;
  k = atomicCAS(keys + s, -1, L);
  return k == -1 || k == L;
}

__device__ __forceinline__ void lds_init(int* keys) {
  for (int i = threadIdx.x; i < HS; i += DNT) keys[i] = -1;
}

// ---------------------------------------------------------------- touched
// touched[r] = r is an endpoint of some edge. With union-find labels that is
// lab[r] != r (hooked under a smaller row: a component of >= 2 rows), or r
// is the label of another row, or r has a self-loop (dg_edges_kernel) -- a
// sequential pass over the labels instead of 2 random byte stores per edge.
// Rows of a wave are consecutive, so in the usual one-giant-component graph
// all lanes share the label and one lane marks it.
__global__ __launch_bounds__(DNT) void dg_touch_kernel(const int* __restrict__ lab, long n,
                                                       unsigned char* __restrict__ touched) {
  const int lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * DNT;
  for (long base = (long)blockIdx.x * DNT; base < n; base += stride) {
    const long r = base + threadIdx.x;
    int L = -1;
    if (r < n) {
      L = lab[r];
      if (L != (int)r) touched[r] = 1;
      else L = -1;
    }
    bool act = L >= 0;
    for (int it = 0; it < MATCH_PASSES; ++it) {
      const unsigned long long m = __ballot(act);
      if (m == 0) break;
      const int leader = __ffsll((long long)m) - 1;
      const int LL = __shfl(L, leader, 64);
      if (lane == leader) touched[LL] = 1;
      act = act && L != LL;
    }
    if (act) touched[L] = 1;
  }
}

// ---------------------------------------------------------------- edges
// Per label of src: sum of weights (fp64), edge count; touched[a] for a
// self-loop (a, a) (every other endpoint is marked by dg_touch_kernel).
__device__ __forceinline__ void push_w(int L, double s, int c, int* keys, double* ssum, int* scnt, double* gsum,
                                       int* gcnt) {
  const int sl = slot_of(L);
  if (lds_claim(keys, sl, L)) {
    atomicAdd(ssum + sl, s);
    atomicAdd(scnt + sl, c);
  } else {
    unsafeAtomicAdd(gsum + L, s);
    atomicAdd(gcnt + L, c);
  }
}

__global__ __launch_bounds__(DNT) void dg_edges_kernel(const int* __restrict__ src, const int* __restrict__ dst,
                                                       const float* __restrict__ w, long ne,
                                                       const int* __restrict__ lab,
                                                       unsigned char* __restrict__ touched, double* __restrict__ gsum,
                                                       int* __restrict__ gcnt) {
  __shared__ int keys[HS];
  __shared__ double ssum[HS];
  __shared__ int scnt[HS];
  lds_init(keys);
  for (int i = threadIdx.x; i < HS; i += DNT) { ssum[i] = 0.0; scnt[i] = 0; }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * DNT;
  for (long base = (long)blockIdx.x * DNT; base < ne; base += stride) {  // block-uniform trip count
    const long e = base + threadIdx.x;
    bool act = e < ne;
    int L = -1;
    double v = 0.0;
    if (act) {
      const int a = src[e];
      if (a == dst[e]) touched[a] = 1;
      L = lab[a];
      v = (double)w[e];
    }
    for (int it = 0; it < MATCH_PASSES; ++it) {
      const unsigned long long m = __ballot(act);
      if (m == 0) break;
      const int leader = __ffsll((long long)m) - 1;
      const int LL = __shfl(L, leader, 64);
      const bool mine = act && L == LL;
      const double s = wave_sum_d(mine ? v : 0.0);
      const int c = __popcll(__ballot(mine));
      if (lane == leader) push_w(LL, s, c, keys, ssum, scnt, gsum, gcnt);
      act = act && !mine;
    }
    if (act) push_w(L, v, 1, keys, ssum, scnt, gsum, gcnt);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < HS; i += DNT) {
    const int L = keys[i];
    if (L >= 0) {
      unsafeAtomicAdd(gsum + L, ssum[i]);
      atomicAdd(gcnt + L, scnt[i]);
    }
  }
}

// ---------------------------------------------------------------- rows
// Members = touched rows that are not free (live nodes and ghost endpoints,
// like the reference DFS that follows edges to missing ids). Per label:
// member count, candidate count (live shard nodes: kind 1, not super), and
// the order key min over live nodes.
__device__ __forceinline__ void push_r(int L, int sz, int cc, long long fk, int* keys, int* ssz, int* scc,
                                       long long* sfk, int* gsize, int* gccnt, long long* gfirst) {
  const int sl = slot_of(L);
  if (lds_claim(keys, sl, L)) {
    atomicAdd(ssz + sl, sz);
    if (cc) atomicAdd(scc + sl, cc);
    if (fk < BIGKEY) atomicMin(sfk + sl, fk);
  } else {
    atomicAdd(gsize + L, sz);
    if (cc) atomicAdd(gccnt + L, cc);
    if (fk < BIGKEY) atomicMin(gfirst + L, fk);
  }
}

__global__ __launch_bounds__(DNT) void dg_rows_kernel(const int* __restrict__ lab,
                                                      const unsigned char* __restrict__ touched,
                                                      const unsigned char* __restrict__ kind,
                                                      const unsigned char* __restrict__ sup,
                                                      const int* __restrict__ shard, long n, int* __restrict__ gsize,
                                                      int* __restrict__ gccnt, long long* __restrict__ gfirst) {
  __shared__ int keys[HS];
  __shared__ int ssz[HS];
  __shared__ int scc[HS];
  __shared__ long long sfk[HS];
  lds_init(keys);
  for (int i = threadIdx.x; i < HS; i += DNT) { ssz[i] = 0; scc[i] = 0; sfk[i] = BIGKEY; }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * DNT;
  for (long base = (long)blockIdx.x * DNT; base < n; base += stride) {
    const long r = base + threadIdx.x;
    bool act = false, cand = false;
    int L = -1;
    long long fk = BIGKEY;
    if (r < n && touched[r]) {
      const unsigned char k = kind[r];
      if (k != 0) {
        act = true;
        L = lab[r];
        if (k == 1) {
          const bool s = sup[r] != 0;
          cand = !s;
          fk = (s ? 0LL : (long long)shard[r] + 1) * (long long)n + r;
        }
      }
    }
    for (int it = 0; it < MATCH_PASSES; ++it) {
      const unsigned long long m = __ballot(act);
      if (m == 0) break;
      const int leader = __ffsll((long long)m) - 1;
      const int LL = __shfl(L, leader, 64);
      const bool mine = act && L == LL;
      const int sz = __popcll(__ballot(mine));
      const int cc = __popcll(__ballot(mine && cand));
      const long long f = wave_min_ll(mine ? fk : BIGKEY);
      if (lane == leader) push_r(LL, sz, cc, f, keys, ssz, scc, sfk, gsize, gccnt, gfirst);
      act = act && !mine;
    }
    if (act) push_r(L, 1, cand ? 1 : 0, fk, keys, ssz, scc, sfk, gsize, gccnt, gfirst);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < HS; i += DNT) {
    const int L = keys[i];
    if (L >= 0) {
      atomicAdd(gsize + L, ssz[i]);
      if (scc[i]) atomicAdd(gccnt + L, scc[i]);
      if (sfk[i] < BIGKEY) atomicMin(gfirst + L, sfk[i]);
    }
  }
}

// ---------------------------------------------------------------- classify
// cls[L]: 0 = not selected, 1 = qualifies with <= take candidates (all of
// them are taken), 2 = qualifies with more (selection rounds). counters[0] +=
// candidates of class-1 labels, counters[1] = number of class-2 labels (also
// appended to biglist), counters[2] = qualifying components.
__global__ __launch_bounds__(DNT) void dg_classify_kernel(long n, int min_size, double min_avg_w, int take,
                                                          const int* __restrict__ gsize,
                                                          const double* __restrict__ gsum,
                                                          const int* __restrict__ gcnt,
                                                          const long long* __restrict__ gfirst,
                                                          const int* __restrict__ gccnt,
                                                          unsigned char* __restrict__ cls, int* __restrict__ biglist,
                                                          int* __restrict__ counters) {
  __shared__ int red[2][DNT / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int direct = 0, nok = 0;
  const long stride = (long)gridDim.x * DNT;
  for (long base = (long)blockIdx.x * DNT; base < n; base += stride) {
    const long L = base + threadIdx.x;
    unsigned char c = 0;
    if (L < n) {
      const int sz = gsize[L], ec = gcnt[L], cc = gccnt[L];
      if (sz >= min_size && ec > 0 && cc > 0 && gfirst[L] < BIGKEY && gsum[L] / (double)ec > min_avg_w) {
        c = cc <= take ? 1 : 2;
        ++nok;
        if (c == 1) direct += cc;
      }
      cls[L] = c;
    }
    const unsigned long long big = __ballot(c == 2);
    if (big) {
      int b0 = 0;
      if (lane == 0) b0 = atomicAdd(counters + 1, __popcll(big));
      b0 = __shfl(b0, 0, 64);
      if (c == 2) biglist[b0 + __popcll(big & ((1ULL << lane) - 1))] = (int)L;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    direct += __shfl_xor(direct, o, 64);
    nok += __shfl_xor(nok, o, 64);
  }
  if (lane == 0) { red[0][wv] = direct; red[1][wv] = nok; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int d = 0, k = 0;
    for (int i = 0; i < DNT / 64; ++i) { d += red[0][i]; k += red[1][i]; }
    if (d) atomicAdd(counters, d);
    if (k) atomicAdd(counters + 2, k);
  }
}

__device__ __forceinline__ bool is_cand(long r, long n, const unsigned char* touched, const unsigned char* kind,
                                        const unsigned char* sup) {
  return r < n && touched[r] && kind[r] == 1 && sup[r] == 0;
}

// Candidates of class-1 components: appended as (order key, row).
__global__ __launch_bounds__(DNT) void dg_direct_kernel(const int* __restrict__ lab,
                                                        const unsigned char* __restrict__ touched,
                                                        const unsigned char* __restrict__ kind,
                                                        const unsigned char* __restrict__ sup, long n,
                                                        const unsigned char* __restrict__ cls,
                                                        const long long* __restrict__ gfirst,
                                                        long long* __restrict__ out_key, int* __restrict__ out_row,
                                                        int cap, int* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * DNT;
  for (long base = (long)blockIdx.x * DNT; base < n; base += stride) {
    const long r = base + threadIdx.x;
    int L = -1;
    bool sel = false;
    if (is_cand(r, n, touched, kind, sup)) {
      L = lab[r];
      sel = cls[L] == 1;
    }
    const unsigned long long m = __ballot(sel);
    if (m == 0) continue;
    int b0 = 0;
    if (lane == 0) b0 = atomicAdd(count, __popcll(m));
    b0 = __shfl(b0, 0, 64);
    const int at = b0 + __popcll(m & ((1ULL << lane) - 1));
    if (sel && at < cap) {
      out_key[at] = gfirst[L];
      out_row[at] = (int)r;
    }
  }
}

// One selection round over the class-2 components, rows [lo, hi): cur[L] =
// smallest candidate row of L in the range above last[L] (the last row
// selected for L, -1 before the first).
__global__ __launch_bounds__(DNT) void dg_round_kernel(const int* __restrict__ lab,
                                                       const unsigned char* __restrict__ touched,
                                                       const unsigned char* __restrict__ kind,
                                                       const unsigned char* __restrict__ sup, long lo, long hi,
                                                       const unsigned char* __restrict__ cls,
                                                       const int* __restrict__ last, int* __restrict__ cur) {
  const int lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * DNT;
  for (long base = lo + (long)blockIdx.x * DNT; base < hi; base += stride) {
    const long r = base + threadIdx.x;
    int L = -1;
    bool act = false;
    if (is_cand(r, hi, touched, kind, sup)) {
      L = lab[r];
      act = cls[L] == 2 && (int)r > last[L];
    }
    while (true) {  // one pass per distinct eligible label in the wave
      const unsigned long long m = __ballot(act);
      if (m == 0) break;
      const int leader = __ffsll((long long)m) - 1;
      const int LL = __shfl(L, leader, 64);
      if (lane == leader) {  // lanes are in row order: the leader holds LL's smallest eligible row
        const int v = __hip_atomic_load(cur + LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((int)r < v) atomicMin(cur + LL, (int)r);
      }
      act = act && L != LL;
    }
  }
}

// After a round: append each class-2 component's selected row (if any),
// advance last[L], count it, retire the component (class 3) once it has
// `take` rows, reset cur[L]; remaining[0] += components still open.
__global__ __launch_bounds__(DNT) void dg_collect_kernel(const int* __restrict__ biglist, int nbig,
                                                         const int* __restrict__ nbig_dev, int take,
                                                         int* __restrict__ cur, int* __restrict__ last,
                                                         int* __restrict__ cnt, unsigned char* __restrict__ cls,
                                                         const long long* __restrict__ gfirst,
                                                         long long* __restrict__ out_key, int* __restrict__ out_row,
                                                         int cap, int* __restrict__ count,
                                                         int* __restrict__ remaining) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * DNT + threadIdx.x;
  if (nbig_dev) nbig = *nbig_dev;  // sync-free mode: the classify pass's count, grid sized for the bound
  int L = -1, v = NOROW;
  bool open = false;
  if (i < nbig) {
    L = biglist[i];
    if (cls[L] == 2) {
      v = cur[L];
      cur[L] = NOROW;
      open = true;
      if (v != NOROW) {
        last[L] = v;
        const int c = cnt[L] + 1;
        cnt[L] = c;
        if (c >= take) { cls[L] = 3; open = false; }
      }
    }
  }
  const bool sel = v != NOROW;
  const unsigned long long m = __ballot(sel);
  const unsigned long long o = __ballot(open);
  if (lane == 0 && o) atomicAdd(remaining, __popcll(o));
  if (m == 0) return;
  int b0 = 0;
  if (lane == 0) b0 = atomicAdd(count, __popcll(m));
  b0 = __shfl(b0, 0, 64);
  const int at = b0 + __popcll(m & ((1ULL << lane) - 1));
  if (sel && at < cap) {
    out_key[at] = gfirst[L];
    out_row[at] = v;
  }
}

// ---------------------------------------------------------------- small graphs
// The whole digest of a graph with at most SD_MAXE edges in ONE block: the
// consolidation buffer at the reference's prune threshold keeps a few
// hundred to a few thousand edges over millions of rows, and consolidate_batch
// reads the digest at ~40 points per step -- a chain of tenant-wide passes
// (or of torch ops over a renumbered index space) costs more in launches
// than the work. Endpoints are sorted (bitonic, LDS) and renumbered to local
// ids u (row order), union-find runs on LDS parents (hook the larger root
// under the smaller: a component's root is its smallest row), the
// per-component reductions go to a small global scratch, `take` selection
// rounds pick each component's first candidate rows, and the (order key,
// row) output is sorted by one more bitonic pass. Same definitions as the
// kernels above (members: touched rows not free; candidates: live shard
// nodes; order key over live nodes with the tenant's n and rows); outputs
// out[0][i] = key, out[1][i] = row for i < count, then (1 << 62, -1).
constexpr int SD_NT = 1024;
constexpr int SD_MAXE = 2048;
constexpr int SD_P = 2 * SD_MAXE;

__device__ __forceinline__ int sd_find(volatile int* par, int x) {
  while (true) {
    const int p = par[x];
    if (p == x) return x;
    x = p;
  }
}

__device__ __forceinline__ int sd_bsearch(const int* a, int n, int v) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

struct SdScratch {  // per local label, in global memory (L2-resident, zeroed here)
  double* wsum;
  int* ecnt;
  int* size;
  int* ccnt;
  long long* first;
  int* cur;
  int* last;
  int* taken;
};

__global__ __launch_bounds__(SD_NT) void dg_small_kernel(const int* __restrict__ src, const int* __restrict__ dst,
                                                         const float* __restrict__ w, int ne,
                                                         const unsigned char* __restrict__ kind,
                                                         const unsigned char* __restrict__ sup,
                                                         const int* __restrict__ shard, long n, int min_size,
                                                         double min_avg_w, int take, SdScratch S,
                                                         long long* __restrict__ out, int cap,
                                                         int* __restrict__ out_cnt) {
  __shared__ int ep[SD_P];       // sorted endpoints, then unique rows (urow)
  __shared__ int par[SD_P];      // union-find parents over local ids
  __shared__ long long sk[SD_P];  // output sort: keys
  __shared__ int su[SD_P];        // output sort: local ids
  __shared__ int s_scan[SD_NT / 64];
  __shared__ int s_U, s_cnt, s_open;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int P = 2;
  while (P < 2 * ne) P <<= 1;
  for (int i = tid; i < P; i += SD_NT) ep[i] = i < ne ? src[i] : (i < 2 * ne ? dst[i - ne] : 0x7fffffff);
  __syncthreads();
  // bitonic sort of the endpoints (ascending)
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += SD_NT) {
        const int l = i ^ j;
        if (l > i) {
          const int a = ep[i], b = ep[l];
          if (((i & k) == 0) == (a > b)) { ep[i] = b; ep[l] = a; }
        }
      }
      __syncthreads();
    }
  // unique -> urow[0 .. U) (in place: a block scan of the first-occurrence
  // flags, values read before the barrier, written after)
  int base = 0;
  for (int c0 = 0; c0 < P; c0 += SD_NT) {
    const int i = c0 + tid;
    int v = 0x7fffffff;
    bool f = false;
    if (i < P) {
      v = ep[i];
      f = v != 0x7fffffff && (i == 0 || ep[i - 1] != v);
    }
    const unsigned long long b = __ballot(f);
    if (lane == 0) s_scan[wv] = __popcll(b);
    __syncthreads();
    int before = 0, tot = 0;
    for (int x = 0; x < SD_NT / 64; ++x) {
      before += x < wv ? s_scan[x] : 0;
      tot += s_scan[x];
    }
    __syncthreads();
    if (f) ep[base + before + __popcll(b & ((1ull << lane) - 1))] = v;
    base += tot;
    __syncthreads();
  }
  const int U = base;
  for (int u = tid; u < P; u += SD_NT) {
    par[u] = u;
    if (u < U) {
      S.wsum[u] = 0.0;
      S.ecnt[u] = 0;
      S.size[u] = 0;
      S.ccnt[u] = 0;
      S.first[u] = BIGKEY;
      S.cur[u] = NOROW;
      S.last[u] = -1;
      S.taken[u] = 0;
    }
  }
  if (tid == 0) { s_U = U; s_cnt = 0; }
  __syncthreads();
  // union-find: hook the larger root under the smaller
  for (int e = tid; e < ne; e += SD_NT) {
    int a = sd_bsearch(ep, U, src[e]), b = sd_bsearch(ep, U, dst[e]);
    while (true) {
      a = sd_find(par, a);
      b = sd_find(par, b);
      if (a == b) break;
      if (a > b) { const int t = a; a = b; b = t; }
      const int old = atomicCAS(&par[b], b, a);
      if (old == b) break;
      b = old;
    }
  }
  __syncthreads();
  for (int u = tid; u < U; u += SD_NT) par[u] = sd_find(par, u);
  __syncthreads();
  __threadfence_block();
  // per-component reductions
  for (int e = tid; e < ne; e += SD_NT) {
    const int L = par[sd_bsearch(ep, U, src[e])];
    atomicAdd(S.wsum + L, (double)w[e]);
    atomicAdd(S.ecnt + L, 1);
  }
  for (int u = tid; u < U; u += SD_NT) {
    const int r = ep[u];
    const unsigned char k = kind[r];
    if (k == 0) continue;
    const int L = par[u];
    atomicAdd(S.size + L, 1);
    if (k == 1) {
      const bool s = sup[r] != 0;
      if (!s) atomicAdd(S.ccnt + L, 1);
      atomicMin(S.first + L, (s ? 0LL : (long long)shard[r] + 1) * (long long)n + r);
    }
  }
  __threadfence();
  __syncthreads();
  // selection: `take` rounds of "smallest candidate above the last one taken"
  for (int round = 0; round < take; ++round) {
    for (int u = tid; u < U; u += SD_NT) {
      const int r = ep[u];
      if (kind[r] != 1 || sup[r] != 0) continue;
      const int L = par[u];
      const int ec = S.ecnt[L];
      if (S.size[L] < min_size || ec <= 0 || S.ccnt[L] <= 0 || S.first[L] >= BIGKEY ||
          !(S.wsum[L] / (double)ec > min_avg_w) || S.taken[L] >= take || u <= S.last[L])
        continue;
      atomicMin(S.cur + L, u);
    }
    __threadfence();
    __syncthreads();
    if (tid == 0) s_open = 0;
    __syncthreads();
    for (int u = tid; u < U; u += SD_NT) {
      if (par[u] != u) continue;  // component roots
      const int c = S.cur[u];
      if (c == NOROW) continue;
      S.cur[u] = NOROW;
      S.last[u] = c;
      S.taken[u] += 1;
      const int at = atomicAdd(&s_cnt, 1);
      sk[at] = S.first[u];
      su[at] = c;
      s_open = 1;
    }
    __threadfence();
    __syncthreads();
    if (!s_open) break;
  }
  const int m = s_cnt;
  int Q = 2;
  while (Q < m) Q <<= 1;
  for (int i = m + tid; i < Q; i += SD_NT) { sk[i] = BIGKEY; su[i] = 0x7fffffff; }
  __syncthreads();
  // (key, local id) ascending = (key, row)
  for (int k = 2; k <= Q; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < Q; i += SD_NT) {
        const int l = i ^ j;
        if (l > i) {
          const long long ka = sk[i], kb = sk[l];
          const int ua = su[i], ub = su[l];
          const bool gt = ka > kb || (ka == kb && ua > ub);
          if (((i & k) == 0) == gt) { sk[i] = kb; sk[l] = ka; su[i] = ub; su[l] = ua; }
        }
      }
      __syncthreads();
    }
  for (int i = tid; i < cap; i += SD_NT) {
    const bool ok = i < m;
    out[i] = ok ? sk[i] : BIGKEY;
    out[cap + i] = ok ? (long long)ep[su[i]] : -1LL;
  }
  if (tid == 0) *out_cnt = m;
}

inline unsigned grid_for(long n, unsigned cap = 4096) {
  const long b = (n + DNT - 1) / DNT;
  return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace

// Stats phase: edge and row reductions + classification. `lab` must be the
// union-find labels (smallest row of the component) of exactly these edges:
// the touched rows are derived from them. Every output array
// is indexed by label (length n) and must be zeroed by the caller, except
// gfirst (filled with 1 << 62) and cls/biglist (written here); counters[3]
// zeroed. The caller reads counters back (one synchronisation) to size the
// selection output: counters[0] + take * counters[1] entries.
LZK_EXPORT int lzk_dg_stats(const int* src, const int* dst, const float* w, long ne, const int* lab, long n,
                            const unsigned char* kind, const unsigned char* sup, const int* shard, int min_size,
                            double min_avg_w, int take, unsigned char* touched, double* gsum, int* gcnt, int* gsize,
                            int* gccnt, long long* gfirst, unsigned char* cls, int* biglist, int* counters,
                            void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (ne > 0) {
    hipLaunchKernelGGL(dg_touch_kernel, dim3(grid_for(n, 4096)), dim3(DNT), 0, st, lab, n, touched);
    hipLaunchKernelGGL(dg_edges_kernel, dim3(grid_for(ne, 2048)), dim3(DNT), 0, st, src, dst, w, ne, lab, touched,
                       gsum, gcnt);
  }
  hipLaunchKernelGGL(dg_rows_kernel, dim3(grid_for(n, 2048)), dim3(DNT), 0, st, lab, touched, kind, sup, shard, n,
                     gsize, gccnt, gfirst);
  hipLaunchKernelGGL(dg_classify_kernel, dim3(grid_for(n, 1024)), dim3(DNT), 0, st, n, min_size, min_avg_w, take,
                     gsize, gsum, gcnt, gfirst, gccnt, cls, biglist, counters);
  return (int)hipGetLastError();
}

// Selection phase: (order key, row) of every selected row, unordered, in
// out_key/out_row[0 : *count]; cap = counters[0] + take * counters[1].
// cur: int[n] filled with 0x7fffffff; last: int[n] filled with -1; cnt:
// int[n] zeroed (only class-2 labels' entries are used). cls is updated
// (class-2 components retire to class 3). First `take` rounds over a prefix
// window of the rows -- a large component's first candidates are nearly
// always there -- then, only for components still open (one synchronising
// read of `remaining`), `take` rounds over the rest.
// nbig_dev (sync-free mode, small n): the class-2 count is read on the
// device (counters + 1 of lzk_dg_stats); nbig is then its upper bound (the
// collect grid), every round runs over all n rows and nothing is read back.
LZK_EXPORT int lzk_dg_select(const int* lab, long n, const unsigned char* touched, const unsigned char* kind,
                             const unsigned char* sup, unsigned char* cls, const long long* gfirst,
                             const int* biglist, int nbig, const int* nbig_dev, int take, int* cur, int* last,
                             int* cnt, long long* out_key, int* out_row, int cap, int* count, int* remaining,
                             long window, void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(dg_direct_kernel, dim3(grid_for(n)), dim3(DNT), 0, st, lab, touched, kind, sup, n, cls, gfirst,
                     out_key, out_row, cap, count);
  if (nbig <= 0) return (int)hipGetLastError();
  const long w = (nbig_dev || window <= 0 || window >= n) ? n : window;
  const unsigned cb = (unsigned)((nbig + DNT - 1) / DNT);
  for (int k = 0; k < take; ++k) {
    hipLaunchKernelGGL(dg_round_kernel, dim3(grid_for(w)), dim3(DNT), 0, st, lab, touched, kind, sup, 0L, w, cls,
                       last, cur);
    (void)hipMemsetAsync(remaining, 0, sizeof(int), st);
    hipLaunchKernelGGL(dg_collect_kernel, dim3(cb), dim3(DNT), 0, st, biglist, nbig, nbig_dev, take, cur, last, cnt,
                       cls, gfirst, out_key, out_row, cap, count, remaining);
  }
  if (w >= n) return (int)hipGetLastError();
  int open = 0;
  if (hipMemcpyAsync(&open, remaining, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess) return (int)hipGetLastError();
  if (hipStreamSynchronize(st) != hipSuccess) return (int)hipGetLastError();
  for (int k = 0; k < take && open > 0; ++k) {
    hipLaunchKernelGGL(dg_round_kernel, dim3(grid_for(n - w)), dim3(DNT), 0, st, lab, touched, kind, sup, w, n, cls,
                       last, cur);
    hipLaunchKernelGGL(dg_collect_kernel, dim3(cb), dim3(DNT), 0, st, biglist, nbig, nbig_dev, take, cur, last, cnt,
                       cls, gfirst, out_key, out_row, cap, count, remaining);
  }
  return (int)hipGetLastError();
}

// One-block digest of a graph with ne <= 2048 edges (dg_small_kernel): out
// int64 [2][cap] (cap >= 2 ne; key row pairs sorted, unused key 1 << 62 /
// row -1), out_cnt int [1]; ws >= lzk_dg_small_ws(ne) bytes. No host
// synchronisation.
LZK_EXPORT long lzk_dg_small_ws(int ne) { return (long)2 * (ne > 0 ? ne : 1) * 48 + 256; }
LZK_EXPORT int lzk_dg_small_max_edges() { return SD_MAXE; }
LZK_EXPORT int lzk_dg_small(const int* src, const int* dst, const float* w, int ne, const unsigned char* kind,
                            const unsigned char* sup, const int* shard, long n, int min_size, double min_avg_w,
                            int take, void* ws, long long* out, int cap, int* out_cnt, void* stream) {
  if (ne <= 0 || ne > SD_MAXE || cap < 2 * ne || take < 1 || min_size < 2) return (int)hipErrorInvalidValue;
  const long U = 2L * ne;
  char* p = (char*)ws;
  SdScratch S;
  S.wsum = (double*)p; p += U * 8;
  S.first = (long long*)p; p += U * 8;
  S.ecnt = (int*)p; p += U * 4;
  S.size = (int*)p; p += U * 4;
  S.ccnt = (int*)p; p += U * 4;
  S.cur = (int*)p; p += U * 4;
  S.last = (int*)p; p += U * 4;
  S.taken = (int*)p;
  hipLaunchKernelGGL(dg_small_kernel, dim3(1), dim3(SD_NT), 0, (hipStream_t)stream, src, dst, w, ne, kind, sup, shard,
                     n, min_size, min_avg_w, take, S, out, cap, out_cnt);
  return (int)hipGetLastError();
}
