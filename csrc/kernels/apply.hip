// Native applier of a consolidation batch's segments (consolidate_batch at the
// reference cadence, reference memory_system.py:580-649, :651-933, :951-1010).
//
// The host planner (csrc/runtime/batch_plan.cpp) decides every insert, link,
// eviction and salience change of B conversations up front; the plan is then
// applied to the tenant's HBM columns in segments that end at the
// run_consolidation points (~43 per 128-conversation step). Driving each
// segment from Python cost ~0.45 ms of interpreter time for ~0.1 ms of GPU
// work, so the GPU sat idle half of a step (profiles/r5/consolidation_device_busy).
//
// Here the whole segment loop is ONE call: Python uploads the batch's data in
// one pinned block and passes a small op program; this loop issues each
// segment's fixed kernel chain back to back -- decay (+ deferred prune flags),
// touched-row updates, node inserts (columns + embeddings), super-node parent
// links, edge appends, the segment end (victims ghosted, edges flagged, ONE
// 8-byte-per-victim read of the survivors / prune counts, stable compaction into
// the other buffer set), and at each run_consolidation point the component
// digest (digest.hip dg_small_kernel) and the profile's first shard rows
// (tg_first_rows_kernel) into per-point capture slots. The host bookkeeping
// (ids, counters, store deletes, captures) is replayed by the caller from
// the per-segment records this call returns (engine/native_apply.py).
//
// The op program (int64 words):
//   DECAY   steps                       edge decay + keep flags over the current
//                                       edges, shard-node salience decay over n
//   ROWS    rows_off row0 m vals_off present consts_off kind_v stored_v
//                                       tg_set_rows (offsets: bytes into the block)
//   EMB     x_row m row0                tg_write_emb of rows x[x_row .. +m) of the
//                                       embedding block at rows row0 ..
//   N       n                           the tenant's row count from here on
//   SHARD   code delta                  host shard-node count (first-rows targets)
//   APPEND  vals_off m                  tg_append_edges at the current edge count
//   SEGEND  vrows_off nv seg            victims + deferred prune + compaction
//   POINT   p                           digest + first rows into slot p
#include <algorithm>
#include <cstring>
#include <utility>
#include <vector>

#include "lzk_common.h"

extern "C" {
int lzk_tg_decay(float* w, long ne, float keep, float thr, unsigned char* flag, int* block_cnt, float* sal,
                 const unsigned char* kind, const unsigned char* sup, long nn, int decay_nodes, int steps,
                 void* stream);
int lzk_tg_set_rows(const long* rows, long row0, int m, const double* vals, int present, const double* consts,
                    float* sal, int* acc, double* last, double* ts, int* shard, unsigned char* sup, int* parent,
                    unsigned char* kind, unsigned char* stored, unsigned char* dirty, int kind_v, int stored_v,
                    void* stream);
int lzk_tg_write_emb(const float* x, long ldx, const unsigned char* has, int m, int D, const long* rows, long row0,
                     float* emb32, long ld32, void* emb16, long ld16, void* emb8, long ld8, float* rs8, float* sqn,
                     double* sumsq, float* rs_max, float* dv_max, unsigned char* has_emb, void* stream);
int lzk_tg_append_edges(const double* vals, int m, long ne, int meta_bits, double now, int* src, int* dst, float* w,
                        int* co, double* lu, int* meta, void* stream);
int lzk_tg_seg_end(const long* vrows, int nv, unsigned char* kind, const unsigned char* sup, const int* shard,
                   unsigned char* stored, int unstore, unsigned* rmb, const int* src, const int* dst, const int* meta,
                   long ne, const unsigned char* prev, long nprev, unsigned char* flag, int* bc, int* info,
                   void* stream);
int lzk_tg_compact(const unsigned char* flag, const int* block_off, long ne, const int* src, const int* dst,
                   const float* w, const int* co, const double* lu, const int* meta, int* osrc, int* odst, float* ow,
                   int* oco, double* olu, int* ometa, int* dsrc, int* ddst, int* dmeta, void* stream);
int lzk_dg_small(const int* src, const int* dst, const float* w, int ne, const unsigned char* kind,
                 const unsigned char* sup, const int* shard, long n, int min_size, double min_avg_w, int take,
                 void* ws, long long* out, int cap, int* out_cnt, void* stream);
int lzk_tg_first_rows(const unsigned char* kind, const unsigned char* sup, const int* shard, long n, const int* tc,
                      const int* tt, const int* to, int nt, long* out, void* stream);
int lzk_dg_small_max_edges();
int lzk_uf_union_sel(const int* src, const int* dst, long ne, const float* w, float wthr, const unsigned char* vmark,
                     int n0, int sel, int* parent, void* stream);
int lzk_cc_compress(int* parent, long n, void* stream);
int lzk_dg_stats(const int* src, const int* dst, const float* w, long ne, const int* lab, long n,
                 const unsigned char* kind, const unsigned char* sup, const int* shard, int min_size, double min_avg_w,
                 int take, unsigned char* touched, double* gsum, int* gcnt, int* gsize, int* gccnt, long long* gfirst,
                 unsigned char* cls, int* biglist, int* counters, void* stream);
int lzk_dg_select(const int* lab, long n, const unsigned char* touched, const unsigned char* kind,
                  const unsigned char* sup, unsigned char* cls, const long long* gfirst, const int* biglist, int nbig,
                  const int* nbig_dev, int take, int* cur, int* last, int* cnt, long long* out_key, int* out_row,
                  int cap, int* count, int* remaining, long window, void* stream);
}

namespace {

enum Op : long { OP_END = 0, OP_DECAY, OP_ROWS, OP_EMB, OP_N, OP_SHARD, OP_APPEND, OP_SEGEND, OP_POINT };

// column pointers, in this order (ApplyCols.* of engine/native_apply.py)
struct Cols {
  float* sal;
  int* acc;
  double* last;
  double* ts;
  int* shard;
  unsigned char* sup;
  int* parent;
  unsigned char* kind;
  unsigned char* stored;
  unsigned char* dirty;
  float* emb32;
  void* emb16;
  void* emb8;
  float* rs8;
  float* sqn;
  double* sumsq;
  float* rs_max;
  float* dv_max;
  unsigned char* has_emb;
  unsigned* rmb;
  // optional (nullptr: every segment's DECAY passes over the shard nodes):
  // per-row decay stamps of the lazy node decay (see lzk_apply_segments)
  int* stamp;
};

struct EdgeSet {
  int* src;
  int* dst;
  float* w;
  int* co;
  double* lu;
  int* meta;
};

inline EdgeSet edge_set(void* const* p) {
  return EdgeSet{(int*)p[0], (int*)p[1], (float*)p[2], (int*)p[3], (double*)p[4], (int*)p[5]};
}

__global__ void ap_iota_kernel(int* __restrict__ a, long lo, long hi) {
  const long i = lo + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < hi) a[i] = (int)i;
}

__global__ void ap_fill64_kernel(long long* __restrict__ a, long n, long long v) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = v;
}

inline unsigned nblk(long n, int per = 256) { return (unsigned)((n + per - 1) / per); }

// Lazy node decay. The segments' DECAY ops each pass over every shard node
// (one fp32 salience decay per conversation, tenant.hip decay_sal); nothing
// on the device reads a node's salience between them (the planner wrote the
// absolute saliences of the rows it touches), so the passes collapse into
// per-row stamps -- the conversation count a row's salience is current at --
// and ONE pass at the end that applies the missing steps one by one in the
// same fp32 order (bit-identical). A victim takes its missing steps at its
// segment end, before it stops being a shard node.
constexpr float kSalFloor = 0.2f;  // = tenant.hip SAL_FLOOR
__device__ __forceinline__ float ap_decay_sal(float s, float keep) {
#pragma clang fp contract(off)
  return s > kSalFloor ? kSalFloor + (s - kSalFloor) * keep : kSalFloor;
}

__global__ void ap_stamp_rows_kernel(const long* __restrict__ rows, long row0, int m, const double* __restrict__ vals,
                                     int present, int* __restrict__ stamp, int cum) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  long r;  // the row tg_set_rows_kernel writes
  if (present & (1 << 15)) r = (long)vals[j];
  else r = rows ? rows[j] : row0 + j;
  if (r >= 0) stamp[r] = cum;
}

__global__ void ap_victim_decay_kernel(const long* __restrict__ vrows, int nv, float* __restrict__ sal,
                                       const unsigned char* __restrict__ kind, const unsigned char* __restrict__ sup,
                                       int* __restrict__ stamp, int cum, float keep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nv) return;
  const long r = vrows[i];
  if (r < 0) return;
  if (kind[r] == 1 && !sup[r]) {
    float s = sal[r];
    for (int t = stamp[r]; t < cum; ++t) s = ap_decay_sal(s, keep);
    sal[r] = s;
  }
  stamp[r] = cum;
}

__global__ void ap_lazy_decay_kernel(float* __restrict__ sal, const unsigned char* __restrict__ kind,
                                     const unsigned char* __restrict__ sup, int* __restrict__ stamp, long n, int cum,
                                     float keep) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int st = stamp[i];
    if (st < cum && kind[i] == 1 && !sup[i]) {
      float s = sal[i];
      for (int t = st; t < cum; ++t) s = ap_decay_sal(s, keep);
      sal[i] = s;
    }
    if (st) stamp[i] = 0;  // every stamp is 0 between calls
  }
}

// Incremental-components digest of one run_consolidation point (the
// partitioned batch of TenantGraph.cc_begin: stable prefix [0, ns) labelled
// once per batch into base_lab over the first n0 rows; this point's labels =
// base, rows inserted since as singletons, unions over the volatile suffix
// [ns, ne); then ops.tenant_ops.component_digest: stats, one read of the
// counters, selection, one read of the count, (key, row) pairs sorted on the
// host). cc slots: see lzk_apply_segments.
struct Cc {
  long ns, mode;
  const int* base_lab;
  long n0;
  int* lab;
  const unsigned char* zero_vm;
  unsigned char* touched;
  double* gsum;
  int* gi;
  long long* gfirst;
  unsigned char* cls;
  int* biglist;
  int* counters;
  long long* keys;
  int* rows;
  long sel_cap;
  int* cur;
  int* last;
  int* cnt;
  int* rem;
  long window;
  long n_cap;
};

Cc cc_args(const long* c) {
  Cc a;
  a.ns = c[0];
  a.mode = c[1];
  a.base_lab = (const int*)c[2];
  a.n0 = c[3];
  a.lab = (int*)c[4];
  a.zero_vm = (const unsigned char*)c[5];
  a.touched = (unsigned char*)c[6];
  a.gsum = (double*)c[7];
  a.gi = (int*)c[8];
  a.gfirst = (long long*)c[9];
  a.cls = (unsigned char*)c[10];
  a.biglist = (int*)c[11];
  a.counters = (int*)c[12];
  a.keys = (long long*)c[13];
  a.rows = (int*)c[14];
  a.sel_cap = c[15];
  a.cur = (int*)c[16];
  a.last = (int*)c[17];
  a.cnt = (int*)c[18];
  a.rem = (int*)c[19];
  a.window = c[20];
  a.n_cap = c[21];
  return a;
}

// the (key, row) pairs of the last call's incremental digests, every point
// appended in order (lzk_apply_dig_size / lzk_apply_dig_copy read them)
thread_local std::vector<long long> g_dig;

// Returns 0 / an error; *m = selected (key, row) pairs appended to g_dig
// (sorted by key, then row).
int cc_digest(const Cc& a, const int* src, const int* dst, const float* w, long ne, long n, const unsigned char* kind,
              const unsigned char* sup, const int* shard, int take, long* m_out, hipStream_t st) {
  void* stream = (void*)st;
  *m_out = 0;
  if (n > a.n_cap || a.ns > ne || n < a.n0) return (int)hipErrorInvalidValue;
  // TenantGraph._cc_labels
  if (hipMemcpyAsync(a.lab, a.base_lab, sizeof(int) * a.n0, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return (int)hipGetLastError();
  if (n > a.n0) hipLaunchKernelGGL(ap_iota_kernel, dim3(nblk(n - a.n0)), dim3(256), 0, st, a.lab, a.n0, n);
  int rc = lzk_uf_union_sel(src + a.ns, dst + a.ns, ne - a.ns, nullptr, -__builtin_huge_valf(), a.zero_vm, (int)n, 0,
                            a.lab, stream);
  if (rc) return rc;
  if ((rc = lzk_cc_compress(a.lab, n, stream))) return rc;
  // ops.tenant_ops.component_digest
  if (hipMemsetAsync(a.touched, 0, n, st) != hipSuccess || hipMemsetAsync(a.gsum, 0, 8 * n, st) != hipSuccess ||
      hipMemsetAsync(a.gi, 0, 12 * n, st) != hipSuccess || hipMemsetAsync(a.counters, 0, 16, st) != hipSuccess)
    return (int)hipGetLastError();
  hipLaunchKernelGGL(ap_fill64_kernel, dim3(nblk(n)), dim3(256), 0, st, a.gfirst, n, 1LL << 62);
  if ((rc = lzk_dg_stats(src, dst, w, ne, a.lab, n, kind, sup, shard, 3, 0.3, take, a.touched, a.gsum, a.gi,
                         a.gi + n, a.gi + 2 * n, a.gfirst, a.cls, a.biglist, a.counters, stream)))
    return rc;
  int ctr[4] = {0, 0, 0, 0};
  if (hipMemcpyAsync(ctr, a.counters, sizeof(ctr), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return (int)hipGetLastError();
  const long direct = ctr[0], nbig = ctr[1];
  const long cap = direct + (long)take * nbig;
  if (cap == 0) return 0;
  if (cap > a.sel_cap) return (int)hipErrorInvalidValue;
  if (nbig) {
    if (hipMemsetD32Async((hipDeviceptr_t)a.cur, 0x7FFFFFFF, n, st) != hipSuccess ||
        hipMemsetD32Async((hipDeviceptr_t)a.last, 0xFFFFFFFFu, n, st) != hipSuccess ||
        hipMemsetAsync(a.cnt, 0, 4 * n, st) != hipSuccess)
      return (int)hipGetLastError();
  }
  if (hipMemsetAsync(a.rem, 0, 4, st) != hipSuccess) return (int)hipGetLastError();
  if ((rc = lzk_dg_select(a.lab, n, a.touched, kind, sup, a.cls, a.gfirst, a.biglist, (int)nbig, nullptr, take,
                          nbig ? a.cur : a.rem, nbig ? a.last : a.rem, nbig ? a.cnt : a.rem, a.keys, a.rows,
                          (int)cap, a.counters + 3, a.rem, a.window, stream)))
    return rc;
  // the selected count and (speculatively) the first `spec` pairs in ONE
  // wait; a longer selection reads its remainder after a second one
  int m = 0;
  const long spec = cap < 8192 ? cap : 8192;
  std::vector<long long> k(spec);
  std::vector<int> r(spec);
  if (hipMemcpyAsync(&m, a.counters + 3, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(k.data(), a.keys, 8L * spec, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(r.data(), a.rows, 4L * spec, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return (int)hipGetLastError();
  if (m > cap) return (int)hipErrorInvalidValue;
  if (m == 0) return 0;
  if (m > spec) {
    k.resize(m);
    r.resize(m);
  }
  if (m > spec &&
      (hipMemcpyAsync(k.data() + spec, a.keys + spec, 8L * (m - spec), hipMemcpyDeviceToHost, st) != hipSuccess ||
       hipMemcpyAsync(r.data() + spec, a.rows + spec, 4L * (m - spec), hipMemcpyDeviceToHost, st) != hipSuccess ||
       hipStreamSynchronize(st) != hipSuccess))
    return (int)hipGetLastError();
  std::vector<std::pair<long long, long long>> kr(m);
  for (int i = 0; i < m; ++i) kr[i] = {k[i], (long long)r[i]};
  std::sort(kr.begin(), kr.end());  // (key, row) ascending: the caller's argsort order
  for (int i = 0; i < m; ++i) {
    g_dig.push_back(kr[i].first);
    g_dig.push_back(kr[i].second);
  }
  *m_out = m;
  return 0;
}

}  // namespace

// Returns 0 or a HIP error / hipErrorInvalidValue (bad program). On return:
//   state[0] = final edge count, state[1] = buffer set holding them (0 = A,
//   1 = B), state[2] = dropped edges written, state[3] = ops executed.
//   seg_out[4 s ..] = (pruned by the decay, surviving edges, dropped edges
//   written by this segment, offset of its victim records in vinfo) per
//   segment; vinfo = (kind, sup, shard) x nv per segment, concatenated.
//   point_out[5 p ..] = (edges at the point, digest kind (0 = no edges: an
//   empty digest, 1 = one-block digest in dg_out slot p, 2 = incremental
//   digest), first-rows entries, offset and count of its (key, row) pairs in
//   the incremental digests' output (lzk_apply_dig_copy)) per point.
// ccp: int64 slots (ns, mode, base_lab, n0, lab, zero_vm, touched, gsum, gi,
//   gfirst, cls, biglist, counters, keys, rows, sel_cap, cur, last, cnt, rem,
//   window, n_cap) -- see Cc.
// shard_count (host, int64 [ncodes]) is updated like the host's counters.
LZK_EXPORT int lzk_apply_segments(const long* prog, long nprog, const char* blk, const float* xblk, int D,
                                  void* const* colp, long ld32, long ld16, long ld8, void* const* ebuf_a,
                                  void* const* ebuf_b, long ne0, long cap_e, float thr, float keep, double now,
                                  int meta_bits, int unstore, unsigned char* flag_a, unsigned char* flag_b, int* bc,
                                  int* info, long info_cap, int* dsrc, int* ddst, int* dmeta, long drop_cap,
                                  long long* dg_out, int dg_cap, void* dg_ws, int* dg_cnt, long* fr_out, int fr_k,
                                  long* shard_count, int ncodes, long* seg_out, int* vinfo, long vinfo_cap,
                                  long* point_out, long* state, const long* ccp, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const Cols& C = *reinterpret_cast<const Cols*>(colp);
  // ccp (optional): a partitioned batch (TenantGraph.cc_begin) -- the stable
  // prefix [0, ns) of buffer set A never changes: flags, survivors and the
  // compaction cover the suffix only (compacted into set B, copied back
  // behind the prefix), and a point's digest is the incremental-components
  // one (mode 1) instead of the one-block digest
  Cc cc{};
  if (ccp) cc = cc_args(ccp);
  const long ns = ccp ? cc.ns : 0;
  long dig_used = 0;
  g_dig.clear();
  EdgeSet E[2] = {edge_set(ebuf_a), edge_set(ebuf_b)};
  int cur = 0;
  long ne = ne0, n = 0, drop_total = 0, vinfo_used = 0;
  long cum = 0;  // conversations decayed so far (lazy node decay)
  // the deferred prune of the open segment: keep flags over its first nprev edges
  unsigned char* prev = nullptr;
  long nprev = 0;
  const int dg_max = lzk_dg_small_max_edges();
  long pc = 0, ops = 0;
  int rc = 0;
#define LZK_RC(x)                  \
  do {                             \
    rc = (x);                      \
    if (rc != 0) goto done;        \
  } while (0)
  while (pc < nprog) {
    const long op = prog[pc];
    ++ops;
    if (op == OP_END) break;
    if (op == OP_DECAY) {
      const int steps = (int)prog[pc + 1];
      pc += 2;
      // flag_a: the decay's keep flags (flag_b: the segment end's); thr = -inf:
      // nothing is pruned, no flags (TenantGraph.segment_begin)
      prev = (ne > 0 && thr > -__builtin_huge_valf()) ? flag_a : nullptr;
      nprev = ne;
      // lazy node decay (C.stamp): the nodes' steps are only counted here
      LZK_RC(lzk_tg_decay(E[cur].w, ne, keep, thr, prev, prev ? bc : nullptr, C.sal, C.kind, C.sup, n,
                          (n && !C.stamp) ? 1 : 0, steps, stream));
      cum += steps;
      // the decay's block counts are only needed by a compaction of these
      // flags alone, which never happens here (the segment end re-flags)
    } else if (op == OP_ROWS) {
      const long rows_off = prog[pc + 1], row0 = prog[pc + 2];
      const int m = (int)prog[pc + 3];
      const long vals_off = prog[pc + 4];
      const int present = (int)prog[pc + 5];
      const long consts_off = prog[pc + 6];
      const int kind_v = (int)prog[pc + 7], stored_v = (int)prog[pc + 8];
      pc += 9;
      LZK_RC(lzk_tg_set_rows(rows_off >= 0 ? (const long*)(blk + rows_off) : nullptr, row0, m,
                             (const double*)(blk + vals_off), present, (const double*)(blk + consts_off), C.sal,
                             C.acc, C.last, C.ts, C.shard, C.sup, C.parent, C.kind, C.stored, C.dirty, kind_v,
                             stored_v, stream));
      // a written salience is current as of now
      if (C.stamp && m > 0 && !(present & (1 << 8)))
        hipLaunchKernelGGL(ap_stamp_rows_kernel, dim3(nblk(m)), dim3(256), 0, st,
                           rows_off >= 0 ? (const long*)(blk + rows_off) : nullptr, row0, m,
                           (const double*)(blk + vals_off), present, C.stamp, (int)cum);
    } else if (op == OP_EMB) {
      const long xr = prog[pc + 1];
      const int m = (int)prog[pc + 2];
      const long row0 = prog[pc + 3];
      pc += 4;
      LZK_RC(lzk_tg_write_emb(xblk + xr * D, D, nullptr, m, D, nullptr, row0, C.emb32, ld32, C.emb16, ld16, C.emb8,
                              ld8, C.rs8, C.sqn, C.sumsq, C.rs_max, C.dv_max, C.has_emb, stream));
    } else if (op == OP_N) {
      n = prog[pc + 1];
      pc += 2;
    } else if (op == OP_SHARD) {
      const long code = prog[pc + 1], delta = prog[pc + 2];
      pc += 3;
      if (code < 0 || code >= ncodes) { rc = (int)hipErrorInvalidValue; goto done; }
      shard_count[code] += delta;
    } else if (op == OP_APPEND) {
      const long vals_off = prog[pc + 1];
      const int m = (int)prog[pc + 2];
      pc += 3;
      if (ne + m > cap_e) { rc = (int)hipErrorInvalidValue; goto done; }
      const EdgeSet& e = E[cur];
      LZK_RC(lzk_tg_append_edges((const double*)(blk + vals_off), m, ne, meta_bits, now, e.src, e.dst, e.w, e.co, e.lu,
                                 e.meta, stream));
      ne += m;
    } else if (op == OP_SEGEND) {
      const long vrows_off = prog[pc + 1];
      const int nv = (int)prog[pc + 2];
      const long s = prog[pc + 3];
      pc += 4;
      long* so = seg_out + 4 * s;
      so[0] = 0;
      so[1] = ne;
      so[2] = 0;
      so[3] = vinfo_used;
      if (nv == 0 && prev == nullptr) continue;  // nothing to flag, nobody removed
      if (3L * nv + 2 > info_cap || vinfo_used + 3L * nv > vinfo_cap || ne < ns || (prev && nprev < ns)) {
        rc = (int)hipErrorInvalidValue;
        goto done;
      }
      if (C.stamp && nv)  // the victims' missing decay steps, while they are still shard nodes
        hipLaunchKernelGGL(ap_victim_decay_kernel, dim3(nblk(nv)), dim3(256), 0, st, (const long*)(blk + vrows_off),
                           nv, C.sal, C.kind, C.sup, C.stamp, (int)cum, keep);
      const EdgeSet& e = E[cur];
      const long nes = ne - ns;  // the suffix the segment end flags
      LZK_RC(lzk_tg_seg_end(nv ? (const long*)(blk + vrows_off) : nullptr, nv, C.kind, C.sup, C.shard, C.stored,
                            unstore, C.rmb, e.src + ns, e.dst + ns, e.meta + ns, nes, prev ? prev + ns : nullptr,
                            prev ? nprev - ns : 0, nes ? flag_b : nullptr, nes ? bc : nullptr, info, stream));
      // the one host read of the segment: victims' (kind, sup, shard),
      // survivors, pruned
      if (nv && hipMemcpyAsync(vinfo + vinfo_used, info, sizeof(int) * (3L * nv), hipMemcpyDeviceToHost, st) !=
                    hipSuccess) {
        rc = (int)hipGetLastError();
        goto done;
      }
      int tail[2] = {0, 0};
      if (hipMemcpyAsync(tail, info + 3L * nv, sizeof(tail), hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess) {
        rc = (int)hipGetLastError();
        goto done;
      }
      const long n_out = nes ? tail[0] : 0;  // survivors of the suffix
      so[0] = prev ? tail[1] : 0;
      // the victims leave the host counters like TenantGraph.segment_end
      for (int i = 0; i < nv; ++i) {
        const int k = vinfo[vinfo_used + i], sp = vinfo[vinfo_used + nv + i], sh = vinfo[vinfo_used + 2 * nv + i];
        if (k == 1 && !sp && sh >= 0 && sh < ncodes) shard_count[sh] -= 1;
      }
      vinfo_used += 3L * nv;
      if (nes && n_out != nes) {
        const long nd = nes - n_out;
        const bool track = dsrc != nullptr;
        if (track && drop_total + nd > drop_cap) { rc = (int)hipErrorInvalidValue; goto done; }
        const EdgeSet& o = E[cur ^ 1];
        LZK_RC(lzk_tg_compact(flag_b, bc, nes, e.src + ns, e.dst + ns, e.w + ns, e.co + ns, e.lu + ns, e.meta + ns,
                              o.src, o.dst, o.w, o.co, o.lu, o.meta, track ? dsrc + drop_total : nullptr,
                              track ? ddst + drop_total : nullptr, track ? dmeta + drop_total : nullptr, stream));
        if (track) {
          so[2] = nd;
          drop_total += nd;
        }
        if (ns) {  // survivors back behind the untouched prefix, in the same buffers
          if (n_out &&
              (hipMemcpyAsync(e.src + ns, o.src, 4 * n_out, hipMemcpyDeviceToDevice, st) != hipSuccess ||
               hipMemcpyAsync(e.dst + ns, o.dst, 4 * n_out, hipMemcpyDeviceToDevice, st) != hipSuccess ||
               hipMemcpyAsync(e.w + ns, o.w, 4 * n_out, hipMemcpyDeviceToDevice, st) != hipSuccess ||
               hipMemcpyAsync(e.co + ns, o.co, 4 * n_out, hipMemcpyDeviceToDevice, st) != hipSuccess ||
               hipMemcpyAsync(e.lu + ns, o.lu, 8 * n_out, hipMemcpyDeviceToDevice, st) != hipSuccess ||
               hipMemcpyAsync(e.meta + ns, o.meta, 4 * n_out, hipMemcpyDeviceToDevice, st) != hipSuccess)) {
            rc = (int)hipGetLastError();
            goto done;
          }
        } else {
          cur ^= 1;
        }
        ne = ns + n_out;
      }
      so[1] = ne;
      prev = nullptr;
      nprev = 0;
    } else if (op == OP_POINT) {
      const long p = prog[pc + 1];
      pc += 2;
      long* po = point_out + 5 * p;
      po[0] = ne;
      po[1] = 0;
      po[2] = 0;
      po[3] = dig_used;
      po[4] = 0;
      if (ne > 0 && ccp && cc.mode == 1) {  // TenantGraph.component_digest with the batch's incremental labels
        long m = 0;
        const EdgeSet& e = E[cur];
        LZK_RC(cc_digest(cc, e.src, e.dst, e.w, ne, n, C.kind, C.sup, C.shard, fr_k, &m, st));
        po[1] = 2;
        po[4] = m;
        dig_used += m;
      } else if (ne > 0) {  // TenantGraph.digest_capture on the one-block digest (ne <= dg_max: the caller's bound)
        if (ne > dg_max || 2L * ne > dg_cap) { rc = (int)hipErrorInvalidValue; goto done; }
        const EdgeSet& e = E[cur];
        LZK_RC(lzk_dg_small(e.src, e.dst, e.w, (int)ne, C.kind, C.sup, C.shard, n, 3, 0.3, fr_k, dg_ws,
                            dg_out + p * 2L * dg_cap, dg_cap, dg_cnt, stream));
        po[1] = 1;
      }
      // TenantGraph._first_rows_dev: per-shard targets from the host counts
      int tc[64], tt[64], to[64], nt = 0, need = fr_k, off = 0;
      for (int c = 0; c < ncodes && need > 0; ++c) {
        const long cnt = shard_count[c];
        if (cnt <= 0) continue;
        if (nt == 64) { rc = (int)hipErrorInvalidValue; goto done; }
        const int t = (int)(cnt < need ? cnt : need);
        tc[nt] = c;
        tt[nt] = t;
        to[nt] = off;
        ++nt;
        off += t;
        need -= t;
      }
      if (nt) LZK_RC(lzk_tg_first_rows(C.kind, C.sup, C.shard, n, tc, tt, to, nt, fr_out + p * (long)fr_k, stream));
      po[2] = off;
    } else {
      rc = (int)hipErrorInvalidValue;
      goto done;
    }
  }
  // the lazy node decay's one pass: every shard node's missing steps
  if (rc == 0 && C.stamp && n > 0) {
    const long g = (long)nblk(n) < 4096 ? (long)nblk(n) : 4096;
    hipLaunchKernelGGL(ap_lazy_decay_kernel, dim3((unsigned)g), dim3(256), 0, st, C.sal, C.kind, C.sup, C.stamp, n,
                       (int)cum, keep);
  }
done:
#undef LZK_RC
  state[0] = ne;
  state[1] = cur;
  state[2] = drop_total;
  state[3] = ops;
  if (rc == 0) rc = (int)hipGetLastError();
  return rc;
}

// The (key, row) pairs of the last lzk_apply_segments call's incremental
// digests (this thread), 2 int64 per pair.
LZK_EXPORT long lzk_apply_dig_size() { return (long)g_dig.size() / 2; }
LZK_EXPORT void lzk_apply_dig_copy(long long* out) {
  if (!g_dig.empty()) std::memcpy(out, g_dig.data(), g_dig.size() * sizeof(long long));
}
