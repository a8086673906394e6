"""TenantGraph: one tenant's memory graph as structure-of-arrays in HBM.

This is the engine under :class:`~lazzaro_amd.core.memory_system.MemorySystem`.
The reference keeps a tenant's graph as Python ``Node``/``Edge`` objects in
per-topic dicts (``core/memory_shard.py:30-88``, ``core/buffer_graph.py``) and
runs every maintenance step as a Python loop over them. Here the graph is a
set of device columns and every step is a kernel or a batched tensor op:

=====================  ==========================================  =====================
reference step          reference code                              here
=====================  ==========================================  =====================
dedupe (top-1, >0.95)   memory_system.py:719-742                    fused MFMA top-k scan
link within shard       memory_system.py:797-836                    label-filtered list of
link to existing        memory_system.py:838-891                    the same dual scan
decay + prune           memory_shard.py:64-84, :624-630, :991       ``tg_decay_kernel``
evict (importance)      memory_system.py:535-578                    ``tg_importance_kernel``
                                                                    + stable select +
                                                                    ``tg_flag_remove``
components              buffer_graph.py:99-120                      ``cc_hook/compress``
neighbour boost         memory_system.py:242-260                    ``tg_boost_kernel``
retrieval touch         buffer_graph.py:79-85                       ``tg_touch_kernel``
super-node centroid     memory_system.py:893-933                    segmented mean
store vector search     vector_store.py:132-140                     fused MFMA top-k +
                                                                    fp32 re-rank
=====================  ==========================================  =====================

Node columns (row-indexed; rows are never reused while referenced):

* ``emb32`` fp32 [cap, D]: exact vectors (the store's precision, reference
  ``vector_store.py:37``); ``emb16`` bf16 [cap, Dp] on the GPU: the operand of
  the MFMA scans (Dp = D rounded up to 64); ``sqn`` fp32 |x|^2.
* ``sal f32, acc i32, last f64, ts f64, shard i32, kind u8, sup u8,
  has_emb u8, parent i32, stored u8, dirty u8``. ``kind``: 0 free, 1 node,
  2 ghost -- an id that is not (or no longer) a node but is still an edge
  endpoint or a store row (the reference keeps dangling edges of removed
  nodes in other shards, and the store may hold rows the graph dropped).
* host lists: ``ids``, ``content``, ``types``; ``children`` (super rows).

Edge columns: ``src/dst i32, w f32, co i32, lu f64, meta i32`` with ``meta =
shard | type << 24 | stored << 29 | dirty << 30``: the shard that stores the edge matters,
because the reference's ``get_neighbors`` only sees edges of the node's own
shard (``buffer_graph.py:72-77``); that visibility drives the neighbour boost.

Decisions are taken in float64 from the fp32 columns (the reference computes
cosine in float64, ``memory_system.py:197-203``); the bf16 MFMA scans only
nominate candidates, which are re-ranked exactly.

Deliberate differences (documented in docs/INVENTORY.md):
* connected components treat an edge as connecting both endpoints whichever
  shard stores it (the reference's recursive DFS sees a cross-shard edge from
  one side only, which makes its components depend on the visit order);
* ties in similarity / importance break by row (insertion) order.
"""
from __future__ import annotations

import math
import os
import threading
import time
from contextlib import contextmanager
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import tenant_ops as T

FREE, NODE, GHOST = 0, 1, 2
NEG_INF = float("-inf")
SHARD_MASK = 0xFFFFFF
TYPE_SHIFT = 24
TYPE_MASK = 0x1F
ESTORED = 1 << 29  # the edge is in the persistent store (its removal must be committed)
EDIRTY = 1 << 30  # changed since the last commit
MAX_ETYPES = TYPE_MASK + 1

# below this many query x row products the exact float64 GEMM is used directly
KERNEL_MIN_WORK = 1 << 22
CAND_SLOTS = 16  # candidates per query from the bf16 scan before the exact re-rank
# fp8 candidate scan of the store search: large batches over large tenants
# (the candidate kernel's regime), margin in standard deviations of the fp8
# score error (see TenantGraph._fp8_candidates)
LOWP_MIN_Q, LOWP_MIN_ROWS, LOWP_MARGIN_Z = 128, 1 << 20, 8.0
# Two int8 margins (TenantGraph._i8_query): a STATISTICAL one (LOWP_MARGIN_Z
# standard deviations of the row-rounding term plus the exact worst case of
# the query term) and a WORST-CASE one (|<x, eta>| <= |x| |eta|, |<delta, q>|
# <= s_max / 2 |q|_1, + fp32 accumulation). ops/search.py flat_topk_i8 /
# flat_topk_dual_i8 set the scan threshold from the first, the re-score cut
# and a per-query certificate from the second (a query whose k-th re-scored
# score does not clear threshold + bound is recomputed by the exact scan).
# LOWP_EXACT picks which margin thresholds a scan:
#   "auto" (default): the worst-case one -- results equal the bf16 search for
#       ANY data -- for the interactive / narrow store searches (< LOWP_MIN_Q
#       queries: HBM-bound, the longer lists cost little) and for
#       consolidation's dual scan (dedupe / link decisions); the statistical
#       one for wide store-search batches, where the worst case costs ~30 %
#       of the headline QPS (profiles/r5/README.md). Statistical means: on
#       random or clustered unit rows the lists equal the bf16 scan's
#       (recall tests, bench recall 1.0), but an adversarial row set could
#       move a true top-k row below the threshold -- the certificate then
#       checks against the same statistical margin, so such a miss is not
#       detected.
#   "1": the worst-case margin everywhere; "0": the statistical one everywhere.
LOWP_EXACT = os.environ.get("LZK_LOWP_EXACT", "auto")
# batches below LOWP_MIN_Q (the interactive turn) take the HBM-bound narrow
# int8 scan (scan8.hip scan8_narrow_kernel); LOWP_NARROW = False: the bf16 lane kernel
LOWP_NARROW = True
# consolidation's dual candidate scan on the int8 copy (flat_topk_dual_i8).
# LZK_DUAL_LOWP=1 always, 0 never, default "auto": int8 while its lists stay
# short, bf16 for the next DUAL_BACKOFF calls of a tenant whose last int8 call
# overflowed lists or averaged more than a quarter of the list capacity.
# Measured: random fact vectors (bench/bench_consolidate.py) 1881 -> 2075
# conversations/s with int8; the clustered-topic row-sharded run lost with it
# (437.9 -> 391.4/s, profiles/r4/sharded_clustered_dual_lowp_*.json): facts
# near a topic centre clear their (link-floor) threshold on thousands of rows,
# so the lists fill up and the re-score / exact fallback outweigh the scan.
_DL = os.environ.get("LZK_DUAL_LOWP", "auto")
DUAL_LOWP = _DL != "0"
DUAL_LOWP_AUTO = _DL not in ("0", "1")
DUAL_OVF_MAX = 0.02
DUAL_BACKOFF = 16
# Lean HBM layout (LZK_LEAN_HBM=1 / TenantGraph.LEAN_HBM): a tenant with the
# int8 scan copy and at least LOWP_MIN_ROWS rows of capacity keeps NO bf16
# copy -- fp32 (the store's precision) + int8 + scale, ~5 bytes per dimension
# instead of ~7: the int8 scans' threshold sample converts its 1/64 of the
# rows on the fly, their re-score reads the fp32 rows, consolidation's scans
# take the int8 dual path, and a k-means pass converts the rows for its
# duration.
LEAN_HBM = os.environ.get("LZK_LEAN_HBM", "0") == "1"
# inserts of at most this many rows write their embedding columns in one launch
WRITE_EMB_MAX_ROWS = 8192
# node columns of an insert in one launch (tenant.hip tg_set_rows_kernel); 0 = per-column writes
SET_ROWS_KERNEL = True
# the int8 search's query quantisation + margin in one launch (I8_QUERY_KERNEL = False: torch ops)
I8_QUERY_KERNEL = True
# wide batches too (I8_QUERY_WIDE = False: the torch formulation of ~25 launches
# for batches >= I8_QUERY_WIDE_MIN). Round 5 once measured the pipelined headline
# at 54k QPS with the kernel; interleaved round-6 runs on one box: 82.5k / 82.7k
# with it vs 82.1k / 79.2k without, store search 8.08 vs 8.40 ms
# (profiles/r6/serving/i8_query_wide_ab/; tests/kernels/test_query_prep_gpu.py, nq = 1024)
I8_QUERY_WIDE = os.environ.get("LZK_I8_QUERY_WIDE", "1") == "1"
I8_QUERY_WIDE_MIN = 128
# consolidate_batch segment ends through tenant.hip lzk_tg_seg_end (SEG_END_KERNEL = False: the torch formulation)
SEG_END_KERNEL = True
# store-search re-rank as one kernel (tenant.hip store_rerank_kernel); 0 = torch chain
RERANK_KERNEL = True
# consolidation's float64 candidate re-rank as one kernel (cos_rerank64_kernel); 0 = torch chain
RERANK64_KERNEL = True
# cos_topk(min_score=): kernel threshold slack below min_score. Unit rows and
# queries rounded to bf16 (relative 2^-9 each) move a cosine by at most
# 2^-8 * sum|q_i x_i| <= 2^-8 ~ 0.0039, plus fp32 accumulation order.
COS_FLOOR_SLACK = 0.01


def _str_column(items=None):
    """A native StrColumn (list-like, not GC-tracked); a list where the host
    runtime is not built."""
    try:
        from .._lib._lzrt import StrColumn  # type: ignore
    except ImportError:  # pragma: no cover - the runtime ships with the package build
        return list(items or [])
    return StrColumn(items)


def _pad64(d: int) -> int:
    return (d + 63) // 64 * 64


def _seg_sum_count(keys: torch.Tensor, vals: torch.Tensor, n: int):
    """(sum of ``vals`` per key, count per key) for keys in [0, n) by sort +
    prefix sum. A float64 ``index_add_`` into few keys (one giant component
    holding millions of edges) is a contended fp64 atomic on one address --
    minutes on the GPU; this is a sort and a scan, and deterministic."""
    dev = keys.device
    sums = torch.zeros(n, dtype=torch.float64, device=dev)
    cnts = torch.zeros(n, dtype=torch.int64, device=dev)
    if keys.numel() == 0:
        return sums, cnts
    o = torch.argsort(keys, stable=True)
    k = keys[o]
    c = torch.cumsum(vals[o].double(), 0)
    last = torch.ones_like(k, dtype=torch.bool)
    last[:-1] = k[1:] != k[:-1]
    idx = torch.nonzero(last).flatten()
    ends = c[idx]
    sums[k[idx]] = ends - torch.cat([ends.new_zeros(1), ends[:-1]])
    cnts[k[idx]] = idx - torch.cat([idx.new_full((1,), -1), idx[:-1]])
    return sums, cnts


def _seg_min(keys: torch.Tensor, vals: torch.Tensor, n: int, fill: int) -> torch.Tensor:
    """Minimum of int64 ``vals`` per key in [0, n) (``fill`` where a key has
    none) by two stable sorts -- no contended atomic min on a huge key."""
    out = torch.full((n,), fill, dtype=torch.long, device=keys.device)
    if keys.numel() == 0:
        return out
    o = torch.argsort(vals, stable=True)
    o = o[torch.argsort(keys[o], stable=True)]
    k = keys[o]
    head = torch.ones_like(k, dtype=torch.bool)
    head[1:] = k[1:] != k[:-1]
    out[k[head]] = vals[o][head]
    return out


_SIDE_STREAMS: Dict[torch.device, "torch.cuda.Stream"] = {}


def _side_stream(dev: torch.device):
    """One side HIP stream per device, shared by every tenant graph on it: a
    rank serving 10^4 tenants must not create 10^4 streams (the hardware has
    a few queues), and tenants' side work needs no mutual concurrency."""
    st = _SIDE_STREAMS.get(dev)
    if st is None:
        st = torch.cuda.Stream(device=dev, priority=SIDE_STREAM_PRIORITY)
        _SIDE_STREAMS[dev] = st
    return st


# priority of the graphs' side stream (0 normal, -1 high, as torch counts)
SIDE_STREAM_PRIORITY = 0


def _host_ints(v, m: int, default: int) -> Optional[np.ndarray]:
    """int64 [m] host values of a per-row argument (scalar, sequence,
    ndarray or CPU tensor); None for a device tensor."""
    if v is None:
        return np.full(m, default, np.int64)
    if torch.is_tensor(v):
        if v.is_cuda:
            return None
        v = v.numpy()
    if isinstance(v, (int, float, bool, np.number)):
        return np.full(m, int(v), np.int64)
    a = np.asarray(v).reshape(-1).astype(np.int64)
    return np.broadcast_to(a, (m,)) if a.size == 1 else a


class Capture:
    """A result of device work read on the host later: the device tensor is
    copied into pinned memory on the graph's stream right away (no host
    wait), and :meth:`get` waits for that copy only when the value is needed
    -- consolidate_batch keeps its segment loop free of host
    synchronisations and reads every run_consolidation digest at the end of
    the batch. ``host``: an already-known host value."""

    __slots__ = ("_h", "_ev", "_fn", "_val")

    def __init__(self, dev_t: Optional[torch.Tensor] = None, fn=None, host=None):
        self._fn, self._val, self._h, self._ev = fn, host, None, None
        if dev_t is not None:
            self._h = torch.empty(tuple(dev_t.shape), dtype=dev_t.dtype, pin_memory=True)
            self._h.copy_(dev_t, non_blocking=True)
            self._ev = torch.cuda.Event()
            self._ev.record()

    def get(self):
        if self._h is not None:
            self._ev.synchronize()
            a = self._h.numpy()
            self._val = self._fn(a) if self._fn is not None else a
            self._h = self._ev = None
        return self._val


_CL_STREAMS: Dict = {}


def _cluster_stream(dev):
    """One side stream per device for background k-means passes."""
    st = _CL_STREAMS.get(dev)
    if st is None:
        st = _CL_STREAMS[dev] = torch.cuda.Stream(dev)
    return st


class _BackgroundJob:
    """``fn()`` on a worker thread; ``result()`` joins it and re-raises."""

    def __init__(self, fn):
        import threading

        self._out = self._err = None

        def run():
            try:
                self._out = fn()
            except BaseException as e:  # noqa: BLE001 -- re-raised by result()
                self._err = e

        self._t = threading.Thread(target=run, name="lzk-cluster", daemon=False)
        self._t.start()

    def result(self):
        self._t.join()
        if self._err is not None:
            raise self._err
        return self._out


class TenantGraph:
    NODE_COLS = (("sal", torch.float32, 0.0), ("acc", torch.int32, 0), ("last", torch.float64, 0.0),
                 ("ts", torch.float64, 0.0), ("shard", torch.int32, -1), ("kind", torch.uint8, FREE),
                 ("sup", torch.uint8, 0), ("has_emb", torch.uint8, 0), ("parent", torch.int32, -1),
                 ("stored", torch.uint8, 0), ("dirty", torch.uint8, 0))

    def __init__(self, device=None, dim: Optional[int] = None, capacity: int = 256):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.on_gpu = self.device.type == "cuda"
        self.dim: Optional[int] = None
        self.Dp = 0
        self.n = 0
        self.cap = 0
        self._init_cap = capacity
        # per-row host strings in native arrays the cyclic collector never
        # traverses (csrc/runtime/strcol.cpp): a 10M-row tenant's lists made
        # the collector's full passes stall serving loops for ms at a time;
        # row_of (str -> int) is an untracked dict already (atomic keys/values)
        self.ids = _str_column()
        self.content = _str_column()
        self.types = _str_column()
        self.row_of: Dict[str, int] = {}
        self.children: Dict[int, List[str]] = {}
        self.odd_emb: Dict[int, list] = {}
        self.shard_names: List[str] = []
        self.shard_code: Dict[str, int] = {}
        self.shard_live: List[bool] = []
        self.shard_count: List[int] = []  # live non-super nodes per shard
        self.n_super = 0
        self.etype_names: List[str] = []
        self.etype_code: Dict[str, int] = {}
        self._max_norm_dev = 0.0  # max | |x| - 1 | over embedded rows (see max_norm_dev)
        self.decay_log = 0.0  # sum of log(1 - rate) over every decay applied
        self.version = 0  # bumps on any mutation (views / caches)
        self.edge_version = 0
        self._hier = None  # the k-means hierarchy (cluster_pass); read through .hier
        self._hier_job = None  # a background cluster_pass in flight (cluster_join)
        self._hier_lock = threading.Lock()  # one joiner publishes the job's hierarchy
        self._csr = None
        self._csr_version = -1
        self._boost_state = T.BoostState()
        self._bias_cache: Dict[str, Tuple[int, torch.Tensor]] = {}
        self._store_version = 0
        self._mirror: Dict[str, Tuple[int, np.ndarray]] = {}
        self.deleted_ids: Dict[str, None] = {}  # node ids to delete from the store at the next commit
        self._deleted_edges: Dict[Tuple[str, str], None] = {}
        # removed edges still on the device, (src, dst, meta) -- resolved to
        # ids when deleted_edges is read (rows never change ids), so removals
        # inside a consolidation batch cost no host synchronisation
        self._drop_pending: List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = []
        self.last_add_rows: Sequence[int] = range(0)
        self._norm_dev_pending: List[torch.Tensor] = []
        self.track = True
        self.stream = _side_stream(self.device) if self.on_gpu else None
        self.on_change = None  # called after every mutation (_bump)
        self.ann_cfg: Optional[Dict] = None  # store index="ivfpq": IVF-PQ for large tenants (HBMStore.attach)
        self._ann = None
        self._ann_covered = 0
        self._ann_stale = False
        self.lock = threading.RLock()
        z = lambda dt: torch.zeros(0, dtype=dt, device=self.device)  # noqa: E731
        self.e = {"src": z(torch.int32), "dst": z(torch.int32), "w": z(torch.float32), "co": z(torch.int32),
                  "lu": z(torch.float64), "meta": z(torch.int32)}
        # edge columns with room to grow: column -> (buffer, length of the view
        # self.e holds); an append writes in place only while self.e[k] is
        # still exactly that view (see _edge_append)
        self._ebuf: Dict[str, Tuple[torch.Tensor, int]] = {}
        self.emb32 = self.emb16 = self.emb8 = self.rs8 = self.sqn = None
        self._rs8_max = None  # device scalar: max per-row int8 scale ever written (error model)
        self.sumsq = None  # per-dimension sum of x_i^2 over inserted rows (fp8 error model)
        self.n_sumsq = 0
        for name, dt, _ in self.NODE_COLS:
            setattr(self, name, z(dt))
        if dim:
            self._set_dim(dim)

    # ------------------------------------------------------------------ streams
    @contextmanager
    def on_stream(self):
        """Run device work on the graph's own HIP stream, ordered after the
        caller's stream and before anything the caller does next."""
        if not self.on_gpu:
            yield
            return
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream == self.stream.cuda_stream:
            yield
            return
        self.stream.wait_stream(cur)
        try:
            with torch.cuda.stream(self.stream):
                yield
        finally:
            cur.wait_stream(self.stream)

    # ------------------------------------------------------------------ storage
    def _set_dim(self, d: int) -> None:
        self.dim = int(d)
        self.Dp = _pad64(self.dim) if self.on_gpu else self.dim
        self._alloc(max(self.cap, self._init_cap))

    def _alloc(self, cap: int) -> None:
        """(Re)allocate every column at ``cap`` rows, keeping rows [0, n).
        Columns move ONE AT A TIME, largest first, each old tensor released
        before the next new one is allocated: the peak is the old footprint
        plus one new column (the caching allocator hands the released block
        to the next, smaller column), not twice the tenant -- at 10M x 768
        rows the difference is ~50 GB of HBM."""
        dev, n = self.device, self.n
        keep = self.cap and n

        def move(name, shape, dt, fill=0):
            old = getattr(self, name, None)
            if fill == 0:
                t = torch.zeros(shape, dtype=dt, device=dev)
            else:
                t = torch.full(shape, fill, dtype=dt, device=dev)
            if keep and old is not None and old.dtype == dt and old.shape[1:] == tuple(shape[1:]):
                t[:n] = old[:n]
            setattr(self, name, t)
            del old

        if self.dim is not None:
            lowp = self._lowp_mode()
            fresh = self.emb32 is None or self.emb32.shape[1] != self.dim
            if fresh:  # first allocation or a width change: nothing to keep
                self.emb32 = self.emb16 = self.emb8 = self.rs8 = self.sqn = None
            move("emb32", (cap, self.dim), torch.float32)
            if self.on_gpu and not (lowp == "i8" and self._lean(cap)):
                move("emb16", (cap, self.Dp), torch.bfloat16)
            else:
                self.emb16 = None  # (lean: released before the int8 column grows)
            if lowp:
                if self.emb8 is not None and self.emb8.dtype != (torch.int8 if lowp == "i8" else torch.uint8):
                    self.emb8 = None
                move("emb8", (cap, self.Dp), torch.int8 if lowp == "i8" else torch.uint8)
            else:
                self.emb8 = None
            move("sqn", (cap,), torch.float32)
            if lowp == "i8":
                move("rs8", (cap,), torch.float32)
            else:
                self.rs8 = None
            rs8 = self.rs8
            if rs8 is not None and self._rs8_max is None:
                self._rs8_max = torch.zeros((), dtype=torch.float32, device=dev)
            if self.sumsq is None or self.sumsq.numel() != self.dim:
                self.sumsq = torch.zeros(self.dim, dtype=torch.float64, device=dev)
        for name, dt, fill in self.NODE_COLS:
            move(name, (cap,), dt, fill)
        self.cap = cap
        self._alloc_gen = getattr(self, "_alloc_gen", 0) + 1

    @classmethod
    def hbm_bytes_per_row(cls, dim: int, lowp: str = "i8", lean: bool = False) -> int:
        """HBM bytes one row of a GPU tenant holds (:meth:`_alloc`'s
        columns): fp32 vector, bf16 scan copy (not in the lean layout), the
        low-precision copy + row scale, |x|^2 and the node columns."""
        dp = _pad64(int(dim))
        b = 4 * int(dim) + (0 if lean else 2 * dp) + 4
        if lowp:
            b += dp + (4 if lowp == "i8" else 0)
        return b + sum(torch.empty((), dtype=dt).element_size() for _, dt, _ in cls.NODE_COLS)

    EDGE_BYTES = 4 + 4 + 4 + 4 + 8 + 4  # src, dst, w, co, lu, meta

    def _dev_rows(self, rows: Sequence[int]) -> torch.Tensor:
        """A short host row list as an int64 device tensor (pinned, async on a
        GPU: no host-blocking pageable copy)."""
        t = torch.as_tensor(rows, dtype=torch.long)
        if self.on_gpu:
            return t.pin_memory().to(self.device, non_blocking=True)
        return t

    def column_ptrs(self) -> Tuple[int, ...]:
        """Base addresses (emb32, sal, acc, kind, sup, shard) of the current
        column allocations, recomputed only after a re-allocation -- for
        pointer tables that index many tenants (parallel/routing.py)."""
        c = getattr(self, "_ptrs", None)
        gen = getattr(self, "_alloc_gen", 0)
        if c is None or c[0] != gen:
            c = self._ptrs = (gen, (self.emb32.data_ptr() if self.emb32 is not None else 0, self.sal.data_ptr(),
                                    self.acc.data_ptr(), self.kind.data_ptr(), self.sup.data_ptr(),
                                    self.shard.data_ptr()))
        return c[1]

    # rows of the mini-batch k-means refinement steps of cluster_pass
    CLUSTER_SAMPLE = 1 << 20
    # component_digest on the GPU: digest.hip keyed reductions (False) or the
    # sort + segmented-scan formulation the CPU runs (True; tests compare them)
    _digest_sorted = False
    _rmb = None  # persistent all-zero removal bitmap of the fused segment end
    _dv_acc = None  # device running max of | |x| - 1 | over small inserts
    _dv_acc_pending = False  # _dv_acc is in _norm_dev_pending
    SAMPLE_TWO_LEVEL = True

    # Low-precision copy of the rows for the store search's candidate scan
    # (LZK_SEARCH_LOWP): "i8" = per-row symmetric int8 + fp32 row scales
    # (ops.search.flat_topk_i8, v_mfma_i32_16x16x64_i8), "fp8" = e4m3 rows
    # scaled by FP8_ROW_SCALE (ops.search.flat_topk_fp8), "off" = bf16 scan.
    # The fp8 path lost (round 2: its 8-sigma margin grew the lists ~5x and the
    # bf16 re-score of every entry cost 5.9 ms, bench/ab_fp8_search.py); int8
    # has ~4x less score error on unit rows and re-scores only the entries
    # above the error cut.
    FP8_ROW_SCALE = 64.0
    LOWP = os.environ.get("LZK_SEARCH_LOWP", "i8")

    def _lean(self, cap: int) -> bool:
        return bool((LEAN_HBM or getattr(self, "LEAN_HBM", False)) and cap >= LOWP_MIN_ROWS)

    @property
    def lean(self) -> bool:
        """No bf16 copy in HBM (see LEAN_HBM)."""
        return self.on_gpu and self.dim is not None and self.emb16 is None and self.emb8 is not None

    def _scan_rows(self, n: int, Q32: torch.Tensor):
        """The bf16 operand of the scans: the bf16 column, or -- lean -- the
        fp32 rows standing in for it (ops/search.py LeanRows)."""
        if self.emb16 is not None:
            return self.emb16[:n]
        from ..ops.search import LeanRows
        return LeanRows(self.emb32[:n], self.Dp, Q32)

    def _lowp_mode(self) -> str:
        if not self.on_gpu or self.Dp % 128 != 0:
            return ""
        if self.LOWP == "i8" and self.Dp <= 1024:
            return "i8"
        return "fp8" if self.LOWP == "fp8" else ""

    def _write_lowp(self, rt, e32: torch.Tensor) -> None:
        if self.emb8 is None:
            return
        if self.emb8.dtype == torch.int8:
            from ..ops.search import quantize_i8_rows
            # quantised from the bf16 rows: the scan then estimates the bf16
            # scores the exact re-score and select rank by
            q, sc = quantize_i8_rows(e32.to(torch.bfloat16))
            self.emb8[rt, : self.dim] = q
            self.rs8[rt] = sc
            if sc.numel():
                torch.maximum(self._rs8_max, sc.max(), out=self._rs8_max)
        else:
            from ..ops.search import quantize_e4m3
            self.emb8[rt, : self.dim] = quantize_e4m3(e32, self.FP8_ROW_SCALE)

    def reserve(self, n: int) -> None:
        if n > self.cap:
            self._alloc(max(n, self._init_cap, int(self.cap * 1.5) + 1))

    def _bump(self, edges: bool = False, store: bool = False) -> None:
        self.version += 1
        if edges:
            self.edge_version += 1
        if store:
            self._store_version += 1
        if self.on_change is not None:  # (e.g. the routed directory of parallel/service.py)
            self.on_change()

    # ------------------------------------------------------------------ codes
    def shard_id(self, name: str, live: bool = True) -> int:
        """Code of shard ``name`` (created on first use). ``live=False`` gives a
        code without making the shard visible in ``MemorySystem.shards``
        (a super-node's or store-only row's label)."""
        c = self.shard_code.get(name)
        if c is None:
            c = len(self.shard_names)
            if c > SHARD_MASK:
                raise OverflowError("too many shards")
            self.shard_names.append(name)
            self.shard_code[name] = c
            self.shard_live.append(live)
            self.shard_count.append(0)
        elif live and not self.shard_live[c]:
            self.shard_live[c] = True
        return c

    def live_shards(self) -> List[str]:
        return [s for s, live in zip(self.shard_names, self.shard_live) if live]

    def etype(self, name: str) -> int:
        c = self.etype_code.get(name)
        if c is None:
            c = len(self.etype_names)
            if c >= MAX_ETYPES:
                raise OverflowError("too many edge types")
            self.etype_names.append(name)
            self.etype_code[name] = c
        return c

    # ------------------------------------------------------------------ nodes
    def _as_emb(self, emb, m: int):
        """(fp32 [m, D] device tensor, None | (has-embedding flags, odd-dim rows))."""
        if torch.is_tensor(emb):
            t = emb.to(self.device, torch.float32)
            if t.dim() == 1:
                t = t[None, :]
            if self.dim is None and t.shape[1] > 0:
                self._set_dim(t.shape[1])
            if t.shape[1] != self.dim:
                raise ValueError(f"embedding dim {t.shape[1]} != tenant dim {self.dim}")
            return t.contiguous(), None
        rows = list(emb) if emb is not None else [None] * m
        if self.dim is None:
            for r in rows:
                if r is not None and len(r) > 0:
                    self._set_dim(len(r))
                    break
        D = self.dim or 0
        out = np.zeros((m, D), dtype=np.float32)
        ok = [False] * m
        odd = {}
        for i, r in enumerate(rows):
            if r is None or len(r) == 0:
                continue
            if len(r) != D:
                odd[i] = list(r)
                continue
            out[i] = np.asarray(r, dtype=np.float32)
            ok[i] = True
        return torch.from_numpy(out).to(self.device), (ok, odd)

    def add_nodes(self, ids: Sequence[str], contents: Sequence[str], emb=None, *, shard=None, types=None,
                  sal=None, acc=None, last=None, ts=None, sup=None, parents: Optional[Sequence[Optional[str]]] = None,
                  children: Optional[Dict[int, List[str]]] = None, stored: bool = False,
                  now: Optional[float] = None, ghost: bool = False, want_rows: bool = True) -> torch.Tensor:
        """Append (or replace, by id) ``m`` nodes. Scalars may be python
        sequences, tensors or scalars; ``shard`` holds shard codes; ``children``
        maps batch position -> child id list (super-nodes). ``ghost``: rows
        that are store members only, not graph nodes. Returns rows [m]."""
        m = len(ids)
        dev = self.device
        if m == 0:
            return torch.zeros(0, dtype=torch.long, device=dev)
        now = time.time() if now is None else now
        with self.on_stream():
            return self._add_nodes(ids, contents, emb, shard, types, sal, acc, last, ts, sup, parents, children,
                                   stored, now, ghost, want_rows)

    def _add_nodes(self, ids, contents, emb, shard, types, sal, acc, last, ts, sup, parents, children, stored, now,
                   ghost=False, want_rows=True):
        m = len(ids)
        dev = self.device
        e32, info = self._as_emb(emb, m)
        tlist = types if (types is not None and not isinstance(types, str)) else None
        tdef = types if isinstance(types, str) else "semantic"
        n0 = self.n
        fresh_map = dict(zip(ids, range(n0, n0 + m))) if not self.row_of else None  # empty graph (a load)
        if (fresh_map is not None and len(fresh_map) == m) or (
                fresh_map is None and len(set(ids)) == m and self.row_of.keys().isdisjoint(ids)):
            # bulk append of fresh ids (loads, large ingests): no per-row loop
            self.reserve(n0 + m)
            self.ids.extend(ids)
            self.content.extend(contents)
            self.types.extend(tlist if tlist is not None else [tdef] * m)
            if fresh_map is not None:
                self.row_of = fresh_map
            else:
                self.row_of.update(zip(ids, range(n0, n0 + m)))
            self.n = n0 + m
            rl = range(n0, n0 + m)
            rt = None  # contiguous rows n0 ..: materialised only where a row list is needed
        else:
            rows = [self.row_of.get(i, -1) for i in ids]
            fresh = sum(1 for r in rows if r < 0)
            self.reserve(self.n + fresh)
            kind_h = self.mirror("kind") if fresh < m else None
            r_next = self.n
            rl = []
            for j, (i, r) in enumerate(zip(ids, rows)):
                t = tlist[j] if tlist is not None else tdef
                if r < 0:
                    r = r_next
                    r_next += 1
                    self.ids.append(i)
                    self.content.append(contents[j])
                    self.types.append(t)
                    self.row_of[i] = r
                else:
                    if r < self._ann_covered:
                        self._ann_stale = True  # re-added id: its row gets a new vector
                    if kind_h is not None and r < len(kind_h) and kind_h[r] == NODE:
                        self._unlink_row(r)
                    self.content[r] = contents[j]
                    self.types[r] = t
                rl.append(r)
            self.n = r_next
            rt = torch.as_tensor(rl, dtype=torch.long).to(dev)

        def rows_t():
            return rt if rt is not None else torch.arange(n0, n0 + m, dtype=torch.long, device=dev)

        # a small batch whose per-row columns are all host values (or
        # scalars): ONE pinned float64 block -> one H2D copy + one kernel
        # writing every node column (tenant.hip tg_set_rows_kernel) --
        # consolidate_batch applies ~40 segments a step, each an insert
        fused = False
        if SET_ROWS_KERNEL and dev.type == "cuda" and m <= (1 << 16) and not (parents is not None and any(parents)):
            fused = self._set_rows_fused(rt, m, shard, sup, sal, acc, last, ts, now, ghost, stored, row0=n0)
        packed = {}
        if fused:
            sh, supv = None, None
        elif dev.type == "cuda" and m <= (1 << 16):
            def hostcol(v):
                if v is None or isinstance(v, (int, float, bool, np.number)):
                    return None
                if torch.is_tensor(v):
                    return v.numpy() if (not v.is_cuda and v.numel() == m) else None
                return v
            host = [(k, hv) for k, hv in ((k, hostcol(v)) for k, v in (("shard", shard), ("sup", sup), ("sal", sal),
                                                                       ("acc", acc), ("last", last), ("ts", ts)))
                    if hv is not None]
            if len(host) > 1:
                blk = torch.empty((len(host), m), dtype=torch.float64).pin_memory()
                bn = blk.numpy()
                for j, (_, v) in enumerate(host):
                    bn[j] = np.asarray(v, dtype=np.float64).reshape(-1)
                dblk = blk.to(dev, non_blocking=True)
                packed = {k: dblk[j] for j, (k, _) in enumerate(host)}

        def col(v, dt, default, name=None):
            if name in packed:
                return packed[name].to(dt)
            if v is None:
                return torch.full((m,), default, dtype=dt, device=dev)
            if torch.is_tensor(v):
                return v.to(dev, dt).reshape(-1).expand(m).contiguous() if v.numel() == 1 else v.to(dev, dt)
            if isinstance(v, (int, float, bool, np.number)):
                return torch.full((m,), v, dtype=dt, device=dev)
            return torch.as_tensor(np.asarray(v)).to(dev, dt)

        if not fused:
            rt = rows_t()
            sh = col(shard, torch.int32, 0, "shard")
            supv = col(sup, torch.uint8, 0, "sup")
            self.sal[rt] = col(sal, torch.float32, 0.5, "sal")
            self.acc[rt] = col(acc, torch.int32, 0, "acc")
            self.last[rt] = col(last, torch.float64, now, "last")
            self.ts[rt] = col(ts, torch.float64, now, "ts")
            self.shard[rt] = sh
            self.kind[rt] = GHOST if ghost else NODE
            self.sup[rt] = supv
            self.stored[rt] = 1 if stored else 0
            self.dirty[rt] = 1
            if parents is not None and any(parents):
                par = [self._ensure_row(p) if p else -1 for p in parents]
                self.parent[rt] = torch.as_tensor(par, dtype=torch.int32).to(dev)
            else:
                self.parent[rt] = -1
        if self.dim is not None:
            if info is None:
                has = None if (self.on_gpu and m <= WRITE_EMB_MAX_ROWS and self.dim <= 1024 and e32.is_cuda) \
                    else torch.ones(m, dtype=torch.bool, device=dev)
            else:
                ok, odd = info
                has = torch.as_tensor(ok, dtype=torch.bool).to(dev)
                for j, v in odd.items():
                    self.odd_emb[rl[j]] = v
            mc = m  # rows left to the chunked path
            if self.on_gpu and m <= WRITE_EMB_MAX_ROWS and self.dim <= 1024 and e32.is_cuda:
                # small inserts (consolidation segments, chat turns): every
                # embedding column in one launch (tenant.hip tg_write_emb_kernel)
                from ..ops.tenant_ops import write_emb
                if self._dv_acc is None:  # running device max of | |x| - 1 | (max_norm_dev)
                    self._dv_acc = torch.zeros(1, dtype=torch.float32, device=dev)
                write_emb(self, e32, None if info is None else has, rt, self._dv_acc, row0=n0, has_emb=True)
                self.n_sumsq += m
                if (info is None or any(info[0])) and not self._dv_acc_pending:
                    self._norm_dev_pending.append(self._dv_acc[0])
                    self._dv_acc_pending = True
                mc = 0  # columns written; skip the chunked path below
            # row chunks: a 10M-row load must not hold fp64 copies of the
            # whole [m, D] block (the squares were 2 x 60 GB of temporaries)
            contig = isinstance(rl, range)
            if mc:
                rt = rows_t()
            nrm2 = torch.empty(mc, dtype=torch.float64, device=dev)
            ch = max(1, (1 << 28) // max(1, 8 * self.dim))  # ~256 MB of fp64 per chunk
            for a in range(0, mc, ch):
                b = min(mc, a + ch)
                x = e32[a:b]
                if info is not None:
                    x = x * has[a:b, None].to(x.dtype)
                r = slice(n0 + a, n0 + b) if contig else rt[a:b]
                self.emb32[r] = x
                x2 = x.double() ** 2
                nrm2[a:b] = x2.sum(1)
                self.sumsq += x2.sum(0)
                del x2
                if self.emb16 is not None:
                    self.emb16[r, : self.dim] = x.to(torch.bfloat16)
                self._write_lowp(rt[a:b], x)
            if mc:
                self.sqn[rt] = nrm2.float()
                self.n_sumsq += m
                self.has_emb[rt] = has.to(torch.uint8)
            if mc and (info is None or any(info[0])):
                dv = torch.where(has, (nrm2.sqrt() - 1.0).abs(), torch.zeros_like(nrm2)).max()
                if dv.is_cuda:
                    self._norm_dev_pending.append(dv)
                    if len(self._norm_dev_pending) >= 256:
                        self._norm_dev_pending = [torch.stack(self._norm_dev_pending).max()]
                else:
                    self._max_norm_dev = max(self._max_norm_dev, float(dv))
        elif info is not None:
            for j, v in info[1].items():
                self.odd_emb[rl[j]] = v
        # host counters: from the caller's host values when it passed them
        # (no device round trip), else from the device columns
        if not ghost:
            sh_h, sup_h = _host_ints(shard, m, 0), _host_ints(sup, m, 0)
            if sh_h is None:
                sh_h = sh.cpu().numpy().astype(np.int64)
            if sup_h is None:
                sup_h = supv.cpu().numpy().astype(np.int64)
            ns = int(np.count_nonzero(sup_h))
            self.n_super += ns
            shs = sh_h[sup_h == 0] if ns else sh_h
            cnt = np.bincount(shs[shs >= 0], minlength=len(self.shard_count))
            for c in np.nonzero(cnt)[0]:
                self.shard_count[int(c)] += int(cnt[c])
        if children is not None:
            for j, ch in children.items():
                self.children[rl[j]] = list(ch)
        if self.deleted_ids:
            for i in ids:
                self.deleted_ids.pop(i, None)
        self.last_add_rows = rl  # host rows of this call (range or list)
        self._bump(store=True)
        return rows_t() if want_rows else None

    def _set_rows_fused(self, rt, m, shard, sup, sal, acc, last, ts, now, ghost, stored, row0=0) -> bool:
        """The node columns of an insert through tg_set_rows_kernel when every
        per-row value is on the host (else False: the caller's column path)."""
        vals = []
        consts = np.empty(7, np.float64)
        present = 0
        for c, (v, default) in enumerate(((sal, 0.5), (acc, 0), (last, now), (ts, now), (shard, 0), (sup, 0),
                                          (None, -1))):
            if v is None:
                consts[c] = default
                continue
            if isinstance(v, (int, float, bool, np.number)):
                consts[c] = float(v)
                continue
            if torch.is_tensor(v):
                if v.is_cuda:
                    return False
                if v.numel() == 1:
                    consts[c] = float(v.reshape(-1)[0])
                    continue
                v = v.numpy()
            a = np.asarray(v).reshape(-1)
            if a.size == 1:
                consts[c] = float(a[0])
                continue
            if a.size != m:
                return False
            consts[c] = 0.0
            vals.append(a)
            present |= 1 << c
        blk = torch.empty(7 + len(vals) * m, dtype=torch.float64).pin_memory()
        bn = blk.numpy()
        bn[:7] = consts
        for j, a in enumerate(vals):
            bn[7 + j * m: 7 + (j + 1) * m] = a
        T.set_rows(self, rt, blk.to(self.device, non_blocking=True), present, GHOST if ghost else NODE,
                   1 if stored else 0, m=m, row0=row0 if rt is None else None)
        return True

    def _ensure_row(self, node_id: str) -> int:
        """Row of ``node_id``; unknown ids become ghost rows (edge endpoints /
        parent references to nodes that do not exist, as the reference allows)."""
        r = self.row_of.get(node_id)
        if r is not None:
            return r
        self.reserve(self.n + 1)
        r = self.n
        self.n += 1
        self.ids.append(node_id)
        self.content.append("")
        self.types.append("semantic")
        self.row_of[node_id] = r
        with self.on_stream():
            self.kind[r] = GHOST
            self.shard[r] = -1
        self._bump()
        return r

    def _unlink_row(self, r: int) -> None:
        """Forget a live node's host counters before its row is replaced."""
        if int(self.mirror("sup")[r]):
            self.n_super -= 1
        else:
            s = int(self.mirror("shard")[r])
            if s >= 0:
                self.shard_count[s] -= 1
        self.children.pop(r, None)
        self.odd_emb.pop(r, None)

    def rows_of(self, ids: Iterable[str]) -> List[int]:
        return [self.row_of.get(i, -1) for i in ids]

    def node_row(self, node_id: str, include_super: bool = True) -> int:
        """Row of a live node (-1 if the id is not a node)."""
        r = self.row_of.get(node_id)
        if r is None or self.kind_h(r) != NODE:
            return -1
        if not include_super and self.sup_h(r):
            return -1
        return r

    def node_rows_of(self, ids: Sequence[str], include_super: bool = True) -> List[int]:
        """:meth:`node_row` for many ids with one small device gather of
        their (kind, sup) -- no whole-column mirror on the per-turn path."""
        rows = [self.row_of.get(i, -1) for i in ids]
        known = [r for r in rows if r >= 0]
        if not known:
            return [-1] * len(rows)
        kind, sup = self.flags_of(known)
        ok = {r: (k == NODE and (include_super or not sp)) for r, k, sp in zip(known, kind.tolist(), sup.tolist())}
        return [r if r >= 0 and ok[r] else -1 for r in rows]

    def _mirror_fresh(self, name: str) -> bool:
        m = self._mirror.get(name)
        return m is not None and m[0] == self.version and len(m[1]) == self.n

    # host mirrors of device columns (refreshed when the graph version moves)
    def mirror(self, name: str) -> np.ndarray:
        m = self._mirror.get(name)
        if m is not None and m[0] == self.version and len(m[1]) == self.n:
            return m[1]
        with self.on_stream():
            a = getattr(self, name)[: self.n].cpu().numpy()
        self._mirror[name] = (self.version, a)
        return a

    def flags_of(self, rows: Sequence[int]) -> Tuple[np.ndarray, np.ndarray]:
        """(kind, sup) of a few rows by one device gather -- the hot paths
        (retrieval, search result mapping) must not mirror whole columns of a
        multi-million-row tenant after every mutation."""
        if len(rows) == 0:
            return np.zeros(0, np.uint8), np.zeros(0, np.uint8)
        m = self._mirror.get("kind")
        if m is not None and m[0] == self.version and len(m[1]) == self.n:
            return m[1][np.asarray(rows)], self.mirror("sup")[np.asarray(rows)]
        with self.on_stream():
            rt = torch.as_tensor(np.asarray(rows), dtype=torch.long).to(self.device)
            both = torch.stack([self.kind[rt], self.sup[rt]]).cpu().numpy()
        return both[0], both[1]

    def kind_h(self, r: int) -> int:
        return int(self.mirror("kind")[r])

    def sup_h(self, r: int) -> int:
        return int(self.mirror("sup")[r])

    def node_rows_where(self, shard_code: Optional[int] = None, super_: Optional[bool] = None) -> np.ndarray:
        """Live node rows (ascending) filtered by shard code / super flag."""
        if super_ is True and shard_code is None and not self._mirror_fresh("kind"):
            # the few super-node rows by a device select: retrieval's
            # super-node step must not mirror two whole columns per turn
            if self.n_super == 0:
                return np.zeros(0, dtype=np.int64)
            n = self.n
            with self.on_stream():
                return torch.nonzero((self.kind[:n] == NODE) & (self.sup[:n] != 0)).flatten().cpu().numpy()
        kind = self.mirror("kind")
        m = kind == NODE
        if shard_code is not None:
            m &= self.mirror("shard") == shard_code
        if super_ is not None:
            m &= (self.mirror("sup") != 0) == super_
        return np.nonzero(m)[0]

    def ordered_node_rows(self) -> np.ndarray:
        """Live node rows in the reference's ``BufferGraph.nodes`` order:
        super-nodes first, then each shard (creation order) in insertion order."""
        kind, sup, sh = self.mirror("kind"), self.mirror("sup"), self.mirror("shard")
        live = np.nonzero(kind == NODE)[0]
        if live.size == 0:
            return live
        key = np.where(sup[live] != 0, -1, sh[live]).astype(np.int64)
        o = np.lexsort((live, key))
        return live[o]

    def ordered_node_rows_dev(self, super_: Optional[bool] = None) -> torch.Tensor:
        """:meth:`ordered_node_rows` as a device sort (no host mirror of the
        columns); ``super_`` filters super / shard nodes."""
        n = self.n
        with self.on_stream():
            m = self.kind[:n] == NODE
            if super_ is not None:
                m &= (self.sup[:n] != 0) == super_
            live = torch.nonzero(m).flatten()
            key = torch.where(self.sup[live] != 0, torch.full_like(live, -1), self.shard[live].long())
            return live[torch.argsort((key + 1) * max(n, 1) + live)]

    def first_node_rows_dev(self, k: int, super_: Optional[bool] = None) -> torch.Tensor:
        """The first ``k`` rows of :meth:`ordered_node_rows_dev` by one top-k
        pass (no sort of the tenant's rows). Shard nodes only (``super_`` is
        False) on a large tenant: shards in code order from the host counts,
        rows found in growing windows from row 0 -- the answer is almost
        always in the first window (no pass over the whole tenant)."""
        n = self.n
        if super_ is False and k > 0 and self.on_gpu:
            t = self._first_rows_dev(k)
            if t is not None:
                # targets the kernel could not fill (host shard counts ahead of
                # the device columns) stay -1: drop them like first_rows_capture
                with self.on_stream():
                    return t[t >= 0]
        if super_ is False and n > self.FIRST_ROWS_WINDOW and k > 0:
            return self._first_shard_rows(k)
        with self.on_stream():
            m = self.kind[:n] == NODE
            if super_ is not None:
                m &= (self.sup[:n] != 0) == super_
            r = torch.arange(n, device=self.device)
            key = torch.where(self.sup[:n] != 0, torch.zeros_like(r), self.shard[:n].long() + 1) * max(n, 1) + r
            key = torch.where(m, key, torch.full_like(key, 1 << 62))
            kk = min(k, int(m.sum()))
            if kk == 0:
                return torch.zeros(0, dtype=torch.long, device=self.device)
            v, i = torch.topk(key, kk, largest=False, sorted=True)
            return i

    FIRST_ROWS_WINDOW = 1 << 16

    def _first_rows_dev(self, k: int) -> Optional[torch.Tensor]:
        """:meth:`first_node_rows_dev` (shard nodes) by tenant.hip
        tg_first_rows_kernel: the per-shard targets come from the host shard
        counts, one block scans the rows from 0 -- no host synchronisation.
        None when there are more than 64 target shards."""
        tgt, need, off = [], k, 0
        for c, cnt in enumerate(self.shard_count):
            if cnt <= 0 or need == 0:
                continue
            t = min(int(cnt), need)
            tgt.append((c, t, off))
            off += t
            need -= t
        dev = self.device
        if not tgt:
            return torch.zeros(0, dtype=torch.long, device=dev)
        if len(tgt) > 64:
            return None
        with self.on_stream():
            out = torch.full((off,), -1, dtype=torch.long, device=dev)  # the kernel writes found rows only
            T.first_rows(self.kind, self.sup, self.shard, self.n, np.asarray(tgt, dtype=np.int32).T, out)
        return out

    def first_rows_capture(self, k: int) -> Capture:
        """The shard-node rows of :meth:`first_node_rows_dev` as a
        :class:`Capture` (no host wait on the GPU)."""
        if self.on_gpu and k > 0:
            t = self._first_rows_dev(k)
            if t is not None:
                with self.on_stream():
                    return Capture(t, fn=lambda a: a[a >= 0])
        return Capture(host=self.first_node_rows_dev(k, super_=False).cpu().numpy())

    def _first_shard_rows(self, k: int) -> torch.Tensor:
        n = self.n
        out = []
        need = k
        with self.on_stream():
            for c, cnt in enumerate(self.shard_count):
                if cnt <= 0 or need == 0:
                    continue
                got, lo, w = 0, 0, self.FIRST_ROWS_WINDOW
                while lo < n and need > 0 and got < cnt:
                    hi = min(n, lo + w)
                    m = (self.kind[lo:hi] == NODE) & (self.sup[lo:hi] == 0) & (self.shard[lo:hi] == c)
                    idx = torch.nonzero(m).flatten()[:need]
                    t = int(idx.numel())
                    if t:
                        out.append(idx + lo)
                        need -= t
                        got += t
                    lo, w = hi, w * 4
            if not out:
                return torch.zeros(0, dtype=torch.long, device=self.device)
            return torch.cat(out)

    def set_scalar(self, r: int, name: str, value) -> None:
        col = getattr(self, name)
        with self.on_stream():
            col[r] = value
            self.dirty[r] = 1
        m = self._mirror.get(name)
        if m is not None and m[0] == self.version and r < len(m[1]):
            m[1][r] = value
        self._mirror.pop("dirty", None)

    def get_scalar(self, r: int, name: str):
        return self.mirror(name)[r].item()

    def embedding(self, r: int) -> list:
        if r in self.odd_emb:
            return list(self.odd_emb[r])
        if self.dim is None or not int(self.mirror("has_emb")[r]):
            return []
        with self.on_stream():
            return self.emb32[r].double().cpu().tolist()

    def set_embedding(self, r: int, emb) -> None:
        self.odd_emb.pop(r, None)
        if r < self._ann_covered:
            self._ann_stale = True  # an indexed row's vector changed: rebuild the IVF-PQ codes
        if emb is None or len(emb) == 0:
            if self.dim is not None:
                with self.on_stream():
                    self.emb32[r] = 0
                    self.sqn[r] = 0
                    self.has_emb[r] = 0
                    if self.emb16 is not None:
                        self.emb16[r] = 0
                    if self.emb8 is not None:
                        self.emb8[r] = 0
                    if self.rs8 is not None:
                        self.rs8[r] = 0.0
            self._bump(store=True)
            return
        if self.dim is None:
            self._set_dim(len(emb))
        if len(emb) != self.dim:
            self.odd_emb[r] = list(emb)
            self._bump(store=True)
            return
        v = torch.as_tensor(np.asarray(emb, dtype=np.float32)).to(self.device)
        with self.on_stream():
            self.emb32[r] = v
            n2 = float((v.double() ** 2).sum())
            self.sqn[r] = n2
            self.has_emb[r] = 1
            self.dirty[r] = 1
            if self.emb16 is not None:
                self.emb16[r, : self.dim] = v.to(torch.bfloat16)
            self._write_lowp(r, v[None, :])
        self._max_norm_dev = max(self._max_norm_dev, abs(math.sqrt(n2) - 1.0))
        self._bump(store=True)

    # ------------------------------------------------------------------ edges
    @property
    def num_edges(self) -> int:
        return int(self.e["src"].numel())

    EDGE_SORT_MIN = 1 << 20  # edge lists shorter than this are never re-ordered

    def _maybe_sort_edges(self) -> bool:
        """Keep the edge list (nearly) ordered by source row: the union-find
        pass of the component digest hooks / finds ``src`` endpoints in edge
        order, and on a 10M-row / 20M-edge graph a src-ordered list runs in
        1.6 ms against 7.5 ms for a random order (a round-4 probe, since removed). Links
        are appended in insertion order (new rows = new sources), so the list
        stays nearly sorted by itself; when more than 1/32 of adjacent pairs
        are out of order (seeded or migrated edges) every edge column is
        permuted by one stable sort. Edge order carries no meaning (every
        consumer is order-free or re-derives its index lists)."""
        ne = self.num_edges
        if ne < self.EDGE_SORT_MIN or (self._cc is not None and self._cc.get("ns") is not None):
            return False  # (a batch's stable/volatile partition is in place)
        with self.on_stream():
            src = self.e["src"]
            if int((src[1:] < src[:-1]).sum()) * 32 <= ne:
                return False
            o = torch.sort(src, stable=True).indices
            self.e = {k: v[o] for k, v in self.e.items()}
        self.edge_version += 1
        return True

    def append_edges(self, src: torch.Tensor, dst: torch.Tensor, w: torch.Tensor, shard: torch.Tensor,
                     etype: int = 0, co=None, lu=None, now: Optional[float] = None) -> None:
        """Append edges known not to exist yet (every edge a consolidation
        creates starts at a node of this batch)."""
        m = int(src.numel())
        if m == 0:
            return
        now = time.time() if now is None else now
        dev = self.device
        with self.on_stream():
            meta = (shard.to(dev, torch.int32) & SHARD_MASK) | (etype << TYPE_SHIFT) | EDIRTY
            self._edge_append({"src": src, "dst": dst, "w": w,
                               "co": co if co is not None else torch.ones(m, dtype=torch.int32, device=dev),
                               "lu": lu if lu is not None else torch.full((m,), now, dtype=torch.float64, device=dev),
                               "meta": meta}, m)
        self._bump(edges=True)

    EDGE_SLACK_MIN = 1 << 14

    def append_edges_host(self, src, dst, w, code, etype: int = 0, now: Optional[float] = None) -> None:
        """:meth:`append_edges` from host arrays (a consolidation segment's
        planned links): one pinned float64 block, one copy, one launch
        (tenant.hip tg_append_edges_kernel) into the columns' spare tails."""
        m = len(src)
        if m == 0:
            return
        now = time.time() if now is None else now
        if not self.on_gpu:
            cols = T.to_dev_packed([src, dst, np.asarray(w, np.float32), code], self.device)
            self.append_edges(cols[0].long(), cols[1].long(), cols[2].float(), cols[3].int(), etype, now=now)
            return
        dev = self.device
        with self.on_stream():
            blk = torch.empty(4 * m, dtype=torch.float64).pin_memory()
            bn = blk.numpy()
            for j, c in enumerate((src, dst, np.asarray(w, np.float32), code)):
                bn[j * m:(j + 1) * m] = np.asarray(c, dtype=np.float64).reshape(-1)
            vals = blk.to(dev, non_blocking=True)
            e = self.e
            ne = int(e["src"].numel())
            for k, dt in (("src", torch.int32), ("dst", torch.int32), ("w", torch.float32), ("co", torch.int32),
                          ("lu", torch.float64), ("meta", torch.int32)):
                v = e[k]
                buf, vn = self._ebuf.get(k, (None, -1))
                if buf is None or vn != ne or v.numel() != ne or buf.numel() < ne + m or v.data_ptr() != buf.data_ptr():
                    buf = torch.empty(ne + m + max((ne + m) >> 3, self.EDGE_SLACK_MIN), dtype=dt, device=dev)
                    buf[:ne].copy_(v)
                e[k] = buf[:ne + m]
                self._ebuf[k] = (buf, ne + m)
            T._lib.check(T._lib.lib().lzk_tg_append_edges(
                vals.data_ptr(), m, ne, (etype << TYPE_SHIFT) | EDIRTY, float(now), e["src"].data_ptr(),
                e["dst"].data_ptr(), e["w"].data_ptr(), e["co"].data_ptr(), e["lu"].data_ptr(), e["meta"].data_ptr(),
                T._st(vals)), "tg_append_edges")
        self._bump(edges=True)

    def _edge_append(self, new: Dict[str, torch.Tensor], m: int) -> None:
        """Append ``m`` edges: into the spare tail of the column's buffer when
        ``self.e[k]`` is still the view this method (or a segment compaction)
        handed out, else into a fresh buffer with 1/8 headroom. A 20M-edge
        graph gaining a few hundred links per consolidation segment no longer
        copies 560 MB per append (``torch.cat``). Older views only ever cover
        a prefix of the buffer, so writing its tail cannot change them."""
        e = self.e
        ne = int(e["src"].numel())
        for k, dt in (("src", torch.int32), ("dst", torch.int32), ("w", torch.float32), ("co", torch.int32),
                      ("lu", torch.float64), ("meta", torch.int32)):
            v, add = e[k], new[k].to(self.device, dt)
            buf, vn = self._ebuf.get(k, (None, -1))
            if buf is None or vn != ne or v.numel() != ne or buf.numel() < ne + m or v.data_ptr() != buf.data_ptr():
                buf = torch.empty(ne + m + max((ne + m) >> 3, self.EDGE_SLACK_MIN), dtype=dt, device=self.device)
                buf[:ne].copy_(v)
            buf[ne:ne + m].copy_(add)
            e[k] = buf[:ne + m]
            self._ebuf[k] = (buf, ne + m)

    def _adopt_edges(self, e: Dict[str, torch.Tensor]) -> None:
        """Make ``e`` (views of over-allocated buffers, T._compact(extra=...))
        the edge list, its spare tails available to :meth:`_edge_append`."""
        self.e = e
        self._ebuf = {k: (v._base if v._base is not None else v, int(v.numel())) for k, v in e.items()}

    def upsert_edges(self, src: torch.Tensor, dst: torch.Tensor, w: torch.Tensor, shard: torch.Tensor,
                     etype: torch.Tensor, co=None, lu=None, now: Optional[float] = None) -> int:
        """``MemoryShard.add_edge`` for a batch, in order (reference
        memory_shard.py:42-52): an edge whose (shard, source, target) already
        exists -- or appeared earlier in the batch -- strengthens it (weight +0.1
        capped at 1, co_occurrence +1) instead of being added. Returns #new."""
        m = int(src.numel())
        if m == 0:
            return 0
        now = time.time() if now is None else now
        with self.on_stream():
            return self._upsert_edges(src, dst, w, shard, etype, co, lu, now)

    def _upsert_edges(self, src, dst, w, shard, etype, co, lu, now):
        m = int(src.numel())
        dev = self.device
        e = self.e
        ne = self.num_edges
        src, dst = src.to(dev, torch.int64), dst.to(dev, torch.int64)
        shard = shard.to(dev, torch.int64)
        s_all = torch.cat([e["src"].long(), src])
        d_all = torch.cat([e["dst"].long(), dst])
        h_all = torch.cat([(e["meta"] & SHARD_MASK).long(), shard])
        # lexicographic stable sort by (shard, src, dst); equal keys keep position order
        o = torch.sort(d_all, stable=True).indices
        o = o[torch.sort(s_all[o], stable=True).indices]
        o = o[torch.sort(h_all[o], stable=True).indices]
        hs, ss, ds = h_all[o], s_all[o], d_all[o]
        newgrp = torch.ones(ne + m, dtype=torch.bool, device=dev)
        newgrp[1:] = (hs[1:] != hs[:-1]) | (ss[1:] != ss[:-1]) | (ds[1:] != ds[:-1])
        gid = torch.cumsum(newgrp.long(), 0) - 1
        head = o[newgrp]  # position of each group's first element
        cnt = torch.zeros(int(head.numel()), dtype=torch.int64, device=dev).index_add_(0, gid, torch.ones_like(gid))
        extra = (cnt - 1).to(torch.float32)  # strengthening adds per group
        old_head = head < ne
        hi, ex = head[old_head], extra[old_head]
        t = ex > 0
        hi, ex = hi[t], ex[t]
        if hi.numel():
            e["w"][hi] = torch.clamp(e["w"][hi] + 0.1 * ex, max=1.0)
            e["co"][hi] = e["co"][hi] + ex.to(torch.int32)
            e["lu"][hi] = now
            e["meta"][hi] = e["meta"][hi] | EDIRTY
        n_new = 0
        new_head = ~old_head
        if bool(new_head.any()):
            bi, oo = torch.sort(head[new_head] - ne)  # batch positions of first occurrences, in order
            ex = extra[new_head][oo]
            w0 = w.to(dev, torch.float32)[bi]
            ww = torch.where(ex > 0, torch.clamp(w0 + 0.1 * ex, max=1.0), w0)
            cc = (co.to(dev, torch.int32)[bi] if co is not None
                  else torch.ones_like(bi, dtype=torch.int32)) + ex.to(torch.int32)
            ll = lu.to(dev, torch.float64)[bi] if lu is not None else None
            self.append_edges(src[bi], dst[bi], ww, shard[bi].to(torch.int32), 0, cc, ll, now)
            k = int(bi.numel())
            et = etype.to(dev, torch.int32)[bi]
            tail = self.e["meta"][-k:]
            self.e["meta"][-k:] = (tail & ~(TYPE_MASK << TYPE_SHIFT)) | (et << TYPE_SHIFT)
            n_new = k
        self._bump(edges=True)
        return n_new

    def edge_index(self, s: int, d: int, shard_code: int) -> int:
        e = self.e
        with self.on_stream():
            m = (e["src"] == s) & (e["dst"] == d) & ((e["meta"] & SHARD_MASK) == shard_code)
            nz = torch.nonzero(m).flatten()
            return int(nz[0]) if nz.numel() else -1

    def edges_of_shard(self, shard_code: int) -> torch.Tensor:
        with self.on_stream():
            return torch.nonzero((self.e["meta"] & SHARD_MASK) == shard_code).flatten()

    def edges_incident(self, r: int, shard_code: Optional[int] = None) -> torch.Tensor:
        e = self.e
        with self.on_stream():
            m = (e["src"] == r) | (e["dst"] == r)
            if shard_code is not None:
                m &= (e["meta"] & SHARD_MASK) == shard_code
            return torch.nonzero(m).flatten()

    def remove_edges(self, idx: torch.Tensor) -> None:
        if idx.numel() == 0:
            return
        with self.on_stream():
            e = self.e
            idx = idx.to(self.device)
            if self.track:
                self._note_dropped(e["src"][idx], e["dst"][idx], e["meta"][idx])
            keep = torch.ones(self.num_edges, dtype=torch.bool, device=self.device)
            keep[idx] = False
            self.e = {k: v[keep] for k, v in e.items()}
        self._bump(edges=True)

    def _note_dropped(self, s: torch.Tensor, d: torch.Tensor, meta: Optional[torch.Tensor] = None) -> None:
        """Queue removed edges for deletion from the store -- only those the
        store holds (ESTORED): an edge created and pruned between two
        commits never reached it. Device tensors wait in _drop_pending until
        deleted_edges is read."""
        if s.numel() == 0:
            return
        if s.is_cuda:
            self._drop_pending.append((s, d, meta))
            return
        self._resolve_dropped(s, d, meta)

    def _resolve_dropped(self, s, d, meta) -> None:
        s, d = s.cpu().numpy(), d.cpu().numpy()
        if meta is not None:
            keep = (meta.cpu().numpy() & ESTORED) != 0
            s, d = s[keep], d[keep]
        ids, de = self.ids, self._deleted_edges
        for a, b in zip(s.tolist(), d.tolist()):
            de[(ids[a], ids[b])] = None

    @property
    def deleted_edges(self) -> Dict[Tuple[str, str], None]:
        """(src id, dst id) of edges to delete from the store at the next commit."""
        if self._drop_pending:
            pend, self._drop_pending = self._drop_pending, []
            with self.on_stream():
                if len(pend) > 1 and all(m is not None for _, _, m in pend):
                    # one device -> host copy for every pending batch (in order)
                    self._resolve_dropped(*(torch.cat([p[i].to(torch.int32) for p in pend]) for i in range(3)))
                else:
                    for s, d, meta in pend:
                        self._resolve_dropped(s, d, meta)
        return self._deleted_edges

    @deleted_edges.setter
    def deleted_edges(self, v: Dict[Tuple[str, str], None]) -> None:
        self._drop_pending = []
        self._deleted_edges = v

    @property
    def max_norm_dev(self) -> float:
        """max | |x| - 1 | over embedded rows; inserts leave their device
        maxima pending (no host synchronisation per insert)."""
        if self._norm_dev_pending:
            pend, self._norm_dev_pending = self._norm_dev_pending, []
            self._dv_acc_pending = False
            with self.on_stream():
                self._max_norm_dev = max(self._max_norm_dev, float(torch.stack(pend).max()))
        return self._max_norm_dev

    @max_norm_dev.setter
    def max_norm_dev(self, v: float) -> None:
        self._norm_dev_pending = []
        self._dv_acc, self._dv_acc_pending = None, False
        self._max_norm_dev = float(v)

    # ------------------------------------------------------------------ maintenance
    def decay(self, rate: float = 0.01, prune_threshold: Optional[float] = None, decay_nodes: bool = True,
              steps: int = 1) -> int:
        """Temporal decay of all edges and shard-node saliences, ``steps``
        rounds (= that many end_conversation calls, each rounded to fp32),
        + optional prune, in one kernel pass. Returns the number of pruned
        edges."""
        if steps <= 0:
            return 0
        if prune_threshold is not None and prune_threshold <= 0.0:
            prune_threshold = None  # weights never go below 0: nothing to prune, no flag / compaction pass
        if rate == 0.0 and prune_threshold is None:
            return 0
        with self.on_stream():
            self.e, n, dropped = T.decay_prune(self.e, self.sal[: self.n], self.kind[: self.n], self.sup[: self.n],
                                               rate, prune_threshold, decay_nodes, want_dropped=self.track,
                                               steps=steps)
        if rate:
            if self._cc is not None:
                self._cc["steps"] += max(int(steps), 0)
            self.decay_log += steps * math.log1p(-rate)
        if dropped is not None and n:
            self._note_dropped(*dropped)
        self._bump(edges=bool(n) or bool(rate))
        return n

    def prune(self, threshold: float) -> int:
        return self.decay(0.0, threshold, decay_nodes=False)

    # ------------------------------------------------------------------ consolidation segments
    def segment_begin(self, rate: float, prune_threshold: Optional[float], steps: int) -> Dict:
        """Start one segment of a batched consolidation: ``steps`` decay rounds
        of the edges and shard-node saliences now, the prune of ``w <
        prune_threshold`` deferred to :meth:`segment_end`, which drops those
        edges together with the segment's victims' in ONE compaction and ONE
        host sync. Between the two calls the edge list still holds the
        to-be-pruned edges: only node inserts / row updates and
        :meth:`append_edges` may run in between. On the CPU this is
        :meth:`decay` followed by :meth:`remove_nodes` in segment_end."""
        if prune_threshold is not None and prune_threshold <= 0.0:
            prune_threshold = None
        if not self.on_gpu:
            return {"pruned": self.decay(rate, prune_threshold, steps=steps)}
        tok = {"flag": None, "ne0": self.num_edges}
        if steps <= 0 or (rate == 0.0 and prune_threshold is None):
            return tok
        with self.on_stream():
            tok["flag"] = T.decay_flags(self.e, self.sal[: self.n], self.kind[: self.n], self.sup[: self.n], rate,
                                        prune_threshold, steps)
        if rate:
            if self._cc is not None:
                self._cc["steps"] += int(steps)
            self.decay_log += steps * math.log1p(-rate)
        self._bump(edges=bool(rate))
        return tok

    def segment_end(self, tok: Dict, victims, unstore: bool = True) -> int:
        """Finish a segment (:meth:`segment_begin`): drop the deferred-pruned
        edges and remove the ``victims`` rows like :meth:`remove_nodes`
        (ghost rows, their shard's incident edges gone). Returns #pruned."""
        vic = victims.tolist() if torch.is_tensor(victims) else list(victims)
        if "pruned" in tok:
            if vic:
                self.remove_nodes(vic, drop_edges=True, unstore=unstore)
            return tok["pruned"]
        cand = sorted({r for r in vic if 0 <= r < self.n})
        prev, ne0 = tok["flag"], tok["ne0"]
        ne = self.num_edges
        if not cand and prev is None:
            return 0
        if SEG_END_KERNEL:
            return self._segment_end_fused(cand, prev, ne, unstore)
        with self.on_stream():
            parts = []
            rt = live_t = None
            if cand:
                rt = self._dev_rows(cand)
                kd = self.kind[rt]
                live_t = kd == NODE
                parts += [kd.int(), self.sup[rt].int(), self.shard[rt]]
            flag = bc = total = None
            if ne and (prev is not None or cand):
                rm = None
                if cand:
                    rm = torch.zeros(self.n, dtype=torch.uint8, device=self.device)
                    rm[rt] = live_t.to(torch.uint8)
                flag, bc, total = T.flag_finish(self.e, rm, self.shard[: self.n], prev)
                parts.append(total)
                if prev is not None:
                    parts.append(ne0 - prev.sum(dtype=torch.int32).view(1))
            if cand:
                self.kind[rt] = torch.where(live_t, torch.full_like(kd, GHOST), kd)
                if unstore:
                    self.stored[rt] = torch.where(live_t, torch.zeros_like(self.stored[rt]), self.stored[rt])
            info = torch.cat(parts).cpu().numpy() if parts else np.zeros(0, np.int64)  # the one host sync
            nc = len(cand)
            pruned = 0
            if flag is not None:
                n_out = int(info[3 * nc])
                if prev is not None:
                    pruned = int(info[3 * nc + 1])
                if n_out != ne:
                    old = self.e
                    out, n = T._compact(old, flag, bc, ne, extra=max(ne >> 3, self.EDGE_SLACK_MIN), total=total,
                                        n_out=n_out)
                    self._adopt_edges(out)
                    if self.track:
                        self._note_dropped(*T._dropped(old, flag, ne, n))
        if cand:
            kinds, sups, shards = info[:nc], info[nc:2 * nc], info[2 * nc:3 * nc]
            for r, k, sp, sh in zip(cand, kinds.tolist(), sups.tolist(), shards.tolist()):
                if k != NODE:
                    continue
                if sp:
                    self.n_super -= 1
                elif sh >= 0:
                    self.shard_count[sh] -= 1
                self.children.pop(r, None)
                self.odd_emb.pop(r, None)
                self.deleted_ids[self.ids[r]] = None
        self._bump(edges=True, store=bool(cand))
        return pruned

    def _segment_end_fused(self, cand: List[int], prev, ne: int, unstore: bool) -> int:
        """:meth:`segment_end` through tenant.hip lzk_tg_seg_end: the victims'
        state, the removal bitmap, the edge flags and both counts in five
        launches, read back in one copy."""
        nc = len(cand)
        dev = self.device
        # the stable prefix of a partitioned batch (cc_begin) loses nothing:
        # flags, survivors and the compaction cover the suffix only
        ns = self._cc.get("ns") if self._cc is not None else None
        if ns is not None and (ns > ne or (prev is not None and prev.numel() < ns)):
            ns = None
        ns = ns or 0
        with self.on_stream():
            words = (self.cap + 31) // 32
            if self._rmb is None or self._rmb.numel() < words:
                self._rmb = torch.zeros(words, dtype=torch.int32, device=dev)
            rt = self._dev_rows(cand) if nc else None
            info = torch.empty(3 * nc + 2, dtype=torch.int32, device=dev)
            es = self.e if ns == 0 else {k: v[ns:] for k, v in self.e.items()}
            ps = prev if (prev is None or ns == 0) else prev[ns:]
            nes = ne - ns
            flag = bc = None
            if nes:
                flag = torch.empty(nes, dtype=torch.uint8, device=dev)
                bc = torch.empty(max(1, (nes + T.NTB - 1) // T.NTB), dtype=torch.int32, device=dev)
            T.seg_end(rt, nc, self.kind, self.sup, self.shard, self.stored, unstore, self._rmb, es, ps, flag, bc,
                      info)
            info_h = info.cpu().numpy()  # the one host sync
            pruned = int(info_h[3 * nc + 1]) if prev is not None else 0
            if nes:
                n_out = int(info_h[3 * nc])
                if n_out != nes:
                    out, n, dr = T._compact(es, flag, bc, nes, extra=0 if ns else max(ne >> 3, self.EDGE_SLACK_MIN),
                                            n_out=n_out, dropped=self.track)
                    if ns:  # survivors back behind the untouched prefix, in the same buffers
                        for k in T.EDGE_COLS:
                            self.e[k][ns:ns + n_out].copy_(out[k])
                        self._adopt_edges({k: v[:ns + n_out] for k, v in self.e.items()})
                    else:
                        self._adopt_edges(out)
                    if dr is not None:
                        self._note_dropped(*dr)
        if nc:
            kinds, sups, shards = info_h[:nc], info_h[nc:2 * nc], info_h[2 * nc:3 * nc]
            for r, k, sp, sh in zip(cand, kinds.tolist(), sups.tolist(), shards.tolist()):
                if k != NODE:
                    continue
                if sp:
                    self.n_super -= 1
                elif sh >= 0:
                    self.shard_count[sh] -= 1
                self.children.pop(r, None)
                self.odd_emb.pop(r, None)
                self.deleted_ids[self.ids[r]] = None
        self._bump(edges=True, store=bool(cand))
        return pruned

    def remove_nodes(self, rows, drop_edges: bool = True, unstore: bool = False) -> int:
        """Remove live nodes: each becomes a ghost row (its id may still be an
        edge endpoint) and -- ``drop_edges`` -- its own shard's incident edges go
        (reference ``_enforce_buffer_limit`` :558-569). Returns #removed."""
        rl = rows.tolist() if torch.is_tensor(rows) else list(rows)
        cand = sorted({r for r in rl if 0 <= r < self.n})
        if not cand:
            return 0
        # kind / sup / shard of just these rows (one small copy, no mirror of
        # the whole tenant's columns)
        with self.on_stream():
            ct = self._dev_rows(cand)
            info = torch.stack([self.kind[ct].int(), self.sup[ct].int(), self.shard[ct]]).cpu().numpy()
        keep = info[0] == NODE
        live = [r for r, k in zip(cand, keep) if k]
        if not live:
            return 0
        for r, sp, sh in zip(live, info[1][keep].tolist(), info[2][keep].tolist()):
            if sp:
                self.n_super -= 1
            elif sh >= 0:
                self.shard_count[sh] -= 1
            self.children.pop(r, None)
            self.odd_emb.pop(r, None)
        with self.on_stream():
            rt = ct if len(live) == len(cand) else self._dev_rows(live)
            if drop_edges and self.num_edges:
                rm = torch.zeros(self.n, dtype=torch.uint8, device=self.device)
                rm[rt] = 1
                self.e, n, dropped = T.remove_edges_of(self.e, rm, self.shard[: self.n], want_dropped=self.track)
                if dropped is not None and n:
                    self._note_dropped(*dropped)
            self.kind[rt] = GHOST
            if unstore:
                self.stored[rt] = 0
        for r in live:
            self.deleted_ids[self.ids[r]] = None
        self._bump(edges=True, store=True)
        return len(live)

    def unstore(self, ids: Iterable[str]) -> None:
        rows = [r for r in self.rows_of(ids) if r >= 0]
        if rows:
            with self.on_stream():
                self.stored[self._dev_rows(rows)] = 0  # pinned async upload, no host block
            self._bump(store=True)

    def mark_stored(self, rows) -> None:
        rows = torch.as_tensor(rows, dtype=torch.long) if not torch.is_tensor(rows) else rows
        if rows.numel():
            with self.on_stream():
                self.stored[rows.to(self.device)] = 1
            self._bump(store=True)

    def evict(self, max_nodes: int, now: Optional[float] = None) -> List[int]:
        """Buffer-limit eviction (reference memory_system.py:535-578): when the
        node count (super-nodes included) exceeds ``max_nodes``, the ``excess``
        shard nodes of lowest importance go, with their shard's edges.
        Victim order: importance, then the reference's iteration order (shard
        creation order, then insertion order). Returns victim rows."""
        total = self.num_nodes()
        if total <= max_nodes:
            return []
        excess = total - max_nodes
        now = time.time() if now is None else now
        n = self.n
        with self.on_stream():
            score = T.importance(self.sal[:n], self.acc[:n], self.last[:n], self.kind[:n], self.sup[:n], now)
            okey = self.shard[:n].long() * (1 << 32) + torch.arange(n, device=self.device)
            if excess * 64 < n:
                # the k-th smallest score (a top-k: torch.kthvalue is ~100x
                # slower on ROCm), then the tied rows in (shard, row) order by
                # a top-k: O(n) passes instead of two full stable sorts
                t = torch.topk(score, excess, largest=False, sorted=False).values.max()
                lt = torch.nonzero(score < t).flatten()
                m = excess - int(lt.numel())
                big = torch.iinfo(torch.int64).max
                tie_key = torch.where(score == t, okey, torch.full_like(okey, big))
                tv, ti = torch.topk(tie_key, m, largest=False, sorted=True)
                ti = ti[tv != big]
                # victims in the sequential order: score, then (shard, row)
                cand = torch.cat([lt, ti])
                o1 = torch.sort(okey[cand], stable=True).indices
                cand = cand[o1]
                order = cand[torch.sort(score[cand], stable=True).indices]
            else:
                o1 = torch.sort(okey, stable=True).indices
                o2 = torch.sort(score[o1], stable=True).indices
                order = o1[o2][:excess]
            order = order[torch.isfinite(score[order])]
            victims = order.tolist()
        self.remove_nodes(victims, drop_edges=True, unstore=True)
        return victims

    def num_nodes(self) -> int:
        return int(sum(self.shard_count) + self.n_super)

    # ------------------------------------------------------------------ queries
    def neighbors(self, r: int, min_weight: float = 0.3) -> List[int]:
        """``MemoryShard.get_neighbors`` of a shard node: other endpoints of the
        edges its shard stores, with w >= min_weight, in edge order."""
        if r < 0 or self.kind_h(r) != NODE or self.sup_h(r):
            return []
        sc = int(self.mirror("shard")[r])
        e = self.e
        with self.on_stream():
            m = ((e["src"] == r) | (e["dst"] == r)) & ((e["meta"] & SHARD_MASK) == sc) & (e["w"] >= min_weight)
            idx = torch.nonzero(m).flatten()
            s, d = e["src"][idx].tolist(), e["dst"][idx].tolist()
        return [b if a == r else a for a, b in zip(s, d)]

    def csr(self):
        if self._csr is None or self._csr_version != self.edge_version or self._csr[0].numel() != self.n + 1:
            with self.on_stream():
                self._csr = T.build_visible_csr(self.e, self.shard[: self.n], self.n)
            self._csr_version = self.edge_version
        return self._csr

    def boost(self, seed_rows: Sequence[int], now: Optional[float] = None, min_w: float = 0.3,
              delta: float = 0.02) -> int:
        seeds = [r for r in seed_rows if r >= 0]
        if not seeds or self.num_edges == 0:
            return 0
        now = time.time() if now is None else now
        csr = self.csr()
        with self.on_stream():
            st = torch.as_tensor(seeds, dtype=torch.int32).to(self.device)
            k = T.neighbor_boost(csr, self.e["w"], st, self.kind, self.sup, self.sal, self.last, self.dirty, now,
                                 self._boost_state, min_w, delta)
        if k:
            self._bump()
        return k

    def touch(self, rows: Sequence[int], now: Optional[float] = None) -> None:
        rows = [r for r in rows if r >= 0]
        if not rows:
            return
        now = time.time() if now is None else now
        # tg_touch_kernel updates each listed row with plain stores, so a row
        # listed twice in one launch would count once: a repeated row is
        # applied in a further launch per repeat (the reference's
        # update_access per occurrence, buffer_graph.py:79-85)
        with self.on_stream():
            while rows:
                seen, rest = set(), []
                for r in rows:
                    (rest.append(r) if r in seen else seen.add(r))
                T.touch(torch.as_tensor(list(dict.fromkeys(rows)), dtype=torch.long).to(self.device), self.acc,
                        self.last, self.sal, self.dirty, now)
                rows = rest
        self._bump()

    def components(self) -> List[np.ndarray]:
        """Connected components containing at least one live node, as arrays of
        rows (ghost endpoints included, like the reference's DFS that follows
        edges to missing ids), ordered by their first member in
        ``ordered_node_rows`` order; members in row order."""
        n = self.n
        if n == 0:
            return []
        with self.on_stream():
            lab = T.components(self.e["src"], self.e["dst"], n)
            lab_h = lab.cpu().numpy() if torch.is_tensor(lab) else np.asarray(lab)
            touched = np.zeros(n, dtype=bool)
            if self.num_edges:
                touched[self.e["src"].cpu().numpy()] = True
                touched[self.e["dst"].cpu().numpy()] = True
        kind = self.mirror("kind")
        order = self.ordered_node_rows()
        member = (kind == NODE) | ((kind == GHOST) & touched)
        rows = np.nonzero(member)[0]
        if rows.size == 0:
            return []
        labs = lab_h[rows]
        o = np.argsort(labs, kind="stable")
        rows, labs = rows[o], labs[o]
        uniq, start = np.unique(labs, return_index=True)
        groups = np.split(rows, start[1:])
        # position of each label's first member in the reference node order
        pos = np.full(n, np.iinfo(np.int64).max, dtype=np.int64)
        pos[order] = np.arange(order.size)
        first = np.full(n, np.iinfo(np.int64).max, dtype=np.int64)
        np.minimum.at(first, lab_h[order], pos[order])
        keyed = [(int(first[lb]), g) for lb, g in zip(uniq.tolist(), groups) if first[lb] < np.iinfo(np.int64).max]
        keyed.sort(key=lambda x: x[0])
        return [g for _, g in keyed]

    def component_digest(self, min_size: int = 3, min_avg_w: float = 0.3, take: int = 10) -> List[np.ndarray]:
        """``run_consolidation``'s view of the components (reference
        memory_system.py:967-990) without materialising them: components
        with >= ``min_size`` members whose mean edge weight exceeds
        ``min_avg_w``, in the order of :meth:`components`, each as the first
        ``take`` of its live shard-node rows (row order) -- the only rows the
        profile prompt reads (:1032). Components with none are left out.
        Labels, sizes, weight sums and the ordering are device reductions;
        only the <= ``take`` rows per qualifying component reach the host.
        On the GPU the reductions are the sort-free kernels of digest.hip
        (ops.tenant_ops.component_digest); the sorted formulation below is
        the CPU path."""
        n = self.n
        if n == 0 or self.num_edges == 0:
            return []
        dev = self.device
        if self._digest_local(min_size, take):
            with self.on_stream():
                return T.digest_lists(self._digest_local_dev(min_size, min_avg_w, take).cpu().numpy())
        if dev.type == "cuda" and min_size >= 2 and take >= 1 and not self._digest_sorted:
            self._maybe_sort_edges()
            with self.on_stream():
                lab = self._cc_labels() if self._cc is not None and "lab" in self._cc else None
                key, rows = T.component_digest(self.e["src"], self.e["dst"], self.e["w"], self.kind[:n],
                                               self.sup[:n], self.shard[:n], n, min_size, min_avg_w, take, lab=lab)
                kr = torch.stack([key, rows.long()]).cpu().numpy()  # one device -> host copy
                key_h, rows_h = kr[0], kr[1]
            if rows_h.size == 0:
                return []
            return np.split(rows_h, np.nonzero(np.diff(key_h))[0] + 1)
        with self.on_stream():
            # Labels over the rows (one union-find pass over the edges); a row
            # no edge touches is a singleton (size 1 < min_size, no edge
            # weight), so only the touched rows are grouped. Every per-component
            # reduction is a sort + scan: a component holding millions of rows
            # would serialise atomics on one address (a scatter "amin" of the
            # first-member keys took 119 ms at 10M rows / 20M edges).
            src, dst = self.e["src"], self.e["dst"]
            lab = T.components(src, dst, n).to(dev).long()
            touched = torch.zeros(n, dtype=torch.bool, device=dev)
            touched[src.long()] = True
            touched[dst.long()] = True
            # members: live nodes and ghost endpoints (the DFS follows edges to them)
            rows = torch.nonzero(touched & (self.kind[:n] != FREE)).flatten()
            if rows.numel() == 0:
                return []
            o = torch.argsort(lab[rows], stable=True)
            rows = rows[o]  # grouped by component, row order inside each group
            L = lab[rows]
            newg = torch.ones_like(L, dtype=torch.bool)
            newg[1:] = L[1:] != L[:-1]
            gid = torch.cumsum(newg.long(), 0) - 1
            starts = torch.nonzero(newg).flatten()
            G = starts.numel()
            size = torch.diff(starts, append=starts.new_full((1,), L.numel()))
            wsum, wcnt = _seg_sum_count(lab[src.long()], self.e["w"], n)
            gl = L[starts]
            ok = (size >= min_size) & (wcnt[gl] > 0) & (wsum[gl] / wcnt[gl].clamp_min(1).double() > min_avg_w)
            # reference order: a component's first member in BufferGraph.nodes
            # order = the smallest (super ? 0 : shard + 1) * n + row among its
            # live nodes; min per group by one sort of (group, key) composites
            BIG = 1 << 62
            kind_r, sup_r = self.kind[rows], self.sup[rows] != 0
            okey = torch.where(sup_r, torch.zeros_like(rows), self.shard[rows].long() + 1) * max(n, 1) + rows
            node = kind_r == NODE
            kbits = max(1, int(okey.max()).bit_length() + 1)
            if kbits + max(1, G.bit_length()) <= 62:
                comp = gid * (1 << kbits) + torch.where(node, okey, torch.full_like(okey, (1 << kbits) - 1))
                cs = torch.sort(comp).values
                fk = cs[starts] & ((1 << kbits) - 1)
                first = torch.where(fk == (1 << kbits) - 1, torch.full_like(fk, BIG), fk)
            else:  # keys too wide to pack
                first = _seg_min(gid, torch.where(node, okey, torch.full_like(okey, BIG)), G, BIG)
            ok &= first < BIG
            cand = ok[gid] & node & ~sup_r
            ci = torch.nonzero(cand).flatten()
            if ci.numel() == 0:
                return []
            # rank of each candidate among its group's candidates (row order)
            cg = gid[ci]
            cnew = torch.ones_like(cg, dtype=torch.bool)
            cnew[1:] = cg[1:] != cg[:-1]
            cstart = torch.nonzero(cnew).flatten()[torch.cumsum(cnew.long(), 0) - 1]
            sel = ci[(torch.arange(ci.numel(), device=dev) - cstart) < take]
            rowsv, key = rows[sel], first[gid[sel]]
            o = torch.argsort(key * n + rowsv)  # (component order, row): at most take rows per component
            rows_h, key_h = rowsv[o].cpu().numpy(), key[o].cpu().numpy()
        cut = np.nonzero(np.diff(key_h))[0] + 1
        return np.split(rows_h, cut)

    # the O(edges) digest when the edges touch at most 1/DIGEST_LOCAL_FRAC of the rows
    DIGEST_LOCAL_FRAC = 8

    def _digest_local(self, min_size: int, take: int) -> bool:
        """The digest over the edges' endpoints only: one block for a few
        thousand edges (T.component_digest_small), the renumbered torch form
        while the edges touch at most 1/DIGEST_LOCAL_FRAC of the rows."""
        ne = self.num_edges
        return (self.on_gpu and min_size >= 2 and take >= 1 and not self._digest_sorted and ne > 0
                and (ne <= T.dg_small_max_edges() or 2 * ne * self.DIGEST_LOCAL_FRAC <= self.n))

    def _digest_local_dev(self, min_size: int, min_avg_w: float, take: int) -> torch.Tensor:
        n = self.n
        if self.num_edges <= T.dg_small_max_edges():  # one launch
            return T.component_digest_small(self.e["src"], self.e["dst"], self.e["w"], self.kind[:n], self.sup[:n],
                                            self.shard[:n], n, min_size, min_avg_w, take)
        return T.component_digest_local(self.e["src"], self.e["dst"], self.e["w"], self.kind[:n], self.sup[:n],
                                        self.shard[:n], min_size, min_avg_w, take)

    # ------------------------------------------------------------------ incremental components
    # Within one consolidation batch the components at every run_consolidation
    # point come from base labels computed ONCE per batch plus a union pass
    # over the few edges that are not stable, instead of a union-find over
    # every edge at every point (the persistent 20M-edge graph: ~43 points
    # per step, ~2 ms each). Exact: the base holds only edges that exist at
    # every point of the batch -- none incident to a batch victim, none that
    # the batch's decays could bring under the prune threshold, none added --
    # so each point's graph is the base plus its volatile edges, and labels
    # (smallest row per component) of a union-find warm-started from the
    # base's compressed labels are those of a full recompute.
    CC_INCREMENTAL = True
    _cc = None

    def cc_begin(self, victims, prune_threshold: Optional[float], keep: float, steps: int) -> bool:
        """Start a batch's incremental components: ``victims`` -- every row
        the batch may evict (rows < n; rows inserted later are volatile by
        index), ``prune_threshold`` / ``keep`` / ``steps`` -- the batch's decay
        (edges whose weight could fall below the threshold within ``steps``
        decays are volatile). Only on the GPU digest path over many edges
        (the O(edges) local digest needs no labels); returns whether it is on."""
        if not (self.on_gpu and self.CC_INCREMENTAL) or self.n == 0 or self.num_edges == 0:
            return False
        if self._digest_local(3, 1) or self._digest_sorted:
            return False
        from ..ops.graph_ops import components_sel
        n0 = self.n
        t0 = -math.inf
        if prune_threshold is not None and prune_threshold > 0.0:
            t0 = float(prune_threshold) * float(keep) ** (-int(steps)) * (1.0 + 1e-4) + 1e-12
        with self.on_stream():
            vmark = torch.zeros(n0, dtype=torch.uint8, device=self.device)
            v = torch.as_tensor(np.asarray(victims, dtype=np.int64).reshape(-1))
            v = v[(v >= 0) & (v < n0)]
            if v.numel():
                vmark[v.to(self.device)] = 1
            ns = None
            if self.PARTITION_EDGES:
                from ..utils.tracing import tracer
                with tracer.stage("cc_partition", self.device):
                    ns = self._partition_stable(vmark, t0)
            if ns is not None:  # base labels: the stable prefix, every edge of it
                zero = torch.zeros(n0, dtype=torch.uint8, device=self.device)
                lab = components_sel(self.e["src"][:ns], self.e["dst"][:ns], n0, None, -math.inf, zero, n0, 0)
            else:
                lab = components_sel(self.e["src"], self.e["dst"], n0, self.e["w"], t0, vmark, n0, 0)
        self._cc = {"lab": lab, "n0": n0, "vmark": vmark, "t0": t0, "keep": float(keep), "steps": 0, "ns": ns}
        return True

    # Within a batch of the incremental components, the edge list is stably
    # partitioned: the edges that survive the whole batch first (never removed,
    # never pruned: cc_begin's definition), the volatile ones after them. Every
    # removal of the batch (victims' edges, decay prunes) and every append then
    # happens in the suffix, so the segment ends flag and compact only the
    # suffix, and each point unions only the suffix -- instead of passing over
    # all 20M edges of a persistent graph twice per point. Edge order carries
    # no meaning (_maybe_sort_edges); the partition keeps src order inside
    # each side.
    PARTITION_EDGES = True

    def _partition_stable(self, vmark: torch.Tensor, t0: float) -> Optional[int]:
        """Stable partition of the edges into (stable | volatile), in place
        of the edge list; returns the stable count (None: nothing to split)."""
        e = self.e
        ne = int(e["src"].numel())
        if ne == 0:
            return None
        # (int32 indices throughout: the gathers move half the index bytes)
        vol = (torch.index_select(vmark, 0, e["src"]) | torch.index_select(vmark, 0, e["dst"])) != 0
        if t0 > -math.inf:
            vol |= e["w"] < t0
        nv = int(vol.sum())
        if nv == ne:
            return None
        src = e["src"]
        if int((src[1:] < src[:-1]).sum()) * 32 > ne:
            # not (nearly) src-ordered: one stable sort by (volatile, src) --
            # the union-find runs ~5x faster over src-ordered edges, and
            # _maybe_sort_edges does not run while the partition is in place
            o = torch.sort(vol.to(torch.int64) * (1 << 32) + src.to(torch.int64), stable=True).indices
            o = o.to(torch.int32)
        elif nv == 0:
            return ne
        else:
            o = torch.cat([torch.nonzero(~vol).flatten(), torch.nonzero(vol).flatten()]).to(torch.int32)
        extra = max(ne >> 3, self.EDGE_SLACK_MIN)
        out = {}
        for k in T.EDGE_COLS:
            buf = torch.empty(ne + extra, dtype=e[k].dtype, device=self.device)
            torch.index_select(e[k], 0, o, out=buf[:ne])
            out[k] = buf[:ne]
        self._adopt_edges(out)
        self._bump(edges=True)
        return ne - nv

    def cc_end(self) -> None:
        self._cc = None

    def _cc_labels(self) -> torch.Tensor:
        """This point's labels: the base's, rows inserted since as singletons,
        then the volatile edges' unions (weights decayed by the segments run
        since cc_begin: the threshold follows them, with slack)."""
        from ..ops.graph_ops import components_sel
        c = self._cc
        n, n0 = self.n, c["n0"]
        lab = torch.empty(n, dtype=torch.int32, device=self.device)
        lab[:n0] = c["lab"]
        if n > n0:
            lab[n0:] = torch.arange(n0, n, dtype=torch.int32, device=self.device)
        ns = c.get("ns")
        if ns is not None and ns <= self.num_edges:  # every suffix edge, on the base of the stable prefix
            z = c.get("zero")
            if z is None or z.numel() < n:
                z = c["zero"] = torch.zeros(max(n, n0 + 65536), dtype=torch.uint8, device=self.device)
            return components_sel(self.e["src"][ns:], self.e["dst"][ns:], n, None, -math.inf, z, n, 0, parent=lab)
        wthr = c["t0"] * c["keep"] ** c["steps"] * (1.0 + 1e-4) if c["t0"] > -math.inf else -math.inf
        return components_sel(self.e["src"], self.e["dst"], n, self.e["w"], wthr, c["vmark"], n0, 1, parent=lab)

    def digest_capture(self, min_size: int = 3, min_avg_w: float = 0.3, take: int = 10) -> Capture:
        """:meth:`component_digest` as a :class:`Capture`: on the GPU with
        few edges (the O(edges) digest, ops.tenant_ops.component_digest_local)
        nothing waits for the device; otherwise the lists are computed now."""
        if self.n and self._digest_local(min_size, take):
            with self.on_stream():
                return Capture(self._digest_local_dev(min_size, min_avg_w, take), fn=T.digest_lists)
        return Capture(host=self.component_digest(min_size, min_avg_w, take))

    def component_edge_stats(self, comps: List[np.ndarray]) -> Tuple[np.ndarray, np.ndarray]:
        """(sum of weights, count) of edges with both endpoints in the same
        component, per component (reference memory_system.py:970-985)."""
        C = len(comps)
        if C == 0 or self.num_edges == 0:
            return np.zeros(C), np.zeros(C, dtype=np.int64)
        cid = np.full(self.n, -1, dtype=np.int64)
        for i, g in enumerate(comps):
            cid[g] = i
        with self.on_stream():
            cid_t = torch.as_tensor(cid).to(self.device)
            cs, ct = cid_t[self.e["src"].long()], cid_t[self.e["dst"].long()]
            ok = (cs >= 0) & (cs == ct)
            wsum, wcnt = _seg_sum_count(cs[ok], self.e["w"][ok], C)
            return wsum.cpu().numpy(), wcnt.cpu().numpy()

    # ------------------------------------------------------------------ search
    def unit_rows(self) -> bool:
        return self.max_norm_dev < 1e-3

    def _exact_cos(self, Qn: torch.Tensor, mask: torch.Tensor, k: int, row_label=None, q_label=None,
                   chunk: int = 1 << 18):
        """Exact float64 cosine top-k (ties -> lower row). Qn: unit fp64 [M, D]."""
        M = Qn.shape[0]
        n = self.n
        dev = self.device
        best_s = torch.full((M, 0), NEG_INF, dtype=torch.float64, device=dev)
        best_i = torch.zeros((M, 0), dtype=torch.long, device=dev)
        for c0 in range(0, n, chunk):
            c1 = min(n, c0 + chunk)
            X = self.emb32[c0:c1].double()
            nrm = self.sqn[c0:c1].double().sqrt()
            s = (Qn @ X.T) / torch.where(nrm > 0, nrm, torch.ones_like(nrm))[None, :]
            ok = mask[c0:c1][None, :].expand(M, -1)
            if row_label is not None:
                ok = ok & (row_label[c0:c1][None, :] == q_label[:, None])
            s = torch.where(ok, s, torch.full_like(s, NEG_INF))
            idx = torch.arange(c0, c1, device=dev).expand(M, -1)
            cs, ci = torch.cat([best_s, s], 1), torch.cat([best_i, idx], 1)
            o = torch.sort(cs, dim=1, descending=True, stable=True).indices[:, :k]
            best_s, best_i = torch.gather(cs, 1, o), torch.gather(ci, 1, o)
        return self._pad_k(best_s, best_i, k)

    @staticmethod
    def _pad_k(s, i, k):
        M = s.shape[0]
        if s.shape[1] < k:
            pad = k - s.shape[1]
            s = torch.cat([s, torch.full((M, pad), NEG_INF, dtype=s.dtype, device=s.device)], 1)
            i = torch.cat([i, torch.full((M, pad), -1, dtype=torch.long, device=i.device)], 1)
        i = torch.where(torch.isneginf(s), torch.full_like(i, -1), i)
        return s, i

    def _rerank_cos(self, Qn: torch.Tensor, cand: torch.Tensor, k: int):
        """Exact float64 cosine of kernel candidates ``cand`` [M, c] (-1 empty),
        sorted (score desc, row asc), cut to k. GPU: one launch
        (tenant.hip cos_rerank64_kernel)."""
        if self.on_gpu and cand.is_cuda and cand.shape[1] <= 64 and k <= cand.shape[1] and RERANK64_KERNEL:
            from ..ops import _lib
            M, C = cand.shape
            qd = Qn.to(self.device, torch.float64).contiguous()
            cd = cand.to(torch.long).contiguous()
            os_ = torch.empty((M, k), dtype=torch.float64, device=self.device)
            oi = torch.empty((M, k), dtype=torch.long, device=self.device)
            _lib.check(_lib.lib().lzk_cos_rerank64(qd.data_ptr(), qd.stride(0), self.emb32.data_ptr(),
                                                    self.emb32.stride(0), self.dim, self.sqn.data_ptr(), cd.data_ptr(),
                                                    C, M, k, os_.data_ptr(), oi.data_ptr(),
                                                    _lib.stream_ptr(self.device)), "lzk_cos_rerank64")
            return os_, oi
        valid = cand >= 0
        rows = cand.clamp_min(0)
        X = self.emb32[rows].double()  # [M, c, D]
        nrm = self.sqn[rows].double().sqrt()
        s = torch.einsum("md,mcd->mc", Qn, X) / torch.where(nrm > 0, nrm, torch.ones_like(nrm))
        s = torch.where(valid, s, torch.full_like(s, NEG_INF))
        key = torch.where(valid, cand, torch.full_like(cand, 1 << 62))
        o = torch.argsort(key, dim=1, stable=True)
        s, cand = torch.gather(s, 1, o), torch.gather(cand, 1, o)
        o = torch.sort(s, dim=1, descending=True, stable=True).indices[:, :k]
        return self._pad_k(torch.gather(s, 1, o), torch.gather(cand, 1, o), k)

    def _use_kernel(self, M: int) -> bool:
        return self.on_gpu and self.unit_rows() and M * self.n >= KERNEL_MIN_WORK

    def _q16(self, Qn: torch.Tensor) -> torch.Tensor:
        q = torch.zeros((Qn.shape[0], self.Dp), dtype=torch.bfloat16, device=self.device)
        q[:, : self.dim] = Qn.to(torch.bfloat16)
        return q

    def cos_topk(self, Q: torch.Tensor, k: int, mask: torch.Tensor, dual_label: Optional[torch.Tensor] = None,
                 min_score: Optional[float] = None):
        """Cosine top-k of each query row among rows where ``mask``. With
        ``dual_label`` (shard code per query) also returns the top-k restricted
        to rows of the query's shard, from the same scan. Scores are exact
        float64 (kernel candidates re-ranked). Returns (s, rows) or
        ((s, rows), (s_shard, rows_shard)).

        ``min_score``: the caller acts only on entries with cos >= min_score;
        the GPU dual scan may then leave lower-scoring slots empty (-inf, -1)
        instead of finding them. Every entry >= min_score is still returned
        exactly (the kernel threshold is lowered by COS_FLOOR_SLACK, which
        exceeds the bf16 score error of unit rows: |err| <= 2^-8)."""
        with self.on_stream():
            return self._cos_topk(Q, k, mask, dual_label, min_score)

    def _cos_topk(self, Q, k, mask, dual_label, min_score=None):
        from ..ops.search import flat_topk, flat_topk_dual
        M = Q.shape[0]
        n = self.n
        dev = self.device
        if n == 0 or M == 0 or self.dim is None:
            e = self._pad_k(torch.zeros((M, 0), dtype=torch.float64, device=dev),
                            torch.zeros((M, 0), dtype=torch.long, device=dev), k)
            return (e, e) if dual_label is not None else e
        Qd = Q.to(dev, torch.float64)
        qn = Qd.norm(dim=1, keepdim=True)
        Qn = Qd / torch.where(qn > 0, qn, torch.ones_like(qn))
        lab = self.shard[:n]
        lean = self.lean
        if lean and not self.unit_rows():  # (no bf16 rows; the int8 error model needs unit rows)
            pass
        elif (self._use_kernel(M) or lean) and k <= CAND_SLOTS:
            if dual_label is not None:
                ra, rb = self._dual_cands(Qn, mask, dual_label, min_score)
                return self._rerank_cos(Qn, ra, k), self._rerank_cos(Qn, rb, k)
            bias = torch.where(mask, 0.0, NEG_INF).to(torch.float32).contiguous()
            q16 = self._q16(Qn)
            X = self._scan_rows(n, Qn)
            lean_w = 2.0 ** -8 * (1.0 + self.max_norm_dev) if self.emb16 is None else 0.0
            if lean:
                from ..ops.search import flat_topk_i8
                q8, qs, margin, margin_rig = self._i8_query(q16, 1.0)
                if self._lowp_exact(True):
                    margin = margin_rig
                else:
                    margin_rig = margin
                if lean_w:
                    margin, margin_rig = (margin + lean_w).contiguous(), (margin_rig + lean_w).contiguous()
                _, ra = flat_topk_i8(self.emb8, self.rs8, q8, qs, X, q16, CAND_SLOTS, bias=bias, margin=margin,
                                     margin_rig=margin_rig)
            else:
                _, ra = flat_topk(X, q16, CAND_SLOTS, bias=bias)
            return self._rerank_cos(Qn, ra, k)
        if dual_label is not None:
            ql = dual_label.to(dev, torch.int32)
            return (self._exact_cos(Qn, mask, k), self._exact_cos(Qn, mask, k, row_label=lab, q_label=ql))
        return self._exact_cos(Qn, mask, k)

    def _dual_cands(self, Qn: torch.Tensor, mask: torch.Tensor, dual_label: torch.Tensor,
                    min_score: Optional[float], keep=None):
        """The candidate scan of the dual :meth:`cos_topk` (kernel path):
        CAND_SLOTS rows per query for list A (every row in ``mask``) and list
        B (rows of the query's shard), holding each list's exact top-k (and
        every entry >= ``min_score``) for the exact float64 re-rank.
        ``keep``: a list that receives the tensors the scan reads (a caller
        running it on a side stream protects them from reuse)."""
        dev = self.device
        n = self.n
        M = Qn.shape[0]
        lab = self.shard[:n]
        lean = self.lean
        bias = torch.where(mask, 0.0, NEG_INF).to(torch.float32).contiguous()
        q16 = self._q16(Qn)
        X = self._scan_rows(n, Qn)
        # lean: the int8 scans' re-score reads fp32 rows with fp32 queries
        # while their threshold sample and margin are bf16-based, so every
        # int8 margin below also covers |<q16, x16> - <q, x>| <= 2^-8 |q| |x|
        # (both operands rounded to bf16; unit queries) -- as _i8_candidates
        lean_w = 2.0 ** -8 * (1.0 + self.max_norm_dev) if self.emb16 is None else 0.0
        ql = dual_label.to(dev, torch.int32).contiguous()
        floor = None if min_score is None else float(min_score) - COS_FLOOR_SLACK
        labc = lab.contiguous()
        if keep is not None:
            keep += [bias, q16, X, ql, labc, self.emb32, self.sqn]
        if lean or (DUAL_LOWP and self.emb8 is not None and self.emb8.dtype == torch.int8
                    and self.unit_rows() and M >= LOWP_MIN_Q and n >= LOWP_MIN_ROWS
                    and self._dual_lowp_ok()):
            # the int8 dual scan: same lists (error cut + bf16 re-score)
            from ..ops.search import flat_topk_dual_i8
            q8, qs, margin, margin_rig = self._i8_query(q16, 1.0)
            if self._lowp_exact(True):  # consolidation's decisions: the worst-case bound by default
                margin = margin_rig
            else:
                margin_rig = margin
            if lean_w:
                margin, margin_rig = (margin + lean_w).contiguous(), (margin_rig + lean_w).contiguous()
            st = [] if (DUAL_LOWP_AUTO and not lean) else None
            if keep is not None:
                keep += [self.emb8, self.rs8, q8, qs, margin, margin_rig]
            (_, ra), (_, rb) = flat_topk_dual_i8(self.emb8, self.rs8, q8, qs, X, q16, CAND_SLOTS,
                                                 row_label=labc, q_label=ql, bias=bias,
                                                 margin=margin, margin_rig=margin_rig, floor=floor,
                                                 floor_tol=0.5 * COS_FLOOR_SLACK, stats=st)
            if st:
                self._dual_stats = st
        else:
            from ..ops.search import flat_topk_dual
            (_, ra), (_, rb) = flat_topk_dual(X, q16, CAND_SLOTS, row_label=labc, q_label=ql,
                                              bias=bias, floor=floor)
        return ra, rb

    # ------------------------------------------------------------------ prefetched candidate scans
    def dual_prefetch_ok(self, M: int, k: int) -> bool:
        """Whether :meth:`cos_topk_prefetch` applies (the dual kernel path)."""
        return (self.on_gpu and self.n > 0 and M > 0 and self.dim is not None and k <= CAND_SLOTS
                and not (self.lean and not self.unit_rows()) and (self._use_kernel(M) or self.lean))

    def cos_topk_prefetch(self, Q: torch.Tensor, mask: torch.Tensor, dual_label: torch.Tensor,
                          min_score: Optional[float], stream) -> Dict:
        """The candidate scan of a dual :meth:`cos_topk` launched on
        ``stream`` against the rows as they are now; :meth:`cos_topk_finish`
        completes it after the graph changed by row INSERTS (rows >= the
        current n) and rows leaving ``mask`` only -- one consolidation batch.
        The caller reserves the rows the batch inserts first (no column
        reallocation under the running scan)."""
        from ..ops import search as S
        dev = self.device
        cur = torch.cuda.current_stream(dev)
        Qd = Q.to(dev, torch.float64)
        qn = Qd.norm(dim=1, keepdim=True)
        Qn = Qd / torch.where(qn > 0, qn, torch.ones_like(qn))
        stream.wait_stream(cur)
        keep: List[torch.Tensor] = [Qn, mask]
        with torch.cuda.stream(stream), S.grid_cap(S.PREFETCH_GRID_FRAC):
            st0 = self._dual_stats
            ra, rb = self._dual_cands(Qn, mask, dual_label, min_score, keep=keep)
            ev = torch.cuda.Event()
            ev.record(stream)
            if self._dual_stats is not None and self._dual_stats is not st0:
                self._dual_stats_ev = ev
        for t in keep + [ra, rb]:
            if t is not None and t.is_cuda:
                t.record_stream(cur)
                t.record_stream(stream)
        return {"n": self.n, "ra": ra, "rb": rb, "ev": ev, "Qn": Qn, "Q": Q, "ql": dual_label.to(dev, torch.int32),
                "min_score": min_score, "keep": keep}

    def cos_topk_finish(self, h: Dict, k: int, mask: torch.Tensor):
        """(list A, list B) of a prefetched dual scan against the graph NOW
        (``mask``: the rows allowed now), exactly :meth:`cos_topk`'s lists
        for every entry the caller acts on (>= its min_score): a query whose
        candidates hold a row that left the mask is recomputed by a fresh
        scan; for the others the candidates still hold the exact top-k of
        the remaining rows, and the rows inserted since join them through
        the same float64 re-rank kernel (64-row chunks), merged by (score
        desc, row asc)."""
        from ..utils.tracing import tracer
        dev = self.device
        if tracer.enabled:  # how long the host would wait for the prefetched scan here
            with tracer.stage("cb_prefetch_wait", "cpu"):
                h["ev"].synchronize()
        torch.cuda.current_stream(dev).wait_event(h["ev"])
        n0, n = h["n"], self.n
        Qn, ra, rb, ql = h["Qn"], h["ra"], h["rb"], h["ql"]
        parts = [[self._rerank_cos(Qn, ra, k)], [self._rerank_cos(Qn, rb, k)]]
        if n > n0:
            pa, pb = self._new_rows_parts(Qn, ql, mask, n0, k, h["min_score"])
            parts[0] += pa
            parts[1] += pb
        outs = [self._merge_parts(pl, k) for pl in parts]
        # queries whose candidates lost a row: a fresh scan of the graph now
        gone_a = (ra >= 0) & ~mask[ra.clamp(0, n - 1)]
        gone_b = (rb >= 0) & ~mask[rb.clamp(0, n - 1)]
        aff = torch.nonzero(gone_a.any(1) | gone_b.any(1)).flatten()
        if aff.numel():
            with tracer.stage("cb_prefetch_affected", dev):
                (sa, ia), (sb, ib) = self._cos_topk(h["Q"][aff], k, mask, ql[aff], h["min_score"])
            outs[0][0][aff], outs[0][1][aff] = sa, ia
            outs[1][0][aff], outs[1][1][aff] = sb, ib
        h.clear()
        return (outs[0][0], outs[0][1]), (outs[1][0], outs[1][1])

    def _new_rows_parts(self, Qn, ql, mask, n0: int, k: int, min_score):
        """Per-query exact top-k lists (list A, list B as parts to merge) over
        the rows >= ``n0`` allowed by ``mask`` only: the float64 re-rank kernel
        on 64-row blocks, rows that cannot reach ``min_score`` (fp32 cosine
        with slack) left out first."""
        dev = self.device
        n = self.n
        M = Qn.shape[0]
        new = torch.nonzero(mask[n0:n]).flatten() + n0
        nn_ = new.numel()
        ca_all = new[None, :].expand(M, nn_)
        cb_all = torch.where(self.shard[:n][new][None, :] == ql[:, None], ca_all, torch.full_like(ca_all, -1))
        if min_score is not None and nn_:
            # only rows that can reach min_score (the caller acts on entries
            # >= min_score only) go to the exact re-rank, compacted to the front
            Xn = self.emb32[new, : self.dim].float()
            nrm = self.sqn[new].float().sqrt()
            S32 = (Qn.float() @ Xn.T) / torch.where(nrm > 0, nrm, torch.ones_like(nrm))[None, :]
            near = S32 >= float(min_score) - 1e-3
            ca_all = torch.where(near, ca_all, torch.full_like(ca_all, -1))
            cb_all = torch.where(near, cb_all, torch.full_like(cb_all, -1))
            width = int(near.sum(1).max())  # one host read
            o = torch.argsort((ca_all < 0).to(torch.uint8), dim=1, stable=True)[:, : max(width, 1)]
            ca_all = torch.gather(ca_all, 1, o)
            o = torch.argsort((cb_all < 0).to(torch.uint8), dim=1, stable=True)[:, : max(width, 1)]
            cb_all = torch.gather(cb_all, 1, o)
        pa, pb = [], []
        w = ca_all.shape[1]
        for a in range(0, w, 64):  # the re-rank kernel takes 64 candidates per query
            for out, cc in ((pa, ca_all), (pb, cb_all)):
                blk = torch.full((M, 64), -1, dtype=torch.long, device=dev)
                blk[:, : min(64, w - a)] = cc[:, a:a + 64]
                out.append(self._rerank_cos(Qn, blk, k))
        return pa, pb

    def _merge_parts(self, parts, k: int):
        """Top-k of several (score, row) lists by (score desc, row asc), as
        _rerank_cos orders."""
        if len(parts) == 1:
            return list(parts[0])
        s_ = torch.cat([p[0] for p in parts], 1)
        r_ = torch.cat([p[1] for p in parts], 1)
        key = torch.where(r_ >= 0, r_, torch.full_like(r_, 1 << 62))
        o = torch.argsort(key, dim=1, stable=True)
        s_, r_ = torch.gather(s_, 1, o), torch.gather(r_, 1, o)
        o = torch.sort(s_, dim=1, descending=True, stable=True).indices[:, :k]
        return list(self._pad_k(torch.gather(s_, 1, o), torch.gather(r_, 1, o), k))

    def cos_topk_new_rows(self, Q: torch.Tensor, k: int, mask: torch.Tensor, n0: int, dual_label: torch.Tensor,
                          min_score: Optional[float]):
        """The dual :meth:`cos_topk` lists restricted to rows >= ``n0``
        (entries >= ``min_score`` exact): for queries whose lists over the
        older rows are known to hold nothing at that score."""
        dev = self.device
        Qd = Q.to(dev, torch.float64)
        qn = Qd.norm(dim=1, keepdim=True)
        Qn = Qd / torch.where(qn > 0, qn, torch.ones_like(qn))
        ql = dual_label.to(dev, torch.int32)
        M = Qn.shape[0]
        e = self._pad_k(torch.zeros((M, 0), dtype=torch.float64, device=dev),
                        torch.zeros((M, 0), dtype=torch.long, device=dev), k)
        if self.n <= n0:
            return (e[0].clone(), e[1].clone()), (e[0].clone(), e[1].clone())
        pa, pb = self._new_rows_parts(Qn, ql, mask, n0, k, min_score)
        return tuple(self._merge_parts([e] + pa, k)), tuple(self._merge_parts([e] + pb, k))

    _dual_stats = None  # (ovf, cnt) x 2 + cap of the last int8 dual scan (auto mode)
    _dual_stats_ev = None  # the side-stream event after a prefetched scan that wrote _dual_stats
    _dual_bf16 = 0  # calls left on the bf16 dual scan (auto mode back-off)

    def _dual_lowp_ok(self) -> bool:
        """Auto mode: read the last int8 dual call's list statistics (its
        kernels finished long ago) and back off to bf16 for DUAL_BACKOFF
        calls when lists overflowed or ran long."""
        if not DUAL_LOWP_AUTO:
            return True
        if self._dual_stats is not None:
            (oa, ca), (ob, cb), cap = self._dual_stats
            self._dual_stats = None
            ev, self._dual_stats_ev = self._dual_stats_ev, None
            if ev is not None:  # written by a prefetched scan on its side stream
                torch.cuda.current_stream(self.device).wait_event(ev)
            with self.on_stream():
                m = torch.stack([((oa != 0) | (ob != 0)).float().mean(),
                                 ((ca & 0x3FFFFFFF).clamp_max(cap).float().mean()
                                  + (cb & 0x3FFFFFFF).clamp_max(cap).float().mean()) / (2 * cap)]).cpu()
            if float(m[0]) > DUAL_OVF_MAX or float(m[1]) > 0.25:
                self._dual_bf16 = DUAL_BACKOFF
        if self._dual_bf16 > 0:
            self._dual_bf16 -= 1
            return False
        return True

    def store_bias(self, metric: str) -> torch.Tensor:
        """Per-row fp32 score bias of the store search: -inf for rows not in
        the store; -|x|^2 for L2 (scores = 2<q,x> - |x|^2)."""
        c = self._bias_cache.get(metric)
        if c is not None and c[0] == self._store_version and c[1].numel() == self.n:
            return c[1]
        n = self.n
        ok = (self.stored[:n] == 1) & (self.kind[:n] != FREE)
        b = torch.where(ok, 0.0, NEG_INF).to(torch.float32)
        if metric == "l2":
            b = b - self.sqn[:n]
        b = b.contiguous()
        self._bias_cache[metric] = (self._store_version, b)
        return b

    def store_search(self, Q: torch.Tensor, k: int, metric: str = "l2", node_rows: bool = False):
        """The store's vector search over this tenant (reference
        ``LanceDBStore.search_nodes``: flat scan, L2 unless told otherwise,
        vector_store.py:132-140). fp32 scores -- -|q-x|^2 for L2, cosine, or
        dot -- higher is closer; bf16 MFMA candidates are re-ranked in fp32.
        Returns (scores [M, k], rows [M, k]). ``node_rows``: rows that are not
        graph nodes come back as -1 (search_memories skips them, reference
        memory_system.py:1467-1472) -- inside the re-rank kernel when it runs."""
        with self.on_stream():
            s, r = self._store_search(Q, k, metric, node_rows)
            if node_rows and not self._nodes_marked:
                r = torch.where((r >= 0) & (self.kind[r.clamp_min(0)] == NODE), r, torch.full_like(r, -1))
            self._nodes_marked = False
            return s, r

    _nodes_marked = False  # the last _store_search already marked non-node rows (re-rank kernel)

    def _store_search(self, Q, k, metric, node_rows=False):
        from ..ops.search import flat_topk
        n = self.n
        dev = self.device
        Qf = Q.to(dev, torch.float32)
        if Qf.dim() == 1:
            Qf = Qf[None, :]
        M = Qf.shape[0]
        if n == 0 or self.dim is None or Qf.shape[1] != self.dim:
            return self._pad_k(torch.zeros((M, 0), device=dev), torch.zeros((M, 0), dtype=torch.long, device=dev), k)
        if metric == "cosine":
            qn = Qf.norm(dim=1, keepdim=True)
            Qf = Qf / torch.where(qn > 0, qn, torch.ones_like(qn))
        bias = self.store_bias("l2" if metric == "l2" else "ip")
        alpha = 2.0 if metric == "l2" else 1.0
        cfg = self.ann_cfg
        if cfg is not None and n >= cfg["min_rows"] and self.unit_rows():
            # IVF-PQ candidates (the store's index="ivfpq"), re-ranked exactly
            # in fp32 against this graph's rows with the store's row mask
            cand = self._ann_candidates(Qf, max(cfg.get("rerank", 1024), k), cfg)
            return self._rerank_store(Qf, cand, k, metric, bias)
        kc = CAND_SLOTS  # the fp32 re-rank sees 16 bf16 candidates for every k <= 16
        if self.on_gpu and k <= CAND_SLOTS and (metric != "cosine" or self.unit_rows()) \
                and M * n >= KERNEL_MIN_WORK // 16:
            q16 = self._q16(Qf)
            narrow = LOWP_NARROW and self.emb8 is not None and self.emb8.dtype == torch.int8
            if self.lean and not self.unit_rows():
                return self._exact_store(Qf, k, metric, bias)  # (no bf16 rows to scan; the error model needs unit rows)
            if self.lean or (self.emb8 is not None and self.unit_rows() and (M >= LOWP_MIN_Q or narrow)
                             and n >= LOWP_MIN_ROWS):
                if self.emb8.dtype == torch.int8:
                    _, cand = self._i8_candidates(Qf, q16, kc, bias, alpha)
                else:
                    _, cand = self._fp8_candidates(Qf, q16, kc, bias, alpha)
            else:
                _, cand = flat_topk(self.emb16[:n], q16, kc, bias=bias, alpha=alpha)
            return self._rerank_store(Qf, cand, k, metric, bias, node_rows)
        return self._exact_store(Qf, k, metric, bias)

    def _ann_candidates(self, Qf: torch.Tensor, R: int, cfg: Dict) -> torch.Tensor:
        """Graph rows [M, R] from the tenant's IVF-PQ index, built on first
        use over the unit rows (ids = rows) and extended with the rows
        appended since; rebuilt when an embedding was rewritten in place.
        Removed / unstored rows stay in the index and are dropped by the
        re-rank's -inf bias."""
        from ..index.ivfpq import IVFPQIndex
        n = self.n
        idx = self._ann
        if idx is None or self._ann_stale or self._ann_covered > n:
            m = cfg["m"] if self.dim % cfg["m"] == 0 else next(d for d in (64, 48, 32, 16, 8) if self.dim % d == 0)
            nlist = max(16, min(cfg["nlist"], n // 64))
            idx = IVFPQIndex(self.dim, nlist=nlist, m=m, device=self.device)
            live = torch.nonzero(self.has_emb[:n] == 1).flatten()
            g = torch.Generator(device="cpu").manual_seed(0)
            pick = live[torch.randperm(live.numel(), generator=g)[: min(live.numel(), 262144)].to(live.device)]
            idx.train(self.emb32[pick], iters=8, pq_iters=8)
            idx.reserve(n)
            self._ann, self._ann_covered, self._ann_stale = idx, 0, False
        step = 1 << 20
        while self._ann_covered < n:
            r1 = min(n, self._ann_covered + step)
            idx.add(self.emb32[self._ann_covered:r1], ids=torch.arange(self._ann_covered, r1))
            self._ann_covered = r1
        return idx.candidate_ids(Qf, R, cfg["nprobe"])

    def _lowp_exact(self, default: bool) -> bool:
        m = getattr(self, "LOWP_EXACT_MODE", None) or LOWP_EXACT
        return True if m == "1" else False if m == "0" else default

    def _i8_candidates(self, Qf: torch.Tensor, q16: torch.Tensor, kc: int, bias: torch.Tensor, alpha: float):
        """Store-search candidates from the int8 scan (``emb8`` / ``rs8``),
        re-scored from the bf16 rows above the error cut and certified per
        query (ops.search.flat_topk_i8), with the worst-case margin of
        :meth:`_i8_query` (the result is the bf16 search's for ANY data) or
        the statistical one (wide batches by default, see LOWP_EXACT)."""
        from ..ops.search import NARROW_MAX_Q, flat_topk_i8
        q8, qs, margin, margin_rig = self._i8_query(q16, alpha)
        if not self._lowp_exact(Qf.shape[0] < NARROW_MAX_Q):
            margin_rig = margin
        else:
            margin = margin_rig
        if self.emb16 is None:
            # lean: the re-score reads the fp32 rows, so both margins also cover
            # |<q16, x16> - <q, x>| <= 2^-8 |q| |x| (both operands rounded to bf16)
            w = alpha * 2.0 ** -8 * Qf.norm(dim=1) * (1.0 + self.max_norm_dev)
            margin, margin_rig = (margin + w).contiguous(), (margin_rig + w).contiguous()
        return flat_topk_i8(self.emb8, self.rs8, q8, qs, self._scan_rows(self.n, Qf), q16, kc, bias=bias,
                            alpha=alpha, margin=margin, margin_rig=margin_rig)

    def _i8_query(self, q16: torch.Tensor, alpha: float):
        """int8 queries, per-query scales and the two error margins of the
        int8 scans (device tensors, no host sync). Error of the int8 score
        against the bf16 one, with the query's rounding error eta (known
        exactly) and a row's rounding error delta (|delta_i| <= s / 2, s <= the
        largest row scale s_max ever written):
          <x^, q^> - <x, q> = <x, eta> + <delta, q> + <delta, eta>
        * statistical (the scan threshold): var <x, eta> = sum_i eta_i^2
          E[x_i^2] (per-dimension second moments of the tenant's rows),
          var <delta, q> <= |q|^2 s_max^2 / 12; LOWP_MARGIN_Z standard
          deviations plus the worst case s_max / 2 |eta|_1 of the last term;
        * worst case (cut + certificate): |x| |eta| + s_max / 2 |q|_1 +
          s_max / 2 |eta|_1 + the fp32 accumulation error of the re-score,
          rows of norm <= 1 + max_norm_dev (bf16-rounded).
        Returns (q8, qs, margin, margin_rig)."""
        from ..ops.search import i8_query, quantize_i8_rows
        d = self.dim
        xn = 1.0 + self.max_norm_dev + 2.0 ** -7
        if self.on_gpu and I8_QUERY_KERNEL and (q16.shape[0] < I8_QUERY_WIDE_MIN or I8_QUERY_WIDE):
            # one launch (search256.hip i8_query_kernel): the narrow batches, where
            # the ~25 torch launches it replaces are most of the query-side time
            return i8_query(q16, d, self.sumsq, self.n_sumsq, self._rs8_max, alpha, LOWP_MARGIN_Z, xn)
        q8, qs = quantize_i8_rows(q16)
        qf = q16.float()
        eta = q8.float() * qs[:, None] - qf
        mu2 = (self.sumsq / max(self.n_sumsq, 1)).float()
        smax = self._rs8_max
        floor = 0.5 * smax * eta.abs().sum(1)
        a = abs(alpha)
        v1 = (eta[:, :d] ** 2 * mu2[None, :]).sum(1)
        q2 = (qf ** 2).sum(1)
        margin = (a * (LOWP_MARGIN_Z * torch.sqrt(v1 + q2 * (smax * smax / 12.0)) + floor)).contiguous()
        bound = eta[:, :d].norm(dim=1) * xn + 0.5 * smax * qf.abs().sum(1) + floor + d * 2.0 ** -23 * xn * q2.sqrt()
        margin_rig = (a * bound * (1.0 + 1e-5) + 1e-6).contiguous()
        return q8, qs, margin, margin_rig

    def _fp8_candidates(self, Qf: torch.Tensor, q16: torch.Tensor, kc: int, bias: torch.Tensor, alpha: float):
        """Store-search candidates from the fp8 scan (rows in ``emb8``),
        re-scored from the bf16 rows. The threshold margin covers the fp8
        rounding of rows and queries: with relative rounding error u = 2^-4
        per element (e4m3), <q,x> is off by about
        u * sqrt(2/3) * sqrt(sum_i q_i^2 E[x_i^2]) (E over the tenant's rows,
        tracked per dimension); the margin is FP8_MARGIN_Z of those, plus the
        subnormal floor."""
        from ..ops.search import flat_topk_fp8, quantize_e4m3
        n = self.n
        qmax = float(Qf.abs().max().clamp_min(1e-30))
        sq = 64.0 / qmax
        q8 = torch.zeros((Qf.shape[0], self.Dp), dtype=torch.uint8, device=self.device)
        q8[:, : self.dim] = quantize_e4m3(Qf, sq)
        mu2 = (self.sumsq / max(self.n_sumsq, 1)).to(torch.float64)
        sig = (2.0 / 3.0) ** 0.5 * 2.0 ** -4 * torch.sqrt((Qf.double() ** 2 * mu2[None, :]).sum(1))
        floor = 2.0 ** -9 * (1.0 / self.FP8_ROW_SCALE + 1.0 / sq) * Qf.double().abs().sum(1).clamp_min(1.0)
        margin = (abs(alpha) * (LOWP_MARGIN_Z * sig + floor)).float().contiguous()
        return flat_topk_fp8(self.emb8, q8, self.FP8_ROW_SCALE * sq, self.emb16[:n], q16, kc, bias=bias,
                             alpha=alpha, margin=margin)

    def _store_scores(self, Qf, X, sqn, bias, metric):
        dot = Qf @ X.T if X.dim() == 2 else torch.einsum("md,mcd->mc", Qf, X)
        if metric == "l2":
            return 2.0 * dot + bias - (Qf * Qf).sum(1, keepdim=True)
        if metric == "cosine":
            nrm = sqn.sqrt()
            return dot / torch.where(nrm > 0, nrm, torch.ones_like(nrm)) + bias
        return dot + bias

    def _exact_store(self, Qf, k, metric, bias, chunk: int = 1 << 18):
        n = self.n
        M = Qf.shape[0]
        best_s = torch.full((M, 0), NEG_INF, device=self.device)
        best_i = torch.zeros((M, 0), dtype=torch.long, device=self.device)
        for c0 in range(0, n, chunk):
            c1 = min(n, c0 + chunk)
            s = self._store_scores(Qf, self.emb32[c0:c1], self.sqn[c0:c1][None, :], bias[c0:c1][None, :], metric)
            idx = torch.arange(c0, c1, device=self.device).expand(M, -1)
            cs, ci = torch.cat([best_s, s], 1), torch.cat([best_i, idx], 1)
            o = torch.sort(cs, dim=1, descending=True, stable=True).indices[:, :k]
            best_s, best_i = torch.gather(cs, 1, o), torch.gather(ci, 1, o)
        return self._pad_k(best_s, best_i, k)

    def _rerank_store(self, Qf, cand, k, metric, bias, node_rows=False):
        if self.on_gpu and RERANK_KERNEL and 0 < cand.shape[1] <= 64 and metric in ("l2", "ip", "cosine"):
            from ..ops.tenant_ops import store_rerank
            self._nodes_marked = bool(node_rows)
            return store_rerank(Qf, self.emb32, self.sqn, bias, cand, k, metric,
                                kind=self.kind if node_rows else None)
        valid = cand >= 0
        rows = cand.clamp_min(0)
        s = self._store_scores(Qf, self.emb32[rows], self.sqn[rows], bias[rows], metric)
        s = torch.where(valid, s, torch.full_like(s, NEG_INF))
        key = torch.where(valid, cand, torch.full_like(cand, 1 << 62))
        o = torch.argsort(key, dim=1, stable=True)
        s, cand = torch.gather(s, 1, o), torch.gather(cand, 1, o)
        o = torch.sort(s, dim=1, descending=True, stable=True).indices[:, :k]
        return self._pad_k(torch.gather(s, 1, o), torch.gather(cand, 1, o), k)

    def search_ids(self, Q, k: int, metric: str = "l2") -> List[List[str]]:
        _, r = self.store_search(Q, k, metric)
        ids = self.ids
        return [[ids[x] for x in row if x >= 0] for row in r.cpu().tolist()]

    # ------------------------------------------------------------------ k-means hierarchy (K16)
    @property
    def hier(self) -> Optional[Dict]:
        """The k-means hierarchy of the last :meth:`cluster_pass` (joins a
        pass still running in the background)."""
        if self._hier_job is not None:
            self.cluster_join()
        return self._hier

    @hier.setter
    def hier(self, value) -> None:
        self.cluster_join()
        self._hier = value

    def has_hier(self) -> bool:
        """Whether a hierarchy exists or is being built (no join)."""
        return self._hier_job is not None or self._hier is not None

    def cluster_pass(self, n_fine: int = 4096, n_top: int = 64, iters: int = 2, seed: int = 0, comm=None,
                     background: bool = False) -> Dict:
        """Two-level hierarchical clustering of the live shard nodes (SURVEY.md
        §2.4 K16; ``MemorySystem(hierarchy_mode="kmeans")``): spherical k-means
        into ``n_fine`` clusters over the tenant's rows in place (fused MFMA
        argmax assign + sorted segment sums; dead rows masked, no gather),
        warm-started from the previous pass, then the fine centroids into
        ``n_top`` topic clusters -- the scalable form of the reference's one
        mean super-node per shard (memory_system.py:893-933). Keeps
        ``self.hier``: top centroids, each row's fine / top label and the
        rows ordered by (top cluster, row) for child lookups.

        ``comm`` (world > 1): the rows are one row-sharded tenant's local part;
        the fine level is the distributed k-means (centroid sums all-reduced,
        SURVEY.md §2.5 C4) and the topic level runs replicated on the
        identical fine centroids, so every rank holds the same hierarchy.

        ``background`` (one GPU tenant, no ``comm``): the pass reads the rows
        as they are NOW -- the live mask and ``n`` are taken on the graph
        stream here -- but runs on a side stream from a worker thread, so the
        graph's next segments (which only append rows >= n and flip flags of
        rows the mask already fixed; no row's vector below n changes) run
        under it. ``hier`` joins it; :meth:`has_hier` does not."""
        self.cluster_join()
        n = self.n
        if n == 0 or self.dim is None:
            return {}
        dist = comm is not None and (comm.world > 1 or comm.enabled)
        with self.on_stream():
            live = (self.kind[:n] == NODE) & (self.sup[:n] == 0) & (self.has_emb[:n] == 1)
            src = self.emb16[:n] if (self.on_gpu and self.emb16 is not None) else None
            if background and self.on_gpu and not dist:
                ev = torch.cuda.Event()
                ev.record()
                graph_st = torch.cuda.current_stream(self.device)
                st = _cluster_stream(self.device)
                prev = self._hier or {}
                version = self.version
                for t in (live, src):
                    if t is not None:
                        t.record_stream(st)
                emb32 = self.emb32[:n] if src is None else None
                if emb32 is not None:
                    emb32.record_stream(st)

                def work():
                    # a new thread starts on device 0: bind this tenant's GPU
                    # (multi-GPU processes) before any launch
                    with torch.cuda.device(self.device), torch.cuda.stream(st):
                        st.wait_event(ev)
                        out = self._cluster_compute(live, src, emb32, n, n_fine, n_top, iters, seed, None, prev,
                                                    version)
                        done = torch.cuda.Event()
                        done.record(st)
                    return out, done, graph_st

                self._hier_job = _BackgroundJob(work)
                return {"background": True}
            emb32 = self.emb32[:n] if src is None else None
            out = self._cluster_compute(live, src, emb32, n, n_fine, n_top, iters, seed, comm if dist else None,
                                        self._hier or {}, self.version)
        if out is None:
            return {}
        self._hier = out
        return {"fine": out["fine_c"].shape[0], "top": out["top_c"].shape[0], "rows": out["rows"]}

    def cluster_join(self) -> None:
        """Wait for a background :meth:`cluster_pass` and publish its
        hierarchy (the graph stream waits for its kernels; its tensors are
        marked in use there). Re-raises the pass's error."""
        with self._hier_lock:
            job = self._hier_job
            if job is None:
                return
            try:
                out, done, graph_st = job.result()
            finally:
                self._hier_job = None
            graph_st.wait_event(done)
            if out is None:
                return
            for t in out.values():
                if torch.is_tensor(t) and t.is_cuda:
                    t.record_stream(graph_st)
            self._hier = out

    def _cluster_compute(self, live, src, emb32, n: int, n_fine: int, n_top: int, iters: int, seed: int, comm,
                         prev: Dict, version: int) -> Optional[Dict]:
        """The body of :meth:`cluster_pass` on the current stream over rows
        [0, n): ``live`` mask, ``src`` the bf16 rows (or None: ``emb32``)."""
        from ..index.kmeans import kmeans

        n_live = int(live.sum())
        if comm is not None:
            t = torch.tensor([n_live], dtype=torch.int64, device=comm.device)
            comm.all_reduce(t)
            n_glob = int(t.item())
        else:
            n_glob = n_live
        if n_glob == 0:
            return None
        if src is not None:
            X = src
        elif self.on_gpu:  # lean: the pass's own bf16 copy, released when it ends
            from ..ops.search import bf16_rows
            X = bf16_rows(emb32, self.Dp)
        else:
            X = emb32 / self.sqn[:n].sqrt().clamp_min(1e-30)[:, None]
        kf = min(n_fine, n_glob)
        kt = min(n_top, kf)
        init_f = prev.get("fine_c") if prev.get("fine_c") is not None and prev["fine_c"].shape[0] == kf else None
        # large tenants: mini-batch refinement steps on a 1M-row sample,
        # then one full assign + update (labels for every row)
        smp = self.CLUSTER_SAMPLE if n_live > 2 * self.CLUSTER_SAMPLE else 0
        # warm passes over large tenants: the full-data assign searches a
        # row's fine clusters only under its nearest previous topic
        fa = None
        if smp and init_f is not None and prev.get("top_c16") is not None and prev.get("top_of_fine") is not None:
            from ..index.kmeans import assign_two_level
            T16, tof = prev["top_c16"], prev["top_of_fine"]
            fa = lambda Xa, C16: assign_two_level(Xa, C16, T16, tof)  # noqa: E731
        # the mini-batch steps: the same two-level assign (SAMPLE_TWO_LEVEL = False: flat over all fine)
        sa = fa if self.SAMPLE_TWO_LEVEL else None
        fc32, fc16, lab = kmeans(X, kf, iters=iters, seed=seed, init=init_f, mask=live, sample=smp,
                                 full_assign=fa, sample_assign=sa, comm=comm)
        init_t = prev.get("top_c") if prev.get("top_c") is not None and prev["top_c"].shape[0] == kt else None
        tc32, tc16, top_of_fine = kmeans(fc16, kt, iters=iters + 2, seed=seed + 1, init=init_t)
        lab = lab.long()
        top = torch.where(lab >= 0, top_of_fine.long()[lab.clamp_min(0)], torch.full_like(lab, -1))
        rows = torch.nonzero(top >= 0).flatten()
        o = torch.argsort(top[rows] * n + rows)
        perm = rows[o]
        cnt = torch.bincount(top[rows], minlength=kt)
        start = torch.zeros(kt + 1, dtype=torch.long, device=self.device)
        start[1:] = torch.cumsum(cnt, 0)
        return {"fine_c": fc32, "top_c": tc32, "fine": lab.to(torch.int32), "top": top.to(torch.int32),
                "perm": perm, "start": start, "n": n, "version": version, "top_c16": tc16,
                "top_of_fine": top_of_fine, "rows": n_glob}

    def hier_children(self, q: torch.Tensor, threshold: float, limit: int) -> List[int]:
        """Hierarchical retrieval over the k-means topics (the reference's
        super-node step, memory_system.py:464-482): the top cluster most
        similar to ``q`` (float64 cosine) if it beats ``threshold``, and its
        first ``limit`` live members (row order). [] otherwise."""
        h = getattr(self, "hier", None)
        if not h or self.dim is None:
            return []
        with self.on_stream():
            C = h["top_c"][:, : self.dim].double()
            qd = q.to(self.device).double().reshape(-1)
            s = (C @ qd) / (C.norm(dim=1) * qd.norm()).clamp_min(1e-30)
            t = int(torch.argmax(s))
            if float(s[t]) <= threshold:
                return []
            a, b = int(h["start"][t]), int(h["start"][t + 1])
            cand = h["perm"][a: min(b, a + 8 * limit)]
            ok = (self.kind[cand] == NODE) & (self.sup[cand] == 0)
            return cand[ok][:limit].tolist()

    # ------------------------------------------------------------------ centroid
    def mean_embedding(self, rows: torch.Tensor) -> Optional[torch.Tensor]:
        """Mean embedding (float64) of the rows that have one (reference
        ``np.mean`` of the children's embeddings, memory_system.py:916-917)."""
        if self.dim is None or rows.numel() == 0:
            return None
        with self.on_stream():
            rows = rows.to(self.device)
            has = self.has_emb[rows].bool()
            if not bool(has.any()):
                return None
            return self.emb32[rows[has]].double().mean(0)

    # ------------------------------------------------------------------ persistence helpers
    def take_dirty_rows(self) -> np.ndarray:
        """Rows changed since the last commit (new / boosted / touched /
        merged), cleared on return."""
        if self.n == 0:
            return np.zeros(0, dtype=np.int64)
        with self.on_stream():
            n = self.n
            d = torch.nonzero(self.dirty[:n]).flatten()
            self.dirty[:n] = 0
            out = d.cpu().numpy()
        self._mirror.pop("dirty", None)
        return out

    def take_dirty_edges(self) -> np.ndarray:
        if self.num_edges == 0:
            return np.zeros(0, dtype=np.int64)
        with self.on_stream():
            m = (self.e["meta"] & EDIRTY) != 0
            idx = torch.nonzero(m).flatten()
            self.e["meta"] &= ~EDIRTY
            self.e["meta"][idx] |= ESTORED
            return idx.cpu().numpy()

    def restore_tracking(self, rows, eidx, del_ids, del_edges) -> None:
        """Undo ``take_*`` after a failed commit (the change set stays pending)."""
        with self.on_stream():
            if len(rows):
                self.dirty[torch.as_tensor(np.asarray(rows), dtype=torch.long).to(self.device)] = 1
            if len(eidx):
                it = torch.as_tensor(np.asarray(eidx), dtype=torch.long).to(self.device)
                self.e["meta"][it] |= EDIRTY
        for i in del_ids:
            self.deleted_ids[i] = None
        for k in del_edges:
            self.deleted_edges[k] = None
        self._mirror.pop("dirty", None)

    def take_deleted(self):
        ids, edges = list(self.deleted_ids), list(self.deleted_edges)
        self.deleted_ids, self.deleted_edges = {}, {}
        return ids, edges

    def clear_tracking(self, stored: bool = True) -> None:
        """Forget pending changes: the caller wrote a full snapshot
        (``stored``), or the graph was filled from data the store does not
        hold and none of it should ever be deleted from it (``stored=False``)."""
        self.take_dirty_rows()
        self.take_dirty_edges()
        self.take_deleted()
        if not stored and self.num_edges:
            with self.on_stream():
                self.e["meta"] &= ~ESTORED
