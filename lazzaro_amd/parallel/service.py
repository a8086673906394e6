"""DistributedMemoryService: the MemorySystem API served by a one-process-per-
GPU job (tenant-DP).

Every tenant (``user_id``) is owned by exactly one rank (rendezvous hashing,
:mod:`.placement`); the owner holds the tenant's ``MemorySystem`` -- its graph
in that GPU's HBM -- and all ranks share one versioned columnar store
directory, so ownership can move (elastic re-placement) by reloading from it.
The reference is a single-process library (memory_system.py:21-1550); its
per-user flows map onto this service as:

* per-tenant calls -- ``chat``, ``search_memories`` (batched per tenant),
  ``end_conversation``, ``add_to_short_term``, ``get_stats``,
  ``get_connected_memories``, ``export_observations``, ``run_consolidation`` ...
  -- execute on the owner. :meth:`serve` is the SPMD entry point: every rank
  passes the requests its front end received (any tenant); requests for
  remote tenants travel to their owner in ONE all-to-all-v of serialized
  bytes (C3 over RCCL/xGMI or gloo), results come back the same way. Local
  requests never touch the network.
* ``get_all_users`` -- the tenant directory: store users plus every rank's
  resident tenants, all-gathered (C7; reference :1430-1439).
* :meth:`search_global` -- one query against EVERY tenant (cross-tenant /
  global search): each rank runs the fused top-k over its resident tenants,
  then an all-gather of the (score, tenant, node) candidates and a merge (C1
  + K2) give every rank the same exact global top-k.

All collective methods must be called by every rank in the same order.
"""
from __future__ import annotations

import inspect
import os
import weakref
from collections import OrderedDict, defaultdict
from collections.abc import Sequence as _SeqABC
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import routing
from .comm import Communicator
from .placement import tenant_rank

# tenant methods a remote request may invoke (the public per-user API)
ALLOWED = {"chat", "search_memories", "end_conversation", "start_conversation", "add_to_short_term",
           "get_stats", "get_connected_memories", "export_observations", "run_consolidation", "get_insights",
           "consolidate_batch", "display_stats", "display_memories", "display_profile", "graph_json"}


def node_dict(n) -> Dict:
    """A Node (or NodeView) as the JSON the service returns."""
    return {"id": n.id, "content": n.content, "type": n.type, "salience": float(n.salience),
            "shard_key": n.shard_key, "access_count": int(n.access_count), "is_super_node": bool(n.is_super_node)}


class SearchHits(_SeqABC):
    """One request's ``search_memories`` result from the fused multi-tenant
    path: columnar -- the hit rows and their gathered fields (one host copy
    per batch) -- and turned into the service's node dicts only when read
    (indexing, iteration, ``==``, JSON export, a reply to another rank). A
    batch of 1024 queries x 10 hits no longer builds 10k dicts that a
    caller may never look at; what a reader sees is
    exactly the eager result. The service materialises every outstanding
    result of a tenant before it runs a mutating request on it (or releases
    / migrates it), so a late read still sees the rows as they were; a
    caller that mutates a tenant directly (``svc.system(u).chat(...)``)
    should read its results first."""
    __slots__ = ("_g", "_cols", "_q", "_limit", "_items", "__weakref__")

    def __init__(self, g, cols: Dict[str, np.ndarray], q: int, limit: int):
        self._g, self._cols, self._q, self._limit, self._items = g, cols, q, limit, None

    def _mat(self) -> List[Dict]:
        if self._items is None:
            c, q, L, g = self._cols, self._q, self._limit, self._g
            rq, kq = c["rows"][q, :L].tolist(), c["kind"][q, :L].tolist()
            sq, aq = c["sal"][q, :L].tolist(), c["acc"][q, :L].tolist()
            pq, hq = c["sup"][q, :L].tolist(), c["shard"][q, :L].tolist()
            ids, content, types, names = g.ids, g.content, g.types, g.shard_names
            self._items = [{"id": ids[r], "content": content[r], "type": types[r], "salience": sq[j],
                            "shard_key": names[hq[j]] if hq[j] >= 0 else "default", "access_count": aq[j],
                            "is_super_node": bool(pq[j])}
                           for j, r in enumerate(rq) if r >= 0 and kq[j] == 1]
            self._g = self._cols = None  # materialised: drop the batch arrays
        return self._items

    def __len__(self) -> int:
        return len(self._mat()) if self._items is not None or self._cols is None else \
            int(((self._cols["rows"][self._q, :self._limit] >= 0) & (self._cols["kind"][self._q, :self._limit] == 1)).sum())

    def __getitem__(self, i):
        return self._mat()[i]

    def __iter__(self):
        return iter(self._mat())

    def __eq__(self, other):
        return isinstance(other, (_SeqABC, list, tuple)) and list(self._mat()) == list(other)

    def __repr__(self) -> str:
        return repr(self._mat())


def _jsonable(v):
    if isinstance(v, SearchHits):
        return list(v)
    if hasattr(v, "id") and hasattr(v, "content") and hasattr(v, "salience"):
        return node_dict(v)
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if torch.is_tensor(v):
        return v.tolist()
    return str(v)


class DistributedMemoryService:
    def __init__(self, comm: Communicator, factory: Callable[[str], object], owner: Callable[[str], int] = None,
                 max_resident: int = 1 << 30, placement=None, embedder=None, force_collectives: bool = None):
        """``factory(user_id)`` builds the tenant's MemorySystem on this rank
        (sharing one store / embedder / device; it must load the tenant from
        the store); ``owner`` overrides the rendezvous-hash placement;
        ``placement`` (an :class:`~.elastic.ElasticPlacement`) places tenants
        over the ORIGINAL ids of the live ranks, so :meth:`reform` after a rank
        failure moves only the dead ranks' tenants. At most ``max_resident``
        tenants stay in memory (LRU; an evicted tenant is persisted and
        reloaded from the store on its next request). ``embedder``: this
        rank's replica of the encoder for the front end's queries on the
        columnar search paths (default: the first resident tenant's).
        ``force_collectives`` (default: env ``LZK_FORCE_COLLECTIVES=1``): run
        every exchange through the communicator even at world 1 -- under a
        1-rank ``torch.distributed.run`` the RCCL all-to-all / all-gather
        calls of an N-GPU job then execute on the one GPU."""
        if force_collectives is None:
            force_collectives = os.environ.get("LZK_FORCE_COLLECTIVES", "0") == "1"
        self.force_collectives = bool(force_collectives) and comm.enabled
        self.comm = comm
        self.factory = factory
        self._owner = owner
        self.placement = placement
        self.max_resident = max_resident
        self.embedder = embedder
        self._moved: Dict[str, int] = {}  # migrate() overrides of the placement
        self._own_memo: Dict[str, int] = {}
        self._lazy: Dict[str, list] = defaultdict(list)  # user -> weakrefs of its unread SearchHits
        self.systems: "OrderedDict[str, object]" = OrderedDict()
        # columnar search routing (routing.py): the device table of resident
        # tenants, tenant names announced to each owner, key -> name
        self._table = None
        self._announced = defaultdict(set)
        self._key_names: Dict[int, str] = {}
        # owner-side directory of the routed path: tenants announced to this
        # rank stay pinned resident under the current epoch (bumped whenever
        # a pinned tenant leaves), so a batch whose senders all know the epoch
        # is served by matching tenant keys on the device
        self._pinned: Dict[int, str] = {}
        self._dir_epoch = 0
        self._ddir = None  # the device directory (see device_directory)
        self._ddir_dirty: set = set()  # pinned tenants mutated since it was built
        self._gdir = None  # the global-search directory (see global_directory)
        self._gdir_dirty: set = set()
        self._membership = 0  # bumps whenever a tenant becomes / stops being resident
        self.route_stats = {"device": 0, "host": 0}  # routed batches served by device key matching / by name
        self._owner_epoch: Dict[int, int] = {}

    # ------------------------------------------------------------ placement
    def owner(self, user: str) -> int:
        """The CURRENT communicator rank that owns ``user`` (memoised: the
        placement hash is computed once per tenant until the placement
        changes -- reform / migrate clear the memo)."""
        r = self._own_memo.get(user)
        if r is None:
            r = self._owner_of(user)
            if len(self._own_memo) < (1 << 22):
                self._own_memo[user] = r
        return r

    def _owner_of(self, user: str) -> int:
        if user in self._moved:
            return self._moved[user]
        if self._owner is not None:
            return self._owner(user)
        if self.placement is not None:
            return self.placement.alive.index(self.placement.owner(user))
        return tenant_rank(user, self.comm.world)

    def reform(self, comm: Communicator, placement) -> List[str]:
        """Adopt the re-formed group after a rank failure
        (:func:`~.elastic.reform_group` + ``ElasticPlacement.remove``):
        tenants this rank no longer owns are persisted and released; tenants
        that moved here are loaded from the shared store by ``factory`` on
        their first request (every durable byte is in the store, so a dead
        rank loses no committed state). Returns the released tenants."""
        self.comm, self.placement, self._owner = comm, placement, None
        self._moved = {}
        self._own_memo = {}
        self._announced = defaultdict(set)  # owners changed: announce names again
        self._owner_epoch = {}
        self._unpin_all()
        gone = [u for u in self.systems if not self.is_local(u)]
        for u in gone:
            self._release(u, self.systems.pop(u))
        return gone

    def _settle(self, user: str) -> None:
        """Materialise the outstanding columnar results of ``user`` (before
        its rows can change)."""
        for r in self._lazy.pop(user, ()):
            h = r()
            if h is not None:
                h._mat()

    # ------------------------------------------------------------ routed directory
    # device key matching serves any number of pinned small tenants (one
    # fused segment_topk over the tenant table) and at most this many pinned
    # large ones (each its own store search over the whole received batch)
    DEVICE_ROUTE_MAX_TENANTS = 2

    def pin(self, user: str) -> None:
        """Keep an announced tenant resident for the routed path (loads it
        if needed); its mutations mark the device directory for refresh."""
        self.system(user)
        key = routing.tenant_key(user)
        if key not in self._pinned:
            self._pinned[key] = user
            self._ddir = None

    def _unpin(self, user: str) -> None:
        if self._pinned.pop(routing.tenant_key(user), None) is not None:
            self._dir_epoch += 1
            self._ddir = None

    def _unpin_all(self) -> None:
        if self._pinned:
            self._pinned = {}
            self._dir_epoch += 1
            self._ddir = None

    def _classify(self, user: str, D: int, K: int) -> Optional[str]:
        """'big' (own store search), 'small' (the fused tenant-table scan) or
        None (the routed owner must serve this tenant by name)."""
        ms = self.systems.get(user)
        g = getattr(ms, "graph", None)
        if g is None or g.dim != D or getattr(ms, "enable_async", False):
            return None  # (a background consolidation may move columns under a raw-pointer scan)
        if g.n >= routing.BIG_ROWS:
            return "big"
        return "small" if routing._fused_ok(ms, D, K) else None

    def device_directory(self, D: int, K: int):
        """The routed owner side's device directory -- sorted pinned tenant
        keys with their table slots and a small/big flag -- or None when some
        pinned tenant cannot be served by key on the device (then the owner
        reads the received keys back). Rebuilt when the pinned set, the width
        or a mutated tenant's class changed; a mutated small tenant only has
        its table entry refreshed."""
        if not self._pinned:
            return None
        d = self._ddir
        if d is not None and d["D"] == D and d["K"] >= K and d["epoch"] == self._dir_epoch:
            if self._ddir_dirty:
                dirty, self._ddir_dirty = self._ddir_dirty, set()
                for u in dirty:
                    if u in d["cls"] and self._classify(u, D, d["K"]) != d["cls"][u]:
                        self._ddir = None
                        return self.device_directory(D, K)
                small = [u for u in dirty if d["cls"].get(u) == "small"]
                if small:
                    d["table"].slots_host(small, self.systems)
            return d
        self._ddir_dirty = set()
        K = max(K, 1)
        cls = {}
        for u in self._pinned.values():
            c = self._classify(u, D, K)
            if c is None:
                return None
            cls[u] = c
        big = sorted(u for u, c in cls.items() if c == "big")
        if len(big) > self.DEVICE_ROUTE_MAX_TENANTS:
            return None
        small = sorted(u for u, c in cls.items() if c == "small")
        table = None
        keys = np.asarray([routing.tenant_key(u) for u in small], np.int64)
        slots = np.zeros(0, np.int64)
        dev = self.systems[(small or big)[0]].graph.device
        if small:
            table = self.tenant_table(dev)
            slots = table.slots_host(small, self.systems)
        o = np.argsort(keys, kind="stable")
        streams = {}
        for u in small:
            st = getattr(self.systems[u].graph, "stream", None)
            if st is not None:
                streams[st.cuda_stream] = st
        self._ddir = {"D": D, "K": K, "epoch": self._dir_epoch, "cls": cls, "big": big, "table": table,
                      "streams": list(streams.values()),
                      "keys": torch.from_numpy(keys[o]).to(dev), "slots": torch.from_numpy(slots[o]).to(dev)}
        return self._ddir

    def device_directory_ok(self, D: int, K: int = 1) -> bool:
        return self.device_directory(D, K) is not None

    def _release(self, user: str, ms) -> None:
        """Persist and close a tenant this rank stops holding."""
        self._membership += 1
        if getattr(ms, "graph", None) is not None:
            ms.graph.on_change = None
        self._unpin(user)
        self._settle(user)
        if self._table is not None:
            self._table.drop(user)
        ms._save_to_persistence()
        ms.close()

    def warm_table(self) -> int:
        """Register every resident GPU tenant in the device pointer table (as
        an index is built at load): the fused search then refreshes only
        tenants whose columns moved since. Returns the tenants registered."""
        gpu = [u for u, ms in self.systems.items() if ms.graph.on_gpu and ms.graph.dim is not None]
        if not gpu:
            return 0
        self.tenant_table(self.systems[gpu[0]].graph.device).slots(gpu, self.systems)
        return len(gpu)

    def tenant_table(self, device=None) -> "routing.TenantTable":
        """The device table of resident tenants' column pointers, on the
        tenants' device (NOT necessarily the communicator's: a CPU/gloo
        communicator can front GPU tenants)."""
        dev = torch.device(device) if device is not None else torch.device(self.comm.device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        if self._table is None or self._table.device != dev:
            self._table = routing.TenantTable(dev)
        return self._table

    def is_local(self, user: str) -> bool:
        return self.owner(user) == self.comm.rank

    def system(self, user: str):
        """The resident MemorySystem of a tenant this rank owns."""
        if not self.is_local(user):
            raise KeyError(f"tenant {user!r} is owned by rank {self.owner(user)}, not {self.comm.rank}")
        ms = self.systems.get(user)
        if ms is None:
            ms = self._build(user)
            self.systems[user] = ms
            self._resident(user, ms)
            while len(self.systems) > self.max_resident:
                u0, old = self.systems.popitem(last=False)
                self._release(u0, old)
        else:
            self.systems.move_to_end(user)
        return ms

    def _resident(self, user: str, ms) -> None:
        """A tenant became resident: its mutations mark the device and
        global directories (TenantGraph.on_change)."""
        self._membership += 1
        g = getattr(ms, "graph", None)
        if g is not None:
            g.on_change = lambda u=user: (self._ddir_dirty.add(u), self._gdir_dirty.add(u))

    def global_directory(self, D: int, k: int):
        """The resident tenants of width ``D`` as global search sees them:
        ``small`` (names, table slots, stable tenant keys as a device array
        indexed by slot, their graph streams, whether any needs its graph
        lock held) for the one-pass tile-table scan, and ``big`` (name, slot)
        for per-tenant store searches. Rebuilt when residency, the width or a
        mutated tenant's class changed; a mutated small tenant only has its
        table entry refreshed -- no per-call pass over thousands of tenants."""
        d = self._gdir
        if d is not None and d["D"] == D and d["k"] >= k and d["membership"] == self._membership:
            if self._gdir_dirty:
                dirty, self._gdir_dirty = self._gdir_dirty, set()
                for u in dirty:
                    ms = self.systems.get(u)
                    if ms is None:
                        continue
                    if self._global_class(ms, D, d["k"]) != d["cls"].get(u):
                        self._gdir = None
                        return self.global_directory(D, k)
                small = [u for u in dirty if d["cls"].get(u) == "small"]
                if small and d["table"] is not None:
                    d["table"].slots_host(small, self.systems)
            return d
        self._gdir_dirty = set()
        k = max(int(k), 1)
        cls = {u: self._global_class(ms, D, k) for u, ms in self.systems.items()}
        small = [u for u, c in cls.items() if c == "small"]
        bigu = [u for u, c in cls.items() if c == "big"]
        table = None
        slots = np.zeros(0, np.int64)
        big = []
        users = small + bigu
        if users:
            table = self.tenant_table(self.systems[users[0]].graph.device)
            sl = table.slots_host(users, self.systems)
            slots = sl[: len(small)]
            big = list(zip(bigu, sl[len(small):].tolist()))
        tk = tkdev = None
        streams = {}
        if small:
            tk = np.full(table.cap, -1, np.int64)
            tk[slots] = [routing.tenant_key(u) for u in small]
            tkdev = torch.from_numpy(tk).to(table.device)
            for u in small:
                st = getattr(self.systems[u].graph, "stream", None)
                if st is not None:
                    streams[st.cuda_stream] = st
        self._gdir = {"D": D, "k": k, "membership": self._membership, "cls": cls, "small": small,
                      "slots": np.asarray(slots, np.int64), "tkeys": tkdev, "big": big, "table": table,
                      "streams": list(streams.values()),
                      "lock": any(getattr(self.systems[u], "enable_async", False) for u in small)}
        return self._gdir

    @staticmethod
    def _global_class(ms, D: int, k: int) -> Optional[str]:
        g = getattr(ms, "graph", None)
        if g is None or g.dim != D or g.n == 0:
            return None
        return "small" if (routing.MT_GLOBAL and routing._fused_ok(ms, D, k)) else "big"

    def migrate(self, moves: Dict[str, int]) -> List[str]:
        """SPMD live re-shard of tenants (C3): ``moves`` = {user: new rank},
        identical on every rank. A resident tenant's owner commits it, exports
        its graph (``MemorySystem.export_state``) and ships it in two
        all-to-all-v exchanges -- the fp32 vector rows device to device over
        RCCL/xGMI, the other columns as serialized bytes -- and the new owner
        rebuilds it with ``import_state`` (no store read). Tenants that are
        not resident anywhere just change owner (loaded from the store on
        first use). Returns the tenants this rank received."""
        comm = self.comm
        me = comm.rank
        out_meta: List[List] = [[] for _ in range(comm.world)]
        out_vec: List[List[torch.Tensor]] = [[] for _ in range(comm.world)]
        for user in sorted(moves):
            dst = int(moves[user])
            if user in self.systems and dst != me:
                self._settle(user)
                self._unpin(user)
                ms = self.systems.pop(user)
                self._membership += 1
                ms.graph.on_change = None
                if self._table is not None:
                    self._table.drop(user)
                ms._save_to_persistence()
                meta, vec = ms.export_state()
                out_meta[dst].append([user, meta, list(vec.shape)])
                out_vec[dst].append(vec.reshape(-1).float())
                ms.close()
        got_meta = self._exchange(out_meta)
        dev = comm.device
        send = [torch.cat(v) if v else torch.zeros(0) for v in out_vec]
        counts = [int(t.numel()) for t in send]
        flat = torch.cat([t.to(dev) for t in send]) if sum(counts) else torch.zeros(0, device=dev)
        rc = comm.host_counts(counts)
        recv = comm.all_to_all_v(flat, counts, rc) if comm.world > 1 or self.force_collectives else flat
        self._moved.update({u: int(r) for u, r in moves.items()})
        for u in moves:
            self._own_memo.pop(u, None)
        self._announced = defaultdict(set)
        self._owner_epoch = {}
        received, off = [], 0
        for src in range(comm.world):
            for user, meta, shape in got_meta[src]:
                n = int(np.prod(shape)) if shape else 0
                vec = recv[off: off + n].reshape(shape)
                off += n
                ms = self._build(user, load=False)
                ms.import_state(meta, vec)
                self.systems[user] = ms
                self._resident(user, ms)
                received.append(user)
        return received

    def _build(self, user: str, load: bool = True):
        """factory(user[, load_from_disk=...]): a factory without the keyword
        always loads the tenant from the store itself."""
        try:
            params = inspect.signature(self.factory).parameters
            kw = "load_from_disk" in params or any(p.kind == p.VAR_KEYWORD for p in params.values())
        except (TypeError, ValueError):
            kw = False
        return self.factory(user, load_from_disk=load) if kw else self.factory(user)

    # ------------------------------------------------------------ request routing
    def _exchange(self, outgoing: List[List]) -> List[List]:
        """outgoing[r] = JSON-able items for rank r -> items received per rank
        (this rank's own items stay in process: no serialisation)."""
        if self.comm.world == 1 and not self.force_collectives:
            return outgoing
        me = self.comm.rank
        send = list(outgoing)
        mine, send[me] = send[me], []
        got = [x if x is not None else [] for x in self.comm.exchange_objects(send)]
        got[me] = mine
        return got

    def serve(self, requests: Sequence[Tuple]) -> List:
        """SPMD: ``requests`` = [(user_id, method, args...)] received by this
        rank's front end. Each runs on the tenant's owner -- remote ones via
        one all-to-all-v there and one back -- in order per tenant; the
        ``search_memories`` requests of all tenants an owner receives run as
        one batch (:meth:`_search_submit`). Returns one JSON-able result per
        request (Nodes as dicts); a ``search_memories`` result served by the
        fused GPU path is a :class:`SearchHits` sequence of those dicts, built
        when first read (``list(r)`` for a plain list, e.g. before
        ``json.dumps``)."""
        return self._serve_finish(self._serve_submit(requests))

    def serve_stream(self, rounds: Iterable[Sequence[Tuple]]):
        """Pipelined :meth:`serve` for serving loops (SPMD, every rank the
        same number of rounds): round i+1's requests are routed and its
        batched search enqueued on the GPU BEFORE round i's results are
        materialised and returned, so the host work of one round hides
        under the device work of the next. Yields one result list per round,
        equal to ``serve`` of that round."""
        prev = None
        for reqs in rounds:
            h = self._serve_submit(reqs, prev)
            if prev is not None:
                yield self._serve_finish(prev)
            prev = h
        if prev is not None:
            yield self._serve_finish(prev)

    def _serve_submit(self, requests: Sequence[Tuple], prev=None):
        """Route and start one round. ``prev``: the still-unfinished state of
        the previous round (serve_stream) -- its batched search is completed
        locally before a mutating request runs on any of its tenants, so the
        rows it gathered are mapped to nodes before they can move."""
        comm = self.comm
        out_req: List[List] = [[] for _ in range(comm.world)]
        for i, req in enumerate(requests):
            user, method = req[0], req[1]
            if method not in ALLOWED:
                raise ValueError(f"method {method!r} is not served")
            out_req[self.owner(user)].append([i, user, method, list(req[2:])])
        inbox = self._exchange(out_req)
        replies: List[List] = [[] for _ in range(comm.world)]
        # searches of every source and tenant run as one batch (one embed,
        # one multi-tenant scan on the GPU); a tenant's mutating request
        # first flushes its pending searches, so per-tenant order holds
        pending: List[Tuple] = []

        def flush():
            if pending:
                for (src, i, *_), r in zip(pending, self._search_finish(self._search_submit(pending))):
                    replies[src].append([i, r])
                pending.clear()
        for src, items in enumerate(inbox):
            for i, user, method, args in items:
                if method == "search_memories":
                    pending.append((src, i, user, args[0], int(args[1]) if len(args) > 1 else 5))
                    continue
                if any(p[2] == user for p in pending):
                    flush()
                if prev is not None and prev[3] is not None and prev[3][0] != "done" and \
                        any(p[2] == user for p in prev[2]):
                    prev[3] = ("done", self._search_finish(prev[3]))
                self._settle(user)
                replies[src].append([i, _jsonable(getattr(self.system(user), method)(*args))])
        handle = self._search_submit(pending) if pending else None
        return [len(requests), replies, list(pending), handle]

    def _serve_finish(self, state) -> List:
        n, replies, pending, handle = state
        if handle is not None:
            for (src, i, *_), r in zip(pending, self._search_finish(handle)):
                replies[src].append([i, r])
        back = self._exchange(replies)
        result: List = [None] * n
        for items in back:
            for i, r in items:
                result[i] = r
        return result

    # fused multi-tenant search: below this many tenants
    # in a batch the per-tenant path is used
    FUSED_MIN_TENANTS = 2

    def _search_submit(self, pending: List[Tuple]):
        """search_memories for (src, i, user, query, limit) requests of many
        tenants. GPU, one shared embedder, L2 stores bound to their graphs:
        ONE embed of all queries and ONE ``segment_topk`` launch in which
        each query scans only its tenant's fp32 rows (score 2<q,x> - |x|^2 -
        |q|^2 = -|q-x|^2 with the store's row mask as bias -- the exact fp32
        L2 of the reference's store search), then one pointer-table gather of
        the result rows' fields, copied to pinned memory asynchronously: the
        returned handle is finished by :meth:`_search_finish` (which holds
        the tenants' graph locks until then). Otherwise per tenant, at once."""
        users = [p[2] for p in pending]
        systems = {u: self.system(u) for u in dict.fromkeys(users)}
        first = next(iter(systems.values()))
        emb0 = first.embedder
        fused = (len(systems) >= self.FUSED_MIN_TENANTS and first.graph.on_gpu
                 and first.graph.dim is not None and first.graph.dim % 32 == 0
                 and max(p[4] for p in pending) <= 16
                 and all(ms.embedder is emb0 and getattr(ms.store, "metric", "l2") == "l2"
                         and ms._store_binds_graph() for ms in systems.values()))
        if not fused:
            out, j = [], 0
            while j < len(pending):  # consecutive same-tenant, same-limit runs batch
                k = j
                while k < len(pending) and pending[k][2] == pending[j][2] and pending[k][4] == pending[j][4]:
                    k += 1
                res = systems[pending[j][2]].search_memories_batch([p[3] for p in pending[j:k]], limit=pending[j][4])
                out += [[node_dict(n) for n in r] for r in res]
                j = k
            return ("done", out)
        from ..ops.search import segment_topk_ptrs
        from ..ops.tenant_ops import gather_fields
        from ..utils.tracing import tracer
        with tracer.stage("mt_embed", first._device):
            embs = first._batch_embed_any([p[3] for p in pending])
        dev = first.graph.device
        Q = (embs if torch.is_tensor(embs) else torch.as_tensor(np.asarray(embs, np.float32))).to(dev, torch.float32)
        locks = [systems[u]._graph_lock for u in sorted(systems)]
        for lk in locks:
            lk.acquire()
        try:
            with tracer.stage("mt_prep", "cpu"):
                D = Q.shape[1]
                graphs = {u: ms.graph for u, ms in systems.items()}
                table = self.tenant_table(dev)
                slots = table.slots(users, systems)
                ptrs = table.d_ptr[:, slots]
                nrows = table.d_n[slots]
                # a tenant of another width contributes no rows
                wrong = [j for j, u in enumerate(users) if graphs[u].dim != D]
                if wrong:
                    nrows = nrows.clone()
                    nrows[torch.as_tensor(wrong, device=dev)] = 0
            qb = -(Q * Q).sum(1)
            k = max(p[4] for p in pending)
            with tracer.stage("mt_scan", first._device):
                _, rows = segment_topk_ptrs(ptrs[0].contiguous(), nrows.contiguous(), D, Q.contiguous(), k,
                                            bptr=ptrs[1].contiguous(), alpha=2.0, qbias=qb)
            # the result rows' fields in one gather over the per-query column
            # pointers of the tenant table (the tenants' columns are separate
            # allocations)
            qg = [graphs[u] for u in users]
            f = gather_fields(rows, None, device_out=True, base=ptrs[2:7].contiguous())
            f["rows"] = rows
            host = {n: torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for n, t in f.items()}
            for n, t in f.items():
                host[n].copy_(t, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            return ("fused", pending, qg, host, ev, locks, (Q, ptrs, nrows, f))
        except BaseException:
            for lk in reversed(locks):
                lk.release()
            raise

    def _search_finish(self, h) -> List[List[Dict]]:
        if h[0] == "done":
            return h[1]
        from ..utils.tracing import tracer
        _, pending, qg, host, ev, locks, _keep = h
        try:
            ev.synchronize()
            with tracer.stage("mt_results", "cpu"):
                cols = {n: t.numpy() for n, t in host.items()}
                me = self.comm.rank
                # columnar per request; a reply to another rank is materialised
                # now (its graph stays here)
                out = [SearchHits(qg[q], cols, q, p[4]) for q, p in enumerate(pending)]
                lazy = self._lazy
                for q, p in enumerate(pending):
                    if p[0] != me:
                        out[q] = list(out[q])
                    else:
                        lst = lazy[p[2]]
                        if len(lst) >= 32:  # drop the refs of results already gone
                            lst[:] = [w for w in lst if w() is not None]
                        lst.append(weakref.ref(out[q]))
            return out
        finally:
            for lk in reversed(locks):
                lk.release()

    # ------------------------------------------------------------ columnar search (routing.py)
    def search_routed(self, users: Sequence[str], queries, limit=5) -> "routing.RoutedHits":
        """SPMD batched search_memories with tensors on the wire: ``queries``
        are texts (embedded here, by this rank's replica of the encoder) or an
        embedding tensor [n, D]; each goes to ``users[q]``'s owner in one
        all-to-all and its (score, row) hits come back in one more. Returns a
        :class:`~.routing.RoutedHits` in the caller's order."""
        Q = self._embed_front(queries)
        return routing.search_routed(self, list(users), Q, limit)

    def search_routed_stream(self, batches, limit=5):
        """Pipelined :meth:`search_routed` for serving loops (the routed
        counterpart of ``MemorySystem.search_memories_stream``): ``batches``
        yields (users, query texts); batch i+1's front-end embed is enqueued
        on a side stream BEFORE batch i's routed search (header exchange, the
        two all-to-alls, the owners' store searches), so the encoder runs
        under the search instead of after it. Every rank must iterate alike.
        Yields one :class:`~.routing.RoutedHits` per batch, in order."""
        dev = self.comm.device
        side = None
        if dev.type == "cuda":
            side = self._routed_side = getattr(self, "_routed_side", None) or torch.cuda.Stream(dev)

        def embed(texts):
            if side is None:
                return self._embed_front(texts), None
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                Q = self._embed_front(texts)
                ev = torch.cuda.Event()
                ev.record(side)
            return Q, ev

        it = iter(batches)
        cur = next(it, None)
        if cur is None:
            return
        q_cur = embed(cur[1])
        while cur is not None:
            nxt = next(it, None)
            q_nxt = embed(nxt[1]) if nxt is not None else None
            Q, ev = q_cur
            if ev is not None:
                main = torch.cuda.current_stream(dev)
                main.wait_event(ev)
                Q.record_stream(main)
            yield routing.search_routed(self, list(cur[0]), Q, limit)
            cur, q_cur = nxt, q_nxt

    def search_global_batch(self, queries, limit: int = 5) -> "routing.GlobalHits":
        """SPMD: this rank's queries against every resident tenant of every
        rank (all-gather of queries, local search, one all-to-all back)."""
        return routing.search_global_batch(self, self._embed_front(queries), limit)

    def resolve(self, hits: "routing.RoutedHits") -> List[List[Dict]]:
        """SPMD: node dicts of routed hits (for callers that need contents)."""
        return routing.resolve(self, hits)

    def _embed_front(self, queries):
        if torch.is_tensor(queries):
            return queries.to(self.comm.device, torch.float32)
        queries = list(queries)
        emb = getattr(self, "embedder", None)
        if emb is None:
            ms = next(iter(self.systems.values()), None)
            emb = ms.embedder if ms is not None else None
        if emb is None or not queries:
            return torch.zeros((0, 0), dtype=torch.float32, device=self.comm.device)
        if getattr(type(emb), "batch_embed_tensor", None) is not None:
            out = emb.batch_embed_tensor(queries)
        else:
            out = torch.as_tensor(np.asarray(emb.batch_embed(queries), np.float32))
        return out.to(self.comm.device, torch.float32)

    # ------------------------------------------------------------ directory (C7)
    def get_all_users(self) -> List[str]:
        mine = set(self.systems)
        for ms in list(self.systems.values())[:1]:
            try:
                mine |= set(ms.get_all_users())
            except Exception:
                pass
        parts = self.comm.all_gather_object(sorted(mine))
        users = sorted({u for p in parts for u in p})
        for u in users:  # the directory also names every tenant key (GlobalHits.users)
            self._key_names[routing.tenant_key(u)] = u
        return users

    # ------------------------------------------------------------ global search (C1 + K2)
    def search_global(self, query_emb: torch.Tensor, limit: int = 5, metric: str = "l2") -> List[Dict]:
        """Top-``limit`` over every resident tenant of every rank for one
        query vector (exact store scores: -|q-x|^2 for L2). Returns the same
        list of {user_id, node...} dicts on every rank."""
        comm = self.comm
        cands = []
        for user, ms in self.systems.items():
            g = ms.graph
            if g.dim is None or g.dim != query_emb.numel():
                continue
            with ms._graph_lock:
                s, r = g.store_search(query_emb.reshape(1, -1).to(g.device), limit, metric)
                s, r = s[0].cpu().tolist(), r[0].cpu().tolist()
                for sc, row in zip(s, r):
                    if row >= 0 and g.kind_h(row) == 1:
                        cands.append((sc, user, row, node_dict(_view(g, row))))
        cands.sort(key=lambda c: (-c[0], c[1], c[2]))
        cands = cands[:limit]
        parts = comm.all_gather_object([(c[0], c[1], c[2], c[3]) for c in cands])
        allc = sorted((c for p in parts for c in p), key=lambda c: (-c[0], c[1], c[2]))[:limit]
        return [dict(user_id=u, score=sc, **nd) for sc, u, _, nd in allc]

    # ------------------------------------------------------------ row-sharded tenants
    def shard_of(self, user: str):
        """This rank's shard of a row-sharded tenant (a tenant too large for
        one GPU: every rank holds the rows whose id hashes to it, persisted
        as tenant ``user@r/world``)."""
        sid = f"{user}@{self.comm.rank}/{self.comm.world}"
        ms = self.sharded.get(sid)
        if ms is None:
            ms = self._build(sid)
            self.sharded[sid] = ms
        return ms

    @property
    def sharded(self) -> Dict[str, object]:
        if not hasattr(self, "_sharded"):
            self._sharded: Dict[str, object] = {}
        return self._sharded

    def add_sharded(self, user: str, ids: Sequence[str], contents: Sequence[str], vectors) -> int:
        """SPMD: rows given on any rank go to the rank their id hashes to --
        one all-to-all-v of the vectors (C3 re-shard) and one of the ids and
        texts -- and are stored there as memories of the tenant's local
        shard. Returns the rows this rank received."""
        comm = self.comm
        V = torch.as_tensor(np.asarray(vectors, np.float32)) if not torch.is_tensor(vectors) else vectors.float()
        D = V.shape[1] if V.dim() == 2 and V.shape[0] else 0
        D = int(max(comm.all_gather_object(D)))
        dest = [tenant_rank(i, comm.world) for i in ids]
        meta: List[List] = [[] for _ in range(comm.world)]
        order = sorted(range(len(ids)), key=lambda j: dest[j])
        for j in order:
            meta[dest[j]].append([ids[j], contents[j]])
        counts = [len(m) * D for m in meta]
        flat = V[torch.as_tensor(order, dtype=torch.long)].reshape(-1) if order else torch.zeros(0)
        rc = comm.host_counts(counts)
        got = comm.all_to_all_v(flat.to(comm.device), counts, rc) if comm.world > 1 or self.force_collectives else flat
        got_meta = self._exchange(meta)
        rows = [m for part in got_meta for m in part]
        if not rows:
            return 0
        ms = self.shard_of(user)
        g = ms.graph
        with ms._graph_lock:
            g.add_nodes([r[0] for r in rows], [r[1] for r in rows], got.reshape(len(rows), D).to(g.device),
                        shard=g.shard_id("default"), stored=ms._store_binds_graph())
            ms._save_to_persistence()
        return len(rows)

    def search_sharded(self, user: str, queries: Sequence[str], limit: int = 5) -> List[List[Dict]]:
        """SPMD search of a row-sharded tenant: every rank embeds the
        queries (replicated encoder, no broadcast: C2), runs the store search
        over its shard, then ONE all-gather of the (score, rank, row)
        candidates and a merge give every rank the exact global top-``limit``
        (C1 + K2); the owner of each winning row supplies its node dict
        through one more all-gather."""
        comm = self.comm
        ms = self.shard_of(user)
        g = ms.graph
        embs = ms._batch_embed_any(list(queries))
        Q = (embs if torch.is_tensor(embs) else torch.as_tensor(np.asarray(embs, np.float32))).float()
        nq = len(queries)
        with ms._graph_lock:
            if g.n and g.dim == Q.shape[1]:
                s, r = g.store_search(Q.to(g.device), limit, getattr(ms.store, "metric", "l2"))
                s, r = s.cpu(), r.cpu()
                kind = g.mirror("kind")
                ok = (r >= 0) & torch.as_tensor(kind)[r.clamp_min(0)].eq(1)
                s = torch.where(ok, s, torch.full_like(s, float("-inf")))
            else:
                s = torch.full((nq, limit), float("-inf"))
                r = torch.full((nq, limit), -1, dtype=torch.long)
        # C1: all-gather of fixed-size candidate lists; K2: merge by (score
        # desc, (rank, row) asc) -- the same total order on every rank
        from .sharded import merge_topk
        key = torch.where(r >= 0, comm.rank * (1 << 40) + r, torch.full_like(r, -1))
        gs = comm.all_gather_rows(s.float().contiguous().to(comm.device))
        gk = comm.all_gather_rows(key.contiguous().to(comm.device))
        W = comm.world
        gs = gs.view(W, nq, -1).permute(1, 0, 2).reshape(nq, -1)
        gk = gk.view(W, nq, -1).permute(1, 0, 2).reshape(nq, -1)
        ms_, mk = merge_topk(gs, gk, limit)
        ms_, mk = ms_.cpu(), mk.cpu()
        winners: List[List[Tuple[int, int]]] = [
            [(int(k_) >> 40, int(k_) & ((1 << 40) - 1)) for sc, k_ in zip(ms_[q].tolist(), mk[q].tolist())
             if k_ >= 0 and sc != float("-inf")] for q in range(nq)]
        mine = {}
        with ms._graph_lock:
            for q in range(nq):
                for rk, row in winners[q]:
                    if rk == comm.rank:
                        mine[(q, row)] = node_dict(_view(g, row))
        parts = comm.all_gather_object(list(mine.items()))
        nodes = {(key[0], rk, key[1]): v for rk, p in enumerate(parts) for key, v in p}
        return [[nodes[(q, rk, row)] for rk, row in winners[q]] for q in range(nq)]

    def close(self) -> None:
        for ms in list(self.systems.values()) + list(self.sharded.values()):
            ms.close()
        self.systems.clear()
        self.sharded.clear()


def _view(g, row):
    from ..engine.views import NodeView
    return NodeView.of(g, row)
