"""Python face of the native segment applier (csrc/kernels/apply.hip
``lzk_apply_segments``).

``consolidate_batch`` applies its plan to the tenant graph in ~43 segments
per 128-conversation step (one per run_consolidation point, reference
memory_system.py:580-649, :651-933, :951-1010). :class:`SegmentProgram`
turns the segments into ONE upload and ONE native call:

* every per-row value of the batch (touched rows, inserted rows' columns,
  super-node children, planned links, victims) goes into one pinned byte
  block, copied to the device once; the inserted rows' embeddings into one
  fp32 block;
* a small int64 op program tells the native loop which kernel chain to issue
  for each segment -- decay + deferred prune flags, set_rows, write_emb,
  append_edges, the segment end with its compaction (one host read per
  segment end, inside the loop), and at each run_consolidation point the
  component digest and the profile's first rows into capture slots;
* the host-side graph bookkeeping (ids, counters, children, deleted ids,
  dropped edges) is done here, in segment order, exactly as
  ``TenantGraph.add_nodes`` / ``segment_end`` do it, from the records the
  native loop returns.

The caller (``ConsolidationMixin._apply_planned_native``) decides what each
segment contains and checks eligibility; the results are bit-identical to
the per-segment Python path (tests/unit/test_consolidate_batch_exact.py
test_batch_equals_sequential_gpu*, tests/kernels/test_tenant_engine_gpu.py).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..ops import _lib
from ..ops import tenant_ops as T
from .tenant_graph import EDIRTY, NODE, TYPE_SHIFT, Capture

OP_END, OP_DECAY, OP_ROWS, OP_EMB, OP_N, OP_SHARD, OP_APPEND, OP_SEGEND, OP_POINT = range(9)

P, I, L, F, D = _lib.P, _lib.I, _lib.L, _lib.F, _lib.D
_lib.register("lzk_apply_segments", I, [
    P, L, P, P, I,            # prog, nprog, blk, xblk, D
    P, L, L, L,               # cols, ld32, ld16, ld8
    P, P, L, L,               # ebuf_a, ebuf_b, ne0, cap_e
    F, F, D, I, I,            # thr, keep, now, meta_bits, unstore
    P, P, P, P, L,            # flag_a, flag_b, bc, info, info_cap
    P, P, P, L,               # dsrc, ddst, dmeta, drop_cap
    P, I, P, P, P, I,         # dg_out, dg_cap, dg_ws, dg_cnt, fr_out, fr_k
    P, I, P, P, L, P, P,      # shard_count, ncodes, seg_out, vinfo, vinfo_cap, point_out, state
    P, P])                    # cc slots (or None), stream
_lib.register("lzk_apply_dig_size", L, [])
_lib.register("lzk_apply_dig_copy", None, [P])

# set_rows column bits (tenant.hip tg_set_rows_kernel): sal acc last ts shard sup parent
_SR_COLS = ("sal", "acc", "last", "ts", "shard", "sup", "parent")
_ROWS_IN_VALS = 1 << 15


def available() -> bool:
    try:
        return getattr(_lib.lib(), "lzk_apply_segments", None) is not None
    except Exception:  # pragma: no cover - no kernel library on this host
        return False



# The segments' node-salience decay as per-row stamps and one pass at the end
# of each run (csrc/kernels/apply.hip, bit-identical to a pass per segment).
# False: a pass over every shard node per segment (A/B).
LAZY_NODE_DECAY = True

class SegmentProgram:
    """Builder of one native apply call over a run of segments of a plan."""

    def __init__(self, g, now: float, thr: float, keep: float, etype: int, k_first: int):
        self.g = g
        self.now, self.thr, self.keep = float(now), float(thr), float(keep)
        self.meta_bits = (int(etype) << TYPE_SHIFT) | EDIRTY
        self.k_first = int(k_first)
        self.prog: List[int] = []
        self._parts: List[np.ndarray] = []
        self._nbytes = 0
        self._x_idx: List[int] = []
        self._x_extra: List[torch.Tensor] = []
        self.x_rows = 0
        self.nseg = 0
        self.npoints = 0
        self.total_app = 0
        self.max_nv = 0
        self.n_vinfo = 0
        self.seg_vic: List[List[int]] = []  # victims per segment (host rows)

    # ---- the byte block
    def _put(self, a: np.ndarray) -> int:
        a = np.ascontiguousarray(a)
        assert a.dtype.itemsize == 8
        off = self._nbytes
        self._parts.append(a.reshape(-1).view(np.uint8))
        self._nbytes += a.nbytes
        return off

    def _consts(self, sal=0.0, acc=0, last=0.0, ts=0.0, shard=0, sup=0, parent=-1) -> int:
        return self._put(np.asarray([sal, acc, last, ts, shard, sup, parent], np.float64))

    # ---- ops
    def n(self, n: int) -> None:
        self.prog += [OP_N, int(n)]

    def decay(self, steps: int) -> None:
        self.prog += [OP_DECAY, int(steps)]

    def touch_rows(self, rows, sal, acc, last) -> None:
        """TenantGraph: per-row sal / acc / last of planned touched rows; ts,
        shard, sup, parent, kind, stored untouched (the Python path's
        T.set_rows(g, None, blk, 0b111 | (0b1111000 << 8), -1, -1))."""
        m = len(rows)
        if m == 0:
            return
        vals = np.stack([np.asarray(c, np.float64).reshape(-1) for c in (rows, sal, acc, last)])
        c = self._consts()
        v = self._put(vals)
        self.prog += [OP_ROWS, -1, 0, m, v, _ROWS_IN_VALS | 0b111 | (0b1111000 << 8), c, -1, -1]

    def insert_rows(self, row0: int, m: int, cols: Dict[str, object], stored: bool) -> None:
        """The node columns of a fresh insert at rows row0 .. row0 + m - 1, as
        TenantGraph._set_rows_fused builds them: a per-row column goes to the
        block (a single value becomes the constant), absent ones take the
        add_nodes defaults (ts = last = now, parent -1, sup 0)."""
        defaults = {"sal": 0.5, "acc": 0, "last": self.now, "ts": self.now, "shard": 0, "sup": 0, "parent": -1}
        consts = []
        vals = []
        present = 0
        for c, name in enumerate(_SR_COLS):
            v = cols.get(name)
            if v is None:
                consts.append(float(defaults[name]))
                continue
            a = np.asarray(v, dtype=np.float64).reshape(-1)
            if a.size == 1:
                consts.append(float(a[0]))
                continue
            assert a.size == m
            consts.append(0.0)
            vals.append(a)
            present |= 1 << c
        co = self._put(np.asarray(consts, np.float64))
        vo = self._put(np.stack(vals)) if vals else co
        self.prog += [OP_ROWS, -1, int(row0), int(m), vo, present, co, NODE, 1 if stored else 0]

    def set_parent(self, rows: Sequence[int], parent: int) -> None:
        """parent[rows] = parent, dirty[rows] = 1 (the super-node's children)."""
        m = len(rows)
        if m == 0:
            return
        c = self._consts(parent=int(parent))
        v = self._put(np.asarray(rows, np.float64))
        self.prog += [OP_ROWS, -1, 0, m, v, _ROWS_IN_VALS | (0b0111111 << 8), c, -1, -1]

    def embeddings(self, idx: Sequence[int], row0: int) -> None:
        """Rows ``idx`` of the embedding source (:meth:`run`'s ``E``, then the
        :meth:`extra_embedding` rows) written at rows row0 .. row0 + m - 1."""
        m = len(idx)
        self._x_idx.extend(int(i) for i in idx)
        self.prog += [OP_EMB, self.x_rows, m, int(row0)]
        self.x_rows += m

    def extra_embedding(self, x: torch.Tensor) -> int:
        """Register one extra embedding row (a super-node's mean); returns
        its index in the embedding source, past the facts' rows."""
        self._x_extra.append(x.reshape(1, -1))
        return -len(self._x_extra)  # resolved against E's row count in run()

    def shard_delta(self, code: int, delta: int) -> None:
        if delta:
            self.prog += [OP_SHARD, int(code), int(delta)]

    def append_edges(self, src, dst, w, code) -> None:
        m = len(src)
        if m == 0:
            return
        vals = np.stack([np.asarray(src, np.float64).reshape(-1), np.asarray(dst, np.float64).reshape(-1),
                         np.asarray(w, np.float32).astype(np.float64).reshape(-1),
                         np.asarray(code, np.float64).reshape(-1)])
        self.prog += [OP_APPEND, self._put(vals), m]
        self.total_app += m

    def segment_end(self, victims: Sequence[int]) -> int:
        """Close a segment (victims: sorted distinct rows < n). Returns its index."""
        v = list(victims)
        off = self._put(np.asarray(v, np.int64)) if v else 0
        s = self.nseg
        self.prog += [OP_SEGEND, off, len(v), s]
        self.seg_vic.append(v)
        self.nseg += 1
        self.max_nv = max(self.max_nv, len(v))
        self.n_vinfo += 3 * len(v)
        return s

    def point(self) -> int:
        p = self.npoints
        self.prog += [OP_POINT, p]
        self.npoints += 1
        return p

    # ---- run
    def run(self, shard_count: List[int], E: Optional[torch.Tensor] = None, cc: Optional[Dict] = None) -> Dict:
        """Upload and execute. ``E``: the facts' embeddings (device fp32 [M, D])
        the :meth:`embeddings` indices refer to. ``cc``: the batch's
        incremental components (TenantGraph._cc with a stable prefix) -- the
        suffix-only segment ends and the incremental digest. Returns the
        per-segment / per-point records and the device outputs (the caller
        adopts the edges and builds captures)."""
        g = self.g
        dev = g.device
        self.prog.append(OP_END)
        prog = np.asarray(self.prog, np.int64)
        # the byte block: one pinned buffer, one copy
        nb = max(self._nbytes, 8)
        hblk = torch.empty(nb, dtype=torch.uint8).pin_memory()
        hb = hblk.numpy()
        o = 0
        for a in self._parts:
            hb[o:o + a.size] = a
            o += a.size
        D = int(g.dim or 1)
        with g.on_stream():
            blk = hblk.to(dev, non_blocking=True)
            if self._x_idx:  # every inserted row's embedding by ONE gather
                src = [E.to(dev, torch.float32)] if E is not None else []
                src += [x.to(dev, torch.float32) for x in self._x_extra]
                base = torch.cat(src) if len(src) > 1 else src[0]
                m0 = int(E.shape[0]) if E is not None else 0
                idx = np.asarray(self._x_idx, np.int64)
                idx = np.where(idx < 0, m0 + (-idx - 1), idx)
                xblk = base[torch.from_numpy(idx).to(dev, non_blocking=False)].contiguous()
            else:
                xblk = torch.zeros((1, D), dtype=torch.float32, device=dev)
            ne0 = g.num_edges
            cap_e = ne0 + self.total_app
            extra = max(cap_e >> 3, g.EDGE_SLACK_MIN)
            ns = int(cc["ns"]) if cc is not None else 0
            sets = [{}, {}]
            for k in T.EDGE_COLS:
                v = g.e[k]
                base_ = v._base if v._base is not None else v
                if ns and v.data_ptr() == base_.data_ptr() and base_.numel() >= cap_e:
                    sets[0][k] = base_  # the partitioned list in place: its prefix never moves
                else:
                    b = torch.empty(cap_e + extra, dtype=v.dtype, device=dev)
                    if ne0:
                        b[:ne0].copy_(v)
                    sets[0][k] = b
                # set B: the ping-pong partner, or (partitioned) the suffix's compaction scratch
                sets[1][k] = torch.empty(max(cap_e - ns, 1) + (0 if ns else extra), dtype=v.dtype, device=dev)
            words = (g.cap + 31) // 32
            if g._rmb is None or g._rmb.numel() < words:
                g._rmb = torch.zeros(words, dtype=torch.int32, device=dev)
            if g._dv_acc is None:
                g._dv_acc = torch.zeros(1, dtype=torch.float32, device=dev)
            flag_a = torch.empty(max(cap_e, 1), dtype=torch.uint8, device=dev)
            flag_b = torch.empty(max(cap_e, 1), dtype=torch.uint8, device=dev)
            bc = torch.empty(max(1, (cap_e + T.NTB - 1) // T.NTB), dtype=torch.int32, device=dev)
            info = torch.empty(3 * self.max_nv + 2, dtype=torch.int32, device=dev)
            track = bool(g.track)
            drop = [torch.empty(max(cap_e, 1), dtype=torch.int32, device=dev) for _ in range(3)] if track else None
            dg_cap = 2 * T.dg_small_max_edges()
            P_ = max(self.npoints, 1)
            dg_out = torch.empty((P_, 2, dg_cap), dtype=torch.int64, device=dev)
            dg_ws = torch.empty(int(_lib.lib().lzk_dg_small_ws(dg_cap // 2)), dtype=torch.uint8, device=dev)
            dg_cnt = torch.empty(1, dtype=torch.int32, device=dev)
            fr_out = torch.full((P_, max(self.k_first, 1)), -1, dtype=torch.int64, device=dev)
            i8 = g.emb8 is not None and g.emb8.dtype == torch.int8
            # lazy node decay (apply.hip): per-row stamps, all zero between runs
            stamp = None
            if LAZY_NODE_DECAY:
                stamp = getattr(g, "_dstamp", None)
                if stamp is None or stamp.numel() < g.cap:
                    stamp = g._dstamp = torch.zeros(g.cap, dtype=torch.int32, device=dev)
            cols = np.asarray([
                g.sal.data_ptr(), g.acc.data_ptr(), g.last.data_ptr(), g.ts.data_ptr(), g.shard.data_ptr(),
                g.sup.data_ptr(), g.parent.data_ptr(), g.kind.data_ptr(), g.stored.data_ptr(), g.dirty.data_ptr(),
                g.emb32.data_ptr(), _lib.ptr(g.emb16), g.emb8.data_ptr() if i8 else 0,
                g.rs8.data_ptr() if i8 else 0, g.sqn.data_ptr(), g.sumsq.data_ptr(),
                g._rs8_max.data_ptr() if i8 else 0, g._dv_acc.data_ptr(), g.has_emb.data_ptr(),
                g._rmb.data_ptr(), stamp.data_ptr() if stamp is not None else 0], dtype=np.uint64)
            eb = [np.asarray([sets[s][k].data_ptr() for k in T.EDGE_COLS], dtype=np.uint64) for s in range(2)]
            sc = np.asarray(list(shard_count) or [0], dtype=np.int64)
            seg_out = np.zeros(4 * max(self.nseg, 1), np.int64)
            vinfo = np.zeros(max(self.n_vinfo, 1), np.int32)
            point_out = np.zeros(5 * P_, np.int64)
            state = np.zeros(4, np.int64)
            ccp = None
            if cc is not None:
                nc = int(g.cap)  # workspace rows: every row the batch can reach
                take = max(self.k_first, 1)
                ws = {"lab": torch.empty(nc, dtype=torch.int32, device=dev),
                      "zero": torch.zeros(max(nc, int(cc["n0"]) + 65536), dtype=torch.uint8, device=dev),
                      "touched": torch.empty(nc, dtype=torch.uint8, device=dev),
                      "gsum": torch.empty(nc, dtype=torch.float64, device=dev),
                      "gi": torch.empty(3 * nc, dtype=torch.int32, device=dev),
                      "gfirst": torch.empty(nc, dtype=torch.int64, device=dev),
                      "cls": torch.empty(nc, dtype=torch.uint8, device=dev),
                      "biglist": torch.empty(nc // (take + 1) + 1, dtype=torch.int32, device=dev),
                      "counters": torch.zeros(4, dtype=torch.int32, device=dev),
                      "keys": torch.empty(nc, dtype=torch.int64, device=dev),
                      "rows": torch.empty(nc, dtype=torch.int32, device=dev),
                      "cur": torch.empty(nc, dtype=torch.int32, device=dev),
                      "last": torch.empty(nc, dtype=torch.int32, device=dev),
                      "cnt": torch.empty(nc, dtype=torch.int32, device=dev),
                      "rem": torch.zeros(1, dtype=torch.int32, device=dev)}
                base_lab = cc["lab"].to(torch.int32).contiguous()
                ws["base"] = base_lab
                ccp = np.asarray([
                    ns, 1, base_lab.data_ptr(), int(cc["n0"]), ws["lab"].data_ptr(), ws["zero"].data_ptr(),
                    ws["touched"].data_ptr(), ws["gsum"].data_ptr(), ws["gi"].data_ptr(), ws["gfirst"].data_ptr(),
                    ws["cls"].data_ptr(), ws["biglist"].data_ptr(), ws["counters"].data_ptr(), ws["keys"].data_ptr(),
                    ws["rows"].data_ptr(), nc, ws["cur"].data_ptr(), ws["last"].data_ptr(), ws["cnt"].data_ptr(),
                    ws["rem"].data_ptr(), int(T.DIGEST_WINDOW), nc], dtype=np.int64)
            rc = _lib.lib().lzk_apply_segments(
                prog.ctypes.data, int(prog.size), blk.data_ptr(), xblk.data_ptr(), D,
                cols.ctypes.data, g.emb32.stride(0), g.emb16.stride(0) if g.emb16 is not None else 0,
                g.emb8.stride(0) if i8 else 0, eb[0].ctypes.data, eb[1].ctypes.data, ne0, cap_e,
                self.thr, self.keep, self.now, self.meta_bits, 1,
                flag_a.data_ptr(), flag_b.data_ptr(), bc.data_ptr(), info.data_ptr(), int(info.numel()),
                *((d.data_ptr() for d in drop) if drop else (None, None, None)), int(cap_e if track else 0),
                dg_out.data_ptr(), dg_cap, dg_ws.data_ptr(), dg_cnt.data_ptr(), fr_out.data_ptr(),
                max(self.k_first, 1), sc.ctypes.data, int(len(shard_count)), seg_out.ctypes.data,
                vinfo.ctypes.data, int(vinfo.size), point_out.ctypes.data, state.ctypes.data,
                ccp.ctypes.data if ccp is not None else None, _lib.stream_ptr(dev))
            if rc != 0 and stamp is not None:
                stamp.zero_()  # a failed run leaves no stale stamps behind
            _lib.check(rc, "lzk_apply_segments")
            ne, cur, nd = int(state[0]), int(state[1]), int(state[2])
            g._adopt_edges({k: sets[cur][k][:ne] for k in T.EDGE_COLS})
            dig = np.zeros(0, np.int64)
            if ccp is not None:
                nd_ = int(_lib.lib().lzk_apply_dig_size())
                dig = np.zeros(2 * nd_, np.int64)
                if nd_:
                    _lib.lib().lzk_apply_dig_copy(dig.ctypes.data)
            # every point's capture slots in one device -> host copy each
            # (the captures slice them after one event)
            P_used = max(self.npoints, 1)
            h_dg = torch.empty((P_used, 2, dg_cap), dtype=torch.int64, pin_memory=True)
            h_fr = torch.empty((P_used, max(self.k_first, 1)), dtype=torch.int64, pin_memory=True)
            if self.npoints:
                h_dg.copy_(dg_out[:P_used], non_blocking=True)
                h_fr.copy_(fr_out[:P_used], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            # the block / workspaces must outlive the queued kernels
            for t in [blk, xblk, flag_a, flag_b, bc, info, dg_ws, dg_cnt] + (drop or []):
                t.record_stream(torch.cuda.current_stream(dev))
        return {"seg_out": seg_out.reshape(-1, 4), "vinfo": vinfo, "point_out": point_out.reshape(-1, 5),
                "shard_count": sc, "h_dg": h_dg, "h_fr": h_fr, "ev": ev, "drop": drop, "n_drop": nd,
                "ne": ne, "dig": dig.reshape(-1, 2)}

    # ---- host replay of a segment end (TenantGraph._segment_end_fused's tail)
    def finish_segment(self, res: Dict, s: int) -> int:
        """Host bookkeeping of segment ``s`` after the run: counters,
        children, deleted ids, dropped edges. Returns the decay's prune count."""
        g = self.g
        so = res["seg_out"][s]
        vic = self.seg_vic[s]
        nv = len(vic)
        if nv:
            vi = res["vinfo"][int(so[3]): int(so[3]) + 3 * nv]
            kinds, sups, shards = vi[:nv], vi[nv:2 * nv], vi[2 * nv:3 * nv]
            for r, k, sp, sh in zip(vic, kinds.tolist(), sups.tolist(), shards.tolist()):
                if k != NODE:
                    continue
                if sp:
                    g.n_super -= 1
                elif sh >= 0:
                    g.shard_count[sh] -= 1
                g.children.pop(r, None)
                g.odd_emb.pop(r, None)
                g.deleted_ids[g.ids[r]] = None
        nd = int(so[2])
        if nd and res["drop"] is not None:
            off = res.setdefault("_drop_off", 0)
            g._note_dropped(*(d[off:off + nd] for d in res["drop"]))
            res["_drop_off"] = off + nd
        g._bump(edges=True, store=bool(nv))
        return int(so[0])

    @staticmethod
    def captures(res: Dict, p: int):
        """(digest, first rows) of point ``p`` as Captures
        (TenantGraph.digest_capture / first_rows_capture): slices of the
        run's bulk host copies, read after its one event."""
        po = res["point_out"][p]
        kind, nf = int(po[1]), int(po[2])
        if kind == 1:
            dig = _Slice(res, lambda r: T.digest_lists(r["h_dg"][p].numpy()))
        elif kind == 2:  # the incremental digest's sorted (key, row) pairs
            o, m = int(po[3]), int(po[4])
            kr = res["dig"][o:o + m]
            dig = Capture(host=np.split(kr[:, 1], np.nonzero(np.diff(kr[:, 0]))[0] + 1) if m else [])
        else:
            dig = Capture(host=[])
        if nf:
            first = _Slice(res, lambda r: (lambda a: a[a >= 0])(r["h_fr"][p, :nf].numpy()))
        else:
            first = Capture(host=np.zeros(0, np.int64))
        return dig, first


class _Slice:
    """A Capture-like view of one point of a native run's bulk host copy."""
    __slots__ = ("_res", "_fn", "_val", "_done")

    def __init__(self, res: Dict, fn):
        self._res, self._fn, self._val, self._done = res, fn, None, False

    def get(self):
        if not self._done:
            self._res["ev"].synchronize()
            self._val = self._fn(self._res)
            self._done = True
            self._res = None
        return self._val
