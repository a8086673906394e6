"""Communicator: one process per GPU over ``torch.distributed``.

Backend ``nccl`` is RCCL on ROCm (GPU tensors, xGMI); ``gloo`` is used for CPU
tensors (tests, host metadata). The collectives this engine needs
(SURVEY.md §2.5):

* ``all_gather_rows``  C1 cross-shard search candidates, C7 tenant directory
* ``all_to_all_v``     C3 re-sharding rows after consolidation (variable sizes,
                       count exchange first); all-to-all uses every xGMI link
                       at once instead of a one-link-bound ring
* ``all_reduce``       C4 k-means partial sums, C5 component labels
* ``barrier``          C6 multi-rank commit

``Communicator.local()`` is the world-of-one stand-in so single-process code
paths call the same API.

Host metadata (split sizes, tenant announcements, directory entries) travels
on a second, gloo group between the same ranks (``host_all_gather``,
``exchange_objects``): reading a count exchanged over RCCL back to the host
would wait for everything queued before it on the GPU stream, so a serving
loop that learns its all-to-all split sizes over gloo never stalls its GPU
pipeline on a device-to-host copy.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..utils.faults import CommError, fault_point


def _guarded(name):
    """Fault point + typed error for one collective."""
    def deco(fn):
        def wrapper(self, *a, **kw):
            fault_point("comm." + name)
            if not self.enabled:
                return fn(self, *a, **kw)
            try:
                return fn(self, *a, **kw)
            except CommError:
                raise
            except (RuntimeError, ValueError) as e:  # DistBackendError / timeouts derive from RuntimeError
                raise CommError(f"{name} failed on rank {self.rank}/{self.world}: {e}") from e
        wrapper.__name__ = fn.__name__
        wrapper.__doc__ = fn.__doc__
        return wrapper
    return deco


class Communicator:
    def __init__(self, group=None, device: Optional[torch.device] = None):
        self.group = group
        self.enabled = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if self.enabled else 0
        self.world = dist.get_world_size(group) if self.enabled else 1
        if device is None:
            be = dist.get_backend(group) if self.enabled else "gloo"
            device = torch.device("cuda", torch.cuda.current_device()) if be == "nccl" else torch.device("cpu")
        self.device = torch.device(device)
        self._host_group = None
        if self.enabled:
            # collective (SPMD): every rank constructs its Communicator together
            be = dist.get_backend(group)
            self._host_group = group if be == "gloo" else dist.new_group(
                ranks=None if group is None else dist.get_process_group_ranks(group), backend="gloo")

    @classmethod
    def local(cls, device=None) -> "Communicator":
        c = cls.__new__(cls)
        c.group, c.enabled, c.rank, c.world = None, False, 0, 1
        c.device = torch.device(device) if device is not None else torch.device("cpu")
        c._host_group = None
        return c

    @classmethod
    def init(cls, backend: Optional[str] = None) -> "Communicator":
        """Initialise from torchrun env vars (RANK/WORLD_SIZE/MASTER_ADDR...)."""
        if not dist.is_initialized():
            if int(os.environ.get("WORLD_SIZE", "1")) == 1 and "MASTER_ADDR" not in os.environ:
                return cls.local()
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            kw = {}
            if backend == "nccl":
                local = int(os.environ.get("LOCAL_RANK", "0"))
                torch.cuda.set_device(local)
                kw["device_id"] = torch.device("cuda", local)
            dist.init_process_group(backend, **kw)
        return cls()

    # ---------------------------------------------------------------- basics
    @_guarded("barrier")
    def barrier(self) -> None:
        if self.enabled:
            dist.barrier(group=self.group)

    @_guarded("all_reduce")
    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.enabled:
            ops = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}
            dist.all_reduce(t, op=ops[op], group=self.group)
        return t

    @_guarded("broadcast")
    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.enabled:
            dist.broadcast(t, src=src, group=self.group)
        return t

    @_guarded("all_gather_rows")
    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate equal-shaped tensors from every rank along dim 0."""
        if not self.enabled:
            return t
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out

    @_guarded("all_gather_object")
    def all_gather_object(self, obj) -> List:
        if not self.enabled:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self._host_group)  # pickled bytes over gloo: no GPU sync
        return out

    # ---------------------------------------------------------------- all-to-all-v
    @_guarded("exchange_counts")
    def exchange_counts(self, send_counts: torch.Tensor) -> torch.Tensor:
        if not self.enabled:
            return send_counts.clone()
        recv = torch.empty_like(send_counts)
        dist.all_to_all_single(recv, send_counts, group=self.group)
        return recv

    @_guarded("host_counts")
    def host_counts(self, send_counts: Sequence[int]) -> List[int]:
        """Host-side count exchange (gloo): ``send_counts[r]`` items for rank
        r -> the count each rank sends here. The split sizes of an
        :meth:`all_to_all_v` without a device-to-host read."""
        if not self.enabled:
            return [int(x) for x in send_counts]
        send = torch.tensor([int(x) for x in send_counts], dtype=torch.int64)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self._host_group)
        return recv.tolist()

    @_guarded("all_to_all_v")
    def all_to_all_v(self, t: torch.Tensor, send_counts: Sequence[int], recv_counts: Sequence[int]) -> torch.Tensor:
        """Rows of ``t`` are grouped by destination rank (send_counts[r] rows
        for rank r, in rank order); returns rows received, grouped by source."""
        if not self.enabled:
            return t
        out = torch.empty((int(sum(recv_counts)),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_to_all_single(out, t.contiguous(), output_split_sizes=list(map(int, recv_counts)),
                               input_split_sizes=list(map(int, send_counts)), group=self.group)
        return out

    # ---------------------------------------------------------------- host metadata (gloo)
    @_guarded("host_all_gather")
    def host_all_gather(self, a) -> "np.ndarray":
        """All-gather of a small host int64 array over the gloo group:
        returns [world, *a.shape] (no GPU stream involved)."""
        import numpy as np
        a = np.ascontiguousarray(np.asarray(a, np.int64))
        if not self.enabled:
            return a[None]
        t = torch.from_numpy(a.reshape(-1).copy())
        out = torch.empty(self.world * t.numel(), dtype=torch.int64)
        dist.all_gather_into_tensor(out, t, group=self._host_group)
        return out.numpy().reshape((self.world,) + a.shape)

    @_guarded("exchange_objects")
    def exchange_objects(self, outgoing: List) -> List:
        """``outgoing[r]`` = a JSON-able object for rank r -> the objects
        received, one per source rank (JSON bytes over one gloo all-to-all-v:
        host metadata never touches the GPU stream)."""
        if not self.enabled:
            return list(outgoing)
        payload = [json.dumps(x).encode() for x in outgoing]
        send = torch.tensor([len(p) for p in payload], dtype=torch.int64)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self._host_group)
        buf = torch.frombuffer(bytearray(b"".join(payload)), dtype=torch.uint8) if sum(map(len, payload)) else \
            torch.zeros(0, dtype=torch.uint8)
        out_t = torch.empty(int(recv.sum()), dtype=torch.uint8)
        dist.all_to_all_single(out_t, buf, output_split_sizes=recv.tolist(), input_split_sizes=send.tolist(),
                               group=self._host_group)
        got = out_t.numpy().tobytes()
        out, off = [], 0
        for n in recv.tolist():
            out.append(json.loads(got[off: off + n].decode()) if n else None)
            off += n
        return out

    def reshard(self, dest: torch.Tensor, *fields: torch.Tensor) -> Tuple[torch.Tensor, ...]:
        """Route every row of each field to rank ``dest[row]`` (C3). Returns the
        fields as received on this rank (grouped by source rank, original
        relative order preserved)."""
        order = torch.argsort(dest, stable=True)
        s_list = torch.bincount(dest.long(), minlength=self.world).to(torch.int64).tolist()
        r_list = self.host_counts(s_list)
        return tuple(self.all_to_all_v(f[order.to(f.device)], s_list, r_list) for f in fields)
