"""Multi-rank atomic commit ("barrier + rank-0 manifest
write ... gives a multi-rank atomic commit, replacing LanceDB MVCC").

Each rank writes its rows as an immutable, unpublished fragment of the shared
columnar table (`ColumnarTable.stage_rows`); the fragment descriptors are
all-gathered; rank 0 publishes every rank's fragment in ONE new manifest
version (`commit_staged`) and broadcasts it. A reader -- another process
polling `get_latest_version`, like the reference's dashboard
(memory_system.py:1412-1428) -- sees either none or all of the ranks' rows.
If any rank fails to stage, nobody commits (the collective raises everywhere).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch

from .comm import Communicator


def distributed_commit(comm: Communicator, table, rows: Sequence[Dict]) -> int:
    """Stage this rank's ``rows`` and publish all ranks' rows atomically.
    Returns the committed version (identical on every rank)."""
    try:
        staged = table.stage_rows(list(rows)) if rows else ("", 0, 0)
        ok = 1
    except Exception:
        staged, ok = ("", 0, 0), 0
    parts: List = comm.all_gather_object((ok, staged))
    if not all(p[0] for p in parts):
        raise RuntimeError("distributed_commit: a rank failed to stage; nothing committed")
    v = torch.zeros(1, dtype=torch.int64)
    if comm.rank == 0:
        v[0] = table.commit_staged([p[1] for p in parts])
    if comm.enabled:
        v = v.to(comm.device)
        comm.broadcast(v, src=0)
    comm.barrier()
    return int(v.item())
