"""Tenant placement across the GPUs of a node ("tenant-DP").

Each tenant (``user_id``) is owned by exactly one rank, chosen by rendezvous
(highest-random-weight) hashing in the native runtime: single-tenant search and
consolidation need no collective, and growing the world from N to N+1 ranks
moves only ~1/(N+1) of the tenants. Very large tenants can additionally be
row-sharded across ranks (``ShardedIndex``).
"""
from __future__ import annotations

from typing import Dict, Iterable, List

import torch


def tenant_rank(tenant: str, world: int) -> int:
    if world <= 1:
        return 0
    from ..store.colstore import _rt
    return int(_rt().tenant_rank(tenant, world))


def tenant_ranks(tenants: Iterable[str], world: int) -> torch.Tensor:
    return torch.tensor([tenant_rank(t, world) for t in tenants], dtype=torch.int64)


class TenantDirectory:
    """Rank-local tenant registry + global view via all-gather (C7)."""

    def __init__(self, comm):
        self.comm = comm
        self.local: Dict[str, int] = {}

    def owner(self, tenant: str) -> int:
        return tenant_rank(tenant, self.comm.world)

    def is_local(self, tenant: str) -> bool:
        return self.owner(tenant) == self.comm.rank

    def register(self, tenant: str, rows: int = 0) -> None:
        self.local[tenant] = self.local.get(tenant, 0) + rows

    def all_tenants(self) -> List[str]:
        parts = self.comm.all_gather_object(sorted(self.local))
        return sorted({t for p in parts for t in p})
