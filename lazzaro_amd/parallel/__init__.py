"""Multi-GPU layer: RCCL communicator, tenant placement, row-sharded search,
all-to-all re-sharding and distributed graph maintenance."""
from .comm import Communicator  # noqa: F401
from .placement import TenantDirectory, tenant_rank  # noqa: F401
from .sharded import ShardedIndex, distributed_components, merge_topk  # noqa: F401
from .sharded_memory import ShardedMemorySystem  # noqa: F401
