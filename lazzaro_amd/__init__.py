"""lazzaro_amd -- an MI355X-native long-term memory engine for AI agents.

Same capabilities and Python API as thelaycon/lazzaro (``MemorySystem`` with
chat / chat_stream / end_conversation / run_consolidation / search_memories,
multi-tenant users, evolving profile, decay & pruning, super-nodes, export,
CLI, dashboard, agent-framework adapters), re-designed around an HBM-resident
vector arena, hand-written CDNA4 HIP kernels and RCCL over xGMI.
"""
__version__ = "0.1.0"

__all__ = ["MemorySystem"]


def __getattr__(name):
    if name == "MemorySystem":
        from .core.memory_system import MemorySystem
        return MemorySystem
    raise AttributeError(name)
