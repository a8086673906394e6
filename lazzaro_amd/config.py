"""MemoryConfig: the configuration system (SURVEY.md §5 "Config / flag system").

A dataclass that is a superset of the reference's 20 ``MemorySystem`` kwargs
(same names and defaults, memory_system.py:63-84) plus the engine knobs of this
framework. Values resolve in order: defaults < environment (``LZK_<NAME>``,
e.g. ``LZK_MAX_BUFFER_SIZE=100``) < explicit arguments. ``MemorySystem.from_config``
builds a system from it; the CLI's ``/set`` keeps mutating attributes at runtime.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

REFERENCE_KWARGS = ("openai_api_key", "model", "enable_sharding", "enable_hierarchy", "enable_caching",
                    "enable_async", "max_shard_size", "super_node_threshold", "auto_consolidate",
                    "consolidate_every", "auto_prune", "prune_threshold", "max_buffer_size", "load_from_disk",
                    "db_dir", "user_id")


@dataclass
class MemoryConfig:
    # ---- reference kwargs (same defaults) ----
    openai_api_key: Optional[str] = None
    model: str = "gpt-4o-mini"
    enable_sharding: bool = True
    enable_hierarchy: bool = True
    enable_caching: bool = True
    enable_async: bool = True
    max_shard_size: int = 500
    super_node_threshold: int = 20
    auto_consolidate: bool = True
    consolidate_every: int = 3
    auto_prune: bool = True
    prune_threshold: float = 0.5
    max_buffer_size: int = 10
    load_from_disk: bool = True
    db_dir: str = "db"
    user_id: str = "default"
    # ---- engine knobs ----
    device: Optional[str] = None          # "cuda", "cuda:3", "cpu" (default: LOCAL_RANK GPU if present)
    metric: str = "l2"                    # store search metric: l2 | cosine | ip
    merge_mode: str = "reference"         # reference | pairwise
    embed_model: Optional[str] = None     # on-device encoder: minilm-l6 | bge-base | e5-large
    embed_weights: Optional[str] = None   # safetensors path (HF BERT layout)
    index: str = "flat"                   # flat | ivfpq (store: IVF-PQ for tenants >= ivf_min_rows)
    nlist: int = 4096
    nprobe: int = 32
    pq_m: int = 64
    ivf_min_rows: int = 1_000_000
    hierarchy_mode: str = "reference"     # reference (one mean super-node per shard) | kmeans (two-level)
    hierarchy_fine: int = 4096            # kmeans: fine clusters
    hierarchy_top: int = 64               # kmeans: top-level clusters
    hierarchy_every: int = 50             # kmeans: re-cluster every N conversations
    strict_errors: bool = False
    verbose: bool = False
    extra: Dict[str, Any] = field(default_factory=dict)

    @classmethod
    def from_env(cls, prefix: str = "LZK_", **overrides) -> "MemoryConfig":
        cfg = cls()
        for f in dataclasses.fields(cls):
            if f.name == "extra":
                continue
            raw = os.environ.get(prefix + f.name.upper())
            if raw is None:
                continue
            setattr(cfg, f.name, _coerce(raw, f.type, getattr(cfg, f.name)))
        for k, v in overrides.items():
            if not hasattr(cfg, k):
                raise TypeError(f"unknown config key {k!r}")
            setattr(cfg, k, v)
        return cfg

    def reference_kwargs(self) -> Dict[str, Any]:
        return {k: getattr(self, k) for k in REFERENCE_KWARGS}

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), indent=2)


def _coerce(raw: str, typ, cur):
    t = str(typ)
    if "bool" in t or isinstance(cur, bool):
        return raw.lower() in ("1", "true", "yes", "on")
    if "int" in t and "Optional" not in t:
        return int(raw)
    if "float" in t:
        return float(raw)
    return raw
