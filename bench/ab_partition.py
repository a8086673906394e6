"""A/B probe: the persistent-graph consolidation (10M rows, 20M edges,
prune_threshold 0) with and without the per-batch stable/volatile edge
partition (TenantGraph.PARTITION_EDGES). argv[1]: 1 / 0. Prints one JSON line
(turns/s and the traced stage p50s)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench_consolidate import run  # noqa: E402
from lazzaro_amd.core.embedders import OnDeviceEmbedder  # noqa: E402
from lazzaro_amd.engine import tenant_graph as TG  # noqa: E402
from lazzaro_amd.parallel import Communicator  # noqa: E402
from lazzaro_amd.utils.tracing import tracer  # noqa: E402


def main():
    TG.TenantGraph.PARTITION_EDGES = sys.argv[1] == "1"
    tracer.enable(True)
    comm = Communicator.init()
    dev = torch.device("cuda", 0)
    enc = OnDeviceEmbedder("bge-base", device=dev, max_len=64)
    r = run(comm, dev, 10_000_000, 128, 8, 5, 2, enc, dim=768, prune_threshold=0.0)
    st = {k: v["p50_ms"] for k, v in (r.get("stages_ms") or {}).items()
          if k in ("cb_apply", "ap_remove", "components", "run_consolidation", "consolidate_batch", "cc_begin",
                   "cc_partition")}
    print(json.dumps({"partition": TG.TenantGraph.PARTITION_EDGES, "turns_per_s": r["turns_per_s"],
                      "ms_per_step": r["ms_per_step"], "stages_p50_ms": st}), flush=True)


if __name__ == "__main__":
    main()
