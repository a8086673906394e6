"""Child of tests/kernels/test_rccl_world1_gpu.py, started by
``torch.distributed.run --nproc-per-node 1`` before it touches the GPU: the
serving and row-sharded paths of an N-GPU job with every exchange forced
through the RCCL (``nccl``) process group at world 1 -- routed search (host
path and device key directory), global search, live migration and the
row-sharded tenant's consolidation -- each checked against its truth.
Prints one JSON line."""
import functools
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from lazzaro_amd.parallel import Communicator
    comm = Communicator.init("nccl")
    import torch
    import torch.distributed as dist

    from lazzaro_amd.parallel import routing
    from tests.distributed import test_routing_gloo as R
    from tests.distributed import test_sharded_memory_gloo as SH
    out = {"backend": dist.get_backend(), "world": comm.world, "device": str(comm.device)}

    def gpu_factory(db, user, load_from_disk=False):
        from lazzaro_amd.core.memory_system import MemorySystem
        from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
        return MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=R.D), enable_async=False,
                            db_dir=db, user_id=user, device="cuda", load_from_disk=load_from_disk,
                            max_buffer_size=10 ** 6)
    R._factory = gpu_factory
    for device_dir in (False, True):
        res = json.loads(R._workload(comm, tempfile.mkdtemp(prefix="rccl_w1_"), force=True, device_dir=device_dir))
        routing.BIG_ROWS = 1 << 18
        qs = R._queries(0)
        names = {int(s): n for s, n in res["names"].items()}
        out[f"routed_dir{int(device_dir)}"] = {
            "exact": res["ids"] == R._truth(qs, res["users"], res["limits"]) and res["same"],
            "global_exact": [[(names[sl], row) for rk, sl, row in q] for q in res["global"]]
            == R._global_truth(qs[:5], 4),
            "route_stats": res["route_stats"], "force": res["force"]}

    # live migration: every tenant "moves" to the rank that holds it -- the
    # exchanges run (zero-row all-to-all-v over RCCL), nothing is rebuilt
    from lazzaro_amd.core.providers import HashEmbedder
    from lazzaro_amd.parallel.service import DistributedMemoryService
    svc = DistributedMemoryService(comm, functools.partial(gpu_factory, tempfile.mkdtemp()),
                                   embedder=HashEmbedder(dim=R.D), force_collectives=True)
    for u in R.USERS[:3]:
        R._fill(svc.system(u), u)
    got = svc.migrate({u: 0 for u in R.USERS[:3]})
    hits = svc.search_routed(R.USERS[:3], R._queries(0, 3), 4)
    out["migrate"] = {"received": got, "resident": sorted(svc.systems),
                      "search_ok": bool((hits.rows >= 0).all())}
    svc.close()

    # row-sharded tenant, batch cadence, every collective on RCCL
    cfg = {"rows": 30_000, "dim": 64, "limit": 30_040, "steps": 2, "convs": 24, "device": "cuda", "force": True}
    sh = SH._sharded(comm, cfg=cfg)
    SH.check_equivalent({0: sh}, 1, cfg["limit"])
    out["sharded_equal"] = True
    # ... and at the reference's per-conversation cadence
    sh = SH._sharded(comm, cfg=dict(cfg, cadence="conversation"))
    SH.check_equivalent({0: sh}, 1, cfg["limit"])
    out["sharded_exact_cadence_equal"] = True
    torch.cuda.synchronize()
    dist.barrier()
    print("RESULT " + json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
