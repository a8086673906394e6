"""BASELINE config 3 through the product API: many small tenants per GPU
served by ``DistributedMemoryService`` -- each tenant a ``MemorySystem`` with
its graph in HBM, every query routed to its tenant's owner (all-to-all-v for
N > 1), the owner's queries answered by ONE embed + ONE multi-tenant
``segment_topk`` launch over the tenants' fp32 rows (exact L2), results
materialised as Node dicts.

Synthetic: random unit memory vectors (``--rows`` per tenant on average),
synthetic query texts, random-init encoder weights. Prints one JSON line
(rank 0). Run under torchrun for N ranks (127.0.0.1 rendezvous).
"""
import argparse
import json
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users-total", type=int, default=100_000)
    ap.add_argument("--rows", type=int, default=800, help="mean memories per user")
    ap.add_argument("--batch", type=int, default=1024, help="queries per rank per step")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="bge-base")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--stream", type=int, default=1, help="1: serve_stream (pipelined rounds), 0: serve per round")
    ap.add_argument("--global-batch", type=int, default=128,
                    help="queries per rank of the global (every-tenant) search; 0 = skip")
    ap.add_argument("--global-steps", type=int, default=5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    import tempfile

    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import LocalLLM
    from lazzaro_amd.core.vector_store import HBMStore
    from lazzaro_amd.parallel import Communicator
    from lazzaro_amd.parallel.service import DistributedMemoryService

    comm = Communicator.init() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else Communicator.local()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    emb = OnDeviceEmbedder(a.model, device=dev, max_len=32)
    db = tempfile.mkdtemp(prefix=f"lzmt{comm.rank}_")
    store = HBMStore(db_dir=db, device=dev)

    def factory(user, load_from_disk=False):
        return MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, enable_async=False, db_dir=db,
                            user_id=user, store=store, device=dev, load_from_disk=load_from_disk,
                            max_buffer_size=10 ** 9, enable_caching=False)
    svc = DistributedMemoryService(comm, factory)
    users = [f"user{i}" for i in range(a.users_total)]
    mine = [u for u in users if svc.is_local(u)]
    rng = random.Random(comm.rank)
    gen = torch.Generator(device=dev).manual_seed(comm.rank)
    t0 = time.time()
    rows_total = 0
    for j, u in enumerate(mine):
        ms = svc.system(u)
        n = rng.randint(a.rows // 4, a.rows * 7 // 4)
        V = torch.randn(n, a.dim, device=dev, generator=gen)
        V /= V.norm(dim=1, keepdim=True)
        g = ms.graph
        g.add_nodes([f"{u}_m{i}" for i in range(n)], [f"memory {i} of {u}" for i in range(n)], V,
                    shard=g.shard_id("default"), stored=True)
        g.store_bias("l2")  # the store's row mask + -|x|^2, built once per tenant version (as after a load)
        rows_total += n
        if j % 2000 == 0:
            log(f"rank {comm.rank}: {j}/{len(mine)} tenants, {rows_total:,} rows ({time.time() - t0:.0f}s)")
    torch.cuda.synchronize()
    t_pop = time.time() - t0
    svc.warm_table()  # the resident tenants' device pointer table, built once at load like an index
    words = "memory user likes python graph kernel music travel project deadline family hobby".split()

    def batch():
        return [(rng.choice(users), "search_memories", " ".join(rng.choice(words) for _ in range(12)), a.k)
                for _ in range(a.batch)]
    for _ in range(a.warmup):
        svc.serve(batch())
    reqs = [batch() for _ in range(a.steps)]
    torch.cuda.synchronize()
    comm.barrier()
    prof = None
    if os.environ.get("LZK_PROF_HOST") == "1":  # host-side profile of the timed loop (stderr)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    outs = list(svc.serve_stream(reqs)) if a.stream else [svc.serve(r) for r in reqs]
    torch.cuda.synchronize()
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(15)
        pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(35)
    comm.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    comm.all_reduce(t, "max")
    el = float(t.item())
    # exactness: this rank's LOCAL requests of the last step against each
    # tenant's own store search with the SAME query embeddings (an encoder
    # batch of 1 rounds differently from a batch of 1024)
    agree = tot = 0
    last = [(i, r) for i, r in enumerate(reqs[-1]) if svc.is_local(r[0])]
    if last:
        E = emb.batch_embed_tensor([r[2] for _, r in last]) if hasattr(emb, "batch_embed_tensor") else None
        E = E[0] if isinstance(E, tuple) else E
        for j, (i, (u, _, q, k)) in enumerate(last[:64]):
            g = svc.system(u).graph
            _, rr = g.store_search(E[j:j + 1].float(), k)
            kind = g.mirror("kind")
            ref = [g.ids[int(r)] for r in rr[0].tolist() if r >= 0 and kind[int(r)] == 1]
            agree += int([n["id"] for n in outs[-1][i]] == ref)
            tot += 1
    ok = torch.tensor([agree, tot], dtype=torch.int64, device=dev)
    comm.all_reduce(ok)
    rt = torch.tensor([rows_total], dtype=torch.int64, device=dev)
    comm.all_reduce(rt)
    res = {"metric": "multi-tenant search_memories QPS through DistributedMemoryService", "value":
           round(comm.world * a.batch * a.steps / el, 1), "unit": "queries/s", "n_gpus": comm.world,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
           "users_total": a.users_total, "users_per_gpu": len(mine), "rows_total": int(rt.item()),
           "batch_per_rank": a.batch, "k": a.k, "model": a.model, "populate_s": round(t_pop, 1),
           "exact_match_vs_per_tenant_search": f"{int(ok[0])}/{int(ok[1])}",
           "path": ("serve_stream() (round i+1 enqueued before round i is materialised)" if a.stream else "serve()")
           + " -> owner's one embed + one segment_topk over tenants' fp32 rows -> Node dicts",
           "data": "synthetic (random unit vectors, synthetic query texts, random-init encoder)"}
    if a.global_batch > 0 and a.global_steps > 0:
        res["global"] = run_global(svc, comm, emb, dev, a, words, rng)
    from lazzaro_amd.utils.tracing import tracer
    if tracer.enabled:
        res["stages_ms"] = {k: v["p50_ms"] for k, v in tracer.summary().items()}
    if comm.rank == 0:
        print(json.dumps(res), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(json.dumps(res) + "\n")
    svc.close()


def run_global(svc, comm, emb, dev, a, words, rng):
    """Global search (every query against EVERY tenant of every rank:
    DistributedMemoryService.search_global_batch) on pre-embedded queries:
    the rank's small tenants in one tile-table MFMA pass (mtscan.hip), the
    candidates all-to-all'ed back to their origin for N > 1. Exactness: the
    first batch against the per-tenant store searches (LZK_MT_GLOBAL=0)."""
    from lazzaro_amd.parallel import routing
    qs = [" ".join(rng.choice(words) for _ in range(12)) for _ in range(a.global_batch * (a.global_steps + 2))]
    E = emb.batch_embed_tensor(qs) if hasattr(emb, "batch_embed_tensor") else None
    E = (E[0] if isinstance(E, tuple) else E).float()
    Eb = [E[i * a.global_batch:(i + 1) * a.global_batch] for i in range(a.global_steps + 2)]
    routing.search_global_batch(svc, Eb[0], a.k)  # warm (tile table build)
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for i in range(a.global_steps):
        got = routing.search_global_batch(svc, Eb[1 + i], a.k)
    torch.cuda.synchronize()
    comm.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    comm.all_reduce(t, "max")
    el = float(t.item())
    chk = routing.search_global_batch(svc, Eb[-1][:64], a.k)
    mt = routing.MT_GLOBAL
    routing.MT_GLOBAL = False
    try:
        ref = routing.search_global_batch(svc, Eb[-1][:64], a.k)
    finally:
        routing.MT_GLOBAL = mt
    same = int(torch.equal(chk.keys, ref.keys))
    ok = torch.tensor([same, 1], dtype=torch.int64, device=dev)
    comm.all_reduce(ok)
    return {"qps": round(comm.world * a.global_batch * a.global_steps / el, 1),
            "qps_per_gpu": round(a.global_batch * a.global_steps / el, 1),
            "ms_per_step": round(el / a.global_steps * 1e3, 3), "batch_per_rank": a.global_batch,
            "exact_match_vs_per_tenant_search": f"{int(ok[0])}/{int(ok[1])} ranks (64 queries each)",
            "path": "routing.search_global_batch: small tenants in one tile-table MFMA pass (mtscan.hip) + "
                    "fp32 re-rank; all-gather of queries / all-to-all of candidates for N > 1"}


if __name__ == "__main__":
    main()
