"""Tenant reload speed (round-1 verdict #8; reference memory_system.py:1304-1410):
persist an N-row tenant (default 10M x 768 fp32 + the reference's columns)
through the incremental commit, then time a fresh ``MemorySystem`` loading it
back into HBM -- store scan (Arrow IPC fragments -> columns) and the bulk load
into the tenant graph (vectors: host -> device copy) timed separately.
Synthetic rows (random unit vectors). The file was just written, so the page
cache is warm: this measures the load path, not the disk.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--db", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from bench import populate
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    from lazzaro_amd.core import memory_system as MSmod

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    db = a.db or tempfile.mkdtemp(prefix="lzk_reload_")

    def make(load):
        return MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=a.dim), enable_async=False,
                            db_dir=db, user_id="big", device=str(dev), load_from_disk=load)
    ms = make(False)
    t0 = time.time()
    populate(ms, a.rows, a.dim, dev, 3)
    g = ms.graph
    with g.on_stream():
        g.stored[: g.n] = 0
        g.dirty[: g.n] = 1
    torch.cuda.synchronize() if dev.type == "cuda" else None
    log(f"populated {a.rows:,} rows in {time.time() - t0:.1f}s")
    t0 = time.time()
    ms._save_to_persistence()
    t_commit = time.time() - t0
    log(f"committed in {t_commit:.1f}s")
    ref = g.emb32[: min(g.n, 1000)].cpu()
    ms.close()
    del ms, g
    torch.cuda.empty_cache() if dev.type == "cuda" else None

    st = {}
    orig_bulk, orig_scan = MSmod.bulk_load, None

    def timed_bulk(*args, **kw):
        t = time.time()
        r = orig_bulk(*args, **kw)
        torch.cuda.synchronize() if dev.type == "cuda" else None
        st["bulk_load_s"] = time.time() - t
        return r
    MSmod.bulk_load = timed_bulk
    from lazzaro_amd.core.vector_store import HBMStore
    orig_scan = HBMStore.load_tenant

    def timed_scan(self, user):
        t = time.time()
        r = orig_scan(self, user)
        st["store_scan_s"] = time.time() - t
        return r
    HBMStore.load_tenant = timed_scan
    prof = None
    if os.environ.get("LZK_PROF_HOST") == "1":  # host-side profile of the reload (stderr)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.time()
    ms2 = make(True)
    torch.cuda.synchronize() if dev.type == "cuda" else None
    t_load = time.time() - t0
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(25)
    ok = ms2.graph.n == a.rows and torch.equal(ms2.graph.emb32[: ref.shape[0]].cpu(), ref)
    du = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(db) for f in fs)
    out = {"metric": "tenant reload (store -> HBM tenant graph)", "rows": a.rows, "dim": a.dim,
           "bytes_on_disk": du, "commit_s": round(t_commit, 2), "reload_s": round(t_load, 2),
           "store_scan_s": round(st.get("store_scan_s", -1), 2), "bulk_load_s": round(st.get("bulk_load_s", -1), 2),
           "rows_per_s": round(a.rows / t_load), "gb_per_s": round(du / t_load / 1e9, 2), "vectors_equal": bool(ok),
           "page_cache": "warm (just written)"}
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    ms2.close()


if __name__ == "__main__":
    main()
