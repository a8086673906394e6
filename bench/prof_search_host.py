"""Host vs device cost of the headline serving step (bench.py's
search_memories_stream over a 10M x 768 tenant): is the pipelined step bound
by the device (embed + scan) or by host work (tokenizer, launches, row ->
Node mapping)? Prints one JSON line; with --cprofile also the top host
functions of 10 streamed steps."""
import argparse
import cProfile
import io
import json
import os
import pstats
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--cprofile", action="store_true")
    a = ap.parse_args()
    from bench import SHARDS, populate, synth_texts  # noqa: F401
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import LocalLLM

    dev = torch.device("cuda", 0)
    emb = OnDeviceEmbedder("bge-base", device=dev, max_len=64, seed=0)
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, device=dev, db_dir="/tmp/lzprof",
                      load_from_disk=False, enable_async=False, max_buffer_size=2 * a.rows, user_id="u")
    populate(ms, a.rows, 768, dev, seed=1)
    g = ms.graph
    rng = random.Random(0)
    pool = [synth_texts(a.batch, rng) for _ in range(4)]
    out = {}

    def timed(fn, n=a.steps):
        fn(2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(n)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    def stream(n):
        for _ in ms.search_memories_stream((pool[i % 4] for i in range(n)), limit=10):
            pass

    out["stream_ms"] = timed(stream)

    # device-bound: pre-tokenized embed + store search, no host mapping, no sync
    toks = [emb.tok.encode_batch(p, emb.max_len) for p in pool]

    def dev_only(n):
        for i in range(n):
            Q = emb.batch_embed_tensor(pool[i % 4])
            g.store_search(Q, 10, "l2")

    out["embed_plus_search_nosync_ms"] = timed(dev_only)

    def embed_only(n):
        for i in range(n):
            emb.batch_embed_tensor(pool[i % 4])

    out["embed_only_ms"] = timed(embed_only)
    Q = emb.batch_embed_tensor(pool[0])

    def search_only(n):
        for _ in range(n):
            g.store_search(Q, 10, "l2")

    out["store_search_only_ms"] = timed(search_only)
    # host wall of each piece (device queue kept busy by the prior work)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        emb.tok.encode_batch(pool[i % 4], emb.max_len)
    out["host_tokenize_ms"] = (time.perf_counter() - t0) / a.steps * 1e3
    h = ms._search_submit(pool[0], 10)
    t0 = time.perf_counter()
    for i in range(a.steps):
        h = ms._search_submit(pool[i % 4], 10)
    out["host_submit_wall_ms"] = (time.perf_counter() - t0) / a.steps * 1e3
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ms._search_finish(h)
    out["host_finish_ms"] = (time.perf_counter() - t0) / a.steps * 1e3
    del toks
    print(json.dumps({k: round(v, 3) for k, v in out.items()}), flush=True)
    if a.cprofile:
        pr = cProfile.Profile()
        pr.enable()
        stream(a.steps)
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
        print(s.getvalue())


if __name__ == "__main__":
    main()
