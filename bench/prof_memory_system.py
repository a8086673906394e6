"""MemorySystem on a large device-resident tenant, through the public API.

A ``--nodes``-memory tenant (random unit fp32 vectors over the reference's
keyword shards, ``--edges`` random association edges) is loaded into a
``MemorySystem(device=cuda)``; then ``--convs`` conversations run the
reference lifecycle -- ``chat`` x2 (embed, hybrid retrieval over super-nodes
+ store search, neighbour boost, touch) and ``end_conversation`` (fact
extraction, batch embed, dedupe + links from the fused scan, decay + prune,
eviction to ``max_buffer_size``, incremental commit), with the automatic
``run_consolidation`` every 3 conversations (components, profile, prune).
Run under ``rocprofv3 --kernel-trace --stats`` to see the tenant kernels
(tg_decay_kernel, tg_boost_kernel, tg_touch_kernel, tg_importance_kernel,
cc_hook_kernel, flat_cand_*) on the API path.

Prints one JSON line with per-call wall times.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import SHARDS, populate  # noqa: E402

TURNS = ["I work on a robotics project with my colleague Ana and we have a deadline on Friday.",
         "My family lives in Lisbon and my hobby is sailing on weekends.",
         "I am learning Japanese from a book and practice every morning.",
         "I go to the gym for exercise and track my sleep and diet.",
         "I started a new project on GPU kernels for a client meeting.",
         "My friend Tom visits home every summer and we cook together."]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=2_000_000)
    ap.add_argument("--convs", type=int, default=6)
    ap.add_argument("--model", default="bge-base")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()
    dev = torch.device(a.device)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)

    def say(msg):
        print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)

    import faulthandler
    faulthandler.dump_traceback_later(45, repeat=True)  # where a slow step is, every 45 s
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import LocalLLM

    emb = OnDeviceEmbedder(a.model, device=dev, max_len=128)
    say("encoder ready")
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, device=dev, db_dir=tempfile.mkdtemp(),
                      load_from_disk=False, enable_async=False, max_buffer_size=a.nodes, super_node_threshold=10 ** 9)
    t0 = time.perf_counter()
    populate(ms, a.nodes, emb.dim, dev, seed=11)
    sync()
    say("populated")
    g = ms.graph
    gen = torch.Generator(device=dev).manual_seed(12)
    src = torch.randint(0, a.nodes, (a.edges,), device=dev, generator=gen, dtype=torch.int64)
    dst = torch.randint(0, a.nodes, (a.edges,), device=dev, generator=gen, dtype=torch.int64)
    w = torch.rand(a.edges, device=dev, generator=gen) * 0.5 + 0.5
    g.append_edges(src.int(), dst.int(), w, g.shard[src.long()], g.etype("relates_to"))
    g.clear_tracking(stored=False)  # the synthetic edges are not in the store
    sync()
    load_s = time.perf_counter() - t0
    say(f"loaded {a.nodes} nodes, {a.edges} edges in {load_s:.1f}s")
    times = {"chat_ms": [], "end_conversation_ms": []}
    for i in range(a.convs):
        ms.start_conversation()
        for j in range(2):
            sync()
            t = time.perf_counter()
            ms.chat(TURNS[(i + j) % len(TURNS)] + f" (conversation {i})")
            sync()
            times["chat_ms"].append((time.perf_counter() - t) * 1e3)
            say(f"chat {i}.{j}: {times['chat_ms'][-1]:.1f} ms")
        t = time.perf_counter()
        ms.end_conversation()
        sync()
        times["end_conversation_ms"].append((time.perf_counter() - t) * 1e3)
        say(f"end_conversation {i}: {times['end_conversation_ms'][-1]:.1f} ms")
    t = time.perf_counter()
    out = ms.run_consolidation()
    sync()
    rc_ms = (time.perf_counter() - t) * 1e3
    say(f"run_consolidation: {rc_ms:.1f} ms")
    t = time.perf_counter()
    res = ms.search_memories_batch(["robotics project deadline"] * 256, limit=10)
    sync()
    s_ms = (time.perf_counter() - t) * 1e3
    st = ms.get_stats()
    line = {"nodes": a.nodes, "edges_initial": a.edges, "model": a.model, "load_s": round(load_s, 2),
            "chat_ms": [round(x, 1) for x in times["chat_ms"]],
            "end_conversation_ms": [round(x, 1) for x in times["end_conversation_ms"]],
            "run_consolidation_ms": round(rc_ms, 1), "run_consolidation": out.splitlines(),
            "search_memories_batch_256_ms": round(s_ms, 1), "hits": len(res[0]),
            "buffer_nodes": st["buffer_nodes"], "buffer_edges": st["buffer_edges"],
            "conversation_count": st["conversation_count"], "shards": list(SHARDS)}
    print(json.dumps(line), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(json.dumps(line) + "\n")
    faulthandler.cancel_dump_traceback_later()
    ms.close()


if __name__ == "__main__":
    main()
