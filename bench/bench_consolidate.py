"""Consolidation at scale (BASELINE.json config 4): a large episodic buffer whose
topic shards are partitioned across the GPUs, consolidating batches of
conversations end to end on device.

One step (= ``--convs`` conversations per rank, ``--facts`` facts each):
  1. embed the extracted fact texts with the on-device encoder (bge-base)
  2. all-to-all: route every fact to the rank owning its topic shard (C3)
  3. all-gather the routed facts; every rank scans its buffer shard with the
     fused MFMA top-k (k=3) for all of them; all-gather the candidates and
     merge (C1/K2) -> global dedupe (top-1 > 0.95) and cross-shard links
  4. owner rank: insert non-duplicates, within-shard links (label-filtered
     top-3), chain edges, duplicate merges (salience=max, access+1)
  5. fused decay (0.99^convs) + prune (K10) and eviction to the buffer limit (K11)
  6. every ``--cluster-every`` steps: two-level hierarchical clustering of the
     whole buffer into super-nodes (distributed spherical k-means, K16/C4)

Fact *texts* are embedded (the cost is paid) but the vectors used for the
graph are synthetic controlled ones (perturbations of existing memories with a
fixed duplicate rate): random-init encoder weights give near-identical
embeddings for every text, which would make dedupe degenerate.
turns/sec = conversations consolidated per second over all ranks.
"""
from __future__ import annotations

import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lazzaro_amd.index.device_graph import DeviceGraph  # noqa: E402
from lazzaro_amd.index.kmeans import kmeans  # noqa: E402
from lazzaro_amd.ops.search import flat_topk, flat_topk_dual  # noqa: E402
from lazzaro_amd.parallel import Communicator  # noqa: E402
from lazzaro_amd.parallel.sharded import merge_topk  # noqa: E402

N_TOPICS = 64
ROW_BITS = 40


def _unit(x):
    return x / x.norm(dim=1, keepdim=True).clamp_min(1e-30)


class ShardedBuffer:
    def __init__(self, comm: Communicator, dim: int, nodes_per_rank: int, device, seed: int = 0):
        self.comm, self.dev = comm, device
        self.g = DeviceGraph(dim, device=device, capacity=int(nodes_per_rank * 1.25) + 1024,
                             edge_capacity=nodes_per_rank * 3)
        gen = torch.Generator(device=device).manual_seed(seed + comm.rank)
        step = 1 << 20
        mine = torch.tensor([t for t in range(N_TOPICS) if t % comm.world == comm.rank], device=device)
        for r0 in range(0, nodes_per_rank, step):
            m = min(step, nodes_per_rank - r0)
            v = _unit(torch.randn((m, dim), device=device, generator=gen))
            topic = mine[torch.randint(0, mine.numel(), (m,), device=device, generator=gen)]
            self.g.add_nodes(v, topic, torch.rand(m, device=device, generator=gen) * 0.8 + 0.2, now=0.0)
        # sparse initial association graph
        ne = nodes_per_rank * 2
        src = torch.randint(0, nodes_per_rank, (ne,), device=device, generator=gen)
        dst = torch.randint(0, nodes_per_rank, (ne,), device=device, generator=gen)
        self.g.add_edges(src, dst, torch.rand(ne, device=device, generator=gen) * 0.5 + 0.5, now=0.0)
        self.limit = int(nodes_per_rank * 1.1)
        self.rows_added = nodes_per_rank  # host-side upper bound on live rows
        self.remote_edges = []
        self.fine = self.super_fine = self.super_top = None

    def owner(self, topic: torch.Tensor) -> torch.Tensor:
        return topic % self.comm.world

    def global_search(self, q: torch.Tensor, k: int, q_label: torch.Tensor = None):
        """All-gather queries, local fused top-k, all-gather candidates, merge.
        With ``q_label`` the same scan (flat_topk_dual) also returns this
        rank's shard-filtered top-k for its own queries (within-shard links)."""
        comm = self.comm
        if comm.world > 1:
            nq = torch.tensor([q.shape[0]], device=self.dev)
            sizes = comm.all_gather_rows(nq).tolist()
            mx = max(sizes) if sizes else 0
            qp = torch.zeros((mx, q.shape[1]), dtype=q.dtype, device=self.dev)
            qp[: q.shape[0]] = q
            allq = comm.all_gather_rows(qp)  # [world*mx, Dp]
        else:
            mx, allq = q.shape[0], q
        n = self.g.n
        lo = comm.rank * mx
        local = None
        if q_label is None:
            s, r = flat_topk(self.g.emb[:n], allq, k, bias=self.g.bias[:n])
        else:
            ql = torch.full((allq.shape[0],), -1, dtype=torch.int32, device=self.dev)
            ql[lo: lo + q.shape[0]] = q_label.to(torch.int32)
            (s, r), (sw, rw) = flat_topk_dual(self.g.emb[:n], allq, k, bias=self.g.bias[:n],
                                              row_label=self.g.shard[:n], q_label=ql, n_labels=N_TOPICS)
            local = (sw[lo: lo + q.shape[0]], rw[lo: lo + q.shape[0]])
        gid = torch.where(r >= 0, (comm.rank << ROW_BITS) + r, r)
        if comm.world > 1:
            S = comm.all_gather_rows(s).view(comm.world, comm.world * mx, k)
            I = comm.all_gather_rows(gid).view(comm.world, comm.world * mx, k)
            S = S[:, lo: lo + q.shape[0]].permute(1, 0, 2).reshape(q.shape[0], -1)
            I = I[:, lo: lo + q.shape[0]].permute(1, 0, 2).reshape(q.shape[0], -1)
            merged = merge_topk(S, I, k)
        else:
            merged = (s, gid)
        return merged if q_label is None else (merged, local)

    def consolidate(self, q: torch.Tensor, topic: torch.Tensor, sal: torch.Tensor, convs_total: int, now: float):
        """One batch, host-sync-free except the edge compaction: duplicates are
        merged by masked index reductions and the batch is ingested with
        DeviceGraph.ingest_fixed (fixed shapes, tombstoned duplicate rows).
        Returns device counts."""
        comm, g = self.comm, self.g
        # (2) route facts to topic owners
        if comm.world > 1:
            q, topic, sal = comm.reshard(self.owner(topic), q, topic, sal)
        # (3) global dedupe + cross-shard link candidates, and (same scan) the
        #     within-shard candidates of this rank's facts
        (s, gid), shard_hits = self.global_search(q, 3, q_label=topic)
        dup = (gid[:, 0] >= 0) & (s[:, 0] > 0.95)
        local_dup = dup & ((gid[:, 0] >> ROW_BITS) == comm.rank)
        rows = torch.where(gid[:, 0] >= 0, gid[:, 0] & ((1 << ROW_BITS) - 1), 0)
        neg = torch.full_like(sal, float("-inf"))
        g.sal.scatter_reduce_(0, rows, torch.where(local_dup, sal.float(), neg), "amax", include_self=True)
        g.acc.index_add_(0, rows, local_dup.to(torch.int32))
        g.last.scatter_reduce_(0, rows, torch.where(local_dup, torch.full_like(neg, now, dtype=torch.float64),
                                                  torch.full_like(neg, float("-inf"), dtype=torch.float64)),
                             "amax", include_self=True)
        # (4) insert + links (within-shard + same-rank global hits; fixed shapes)
        n0 = g.n
        own = (gid >= 0) & ((gid >> ROW_BITS) == comm.rank)
        local_g = (torch.where(own, s, neg[:, None].expand_as(s)), torch.where(own, gid & ((1 << ROW_BITS) - 1), -1))
        out = g.ingest_fixed(q, topic, sal, dup, shard_hits, global_hits=local_g, now=now)
        self.rows_added += q.shape[0]
        n_cross = torch.zeros((), dtype=torch.int64, device=self.dev)
        if comm.world > 1:  # cross-rank associations: local source row -> global target id
            cross = (s > 0.5) & (gid >= 0) & ~own & ~dup[:, None]
            src = torch.arange(n0, g.n, device=self.dev)[:, None].expand(-1, 3)
            self.remote_edges.append((src[cross], gid[cross], s[cross] * 0.8))
            n_cross = cross.sum()
        # (5) decay + prune + eviction
        pruned = g.decay_prune(0.01, 0.5, conversations=convs_total)
        pruned = pruned - out["placeholders"]  # ingest_fixed's untaken-link placeholders are not prunes
        evicted = g.enforce_limit(self.limit, now=now, alive_upper=self.rows_added)
        return {"routed": q.shape[0], "dup": dup.sum(), "inserted": out["inserted"],
                "linked": out["linked"] + n_cross, "pruned": pruned, "evicted": evicted}

    def cluster(self, n_fine: int, n_top: int, iters: int) -> None:
        """Two-level hierarchical clustering of the whole buffer (K16; the
        scalable form of the reference's per-shard mean super-node,
        memory_system.py:893-933): spherical k-means into ``n_fine``
        super-nodes over every rank's rows (fused MFMA top-1 assign, segmented
        mean, one all-reduce of partial sums per iteration, C4), warm-started
        from the previous pass; then the fine centroids (identical on every
        rank) into ``n_top`` topic super-nodes. Tombstoned rows keep label -1."""
        g = self.g
        X = g.emb[: g.n]
        comm = self.comm if self.comm.world > 1 else None
        c32, c16, lab = kmeans(X, n_fine, iters=iters, comm=comm, init=self.fine)
        self.fine = c32
        _, _, top = kmeans(c16, n_top, iters=iters + 2, seed=1)
        lab = torch.where(g.alive[: g.n] > 0, lab, torch.full_like(lab, -1))
        self.super_fine = lab
        self.super_top = torch.where(lab >= 0, top.to(lab.dtype)[lab.clamp_min(0).long()], lab)


def synth_facts(buf: ShardedBuffer, n: int, dim: int, dup_rate: float, gen):
    dev = buf.dev
    g = buf.g
    base_rows = torch.randint(0, g.n, (n,), device=dev, generator=gen)
    base = g.emb[base_rows, :dim].float()
    noise = torch.randn((n, dim), device=dev, generator=gen)
    is_dup = torch.rand(n, device=dev, generator=gen) < dup_rate
    noise = noise / (dim ** 0.5)  # unit-scale perturbation: cos ~0.995 (dup) / ~0.64 (related)
    q = torch.where(is_dup[:, None], _unit(base + 0.1 * noise), _unit(base + 1.2 * noise))
    topic = torch.randint(0, N_TOPICS, (n,), device=dev, generator=gen).to(torch.int32)
    sal = torch.rand(n, device=dev, generator=gen) * 0.5 + 0.5
    Dp = g.emb.shape[1]
    qp = torch.zeros((n, Dp), dtype=g.emb.dtype, device=dev)
    qp[:, :dim] = q.to(g.emb.dtype)
    return qp, topic, sal


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


WORDS = "user likes prefers works lives started visited learned project team python rust garden music".split()


def run(comm: Communicator, dev, nodes: int, convs: int, facts: int, steps: int, warmup: int,
        encoder=None, dim: int = 768, dup_rate: float = 0.1, seed: int = 7,
        cluster_every: int = 0, n_fine: int = 4096, n_top: int = 64, cluster_iters: int = 2):
    buf = ShardedBuffer(comm, dim, nodes, dev, seed)
    gen = torch.Generator(device=dev).manual_seed(seed + 100 + comm.rank)
    rng = random.Random(seed + comm.rank)
    texts = [" ".join(rng.choice(WORDS) for _ in range(12)) for _ in range(convs * facts)]
    now = [1000.0]

    # Fact embedding is pipelined one batch ahead on a side stream (as the
    # MemorySystem's background consolidation does): batch i+1's encoder
    # kernels fill the GPU while the host waits on batch i's data-dependent
    # steps (compaction sizes, counts). The main stream waits for the batch's
    # own embedding before consolidating it.
    side = torch.cuda.Stream(dev) if encoder is not None and dev.type == "cuda" else None
    # sub-batch streams of the fact embed: 1 (14k tokens; two streams measured 6.50k vs 6.75k
    # turns/s in bench.py, profiles/ab_splitk_r1.json -- unlike the 22.6k-token query batch)
    parts = int(os.environ.get("LZK_FACT_PARTS", "1"))
    pending = []
    tokens = []  # host-tokenised batches, one step ahead of their embedding launch

    def tokenize():
        if encoder is not None:
            tokens.append(encoder.tok.encode_batch(texts, 64))

    def launch_embed():
        if encoder is None:
            return
        if not tokens:
            tokenize()
        ids, lens = tokens.pop(0)
        if side is None:
            encoder.encoder.forward_streams(ids, lens, pad_to=buf.g.emb.shape[1], parts=parts)
            return
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            encoder.encoder.forward_streams(ids, lens, pad_to=buf.g.emb.shape[1], parts=parts)
            ev = torch.cuda.Event()
            ev.record(side)
        pending.append(ev)

    def step():
        if encoder is not None and not pending:
            launch_embed()
        if pending:
            torch.cuda.current_stream(dev).wait_event(pending.pop(0))
        launch_embed()  # next batch's facts, overlapped with this batch's consolidation
        tokenize()      # the batch after next, on the host while the GPU has queued work
        q, topic, sal = synth_facts(buf, convs * facts, dim, dup_rate, gen)
        now[0] += 60.0
        out = buf.consolidate(q, topic, sal, convs * comm.world, now[0])
        n_steps[0] += 1
        if cluster_every and n_steps[0] % cluster_every == 0:
            buf.cluster(n_fine, n_top, cluster_iters)
        return out

    n_steps = [0]
    clus_ms = None
    if cluster_every:
        # first pass seeds the fine centroids (farthest-first); it is not
        # part of the steady state, so it runs (and is timed) before warmup
        _sync(dev)
        t0 = time.perf_counter()
        buf.cluster(n_fine, n_top, cluster_iters)
        _sync(dev)
        t1 = time.perf_counter()
        buf.cluster(n_fine, n_top, cluster_iters)
        _sync(dev)
        clus_ms = {"seed_pass": round((t1 - t0) * 1e3, 1), "warm_pass": round((time.perf_counter() - t1) * 1e3, 1)}
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    comm.barrier()
    t0 = time.perf_counter()
    agg = {}
    for _ in range(steps):
        r = step()
        for k, v in r.items():  # device counts stay on device until the end
            agg[k] = agg.get(k, 0) + v
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    agg = {k: float(v) for k, v in agg.items()}
    comm.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev if comm.enabled and dev.type == "cuda" else "cpu")
    comm.all_reduce(t, "max")
    el = float(t.item())
    return {"turns_per_s": round(convs * comm.world * steps / el, 2), "ms_per_step": round(el / steps * 1e3, 3),
            "nodes_per_rank": nodes, "convs_per_rank_step": convs, "facts_per_conv": facts,
            "buffer_nodes_total": nodes * comm.world, "edges_rank0": buf.g.num_edges, "per_step_rank0": {
                k: round(v / steps, 1) for k, v in agg.items()},
            "hierarchical_clustering": None if not cluster_every else {
                "every_steps": cluster_every, "fine_super_nodes": n_fine, "top_super_nodes": n_top,
                "iters_per_pass": cluster_iters, "ms_rank0": clus_ms,
                "fine_clusters_used": int((torch.bincount(buf.super_fine[buf.super_fine >= 0].long(),
                                                          minlength=n_fine) > 0).sum())}}


if __name__ == "__main__":
    import argparse
    import json

    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=12_500_000)
    ap.add_argument("--convs", type=int, default=128)
    ap.add_argument("--facts", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-embed", action="store_true")
    ap.add_argument("--cluster-every", type=int, default=10, help="steps between hierarchical clustering passes (0=off)")
    ap.add_argument("--fine", type=int, default=4096, help="fine super-nodes (k-means level 1)")
    ap.add_argument("--top", type=int, default=64, help="topic super-nodes (k-means level 2)")
    ap.add_argument("--cluster-iters", type=int, default=2)
    a = ap.parse_args()
    comm = Communicator.init()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    enc = None
    if not a.no_embed and dev.type == "cuda":
        from lazzaro_amd.core.embedders import OnDeviceEmbedder
        enc = OnDeviceEmbedder("bge-base", device=dev, max_len=64)
    res = run(comm, dev, a.nodes, a.convs, a.facts, a.steps, a.warmup, enc, cluster_every=a.cluster_every,
              n_fine=a.fine, n_top=a.top, cluster_iters=a.cluster_iters)
    if comm.rank == 0:
        print(json.dumps({"metric": "consolidate turns/sec", "n_gpus": comm.world, **res}), flush=True)
