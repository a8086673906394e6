"""bench.py's multi-rank flow (DistributedMemoryService serving, routed
search, global search, consolidation) as a 2-rank gloo/CPU dry run launched
exactly like the driver launches the GPU bench (torch.distributed.run)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_cpu(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--cpu", "--gpus", "2", "--rows", "6000", "--dim", "128", "--model", "tiny", "--batch", "32",
           "--steps", "2", "--warmup", "1", "--prewarm-s", "0.2", "--recall-queries", "8", "--consolidate-steps", "1",
           "--consolidate-convs", "4"]
    env = dict(os.environ, PYTHONPATH=ROOT, LZK_BENCH_DB=str(tmp_path / "db"))
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 prints ONE json line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["steps"] == 2 and d["warmup"] == 1
    assert d["recall_at_10"] == 1.0 and d["recall_at_10_random_queries"] == 1.0
    assert d["serving"]["routed_queries_per_rank"] == 32 and d["serving"]["global_search_ms"] > 0
    assert d["consolidate_turns_per_s"] > 0 and d["consolidate"]["per_step_rank0"]["evicted"] > 0
