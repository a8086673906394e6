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
           "--consolidate-convs", "4", "--sharded-persistent-steps", "0"]
    env = dict(os.environ, PYTHONPATH=ROOT, LZK_BENCH_DB=str(tmp_path / "db"))
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 prints ONE json line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["steps"] == 2 and d["warmup"] == 1
    assert d["recall_at_10"] == 1.0 and d["recall_at_10_random_queries"] == 1.0
    _check_serving(d, 32)
    assert d["consolidate_turns_per_s"] > 0 and d["consolidate"]["per_step_rank0"]["evicted"] > 0


def _check_serving(d, batch):
    sv = d["serving"]
    assert sv["routed_queries_per_rank"] == batch and sv["routed_qps"] > 0 and sv["global_qps"] > 0
    ok, tot = map(int, sv["routed_exact_check"].split("/"))
    assert tot > 0 and ok == tot  # every routed answer equals the owner's own store search
    assert 0 < sv["routed_remote_frac_rank0"] < 1


SMALL = ["--cpu", "--rows", "6000", "--dim", "128", "--model", "tiny", "--batch", "32", "--steps", "2", "--warmup",
         "1", "--prewarm-s", "0.2", "--recall-queries", "8", "--consolidate-steps", "1", "--consolidate-convs", "4",
         "--no-persistent-graph", "--sharded-steps", "1", "--global-batch", "8", "--sharded-persistent-steps", "0"]


def test_bench_self_launches_ranks(tmp_path):
    """``bench.py --gpus 2`` without a torchrun environment launches the two
    ranks itself (the parent stays GPU-free) and reports n_gpus == 2 with the
    RCCL-path numbers (routed / global search, row-sharded consolidation)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env.update(PYTHONPATH=ROOT, LZK_BENCH_DB=str(tmp_path / "db"))
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"].endswith("2")
    _check_serving(d, 32)
    assert d["consolidate_sharded"]["turns_per_s"] > 0


def test_bench_rejects_gpus_world_mismatch(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL, cwd=str(tmp_path),
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stdout + r.stderr)


def test_bench_eight_ranks_cpu(tmp_path):
    """The 8-GPU job's flow rehearsed on 8 gloo/CPU ranks, launched exactly as
    the driver launches the scaling run (torch.distributed.run, 8 processes):
    headline, routed search (7/8 of each front end's queries remote, every
    answer equal to its owner's own search), global search, per-rank
    consolidation and the row-sharded buffer over all 8 ranks."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--rows", "5000", "--dim", "128", "--model", "tiny", "--batch", "16", "--steps", "1",
           "--warmup", "1", "--prewarm-s", "0", "--recall-queries", "4", "--consolidate-steps", "1",
           "--consolidate-convs", "2", "--no-persistent-graph", "--sharded-steps", "1", "--global-batch", "4",
           "--sharded-persistent-steps", "1", "--cpu"]
    env = dict(os.environ, PYTHONPATH=ROOT, LZK_BENCH_DB=str(tmp_path / "db"), OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "tenant-dp8" and d["value"] > 0
    assert d["config"]["global_batch"] == 8 * 16
    _check_serving(d, 16)
    assert d["consolidate_turns_per_s"] > 0
    sh = d["consolidate_sharded"]
    assert sh["turns_per_s"] > 0 and sh["buffer_nodes_total"] == 8 * 5000
    # the persistent-graph buffer (8 x 10k seeded edges kept): the incremental
    # digest served the run_consolidation points from a replicated stable base
    pg = d["consolidate_sharded_persistent_graph"]
    assert pg["turns_per_s"] > 0 and pg["edges_total_at_start"] == 8 * 10000
    assert pg["incremental_digest_points"] > 0 and pg["incremental_digest_base_edges_max"] > 0


def test_hbm_plan_eight_gpus_ten_million_rows_fits():
    """Every section of the 8-GPU job at the headline size (10M x 768 rows per
    rank) fits one MI355X's HBM with room to spare (bench.py hbm_plan; the GPU
    run reports the measured per-section peaks next to it)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--hbm-check", "--gpus", "8", "--rows",
                        "10000000"], env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 8 and d["fits"]
    assert set(d["sections_gib"]) == {"headline", "consolidate", "consolidate_persistent_graph", "consolidate_sharded",
                                      "consolidate_sharded_persistent_graph"}
    assert d["peak_gib"] < 0.5 * d["hbm_gib"]
