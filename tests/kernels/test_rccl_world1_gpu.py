"""The multi-GPU code paths on the one GPU of the test box: a 1-rank
``torch.distributed.run`` job on the ``nccl`` (RCCL) backend with
``force_collectives`` runs the routed / global search, migration and the
row-sharded consolidation through real RCCL all-to-all / all-gather /
all-reduce calls on device tensors (rccl_world1_worker.py) and checks each
against its truth."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world1_serving_and_sharded_paths():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "tests", "kernels", "rccl_world1_worker.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=280)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and lines, r.stdout[-4000:]
    out = json.loads(lines[-1][len("RESULT "):])
    assert out["backend"] == "nccl" and out["world"] == 1 and out["device"].startswith("cuda")
    for k in ("routed_dir0", "routed_dir1"):
        assert out[k]["exact"] and out[k]["global_exact"] and out[k]["force"], out[k]
    # small GPU tenants: the owner matches keys in the device directory and
    # serves them with one fused tenant-table scan (no key read-back)
    assert out["routed_dir0"]["route_stats"]["device"] >= 1, out["routed_dir0"]
    assert out["routed_dir1"]["route_stats"]["device"] >= 1, out["routed_dir1"]
    assert out["migrate"]["received"] == [] and out["migrate"]["search_ok"]
    assert out["sharded_equal"] and out["sharded_exact_cadence_equal"]
