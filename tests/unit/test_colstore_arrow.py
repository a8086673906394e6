"""Columnar store v2 (csrc/runtime/colstore.cpp): Arrow IPC fragments that
pyarrow reads without the runtime, keyed upserts / deletes that touch only the
changed rows, cross-process (second Table object) visibility, and the
MemorySystem's incremental commits on top of it."""
import os
import time

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")

from lazzaro_amd.store.colstore import NODE_SCHEMA, ColumnarTable, read_fragments  # noqa: E402


def _cols(ids, user="u", dim=8, seed=0):
    rng = np.random.default_rng(seed)
    n = len(ids)
    return {"id": list(ids), "user_id": [user] * n, "content": [f"c-{i}" for i in ids],
            "vector": rng.standard_normal((n, dim)).astype(np.float32), "type": ["semantic"] * n,
            "timestamp": np.arange(n, dtype=np.float64), "access_count": np.zeros(n, np.int32),
            "last_accessed": np.zeros(n), "salience": np.full(n, 0.5, np.float32),
            "is_super_node": np.zeros(n, np.uint8), "child_ids": ["[]"] * n, "parent_id": [""] * n,
            "shard_key": ["work"] * n, "metadata": ["{}"] * n, "decay_clock": np.zeros(n)}


def test_fragments_are_arrow_ipc_readable_by_pyarrow(tmp_path):
    t = ColumnarTable(str(tmp_path), "nodes", NODE_SCHEMA)
    t.add_columns(_cols([f"n{i}" for i in range(100)]))
    t.upsert_columns([("user_id", "u")], "id", ["n3", "n7", "zz"], _cols(["n3", "zz"], seed=1))
    t.delete([("user_id", "u")], "id", ["n10"])
    files = t.fragment_files()
    assert files and all(f.endswith(".arrow") for f in files)
    for f in files:  # every file on disk opens with pyarrow alone
        pa.ipc.open_file(f).read_all()
    tab = read_fragments(t.path)
    ids = sorted(tab.column("id").to_pylist())
    want = sorted([f"n{i}" for i in range(100) if i not in (3, 7, 10)] + ["n3", "zz"])
    assert ids == want
    assert tab.schema.field("vector").type == pa.list_(pa.float32(), 8)
    assert sorted(t.scan_columns([("user_id", "u")])["id"]) == want
    assert t.to_arrow().num_rows == len(want)


def test_keyed_upsert_cost_does_not_grow_with_the_table(tmp_path):
    small = ColumnarTable(str(tmp_path / "s"), "nodes", NODE_SCHEMA)
    big = ColumnarTable(str(tmp_path / "b"), "nodes", NODE_SCHEMA)
    small.add_columns(_cols([f"n{i}" for i in range(2_000)]))
    for c in range(0, 400_000, 100_000):
        big.add_columns(_cols([f"n{i}" for i in range(c, c + 100_000)]))

    def upserts(t):
        t.upsert_columns([("user_id", "u")], "id", ["n5"], _cols(["n5"], seed=9))  # builds the index once
        t0 = time.perf_counter()
        for j in range(20):
            t.upsert_columns([("user_id", "u")], "id", [f"n{j}", f"n{j + 100}"], _cols([f"n{j}"], seed=j))
        return time.perf_counter() - t0

    ts, tb = upserts(small), upserts(big)
    assert tb < 5 * ts + 0.05, (ts, tb)
    assert big.count() == 400_000 - 20  # n{j+100} deleted, n{j} re-added
    # each commit wrote one small fragment, nothing was rewritten
    newest = max(big.fragment_files(), key=os.path.getmtime)
    assert pa.ipc.open_file(newest).read_all().num_rows <= 100


def test_second_table_object_sees_commits(tmp_path):
    a = ColumnarTable(str(tmp_path), "nodes", NODE_SCHEMA)
    b = ColumnarTable(str(tmp_path), "nodes", NODE_SCHEMA)
    a.add_columns(_cols(["x1", "x2", "x3"]))
    assert b.version == a.version and sorted(b.scan_columns()["id"]) == ["x1", "x2", "x3"]
    b.delete([("user_id", "u")], "id", ["x2"])  # b indexes + deletes; a must rebuild
    assert a.upsert_columns([("user_id", "u")], "id", ["x3"], _cols(["x3"], seed=4))[0] == 1
    assert sorted(a.scan_columns()["id"]) == ["x1", "x3"] == sorted(b.scan_columns()["id"])
    a.compact()
    assert b.count() == 2 and len([f for f in b.fragment_files() if "/data/" in f]) >= 1


def test_duplicate_keys_all_deleted(tmp_path):
    t = ColumnarTable(str(tmp_path), "edges", __import__("lazzaro_amd.store.colstore", fromlist=["x"]).EDGE_SCHEMA)
    n = 3
    cols = {"id": ["a_b"] * n, "user_id": ["u"] * n, "source_id": ["a"] * n, "target_id": ["b"] * n,
            "weight": np.ones(n, np.float32), "edge_type": ["relates_to"] * n, "co_occurrence": np.ones(n, np.int32),
            "last_updated": np.zeros(n), "metadata": ["{}"] * n, "decay_clock": np.zeros(n)}
    t.add_columns(cols)
    assert t.delete([("user_id", "u")], "id", ["a_b"])[0] == 3 and t.count() == 0


def test_memory_system_commit_writes_only_changes(tmp_path):
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM

    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=16), enable_async=False,
                      db_dir=str(tmp_path), max_buffer_size=10 ** 6)
    g = ms.graph
    n = 20_000
    rng = np.random.default_rng(0)
    g.add_nodes([f"node_{i + 1}" for i in range(n)], [f"m{i}" for i in range(n)],
                rng.standard_normal((n, 16)).astype(np.float32).tolist(), shard=g.shard_id("work"))
    ms.node_counter = n
    ms._save_to_persistence()  # first commit: every row
    nodes = ms.store._nodes_table
    assert nodes.count() == n
    for turn in ("I work on a robotics project with a deadline.", "My family visits home every summer."):
        # (the first one also creates the "work" super-node, which re-parents --
        # and so rewrites -- its 20k children once, as in the reference)
        ms.start_conversation()
        ms.chat(turn)
        ms.end_conversation()
    newest = max((f for f in nodes.fragment_files() if "/data/" in f), key=os.path.getmtime)
    assert pa.ipc.open_file(newest).read_all().num_rows < 100  # O(changes), not O(tenant)
    ms.close()
    ms2 = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=16), enable_async=False,
                       db_dir=str(tmp_path), max_buffer_size=10 ** 6)
    assert ms2.get_stats()["buffer_nodes"] == ms.get_stats()["buffer_nodes"] == nodes.count()
    ms2.close()


def test_fragment_written_as_several_record_batches(tmp_path):
    """A fragment larger than one Arrow array's capacity is written as several
    record batches (a 10M x 768 vector column is 7.7G floats > 2^31); the
    runtime and pyarrow both read every batch back in order."""
    import subprocess
    import sys
    import textwrap
    code = textwrap.dedent(f"""
        import numpy as np, pyarrow.ipc as ipc
        from lazzaro_amd.store.colstore import ColumnarTable, NODE_SCHEMA, read_fragments
        t = ColumnarTable({str(tmp_path)!r}, "nodes", NODE_SCHEMA)
        n = 1000
        rows = [dict(id=f"n{{i}}", user_id="u", content="c" * (i % 7), vector=[float(i)] * 8, type="semantic",
                     timestamp=float(i), access_count=i, last_accessed=0.0, salience=0.5, is_super_node=False,
                     child_ids="[]", parent_id="", shard_key="s", metadata="{{}}") for i in range(n)]
        t.add_rows(rows)
        f = t.fragment_files()[0]
        assert ipc.open_file(f).num_record_batches > 1
        got = t.scan_columns([("user_id", "u")])
        assert list(got["id"]) == [f"n{{i}}" for i in range(n)]
        assert np.array_equal(got["vector"][:, 0], np.arange(n, dtype=np.float32))
        pa_t = read_fragments(t.path)
        assert pa_t.num_rows == n and pa_t.column("id").to_pylist() == [f"n{{i}}" for i in range(n)]
        print("ok")
    """)
    import os
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, LZK_COLSTORE_BATCH_VALUES="1000", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


_PAR_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, {root!r})
from tests.unit.test_colstore_arrow import _cols
from lazzaro_amd.store.colstore import NODE_SCHEMA, ColumnarTable
t = ColumnarTable({path!r}, "nodes", NODE_SCHEMA)
ids = [f"n{{i}}" for i in range(1000)]
c = _cols(ids, seed=3)
c2 = _cols([f"m{{i}}" for i in range(300)], user="v", seed=4)
t.add_columns(c)           # 1000 rows -> 15 fragments of ~67 rows, written by parallel threads
t.add_columns(c2)
t.upsert_columns([("user_id", "u")], "id", ["n5", "n500", "n999"], _cols(["n5", "new"], seed=5))
nfrag = len([f for f in t.fragment_files() if "_deletions" not in f])
got = t.scan_columns([("user_id", "u")])
pos = {{k: j for j, k in enumerate(got["id"])}}
want = [i for i in ids if i not in ("n5", "n500", "n999")] + ["n5", "new"]
assert got["id"] == want, got["id"][:5]
ref = {{k: j for j, k in enumerate(ids)}}
for k in want[:-2]:
    assert np.array_equal(got["vector"][pos[k]], c["vector"][ref[k]])
    assert got["content"][pos[k]] == c["content"][ref[k]]
assert np.array_equal(got["vector"][pos["new"]], _cols(["n5", "new"], seed=5)["vector"][1])
assert t.scan_columns([("user_id", "v")])["id"] == c2["id"]
print("OK", nfrag)
"""


def test_parallel_fragment_commit_and_parallel_scan(tmp_path):
    """Past LZK_COLSTORE_PAR_ROWS rows a commit is written as several
    fragments by parallel threads (one version); the scan decodes many
    fragments in parallel into presized columns -- row order, vectors,
    strings, upserts and another tenant's rows all as before."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    code = _PAR_SCRIPT.format(root=root, path=str(tmp_path))
    env = dict(os.environ, LZK_COLSTORE_PAR_ROWS="64")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("OK") and int(r.stdout.split()[1]) > 8
