"""Host-side helpers added with the round-4 segment / narrow-path work:
digest list splitting, the two-level merge grouping, the capture object and
the super-node id freshness check of deferred consolidation points."""
import numpy as np
import torch


def test_digest_lists_splits_by_key_and_drops_unused():
    from lazzaro_amd.ops.tenant_ops import digest_lists
    kr = np.array([[5, 5, 9, 12, 12, 12, 1 << 62, 1 << 62],
                   [3, 7, 2, 1, 4, 8, -1, -1]], dtype=np.int64)
    got = [x.tolist() for x in digest_lists(kr)]
    assert got == [[3, 7], [2], [1, 4, 8]]
    assert digest_lists(np.array([[1 << 62], [-1]], dtype=np.int64)) == []


def test_merge_groups_divides_and_bounds():
    from lazzaro_amd.ops.search import _merge_groups
    assert _merge_groups(1024, 512) == 1          # wide batches: one level
    assert _merge_groups(1, 13) == 1              # too few chunks
    for nq, nch in [(1, 407), (1, 512), (4, 407), (8, 1221), (2, 100)]:
        G = _merge_groups(nq, nch)
        assert G > 1 and nch % G == 0 and nch // G >= 8 and G <= 64 and nq * G <= 512


def test_capture_host_value():
    from lazzaro_amd.engine.tenant_graph import Capture
    c = Capture(host=[1, 2, 3])
    assert c.get() == [1, 2, 3] and c.get() == [1, 2, 3]


def test_supers_fresh_rejects_reused_ids():
    from lazzaro_amd.core.memory_system import MemorySystem

    class Emb:
        def embed(self, t):
            return [1.0, 0.0, 0.0, 0.0]

        def batch_embed(self, ts):
            return [self.embed(t) for t in ts]

    class LLM:
        def completion(self, messages, response_format=None):
            return '{"memories": []}'

    import tempfile
    ms = MemorySystem(llm_provider=LLM(), embedding_provider=Emb(), enable_async=False, load_from_disk=False,
                      db_dir=tempfile.mkdtemp(), device="cpu", enable_caching=False)
    g = ms.graph
    code = g.shard_id("work")
    plan = {"supers": [{"code": code}]}
    assert ms._supers_fresh(plan, 1000.0)
    assert not ms._supers_fresh({"supers": [{"code": code}, {"code": code}]}, 1000.0)  # same id twice
    g.add_nodes(["super_work_1000"], ["s"], torch.zeros(1, 4), shard=[code], sup=[1])
    assert not ms._supers_fresh(plan, 1000.0)  # id already a row
    ms.close()
