"""Failure detection / fault injection: typed errors, armed
fault points at provider / store / collective / kernel boundaries, and the
recovery policies (re-queued consolidation, retried persistence, atomic
per-tenant store rewrite)."""
import json
import os

import pytest

from lazzaro_amd.core.memory_system import MemorySystem
from lazzaro_amd.core.providers import HashEmbedder, LocalLLM, ScriptedLLM
from lazzaro_amd.utils import faults
from lazzaro_amd.utils.faults import (CommError, EmbeddingError, InjectedFault, ProviderError, StoreError, armed,
                                      retry)


def _facts(*cs):
    return json.dumps({"memories": [dict(content=c, type="semantic", salience=0.8, topic="work") for c in cs]})


def test_fault_point_arming_and_env_spec():
    inj = faults.FaultInjector()
    inj.load_spec("a.b:2:StoreError, c:1")
    with pytest.raises(StoreError):
        inj.check("a.b")
    with pytest.raises(StoreError):
        inj.check("a.b")
    inj.check("a.b")  # exhausted
    with pytest.raises(InjectedFault):
        inj.check("c")
    assert inj.hits("a.b") == 2


def test_retry_backoff():
    calls = []

    def flaky():
        calls.append(1)
        if len(calls) < 3:
            raise ProviderError("transient")
        return "ok"
    assert retry(flaky, attempts=3, base_delay=0.001) == "ok" and len(calls) == 3
    with pytest.raises(ProviderError):
        retry(lambda: (_ for _ in ()).throw(ProviderError("down")), attempts=2, base_delay=0.001)


def test_llm_failure_requeues_consolidation_instead_of_losing_memories(tmp_path):
    llm = ScriptedLLM([_facts("User works on the Rust compiler team"), _facts("User likes green tea a lot")])
    ms = MemorySystem(llm_provider=llm, embedding_provider=HashEmbedder(), enable_async=False,
                      db_dir=str(tmp_path), max_buffer_size=100)
    ms.start_conversation()
    ms.add_to_short_term("I work on the Rust compiler team")
    with armed("provider.llm", 1, ProviderError):
        ms.end_conversation()
    assert ms.buffer.size()[0] == 0
    assert len(ms.consolidation_queue) == 1 and ms.metrics["consolidation_failures"] == 1
    # next conversation consolidates the re-queued batch together with the new one
    ms.start_conversation()
    ms.add_to_short_term("I like green tea")
    ms.end_conversation()
    assert ms.consolidation_queue == []
    assert ms.buffer.size()[0] == 1  # scripted response for the merged batch
    ms.close()


def test_batches_dropped_after_max_retries(tmp_path):
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                      db_dir=str(tmp_path), max_consolidation_retries=2)
    ms.start_conversation()
    ms.add_to_short_term("I moved to Lisbon last spring")
    with armed("provider.llm", 5, ProviderError):
        ms.end_conversation()
        ms._async_consolidate()
    assert ms.consolidation_queue == [] and ms.metrics["dropped_batches"] == 1
    ms.close()


def test_degenerate_embeddings_are_rejected_not_stored(tmp_path):
    class ZeroEmb(HashEmbedder):
        def batch_embed(self, texts):
            return [[0.0] * self.dim for _ in texts]
    ms = MemorySystem(llm_provider=ScriptedLLM([_facts("User started learning the cello")]),
                      embedding_provider=ZeroEmb(), enable_async=False, db_dir=str(tmp_path))
    ms.start_conversation()
    ms.add_to_short_term("I started learning the cello")
    ms.end_conversation()
    assert ms.buffer.size()[0] == 0
    assert ms.metrics["consolidation_failures"] == 1 and len(ms.consolidation_queue) == 1
    ms.close()
    assert faults.degenerate_embedding([0.0, float("nan")]) and not faults.degenerate_embedding([0.1])
    assert isinstance(EmbeddingError("x"), ProviderError)


def test_store_failure_keeps_graph_and_retries_on_next_save(tmp_path):
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                      db_dir=str(tmp_path), max_buffer_size=100)
    ms.start_conversation()
    ms.chat("My sister lives in Osaka and teaches math.")
    ms.end_conversation()
    ms._get_or_create_shard("default")
    with armed("store.commit", 1, StoreError):
        ms._save_to_persistence()
    n = ms.buffer.size()[0]
    assert n >= 1 and ms.metrics["persist_failures"] == 1 and ms._persist_pending
    ms._save_to_persistence()
    assert not ms._persist_pending
    ms.close()
    ms2 = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                       db_dir=str(tmp_path))
    assert ms2.buffer.size()[0] == n
    ms2.close()


def test_store_failure_during_ingest_rolls_back_then_retries(tmp_path):
    """Third-party store (not graph-bound): the reference's add_nodes at
    ingest fails -> the graph is rolled back and the batch re-queued."""
    from lazzaro_amd.core.vector_store import HBMStore

    class PlainStore(HBMStore):  # opts out of graph binding: behaves like any Store
        attach = None

    llm = ScriptedLLM([_facts("User keeps bees on a rooftop")] * 2)
    ms = MemorySystem(llm_provider=llm, embedding_provider=HashEmbedder(), enable_async=False,
                      store=PlainStore(db_dir=str(tmp_path)), max_buffer_size=100)
    ms.start_conversation()
    ms.add_to_short_term("I keep bees on a rooftop")
    with armed("store.commit", 1, StoreError):
        ms.end_conversation()
    assert ms.buffer.size()[0] == 0 and len(ms.consolidation_queue) == 1
    ms._async_consolidate()
    assert ms.buffer.size()[0] == 1 and ms.consolidation_queue == []
    assert len(ms.store.get_nodes(user_id="default")) == 1
    ms.close()


def test_bound_store_commit_failure_stays_pending(tmp_path):
    """Graph-bound store: the batch is in the graph; the failed incremental
    commit keeps its change set pending and the next save writes it once."""
    llm = ScriptedLLM([_facts("User keeps bees on a rooftop")])
    ms = MemorySystem(llm_provider=llm, embedding_provider=HashEmbedder(), enable_async=False,
                      db_dir=str(tmp_path), max_buffer_size=100)
    ms.start_conversation()
    ms.add_to_short_term("I keep bees on a rooftop")
    with armed("store.commit", 2, StoreError):  # both saves of a sync end_conversation
        ms.end_conversation()
    assert ms.buffer.size()[0] == 1 and ms._persist_pending
    assert ms.metrics["persist_failures"] == 2 and ms.store.get_nodes(user_id="default") == []
    ms._save_to_persistence()
    assert not ms._persist_pending and len(ms.store.get_nodes(user_id="default")) == 1
    ms._save_to_persistence()
    assert len(ms.store.get_nodes(user_id="default")) == 1
    ms.close()


def test_strict_errors_raise_typed(tmp_path):
    ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), enable_async=False,
                      db_dir=str(tmp_path), strict_errors=True)
    ms._get_or_create_shard("default")
    with armed("store.commit", 1, StoreError):
        with pytest.raises(StoreError):
            ms._save_to_persistence()
    ms.close()


def test_replace_rows_is_one_atomic_version(tmp_path):
    from lazzaro_amd.store.colstore import EDGE_SCHEMA, ColumnarTable
    t = ColumnarTable(str(tmp_path), "edges", EDGE_SCHEMA)
    row = dict(id="a_b", user_id="u", source_id="a", target_id="b", weight=0.5, edge_type="r", co_occurrence=1,
               last_updated=0.0, metadata="{}")
    t.add_rows([row, dict(row, user_id="v")])
    v0 = t.version
    n, v1 = t.replace_rows([("user_id", "u")], [dict(row, weight=0.9), dict(row, id="a_c", target_id="c")])
    assert n == 1 and v1 == v0 + 1
    rows = t.scan([("user_id", "u")])
    assert sorted(r["id"] for r in rows) == ["a_b", "a_c"] and len(t.scan([("user_id", "v")])) == 1
    n, v2 = t.replace_rows([("user_id", "u")], [])
    assert n == 2 and v2 == v1 + 1 and t.scan([("user_id", "u")]) == []


def test_comm_fault_is_typed():
    from lazzaro_amd.parallel import Communicator
    import torch
    c = Communicator.local()
    with armed("comm.all_reduce", 1, CommError):
        with pytest.raises(CommError):
            c.all_reduce(torch.ones(2))
    assert c.all_reduce(torch.ones(2)).sum() == 2


def test_kernel_check_is_typed():
    from lazzaro_amd.ops import _lib
    with pytest.raises(faults.KernelError):
        _lib.check(1, "lzk_fake")


def test_elastic_placement_moves_only_dead_ranks_tenants():
    from lazzaro_amd.parallel.elastic import ElasticPlacement
    tenants = [f"user{i}" for i in range(2000)]
    p = ElasticPlacement(8)
    q = p.remove([3])
    moved = p.moved(tenants, q)
    assert moved and all(p.owner(t) == 3 for t in moved) and all(v != 3 for v in moved.values())
    assert all(q.owner(t) == p.owner(t) for t in tenants if t not in moved)


def test_commit_retry_after_partial_write_has_no_duplicate_ids(tmp_path):
    """The nodes table is written, the edges write fails: the retry must go
    through the keyed upsert (rows reported 'fresh' by the failed attempt
    may already be in the table) -- no node id twice, edges land once."""
    # 22 facts of one topic: the shard passes super_node_threshold, and the
    # super-node row is written by the commit itself (never stored before)
    facts = [f"User fact number {i} about beekeeping on the rooftop" for i in range(22)]
    ms = MemorySystem(llm_provider=ScriptedLLM([_facts(*facts)]), embedding_provider=HashEmbedder(),
                      enable_async=False, db_dir=str(tmp_path), max_buffer_size=100)
    ms.start_conversation()
    ms.add_to_short_term("I keep bees on a rooftop and sell the honey")
    with armed("store.commit.edges", 1, StoreError):  # the consolidation save's edge upsert fails
        ms.end_conversation()
    assert ms.metrics["persist_failures"] >= 1 and ms.super_nodes
    for _ in range(2):
        ms._save_to_persistence()
        ids = [r["id"] for r in ms.store.get_nodes(user_id="default")]
        assert len(ids) == len(set(ids)) == 23, sorted(ids)
    ms.close()


def test_write_behind_retry_after_partial_write_has_no_duplicate_ids(tmp_path):
    facts = [f"User fact number {i} about beekeeping on the rooftop" for i in range(22)]
    ms = MemorySystem(llm_provider=ScriptedLLM([_facts(*facts)]), embedding_provider=HashEmbedder(),
                      enable_async=False, db_dir=str(tmp_path), max_buffer_size=100, persist_async=True)
    ms.start_conversation()
    ms.add_to_short_term("I keep bees on a rooftop and sell the honey")
    with armed("store.commit.edges", 1, StoreError):
        ms.end_conversation()
        ms.flush_persistence()
    ms.flush_persistence()
    ms._save_to_persistence()
    ms.flush_persistence()
    ids = [r["id"] for r in ms.store.get_nodes(user_id="default")]
    assert len(ids) == len(set(ids)) == 23, sorted(ids)
    ms.close()
