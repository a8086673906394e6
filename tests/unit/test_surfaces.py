"""CLI, dashboard API and agent-framework adapters (offline, CPU)."""
import json

from fastapi.testclient import TestClient

from lazzaro_amd.cli.main import handle_command, interactive_chat
from lazzaro_amd.core.memory_system import MemorySystem
from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
from lazzaro_amd.integrations import (LazzaroADKPlugin, LazzaroAutogenAgent, LazzaroLangChainMemory,
                                      LazzaroLangGraph)


def _ms(**kw):
    kw.setdefault("enable_async", False)
    kw.setdefault("load_from_disk", False)
    return MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(), **kw)


def _seed(ms):
    ms.start_conversation()
    ms.chat("I love hiking in the Alps every summer. My favorite language is Python.")
    ms.chat("I work on GPU kernels for memory systems at my job.")
    ms.end_conversation()


def test_cli_commands_and_chat():
    ms = _ms()
    out = []
    inputs = iter(["/start", "Hello there, I like coffee a lot.", "/end", "/stats", "/memories 3", "/profile",
                   "/config", "/set max_buffer_size 50", "/set prune_threshold abc", "/prune 0.3",
                   "/merge", "/consolidate", "/save state.json", "/load state.json", "/load", "/help", "/bogus",
                   "/quit"])
    interactive_chat(ms, input_fn=lambda _: next(inputs), out=lambda *a, **k: out.append(" ".join(map(str, a))))
    text = "\n".join(out)
    assert "Assistant:" in text and "Conversation started" in text
    assert "SCALABLE MEMORY SYSTEM STATS" in text and "Set max_buffer_size = 50" in text
    assert ms.max_buffer_size == 50 and "Invalid value for prune_threshold" in text
    assert "State saved to state.json" in text and "State loaded from state.json" in text
    assert "Unknown command" in text and "Goodbye" in text
    assert handle_command(ms, "/quit", out=lambda *a: None) is False
    ms.close()


def test_dashboard_routes():
    from lazzaro_amd.dashboard import api
    ms = _ms(user_id="alice")
    _seed(ms)
    api.set_memory_system(ms)
    c = TestClient(api.app)
    assert "<canvas" in c.get("/").text
    s = c.get("/api/stats").json()
    assert s["user_id"] == "alice" and s["buffer_nodes"] >= 1 and "performance" in s
    g = c.get("/api/graph").json()
    assert len(g["nodes"]) == s["buffer_nodes"] and {"source", "target", "weight", "type"} <= set(
        g["links"][0].keys()) if g["links"] else True
    assert "alice" in c.get("/api/users").json()
    assert "data" in c.get("/api/profile").json()
    assert "Memory Observations for alice" in c.get("/api/export").json()["content"]
    assert isinstance(json.loads(c.get("/api/export?format=json").json()["content"]), list)
    assert "insights" in c.get("/api/insights").json()
    assert "status" in c.post("/api/consolidate").json()
    assert c.get("/api/search", params={"q": "hiking"}).json()
    assert c.get("/api/engine").json()["store"] == "HBMStore"
    r = c.post("/api/users/switch", json={"user_id": "bob"}).json()
    assert r == {"status": "success", "user_id": "bob"} and ms.buffer.size()[0] == 0
    assert c.post("/api/users/switch", json={}).json() == {"error": "User ID required"}
    api.set_memory_system(None)
    assert c.get("/api/stats").json() == {"error": "Memory system not initialized"}
    ms.close()


def test_langchain_adapter():
    ms = _ms()
    _seed(ms)
    mem = LazzaroLangChainMemory(memory_system=ms)
    assert mem.memory_variables == ["history"]
    v = mem.load_memory_variables({"input": "hiking in the Alps"})["history"]
    assert "Relevant Past Memories:" in v and "Alps" in v
    assert mem.load_memory_variables({"input": ""}) == {"history": ""}
    mem.save_context({"input": "I moved to Berlin."}, {"output": "Nice!"})
    assert ms.short_term_memory[-2]["type"] == "episodic" and ms.conversation_active
    mem.clear()
    assert not ms.conversation_active
    ms.close()


def test_langgraph_adapter():
    ms = _ms()
    _seed(ms)
    lg = LazzaroLangGraph(ms)
    ctx = lg.get_memory_node()({"messages": [{"content": "Python language"}]})
    assert "Past Memories:" in ctx["lazzaro_context"]
    assert lg.get_memory_node()({"input": ""}) == {"lazzaro_context": ""}
    assert lg.get_record_node()({"messages": [{"content": "hi"}, {"content": "hello"}]}) == {}
    assert [m["role"] for m in ms.conversation_history[-2:]] == ["user", "assistant"]
    ms.close()


class _FakeAgent:
    def __init__(self):
        self.system_message = "You are helpful."
        self.hooks = []

    def register_reply(self, triggers, reply_func, position=0):
        self.hooks.insert(position, reply_func)

    def update_system_message(self, m):
        self.system_message = m


def test_autogen_adapter_with_duck_typed_agent():
    ms = _ms()
    _seed(ms)
    ag = _FakeAgent()
    LazzaroAutogenAgent(ag, ms)
    hook = ag.hooks[0]
    assert hook(ag, [{"content": "tell me about hiking"}]) is None
    assert "[LAZZARO MEMORY CONTEXT]" in ag.system_message and ag.system_message.startswith("You are helpful.")
    hook(ag, [{"content": "what about Python?"}])
    assert ag.system_message.count("[LAZZARO MEMORY CONTEXT]") == 1
    assert hook(ag, []) is None
    ms.close()


def test_adk_plugin():
    ms = _ms()
    _seed(ms)
    p = LazzaroADKPlugin(ms)
    tool = p.as_tool()
    assert tool["name"] == "lazzaro_memory_retrieval" and tool["parameters"]["required"] == ["query"]
    assert "Relevant Memories:" in tool["func"]("hiking")
    p.observe("I adopted a cat.", "Congrats!")
    assert ms.short_term_memory[-1]["content"] == "Congrats!"
    empty = _ms(db_dir="other")
    assert LazzaroADKPlugin(empty).retrieve("x") == "No relevant memories found."
    ms.close()


def _graph_via_views(ms):
    """The reference's /api/graph construction over the shard/super-node façades."""
    nodes, links = [], []
    for key, sh in ms.shards.items():
        for nid, n in sh.nodes.items():
            nodes.append({"id": nid, "content": n.content, "type": n.type, "salience": n.salience, "shard": key,
                          "access_count": n.access_count, "is_super_node": n.is_super_node})
        for (s, t), e in sh.edges.items():
            links.append({"source": s, "target": t, "weight": e.weight, "type": e.edge_type})
    for nid, n in ms.super_nodes.items():
        nodes.append({"id": nid, "content": n.content, "type": "super_node", "salience": n.salience,
                      "shard": "global", "is_super_node": True})
    return {"nodes": nodes, "links": links}


def test_graph_json_matches_views_and_dashboard_polls_during_async_consolidation():
    import threading

    from lazzaro_amd.dashboard import api
    ms = _ms(super_node_threshold=2, max_buffer_size=200)
    for i in range(4):
        _seed(ms)
        ms.start_conversation()
        ms.chat(f"My project number {i} has a deadline with client {i}. I read book {i} for my course.")
        ms.end_conversation()
    assert ms.graph_json() == _graph_via_views(ms) and ms.graph_json()["links"]
    ms.close()
    # the dashboard reads while the background worker consolidates
    ms = _ms(enable_async=True, super_node_threshold=2, max_buffer_size=200)
    api.set_memory_system(ms)
    c = TestClient(api.app)
    errors, stop = [], threading.Event()

    def poll():
        try:
            while not stop.is_set():
                for route in ("/api/graph", "/api/profile", "/api/stats", "/api/export"):
                    assert c.get(route).status_code == 200
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    t = threading.Thread(target=poll)
    t.start()
    for i in range(6):
        ms.start_conversation()
        ms.chat(f"I work on project {i} with a colleague and exercise at the gym {i} times a week.")
        ms.chat(f"My family visits home in summer {i} and I study a course on kernels.")
        ms.end_conversation()
    ms.flush()
    stop.set()
    t.join()
    assert not errors, errors
    g = c.get("/api/graph").json()
    assert len(g["nodes"]) == ms.get_stats()["buffer_nodes"]
    api.set_memory_system(None)
    ms.close()
