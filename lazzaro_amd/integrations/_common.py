"""Shared retrieval/record helpers for the agent-framework adapters
(the reference duplicates this block in each adapter, e.g.
langchain_integration.py:32-51, autogen_integration.py:40-56)."""
from __future__ import annotations

from contextlib import nullcontext
from typing import List, Tuple

from ..core.profile import EMPTY_CONTEXT


def retrieve(ms, query: str) -> Tuple[str, List[str]]:
    """(profile context or "", retrieved memory contents) for ``query``.
    The graph read runs under the MemorySystem's graph lock: a background
    consolidation may be writing the same tenant graph."""
    q = ms._get_embedding(query)
    with getattr(ms, "_graph_lock", None) or nullcontext():
        ids = ms._optimized_retrieval(q, query)
        prof = ms.profile.get_context()
        texts = [n.content for n in (ms.buffer.get_node(i) for i in ids) if n is not None]
    prof = prof if prof and prof != EMPTY_CONTEXT else ""
    return prof, texts


def context_block(ms, query: str, heading: str, profile_prefix: str = "User Profile: ") -> str:
    prof, texts = retrieve(ms, query)
    parts = []
    if prof:
        parts.append(f"{profile_prefix}{prof}")
    if texts:
        parts.append(heading + "\n" + "\n".join(texts))
    return "\n\n".join(parts)


def record_turn(ms, user_text: str = "", ai_text: str = "") -> None:
    if not ms.conversation_active:
        ms.start_conversation()
    if user_text:
        ms.add_to_short_term(user_text, "episodic", salience=0.7)
        ms.conversation_history.append({"role": "user", "content": user_text})
    if ai_text:
        ms.add_to_short_term(ai_text, "semantic", salience=0.5)
        ms.conversation_history.append({"role": "assistant", "content": ai_text})
