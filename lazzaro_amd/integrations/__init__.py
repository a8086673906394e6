"""Agent-framework adapters. All import without their frameworks installed
(the reference silently drops LangChain/AutoGen when missing and never exports
LangGraph, integrations/__init__.py:1-15; here all four are exported)."""
from .adk_integration import LazzaroADKPlugin  # noqa: F401
from .autogen_integration import LazzaroAutogenAgent  # noqa: F401
from .langchain_integration import LazzaroLangChainMemory  # noqa: F401
from .langgraph_integration import LazzaroLangGraph  # noqa: F401

__all__ = ["LazzaroLangChainMemory", "LazzaroLangGraph", "LazzaroAutogenAgent", "LazzaroADKPlugin"]
