"""AutoGen adapter (reference integrations/autogen_integration.py:5-89): a reply
hook registered at position 0 injects a ``[LAZZARO MEMORY CONTEXT]`` block into
the agent's system message and records the incoming message; it returns None so
AutoGen's normal reply generation continues."""
from __future__ import annotations

import re
from typing import Any, Dict, List, Optional, Union

from ._common import context_block, record_turn

MARK = "[LAZZARO MEMORY CONTEXT]"


class LazzaroAutogenAgent:
    def __init__(self, agent: Any, memory_system):
        self.agent = agent
        self.memory_system = memory_system
        self._setup_hooks()

    def _setup_hooks(self) -> None:
        try:
            from autogen import Agent, ConversableAgent  # type: ignore
        except Exception:
            register = getattr(self.agent, "register_reply", None)
            if callable(register):  # duck-typed agents (tests, forks)
                register([object, None], reply_func=self._generate_memory_aware_reply, position=0)
            return
        if isinstance(self.agent, ConversableAgent):
            self.agent.register_reply([Agent, None], reply_func=self._generate_memory_aware_reply, position=0)

    def _generate_memory_aware_reply(self, recipient: Any, messages: Optional[List[Dict]] = None,
                                     sender: Optional[Any] = None, config: Optional[Any] = None) -> Union[str, Dict, None]:
        if not messages:
            return None
        last = messages[-1].get("content", "")
        if not last:
            return None
        ctx = context_block(self.memory_system, last, "Relevant Context:")
        if ctx:
            block = f"\n\n{MARK}\n" + ctx
            cur = self.agent.system_message
            if MARK not in cur:
                self.agent.update_system_message(cur + block)
            else:
                self.agent.update_system_message(re.sub(r"\n*\[LAZZARO MEMORY CONTEXT\].*$", block, cur,
                                                        flags=re.DOTALL))
        record_turn(self.memory_system, last, "")
        return None
