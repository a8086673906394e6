"""Five-domain evolving user persona (reference ``core/profile.py:3-59``)."""
from __future__ import annotations

import time
from typing import Dict

DOMAINS = ("preferences", "personality_traits", "knowledge_domains",
           "interaction_style", "key_experiences")
EMPTY_CONTEXT = "No profile data yet."


class Profile:
    def __init__(self):
        self.data: Dict[str, str] = {d: "" for d in DOMAINS}
        self.last_updated = time.time()

    def update_domain(self, domain: str, content: str) -> None:
        if domain not in self.data:
            return
        self.data[domain] = content
        self.last_updated = time.time()

    def get_context(self) -> str:
        lines = [f"{k.replace('_', ' ').title()}: {v}" for k, v in self.data.items() if v]
        return "\n".join(lines) if lines else EMPTY_CONTEXT

    def filled(self) -> int:
        return sum(1 for v in self.data.values() if v)

    def to_dict(self) -> Dict:
        return {"data": self.data, "last_updated": self.last_updated}

    @classmethod
    def from_dict(cls, d: Dict) -> "Profile":
        p = cls()
        p.data = d.get("data", p.data)
        p.last_updated = d.get("last_updated", p.last_updated)
        return p
