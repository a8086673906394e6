"""LLM and embedding providers (reference ``core/providers.py:5-196``).

The reference ships thin wrappers over vendor SDKs (openai, google-generativeai,
together). This framework does not depend on any vendor SDK:

* :data:`openai` is a small OpenAI-compatible HTTP client (httpx) exposing the
  subset of the SDK surface the providers use (``OpenAI(...).chat.completions
  .create`` incl. SSE streaming, ``.embeddings.create``). It is a module-level
  name so code/tests that patch ``...providers.openai`` keep working.
* ``OpenAILLM/OpenAIEmbedder`` (api.openai.com or any compatible server via
  ``base_url``), ``TogetherLLM/TogetherEmbedder`` (OpenAI-compatible endpoint)
  and ``GeminiLLM/GeminiEmbedder`` (Generative Language REST API).
* Local, network-free providers for tests/benchmarks and offline use:
  :class:`LocalLLM` (deterministic rule-based fact/profile extractor and chat
  responder) and :class:`HashEmbedder` (feature-hashed lexical embeddings).
  The on-device transformer encoders live in :mod:`lazzaro_amd.core.embedders`.

Error policy matches the reference: remote failures are logged and turn into
``""`` (LLM) or zero vectors (embeddings); MemorySystem refuses to store
zero-vector facts (see ``memory_system._consolidate_batch``).
"""
from __future__ import annotations

import hashlib
import json
import logging
import math
import os
import re
import types
from typing import Dict, Iterator, List, Optional

import numpy as np

from .interfaces import EmbeddingProvider, LLMProvider

log = logging.getLogger("lazzaro_amd.providers")


# --------------------------------------------------------------------------
# Minimal OpenAI-compatible HTTP client
# --------------------------------------------------------------------------
def _ns(obj):
    if isinstance(obj, dict):
        return types.SimpleNamespace(**{k: _ns(v) for k, v in obj.items()})
    if isinstance(obj, list):
        return [_ns(v) for v in obj]
    return obj


class _HTTP:
    def __init__(self, api_key: Optional[str], base_url: str, timeout: float):
        self.api_key = api_key
        self.base_url = base_url.rstrip("/")
        self.timeout = timeout

    def post(self, path: str, payload: dict, stream: bool = False):
        import httpx

        headers = {"Content-Type": "application/json"}
        if self.api_key:
            headers["Authorization"] = f"Bearer {self.api_key}"
        url = self.base_url + path
        if not stream:
            r = httpx.post(url, json=payload, headers=headers, timeout=self.timeout)
            r.raise_for_status()
            return r.json()

        def gen():
            with httpx.stream("POST", url, json=payload, headers=headers, timeout=self.timeout) as r:
                r.raise_for_status()
                for line in r.iter_lines():
                    if not line or not line.startswith("data:"):
                        continue
                    data = line[5:].strip()
                    if data == "[DONE]":
                        break
                    yield _ns(json.loads(data))
        return gen()


class _ChatCompletions:
    def __init__(self, http: _HTTP):
        self._http = http

    def create(self, model: str, messages: List[Dict], temperature: float = 0.7,
               response_format: Optional[Dict] = None, stream: bool = False, **kw):
        payload = {"model": model, "messages": messages, "temperature": temperature}
        if response_format:
            payload["response_format"] = response_format
        if stream:
            payload["stream"] = True
            return self._http.post("/chat/completions", payload, stream=True)
        return _ns(self._http.post("/chat/completions", payload))


class _Embeddings:
    def __init__(self, http: _HTTP):
        self._http = http

    def create(self, model: str, input, **kw):
        return _ns(self._http.post("/embeddings", {"model": model, "input": input}))


class _OpenAIClient:
    def __init__(self, api_key: Optional[str] = None, base_url: Optional[str] = None,
                 timeout: float = 60.0):
        api_key = api_key or os.environ.get("OPENAI_API_KEY")
        base_url = base_url or os.environ.get("OPENAI_BASE_URL", "https://api.openai.com/v1")
        http = _HTTP(api_key, base_url, timeout)
        self.chat = types.SimpleNamespace(completions=_ChatCompletions(http))
        self.embeddings = _Embeddings(http)


# module-like handle (patchable in tests exactly like the reference's `openai`)
openai = types.SimpleNamespace(OpenAI=_OpenAIClient)


# --------------------------------------------------------------------------
# Remote providers
# --------------------------------------------------------------------------
class OpenAILLM(LLMProvider):
    def __init__(self, api_key: Optional[str] = None, model: str = "gpt-4o-mini",
                 base_url: Optional[str] = None, temperature: float = 0.7):
        kw = {"api_key": api_key}
        if base_url:
            kw["base_url"] = base_url
        self.client = openai.OpenAI(**kw)
        self.model = model
        self.temperature = temperature

    def completion(self, messages, response_format=None) -> str:
        try:
            kw = {"model": self.model, "messages": messages, "temperature": self.temperature}
            if response_format:
                kw["response_format"] = response_format
            r = self.client.chat.completions.create(**kw)
            return r.choices[0].message.content or ""
        except Exception as e:  # parity: log and degrade to ""
            log.warning("LLM error: %s", e)
            return ""

    def completion_stream(self, messages, response_format=None) -> Iterator[str]:
        try:
            kw = {"model": self.model, "messages": messages, "temperature": self.temperature,
                  "stream": True}
            if response_format:
                kw["response_format"] = response_format
            for chunk in self.client.chat.completions.create(**kw):
                piece = chunk.choices[0].delta.content
                if piece:
                    yield piece
        except Exception as e:
            log.warning("LLM stream error: %s", e)
            yield ""


class OpenAIEmbedder(EmbeddingProvider):
    dim = 1536

    def __init__(self, api_key: Optional[str] = None, model: str = "text-embedding-3-small",
                 base_url: Optional[str] = None, dim: int = 1536):
        kw = {"api_key": api_key}
        if base_url:
            kw["base_url"] = base_url
        self.client = openai.OpenAI(**kw)
        self.model = model
        self.dim = dim

    def embed(self, text: str) -> List[float]:
        try:
            return list(self.client.embeddings.create(model=self.model, input=text).data[0].embedding)
        except Exception as e:
            log.warning("Embedding error: %s", e)
            return [0.0] * self.dim

    def batch_embed(self, texts: List[str]) -> List[List[float]]:
        if not texts:
            return []
        try:
            r = self.client.embeddings.create(model=self.model, input=texts)
            return [list(d.embedding) for d in r.data]
        except Exception as e:
            log.warning("Batch embedding error: %s", e)
            return [[0.0] * self.dim for _ in texts]


TOGETHER_URL = "https://api.together.xyz/v1"


class TogetherLLM(OpenAILLM):
    """Together AI chat (OpenAI-compatible endpoint). Like the reference it
    ignores ``response_format`` (providers.py:130-168)."""

    def __init__(self, api_key: Optional[str] = None,
                 model: str = "mistralai/Mixtral-8x7B-Instruct-v0.1"):
        super().__init__(api_key=api_key or os.environ.get("TOGETHER_API_KEY"), model=model,
                         base_url=TOGETHER_URL)

    def completion(self, messages, response_format=None) -> str:
        return super().completion(messages, None)

    def completion_stream(self, messages, response_format=None):
        return super().completion_stream(messages, None)


class TogetherEmbedder(OpenAIEmbedder):
    def __init__(self, api_key: Optional[str] = None,
                 model: str = "togethercomputer/m2-bert-80m-8k-retrieval"):
        super().__init__(api_key=api_key or os.environ.get("TOGETHER_API_KEY"), model=model,
                         base_url=TOGETHER_URL, dim=768)


GEMINI_URL = "https://generativelanguage.googleapis.com/v1beta"


def _flatten_messages(messages: List[Dict[str, str]]) -> str:
    # reference providers.py:74-77: everything not 'user' is rendered as Assistant
    return "".join(f"{'User' if m['role'] == 'user' else 'Assistant'}: {m['content']}\n"
                   for m in messages)


class GeminiLLM(LLMProvider):
    def __init__(self, api_key: Optional[str] = None, model: str = "gemini-1.5-flash"):
        self.api_key = api_key or os.environ.get("GEMINI_API_KEY")
        self.model_name = model

    def _url(self, verb: str) -> str:
        return f"{GEMINI_URL}/models/{self.model_name}:{verb}?key={self.api_key}"

    def completion(self, messages, response_format=None) -> str:
        try:
            import httpx

            body = {"contents": [{"parts": [{"text": _flatten_messages(messages)}]}]}
            r = httpx.post(self._url("generateContent"), json=body, timeout=60)
            r.raise_for_status()
            return r.json()["candidates"][0]["content"]["parts"][0]["text"]
        except Exception as e:
            log.warning("Gemini error: %s", e)
            return ""

    def completion_stream(self, messages, response_format=None):
        text = self.completion(messages, response_format)
        yield text


class GeminiEmbedder(EmbeddingProvider):
    dim = 768

    def __init__(self, api_key: Optional[str] = None, model: str = "models/embedding-001"):
        self.api_key = api_key or os.environ.get("GEMINI_API_KEY")
        self.model = model

    def _post(self, verb, body):
        import httpx

        r = httpx.post(f"{GEMINI_URL}/{self.model}:{verb}?key={self.api_key}", json=body, timeout=60)
        r.raise_for_status()
        return r.json()

    def embed(self, text: str) -> List[float]:
        try:
            return self._post("embedContent", {"content": {"parts": [{"text": text}]}})["embedding"]["values"]
        except Exception as e:
            log.warning("Gemini embedding error: %s", e)
            return [0.0] * self.dim

    def batch_embed(self, texts: List[str]) -> List[List[float]]:
        if not texts:
            return []
        try:
            reqs = [{"model": self.model, "content": {"parts": [{"text": t}]}} for t in texts]
            out = self._post("batchEmbedContents", {"requests": reqs})
            return [e["values"] for e in out["embeddings"]]
        except Exception as e:
            log.warning("Gemini batch embedding error: %s", e)
            return [[0.0] * self.dim for _ in texts]


# --------------------------------------------------------------------------
# Local, network-free providers
# --------------------------------------------------------------------------
_WORD = re.compile(r"[a-z0-9']+")


class HashEmbedder(EmbeddingProvider):
    """Deterministic lexical embeddings: signed feature hashing of word unigrams
    and bigrams (+ char trigrams of each word), L2-normalised. Similar wording ->
    high cosine; unrelated text -> ~0. CPU numpy; cheap enough for the
    1k-turn plumbing config. Batch calls can be moved to the device encoder by
    using :class:`lazzaro_amd.core.embedders.OnDeviceEmbedder` instead."""

    def __init__(self, dim: int = 384, seed: int = 0):
        self.dim = dim
        self.seed = seed

    def _h(self, tok: str):
        d = hashlib.blake2b(tok.encode(), digest_size=8, key=str(self.seed).encode()).digest()
        v = int.from_bytes(d, "little")
        return v % self.dim, 1.0 if (v >> 63) & 1 else -1.0

    def _vec(self, text: str) -> np.ndarray:
        words = _WORD.findall(text.lower())
        v = np.zeros(self.dim, dtype=np.float64)
        feats = list(words) + [a + "_" + b for a, b in zip(words, words[1:])]
        for w in words:
            p = f"#{w}#"
            feats.extend(p[i:i + 3] for i in range(max(1, len(p) - 2)))
        for f in feats:
            i, s = self._h(f)
            v[i] += s
        n = np.linalg.norm(v)
        return v / n if n > 0 else v

    def embed(self, text: str) -> List[float]:
        return self._vec(text).tolist()

    def batch_embed(self, texts: List[str]) -> List[List[float]]:
        return [self._vec(t).tolist() for t in texts]


_TOPIC_WORDS = {
    "work": ("work", "project", "meeting", "deadline", "client", "colleague", "job", "office"),
    "personal": ("family", "friend", "hobby", "home", "personal", "wife", "husband", "kids"),
    "learning": ("learn", "study", "course", "book", "tutorial", "practice", "reading"),
    "health": ("health", "exercise", "diet", "sleep", "medical", "fitness", "run", "gym"),
}
_DOMAIN_HINTS = {
    "preferences": ("like", "love", "prefer", "favorite", "favourite", "enjoy", "hate"),
    "personality_traits": ("tend", "patient", "curious", "detail", "careful", "introvert", "extrovert"),
    "knowledge_domains": ("experience", "expert", "know", "years", "skilled", "engineer", "study"),
    "interaction_style": ("communication", "concise", "direct", "verbose", "meetings", "talk"),
    "key_experiences": ("started", "moved", "graduated", "born", "won", "lost", "finished"),
}

_DOMAIN_RX = {d: re.compile("|".join(map(re.escape, h))) for d, h in _DOMAIN_HINTS.items()}


def _topic(text: str) -> str:
    low = text.lower()
    for k, words in _TOPIC_WORDS.items():
        if any(w in low for w in words):
            return k
    return "other"


def _third_person(s: str) -> str:
    s = s.strip().rstrip(".!?")
    rep = [(r"\bI am\b", "User is"), (r"\bI'm\b", "User is"), (r"\bI've\b", "User has"),
           (r"\bI\b", "User"), (r"\bmy\b", "their"), (r"\bMy\b", "Their"), (r"\bme\b", "them")]
    for a, b in rep:
        s = re.sub(a, b, s)
    if not s.lower().startswith("user"):
        s = "User says: " + s
    return s + "."


class LocalLLM(LLMProvider):
    """Deterministic offline stand-in for a chat LLM.

    Recognises the framework's three prompt kinds by their system prompt and
    answers in the requested JSON shape:
      * fact extraction -> {"memories": [...]} from the user's sentences
      * profile extraction -> {domain: insight} by keyword routing
      * anything else -> a short grounded reply quoting retrieved memories
    Used by the benchmarks (synthetic conversations) and offline demos.
    """

    def __init__(self, max_facts: int = 8):
        self.max_facts = max_facts
        self.calls = 0

    def completion(self, messages, response_format=None) -> str:
        self.calls += 1
        sys_txt = " ".join(m["content"] for m in messages if m["role"] == "system")
        user_txt = "\n".join(m["content"] for m in messages if m["role"] == "user")
        if "Extract distinct, atomic facts" in sys_txt:
            return json.dumps({"memories": self._facts(user_txt)})
        if "Analyze these related memories" in sys_txt:
            return json.dumps(self._profile(user_txt))
        if "psychological and knowledge profile" in sys_txt:
            return "1. **Personality Traits**: (local model) derived from stored observations.\n" + \
                   "\n".join(user_txt.splitlines()[:5])
        ctx = [l[2:] for l in sys_txt.splitlines() if l.startswith("- ")]
        last = user_txt.splitlines()[-1] if user_txt else ""
        if ctx:
            return f"Noted: {last[:80]}. I remember that {ctx[0]}"
        return f"Noted: {last[:80]}."

    def completion_stream(self, messages, response_format=None):
        text = self.completion(messages, response_format)
        for i in range(0, len(text), 16):
            yield text[i:i + 16]

    def _facts(self, conv_json: str) -> List[Dict]:
        try:
            mems = json.loads(conv_json)
        except Exception:
            mems = [{"content": conv_json, "type": "episodic"}]
        out = []
        for m in mems:
            if not isinstance(m, dict) or m.get("type") != "episodic":
                continue  # user turns are episodic; assistant turns are not facts
            for sent in re.split(r"(?<=[.!?])\s+", str(m.get("content", ""))):
                if len(sent.strip()) < 8:
                    continue
                fact = _third_person(sent)
                low = fact.lower()
                kind = "procedural" if any(w in low for w in ("always", "usually", "workflow", "process")) else \
                    ("episodic" if any(w in low for w in ("today", "yesterday", "started", "just")) else "semantic")
                sal = min(1.0, 0.5 + 0.05 * len(_WORD.findall(low)) / 4)
                out.append({"content": fact, "type": kind, "salience": round(sal, 3),
                            "topic": _topic(fact)})
                if len(out) >= self.max_facts:
                    return out
        return out

    def _profile(self, prompt: str) -> Dict[str, str]:
        lines = [l[2:] for l in prompt.splitlines() if l.startswith("- ")]
        low = [l.lower() for l in lines]
        out: Dict[str, str] = {}
        for dom, rx in _DOMAIN_RX.items():  # substring match of any hint, one scan per line
            hit = [l for l, lo in zip(lines, low) if rx.search(lo)]
            if hit:
                out[dom] = "; ".join(hit[:2])
        return out


class ScriptedLLM(LLMProvider):
    """Returns canned responses in order (tests / reproducible demos)."""

    def __init__(self, responses: List[str], default: str = "{}"):
        self.responses = list(responses)
        self.default = default

    def completion(self, messages, response_format=None) -> str:
        return self.responses.pop(0) if self.responses else self.default

    def completion_stream(self, messages, response_format=None):
        yield self.completion(messages, response_format)


def cosine(a, b) -> float:
    """Host cosine for single pairs (reference memory_system.py:197-203)."""
    if a is None or b is None or len(a) == 0 or len(b) == 0:
        return 0.0
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    n = math.sqrt(float(a @ a)) * math.sqrt(float(b @ b))
    return float(a @ b) / n if n > 0 else 0.0
