"""Port of reference tests/test_providers.py (provider injection, default
OpenAI providers against a patched client)."""
from unittest.mock import MagicMock, patch

from lazzaro_amd.core.interfaces import EmbeddingProvider, LLMProvider
from lazzaro_amd.core.memory_system import MemorySystem


class MockLLM(LLMProvider):
    def completion(self, messages, response_format=None):
        return "Mock response"


class MockEmbedder(EmbeddingProvider):
    def embed(self, text):
        return [0.1] * 1536

    def batch_embed(self, texts):
        return [[0.1] * 1536 for _ in texts]


def test_custom_providers():
    ms = MemorySystem(openai_api_key="fake", enable_async=False, load_from_disk=False,
                      llm_provider=MockLLM(), embedding_provider=MockEmbedder())
    ms.start_conversation()
    assert ms.chat("Hello") == "Mock response"
    assert ms.metrics["llm_calls"] == 1 and ms.metrics["embedding_calls"] == 1
    ms.close()


@patch("lazzaro_amd.core.providers.openai")
def test_default_providers(mock_openai):
    client = MagicMock()
    mock_openai.OpenAI.return_value = client
    comp = MagicMock()
    comp.choices[0].message.content = "OpenAI response"
    client.chat.completions.create.return_value = comp
    emb = MagicMock()
    emb.data[0].embedding = [0.2] * 1536
    client.embeddings.create.return_value = emb
    ms = MemorySystem(openai_api_key="fake", enable_async=False, load_from_disk=False)
    ms.start_conversation()
    assert ms.chat("Hello") == "OpenAI response"
    client.chat.completions.create.assert_called()
    client.embeddings.create.assert_called()
    ms.close()


def test_chat_stream_yields_info_then_tokens():
    from lazzaro_amd.core.providers import LocalLLM
    ms = MemorySystem(enable_async=False, load_from_disk=False, llm_provider=LocalLLM(),
                      embedding_provider=MockEmbedder())
    ev = list(ms.chat_stream("I love hiking in the mountains."))
    assert ev[0]["type"] == "info" and "Retrieval" in ev[0]["content"]
    toks = "".join(e["content"] for e in ev if e["type"] == "token")
    assert toks and ms.conversation_history[-1]["content"] == toks
    ms.close()
