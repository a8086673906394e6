"""CPU tier of the encoder stack: tokenizer + reference forward shapes/norms."""
import pytest
import torch

from lazzaro_amd.core.embedders import OnDeviceEmbedder, Tokenizer
from lazzaro_amd.models.encoder import CONFIGS, SentenceEncoder, get_config


def test_tokenizer_hashed_vocab_is_deterministic():
    t = Tokenizer()
    a = t.encode("Hello, World! I love Rust.")
    assert a[0] == 101 and a[-1] == 102 and len(a) == 2 + 8
    assert a == t.encode("hello , world ! i love rust .")
    ids, lens = t.encode_batch(["a b c", "hello world"], 16)
    assert ids.shape[0] == 2 and ids.shape[1] % 8 == 0 and lens.tolist() == [5, 4]
    assert (ids[1, 4:] == 0).all()


def test_tokenizer_wordpiece_with_vocab(tmp_path):
    vocab = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "play", "##ing", "the"]
    p = tmp_path / "vocab.txt"
    p.write_text("\n".join(vocab))
    t = Tokenizer(str(p))
    assert t.encode("the playing xyz") == [101, 105, 103, 104, 100, 102]


def test_configs():
    assert get_config("BAAI/bge-base-en-v1.5").hidden == 768
    assert get_config("all-MiniLM-L6-v2").heads * 32 == 384
    assert get_config("e5-large-v2").layers == 24 and CONFIGS["bge-base"].pooling == "cls"


def test_tiny_encoder_cpu_forward():
    enc = SentenceEncoder("tiny", device="cpu")
    ids = torch.randint(1000, 4096, (3, 16), dtype=torch.int32)
    lens = torch.tensor([16, 5, 9], dtype=torch.int32)
    v, v16 = enc.forward(ids, lens, pad_to=192)
    assert v.shape == (3, 128) and torch.allclose(v.norm(dim=1), torch.ones(3), atol=1e-5)
    assert v16.shape == (3, 192) and (v16[:, 128:] == 0).all()
    # padding positions must not influence the result
    ids2 = ids.clone()
    ids2[1, 5:] = 1234
    v2, _ = enc.forward(ids2, lens)
    assert torch.allclose(v[1], v2[1], atol=1e-3)


def test_on_device_embedder_cpu():
    e = OnDeviceEmbedder("tiny", device="cpu")
    out = e.batch_embed(["first text here", "second", "a much longer third text with more words"])
    assert len(out) == 3 and len(out[0]) == 128
    assert abs(sum(x * x for x in out[1]) - 1.0) < 1e-3
    assert e.embed("second") == out[1] or max(abs(a - b) for a, b in zip(e.embed("second"), out[1])) < 1e-4


def test_long_text_chunking_windows_and_mean():
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    emb = OnDeviceEmbedder("tiny", device="cpu", max_len=32)
    long = " ".join(f"word{i}" for i in range(100))  # 100 pieces > 30 per window
    ids, lens, owner = emb.tok.encode_chunks(["short text", long], 32, 8)
    # body 30, stride 22: windows start at 0, 22, 44, 66 (ends at 96, 100)
    assert owner.tolist() == [0, 1, 1, 1, 1, 1] and int(lens.max()) == 32
    assert ids[1, 0] == 101 and ids[1, 31] == 102
    v = emb.embed_long(["short text", long], overlap=8)
    assert torch.allclose(v.norm(dim=1), torch.ones(2), atol=1e-5)
    short_direct = torch.tensor(emb.embed("short text"))
    assert torch.allclose(v[0], short_direct, atol=1e-5)
    # batch_embed routes long texts through the chunked path
    out = emb.batch_embed(["short text", long * 3])
    assert len(out) == 2 and abs(sum(x * x for x in out[1]) - 1.0) < 1e-4


def test_packed_varlen_forward_matches_padded():
    from lazzaro_amd.models.encoder import SentenceEncoder
    enc = SentenceEncoder("tiny", seed=2)
    ids = torch.randint(1000, 4000, (4, 24), dtype=torch.int32)
    lens = torch.tensor([24, 7, 15, 2], dtype=torch.int32)
    for b in range(4):
        ids[b, lens[b]:] = 0
    a, _ = enc.forward(ids, lens, packed=False)
    b, _ = enc.forward(ids, lens, packed=True)
    torch.testing.assert_close(a, b, atol=2e-2, rtol=0)  # bf16 CPU reference, same math
    assert ((a * b).sum(1) > 0.9999).all()


@pytest.mark.parametrize("packed", [False, True])
def test_cls_pooling_last_layer_on_cls_rows_only(packed, monkeypatch):
    """CLS pooling: the last layer's post-attention work on the CLS rows only
    gives the same embedding as the full last layer (packed and padded)."""
    import dataclasses

    from lazzaro_amd.models import encoder as M
    cfg = dataclasses.replace(M.CONFIGS["tiny"], pooling="cls")
    monkeypatch.setitem(M.CONFIGS, "tiny-cls", cfg)
    enc = M.SentenceEncoder("tiny-cls", seed=4)
    ids = torch.randint(1000, 4000, (5, 20), dtype=torch.int32, generator=torch.Generator().manual_seed(11))
    lens = torch.tensor([20, 3, 11, 1, 7], dtype=torch.int32)
    monkeypatch.setattr(M.SentenceEncoder, "CLS_LAST", False)
    full, _ = enc.forward(ids, lens, packed=packed)
    monkeypatch.setattr(M.SentenceEncoder, "CLS_LAST", True)
    cls, _ = enc.forward(ids, lens, packed=packed)
    torch.testing.assert_close(cls, full, atol=1e-6, rtol=0)
