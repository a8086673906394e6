"""Encoder parity against an independent BERT implementation: a random-init
``transformers.BertModel`` per north-star config is saved as safetensors,
loaded through ``SentenceEncoder.load_safetensors`` (HF parameter names) and
compared token by token (last hidden state) and after pooling. CPU tier: the
fp32 path. The bf16 HIP-kernel path is compared in
tests/kernels/test_encoder_parity_gpu.py. (No real checkpoints offline, so
the weights are random; every LayerNorm / bias is randomised too so no
parameter sits at a trivially-correct value.)"""
import os

import pytest
import torch

transformers = pytest.importorskip("transformers")
pytest.importorskip("safetensors")

from lazzaro_amd.core.embedders import Tokenizer  # noqa: E402
from lazzaro_amd.models.encoder import SentenceEncoder, get_config  # noqa: E402

TEXTS = ["The quick brown fox jumps over the lazy dog.",
         "I work on GPU kernels for agent memory systems at my job in Lisbon.",
         "short",
         "Memory consolidation links related facts, decays weak edges and prunes them over many conversations."]


def hf_bert(name: str, path: str, seed: int = 0):
    """Random-init HF BertModel with the config's shape, saved to ``path``."""
    from safetensors.torch import save_file

    c = get_config(name)
    cfg = transformers.BertConfig(vocab_size=c.vocab, hidden_size=c.hidden, num_hidden_layers=c.layers,
                                  num_attention_heads=c.heads, intermediate_size=c.ffn,
                                  max_position_embeddings=c.max_pos, hidden_act="gelu", layer_norm_eps=c.eps,
                                  type_vocab_size=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    torch.manual_seed(seed)
    m = transformers.BertModel(cfg, add_pooling_layer=False).eval()
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("LayerNorm.weight"):
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=g))
            elif n.endswith("bias"):
                p.copy_(0.02 * torch.randn(p.shape, generator=g))
    save_file({("bert." + k): v.contiguous() for k, v in m.state_dict().items()}, path)
    return m


def batch(tok_max=64, vocab=30522):
    tok = Tokenizer(vocab_size=vocab)
    ids, lens = tok.encode_batch(TEXTS, tok_max)
    mask = (torch.arange(ids.shape[1])[None, :] < lens[:, None]).long()
    return ids.long(), lens, mask


def hf_reference(m, ids, mask, pooling):
    with torch.no_grad():
        h = m(input_ids=ids, attention_mask=mask).last_hidden_state.float()
    h = h * mask[..., None]
    if pooling == "cls":
        p = h[:, 0]
    else:
        p = h.sum(1) / mask.sum(1, keepdim=True)
    return h, p / p.norm(dim=1, keepdim=True)


def rel_err(a, b):
    return float((a - b).norm() / b.norm())


@pytest.mark.parametrize("name", ["minilm-l6", "bge-base"])
def test_cpu_fp32_matches_hf_bert(name, tmp_path):
    path = str(tmp_path / f"{name}.safetensors")
    m = hf_bert(name, path)
    enc = SentenceEncoder(name, device="cpu", weights=path, dtype=torch.float32)
    ids, lens, mask = batch()
    h_ref, p_ref = hf_reference(m, ids, mask, enc.cfg.pooling)
    h = enc.hidden_states(ids, lens)
    for b in range(len(TEXTS)):
        n = int(lens[b])
        assert rel_err(h[b, :n], h_ref[b, :n]) < 1e-4, (name, b)
    p, _ = enc.forward(ids, lens)
    assert rel_err(p, p_ref) < 1e-4
    # centred cosine of the pooled vectors (random-init vectors share a large
    # common component; centring removes it so the check keeps its power)
    pc, rc = p - p.mean(0), p_ref - p_ref.mean(0)
    cos = torch.nn.functional.cosine_similarity(pc, rc, dim=1)
    assert float(cos.min()) > 0.9999
