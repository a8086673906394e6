"""HIP encoder (bf16 MFMA kernels, packed varlen layout) against a random-init
``transformers.BertModel`` run in fp32, for the three north-star configs
(MiniLM-L6 / bge-base / e5-large). Weights go through
``SentenceEncoder.load_safetensors``; see tests/unit/test_encoder_parity.py."""
import pytest
import torch

from tests.unit.test_encoder_parity import TEXTS, batch, hf_bert, hf_reference, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("name,tol_tok,tol_pool", [("minilm-l6", 2e-2, 1e-2), ("bge-base", 3e-2, 1.5e-2),
                                                   ("e5-large", 4e-2, 2e-2)])
def test_gpu_bf16_matches_hf_bert(name, tol_tok, tol_pool, tmp_path):
    from lazzaro_amd.models.encoder import SentenceEncoder

    path = str(tmp_path / f"{name}.safetensors")
    m = hf_bert(name, path).to(DEV)
    enc = SentenceEncoder(name, device=DEV, weights=path)
    ids, lens, mask = batch()
    h_ref, p_ref = hf_reference(m, ids.to(DEV), mask.to(DEV), enc.cfg.pooling)
    h = enc.hidden_states(ids, lens)
    worst = 0.0
    for b in range(len(TEXTS)):
        n = int(lens[b])
        for t in range(n):
            worst = max(worst, rel_err(h[b, t], h_ref[b, t]))
    assert worst < tol_tok, worst
    p, _ = enc.forward(ids, lens)
    assert rel_err(p, p_ref) < tol_pool
    pc, rc = p - p.mean(0), p_ref - p_ref.mean(0)
    assert float(torch.nn.functional.cosine_similarity(pc, rc, dim=1).min()) > 0.99
    # the fp8 projection path stays close to the same reference
    enc8 = SentenceEncoder(name, device=DEV, weights=path, precision="fp8")
    p8, _ = enc8.forward(ids, lens)
    assert float(torch.nn.functional.cosine_similarity(p8, p_ref, dim=1).min()) > 0.98
