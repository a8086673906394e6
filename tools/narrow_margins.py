"""Diagnostic: the single-query int8 store search's margins and list sizes
over a 10M x 768 tenant (bench.py's populate): the statistical and
worst-case margins of TenantGraph._i8_query, the sample threshold tau, the
true 10th score, and how many rows clear tau - margin (the scan's list) for
each margin. Prints one JSON line."""
import json
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bench import populate
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import LocalLLM
    from lazzaro_amd.ops.search import _flat_topk_lane
    dev = torch.device("cuda", 0)
    emb = OnDeviceEmbedder("bge-base", device=dev, max_len=64)
    n = int(os.environ.get("ROWS", 10_000_000))
    out = {}
    with tempfile.TemporaryDirectory() as d:
        ms = MemorySystem(llm_provider=LocalLLM(), embedding_provider=emb, device=dev, db_dir=d, load_from_disk=False,
                          enable_async=False, enable_caching=False, max_buffer_size=2 * n)
        populate(ms, n, 768, dev, seed=1)
        g = ms.graph
        texts = ["what did I say about moving to Lisbon and learning the cello?", "my sister's birthday plans"]
        gen = torch.Generator(device=dev).manual_seed(3)
        Qr = torch.randn(4, 768, device=dev, generator=gen)
        Qr = Qr / Qr.norm(dim=1, keepdim=True)
        Q = torch.cat([emb.embed_tensor(texts)[0].float(), Qr])
        bias = g.store_bias("l2")
        for i in range(Q.shape[0]):
            qf = Q[i:i + 1]
            q16 = g._q16(qf)
            q8, qs, m_stat, m_rig = g._i8_query(q16, 2.0)
            X16 = g.emb16[:g.n]
            s_all = []
            for c0 in range(0, g.n, 1 << 20):
                c1 = min(g.n, c0 + (1 << 20))
                s_all.append(2.0 * (X16[c0:c1].float() @ q16[0].float()) + bias[c0:c1])
            sc = torch.cat(s_all)
            top = torch.topk(sc, 10).values
            rec = {"t10": float(top[-1]), "t1": float(top[0]), "m_stat": float(m_stat[0]), "m_rig": float(m_rig[0])}
            for S, J in ((64, 3), (256, 3)):
                bs = bias[:g.n:S].contiguous()
                ts, _ = _flat_topk_lane(X16[::S], q16, 16, 16, bs, None, None, 2.0, 0, None)
                tau = float(ts[0, J - 1])
                rec[f"tau_S{S}"] = tau
                for name, m in (("stat", rec["m_stat"]), ("rig", rec["m_rig"])):
                    # rows whose bf16 score clears thr - m (int8 score >= thr needs bf16 >= thr - m at worst)
                    rec[f"rows_S{S}_{name}"] = int((sc >= tau - m - m).sum())
                    rec[f"rows_S{S}_{name}_exact"] = int((sc >= tau - m).sum())
            rec["rows_above_t10_minus_2rig"] = int((sc >= rec["t10"] - 2 * rec["m_rig"]).sum())
            out[f"q{i}"] = rec
        ms.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
