"""A/B of the split-K O / FFN2 projections (models/encoder.py _lin_ln,
LZK_SPLITK: 0 off, 1 FFN2, 2 O + FFN2) in the bge-base forward of the bench
batch (1024 synthetic queries) on 1 and 2 sub-batch streams, and of the fact
batch of the consolidation bench (1024 x 12 words). Interleaved rounds in one
process; prints one JSON object."""
import json
import os
import random
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from lazzaro_amd.core.embedders import OnDeviceEmbedder  # noqa: E402
from lazzaro_amd.models.encoder import SentenceEncoder  # noqa: E402


WORDS = "user likes prefers works lives started visited learned project team python rust garden music".split()


def main():
    dev = torch.device("cuda", 0)
    emb = OnDeviceEmbedder("bge-base", device=dev, max_len=64, seed=0)
    texts = bench.synth_texts(1024, random.Random(1234))
    q_ids, q_lens = emb.tok.encode_batch(texts, emb.max_len)
    rng = random.Random(7)
    facts = [" ".join(rng.choice(WORDS) for _ in range(12)) for _ in range(1024)]
    f_ids, f_lens = emb.tok.encode_batch(facts, 64)
    out = {"query_tokens": int(q_lens.sum()), "fact_tokens": int(f_lens.sum())}
    arms = {f"split{m}_{name}_{p}s": (m, ids, lens, p) for m in (0, 1, 2)
            for name, (ids, lens) in (("query", (q_ids, q_lens)), ("fact", (f_ids, f_lens))) for p in (1, 2)}
    ref = {}
    for a, (m, ids, lens, p) in arms.items():
        SentenceEncoder.SPLITK = m
        o, _ = emb.encoder.forward_streams(ids, lens, pad_to=768, parts=p)
        key = id(ids)
        if key not in ref:
            ref[key] = o
        out.setdefault("cos_min", {})[a] = float((o * ref[key]).sum(1).min())
    ts = {a: [] for a in arms}
    for _ in range(5):
        for a, (m, ids, lens, p) in arms.items():
            SentenceEncoder.SPLITK = m
            emb.encoder.forward_streams(ids, lens, pad_to=768, parts=p)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                emb.encoder.forward_streams(ids, lens, pad_to=768, parts=p)
            torch.cuda.synchronize()
            ts[a].append((time.perf_counter() - t0) / 3)
    out["ms_median"] = {a: round(statistics.median(v) * 1e3, 3) for a, v in ts.items()}
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
