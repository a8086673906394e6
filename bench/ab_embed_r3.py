"""Round-3 A/B of the bench's query embed (bge-base, 1024 synthetic texts,
packed varlen, CLS-only last layer): sub-batch stream split (parts, uneven
first share) and split-K of the N = 768 projections (SentenceEncoder.SPLITK),
interleaved rounds in one process, median ms. One JSON line."""
import json
import os
import random
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from bench import synth_texts
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    from lazzaro_amd.models.encoder import SentenceEncoder

    dev = torch.device("cuda", 0)
    emb = OnDeviceEmbedder("bge-base", device=dev, max_len=64, seed=0)
    texts = synth_texts(1024, random.Random(1234))
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    enc = emb.encoder
    arms = {"p1": (1, 0.0, 0), "p2": (2, 0.0, 0), "p3": (3, 0.0, 0), "p2_f35": (2, 0.35, 0), "p2_f65": (2, 0.65, 0),
            "p2_sk1": (2, 0.0, 1), "p2_sk2": (2, 0.0, 2), "p1_sk2": (1, 0.0, 2)}
    ref = enc.forward(ids, lens)[0]

    def run(a):
        parts, ff, sk = arms[a]
        SentenceEncoder.SPLITK = sk
        out = enc.forward_streams(ids, lens, parts=parts, first_frac=ff)[0]
        SentenceEncoder.SPLITK = 0
        return out

    cos = {a: float(torch.nn.functional.cosine_similarity(run(a).float(), ref.float(), dim=1).min()) for a in arms}
    t_end = time.perf_counter() + 3.0
    while time.perf_counter() < t_end:
        run("p2")
        torch.cuda.synchronize()
    ts = {a: [] for a in arms}
    for _ in range(7):
        for a in arms:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                run(a)
            torch.cuda.synchronize()
            ts[a].append((time.perf_counter() - t0) / 10 * 1e3)
    print(json.dumps({"ms_median": {a: round(statistics.median(v), 3) for a, v in ts.items()},
                      "min_cos_vs_single_forward": cos}), flush=True)


if __name__ == "__main__":
    main()
