"""A/B of the large-batch query embed split into 1-4 sub-batches on separate
HIP streams (OnDeviceEmbedder, LZK_EMBED_PARTS): bge-base, the bench's 1024
synthetic query texts, interleaved rounds in one process; also checks that
every split gives the same vectors as the single forward. Prints one JSON."""
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

    dev = torch.device("cuda", 0)
    emb = OnDeviceEmbedder("bge-base", device=dev, max_len=64, seed=0)
    texts = synth_texts(1024, random.Random(1234))
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    enc = emb.encoder
    arms = [1, 2, 3, 4]
    ref = enc.forward(ids, lens)[0]
    cos = {}
    for p in arms[1:]:
        v = enc.forward_streams(ids, lens, parts=p)[0]
        cos[p] = float(torch.nn.functional.cosine_similarity(v.float(), ref.float(), dim=1).min())
    t_end = time.perf_counter() + 3.0  # clock ramp
    while time.perf_counter() < t_end:
        enc.forward_streams(ids, lens, parts=2)
        torch.cuda.synchronize()
    ts = {p: [] for p in arms}
    for _ in range(7):
        for p in arms:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                enc.forward_streams(ids, lens, parts=p)
            torch.cuda.synchronize()
            ts[p].append((time.perf_counter() - t0) / 5)
    print(json.dumps({"model": "bge-base", "texts": len(texts), "tokens": int(lens.sum()),
                      "min_cos_vs_single": cos,
                      "ms_median": {p: round(statistics.median(v) * 1e3, 3) for p, v in ts.items()}}, indent=1))


if __name__ == "__main__":
    main()
