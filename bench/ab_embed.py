"""A/B of the bge-base batch embed (1024 synthetic queries, packed varlen):
one stream vs the batch split over 2 / 3 / 4 HIP streams (tail filling)."""
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


def main():
    dev = torch.device("cuda", 0)
    emb = OnDeviceEmbedder("bge-base", device=dev, max_len=64)
    texts = bench.synth_texts(1024, random.Random(1234))
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    ref, _ = emb.encoder.forward(ids, lens, pad_to=768)
    res = {}
    for parts in (1, 2, 3, 4):
        o, _ = emb.encoder.forward_streams(ids, lens, pad_to=768, parts=parts)
        torch.cuda.synchronize()
        diff = float((o - ref).abs().max())
        ts = []
        for _ in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                emb.encoder.forward_streams(ids, lens, pad_to=768, parts=parts)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / 3)
        res[parts] = {"ms_median": round(statistics.median(ts) * 1e3, 3), "max_abs_diff": diff}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
