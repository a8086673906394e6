"""Kernel-time profile target for the bge-base batch embed (1024 synthetic
queries, packed varlen, one stream so per-kernel durations do not overlap).
Run under: rocprofv3 --kernel-trace --stats -- python bench/prof_embed.py"""
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from lazzaro_amd.core.embedders import OnDeviceEmbedder  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = os.environ.get("P_MODEL", "bge-base")
    kw = {"precision": os.environ["P_PREC"]} if os.environ.get("P_PREC") else {}
    emb = OnDeviceEmbedder(model, device=dev, max_len=64, **kw)
    texts = bench.synth_texts(1024, random.Random(1234))
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    parts = int(os.environ.get("P_PARTS", "1"))
    for _ in range(int(os.environ.get("P_REPS", "10"))):
        emb.encoder.forward_streams(ids, lens, pad_to=emb.encoder.cfg.hidden, parts=parts)
    torch.cuda.synchronize()
    print("tokens", int(lens.sum()), flush=True)


if __name__ == "__main__":
    main()
