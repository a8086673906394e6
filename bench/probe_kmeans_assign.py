"""Probe (diagnostic): k-means at the IVF-PQ bench's coarse-quantiser shape
(524k x 1024 training rows, 16,384 centroids): does the MFMA argmax assign
(flat_top1) agree with a plain fp32 argmax, and how tight are the clusters.
Prints one JSON line."""
import json
import sys

import torch

sys.path.insert(0, "bench")
sys.path.insert(1, ".")
from bench_ivfpq_scale import Mixture  # noqa: E402
from lazzaro_amd.index import kmeans as KM  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    d = 1024
    mix = Mixture(d, 100_000, 1.0, 1, dev)
    X = torch.cat([mix.chunk(0, 1 << 19)])
    X16 = torch.zeros((X.shape[0], d), dtype=torch.bfloat16, device=dev)
    X16[:] = X.to(torch.bfloat16)
    out = {}
    for k in (1024, 16384):
        c32, c16, lab = KM.kmeans(X16, k, iters=8, seed=0)
        ref = torch.argmax(X16.float() @ c16.float().T, dim=1)
        s_lab = (X16.float() * c16.float()[lab.long()]).sum(1)
        s_ref = (X16.float() * c16.float()[ref]).sum(1)
        lab2, _ = KM.assign(X16, c16)
        out[f"k{k}"] = {"kmeans_label_agree_exact": round(float((lab.long() == ref).float().mean()), 5),
                        "assign_agree_exact": round(float((lab2.long() == ref).float().mean()), 5),
                        "score_gap_max": float((s_ref - s_lab).max()),
                        "mean_cos_to_centroid": round(float(s_ref.mean()), 5),
                        "empty_clusters": int((torch.bincount(ref, minlength=k) == 0).sum())}
        print(k, out[f"k{k}"], file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
