"""CU-masked streams (hipExtStreamCreateWithCUMask): how the mask bits map to
CUs (a GEMM's time vs. the mask), and whether the headline's two halves --
the bge-base query embed and the 10M x 768 int8 store search -- run faster
side by side on disjoint CU sets than one after the other on the whole chip.
Prints JSON. Diagnostic only."""
import ctypes
import json
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(bits):
    m = (ctypes.c_uint32 * 8)()
    for b in bits:
        m[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, m)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it * 1e3


def main():
    from lazzaro_amd.ops import _lib
    from lazzaro_amd.ops import encoder_ops as E
    L = _lib.lib()
    L.lzk_set_cu_budget.argtypes = [ctypes.c_int]
    dev = torch.device("cuda", 0)
    out = {}
    T, N, K = 22585, 3072, 768
    x = torch.randn(T, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    y = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
    gemm = {}
    for name, bits in [("all256", range(256)), ("first128", range(128)), ("even128", range(0, 256, 2)),
                       ("first64", range(64)), ("every4_64", range(0, 256, 4)), ("first32", range(32))]:
        st = masked_stream(list(bits))
        with torch.cuda.stream(st):
            gemm[name] = round(timeit(lambda: E.linear(x, w, b, act="gelu", out=y)), 3)
    out["ffn1_gemm_ms_by_mask"] = gemm
    print(json.dumps(out), flush=True)

    from lazzaro_amd.engine.tenant_graph import TenantGraph
    from lazzaro_amd.core.embedders import OnDeviceEmbedder
    import bench
    g = TenantGraph(device=dev)
    g._set_dim(768)
    rows = int(os.environ.get("P_ROWS", 10_000_000))
    g.reserve(rows)
    gen = torch.Generator(device=dev).manual_seed(1)
    for r0 in range(0, rows, 1 << 20):
        r1 = min(rows, r0 + (1 << 20))
        v = torch.randn(r1 - r0, 768, device=dev, generator=gen)
        g.add_nodes([f"n{i}" for i in range(r0, r1)], [""] * (r1 - r0), v / v.norm(dim=1, keepdim=True),
                    shard=g.shard_id("w"), stored=True)
    emb = OnDeviceEmbedder("bge-base", device=dev, max_len=64)
    texts = bench.synth_texts(1024, random.Random(1))
    ids, lens = emb.tok.encode_batch(texts, emb.max_len)
    Q = emb.encoder.forward_streams(ids, lens, pad_to=0, parts=1)[0]
    torch.cuda.synchronize()

    def search():
        g.store_search(Q, 10, "l2")

    def embed():
        emb.encoder.forward_streams(ids, lens, pad_to=768, parts=1)

    res = {"seq_embed_ms": round(timeit(embed), 3), "seq_search_ms": round(timeit(search), 3)}
    for ne in (64, 80, 96):
        # encoder on every (256/ne)-th... CU set chosen by bit striding; search on the rest
        step = 256 / ne
        ebits = sorted({int(i * step) for i in range(ne)})
        sbits = [i for i in range(256) if i not in set(ebits)]
        se, ss = masked_stream(ebits), masked_stream(sbits)
        L.lzk_set_cu_budget(len(sbits))
        with torch.cuda.stream(se):
            te = timeit(embed)
        with torch.cuda.stream(ss):
            ts = timeit(search)

        def both():
            se.wait_stream(torch.cuda.current_stream())
            ss.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(se):
                embed()
            with torch.cuda.stream(ss):
                search()
            torch.cuda.current_stream().wait_stream(se)
            torch.cuda.current_stream().wait_stream(ss)
        tb = timeit(both)
        res[f"ne{ne}"] = {"embed_alone_ms": round(te, 3), "search_alone_ms": round(ts, 3), "both_ms": round(tb, 3)}
        L.lzk_set_cu_budget(0)
        print(json.dumps(res), flush=True)
    out["split"] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
