"""Host reads of a pinned result tensor: tolist() straight from the pinned
buffer a device copy landed in vs from a pageable copy of it."""
import json
import time

import torch


def t(fn, n=50):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e3, 4)


def main():
    dev = torch.device("cuda", 0)
    rows = torch.randint(0, 10_000_000, (1024, 10), device=dev)
    host = torch.empty(rows.shape, dtype=rows.dtype, pin_memory=True)
    host.copy_(rows, non_blocking=True)
    torch.cuda.synchronize()
    page = host.clone()
    out = {"pinned_tolist_ms": t(lambda: host.tolist()), "pageable_tolist_ms": t(lambda: page.tolist()),
           "pinned_clone_then_tolist_ms": t(lambda: host.clone().tolist()),
           "pinned_numpy_copy_tolist_ms": t(lambda: host.numpy().copy().tolist()),
           "pinned_clone_ms": t(lambda: host.clone())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
