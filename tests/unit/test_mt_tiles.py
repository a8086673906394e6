"""Tile table of the cross-tenant global search (ops/search.py MtTiles,
csrc/kernels/mtscan.hip): every tenant's rows are covered by 256-row tiles
exactly once, addresses step by the bf16 row stride, and the threshold
sample is every 64th row of every tile."""
import numpy as np
import torch


def test_tile_table_covers_every_row_once():
    from lazzaro_amd.ops.search import MT_STRIDE, MT_TILE, MtTiles
    slots = np.array([3, 0, 7, 5, 9], np.int64)
    nrows = np.array([1, 256, 257, 800, 0], np.int64)
    e16 = np.array([1 << 20, 2 << 20, 3 << 20, 4 << 20, 5 << 20], np.int64)
    bias = e16 + 7
    ld = 832
    t = MtTiles(slots, nrows, e16, bias, ld, "cpu")
    assert t.n_tiles == 1 + 1 + 2 + 4 and t.rows == int(nrows.sum())
    seen = {}
    for i in range(t.n_tiles):
        s, r0, n = int(t.slot[i]), int(t.row0[i]), int(t.n[i])
        assert 1 <= n <= MT_TILE and r0 % MT_TILE == 0
        j = int(np.nonzero(slots == s)[0][0])
        assert int(t.x[i]) == e16[j] + r0 * ld * 2 and int(t.b[i]) == bias[j] + r0 * 4
        for r in range(r0, r0 + n):
            assert (s, r) not in seen
            seen[(s, r)] = i
    assert len(seen) == int(nrows.sum())
    want = sum(-(-int(t.n[i]) // MT_STRIDE) for i in range(t.n_tiles))
    assert t.n_sample == want
    for ti, r in zip(t.s_tile.tolist(), t.s_row.tolist()):
        assert r % MT_STRIDE == 0 and r < int(t.n[ti])
