"""Host-side checks of two index rules the pixel kernels rely on (rc_kernels.hip), restated in
Python: the XCD-aware tile order must visit every tile exactly once, and the key-writer filter
of phase A must keep every writer carry-out that the compaction (segment keys) or the row
shards (in-row writer before a DEP pixel, a row's last writer) can read."""
import numpy as np
import pytest


def xcd_tile(lin, n, order):
    """rc_kernels.hip xcd_tile(): tile index of linear workgroup id `lin` of `n`."""
    if order == 1:
        xcd, k, q, r = lin & 7, lin >> 3, n >> 3, n & 7
        return xcd * (q + 1) + k if xcd < r else r * (q + 1) + (xcd - r) * q + k
    if order == 2 and lin < (n & ~63):
        xcd, k = lin & 7, lin >> 3
        return ((k >> 3) * 8 + xcd) * 8 + (k & 7)
    return lin


@pytest.mark.parametrize("order", [1, 2])
@pytest.mark.parametrize("w,h", [(4096, 4096), (8192, 8192), (2048, 2048), (1024, 1024),
                                 (333, 517), (160, 120), (1, 1), (17, 33), (4096, 16)])
def test_xcd_tile_order_is_a_bijection(order, w, h):
    nx, ny = (w + 15) // 16, (h + 15) // 16
    n = nx * ny
    t = [xcd_tile(i, n, order) for i in range(n)]
    assert sorted(t) == list(range(n))
    if order == 2 and n >= 64:
        # the 8 tiles of a chunk run on one XCD (workgroup ids congruent mod 8)
        inv = np.empty(n, dtype=np.int64)
        inv[t] = np.arange(n)
        full = (n & ~63) // 8
        for c in range(full):
            assert len({int(inv[c * 8 + j]) % 8 for j in range(8)}) == 1


def writer_may_key(cls_frag, lane):
    """rc_kernels.hip writer_may_key() for lane `lane` (0..7) of an 8-pixel row fragment."""
    nxt = [j for j in range(lane + 1, 8) if cls_frag[j] == 1]
    if not nxt:
        return True
    return any(cls_frag[j] == 2 for j in range(lane + 1, nxt[0]))


@pytest.mark.parametrize("seed", range(6))
def test_key_writer_filter_keeps_every_read_carry(seed):
    rng = np.random.default_rng(seed)
    H, W = 24, int(rng.integers(1, 70))
    # classes: 0 ident, 1 writer, 2 DEP, with runs like a real image
    p = rng.dirichlet([1, 1, 1])
    cls = rng.choice(3, size=(H, W), p=p)
    stored = np.zeros((H, W), dtype=bool)
    for y in range(H):
        for x0 in range(0, W, 8):
            frag = [int(cls[y, x]) if x < W else -1 for x in range(x0, x0 + 8)]
            for l in range(8):
                if x0 + l < W and frag[l] == 1:
                    stored[y, x0 + l] = writer_may_key(frag, l)
    flat = cls.reshape(-1)
    # segment keys: the last writer before each DEP pixel in scan order
    last_w = -1
    for i, c in enumerate(flat):
        if c == 1:
            last_w = i
        elif c == 2 and last_w >= 0:
            assert stored.reshape(-1)[last_w], ("segment key", i, last_w)
    for y in range(H):
        row = cls[y]
        ws = np.nonzero(row == 1)[0]
        if len(ws):   # a row's last writer (k_shard_pack row summaries)
            assert stored[y, ws[-1]]
        lw = -1
        for x in range(W):   # the in-row writer before each DEP pixel (k_shard_pack kw)
            if row[x] == 1:
                lw = x
            elif row[x] == 2 and lw >= 0:
                assert stored[y, lw]
