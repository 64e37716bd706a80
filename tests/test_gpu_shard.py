"""GPU tests of the row-sharded path (rc_group / rc_render_sharded) through the
C-ABI: rows dealt cyclically over G ranks, the root gathers the row blocks; in parity mode the
root also gathers every rank's DEP entries (with their primary shades), resolves the scan-order
carry chain and shades every DEP entry into its image (phase C inside its resolver).  Every
image must be byte-identical to the reference's (golden md5) or to the CPU oracle.

The box has one GPU, so G > 1 runs as G ranks on device 0 with device copies between their
buffers (RC_XFER_COPY: the same kernels, wire records and exchange order as RCCL); the RCCL
transport itself runs with one rank (ncclGather / group calls with a single communicator),
both from one process (ncclCommInitAll) and as a rank of a multi-process job
(ncclCommInitRank)."""
import json
import os

import numpy as np
import pytest

from helpers import GOLDEN, golden_key, golden_table, oracle_render, p3_md5, rc, scene_path

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SMALL = ["simple", "reflection", "quadric", "example2", "example3", "quadric2"]


@pytest.fixture(scope="module")
def table():
    return golden_table()


@pytest.fixture(scope="module")
def scenes():
    return {n: rc.Scene.from_file(scene_path(n)) for n in SMALL + ["phantom_four", "phantom_two"]}


_groups = {}


def group(devices, transport):
    key = (tuple(devices), transport)
    if key not in _groups:
        _groups[key] = rc.Group.local(devices, transport)
    return _groups[key]


def sharded(g, scene, w, h, depth, mode, timing=None):
    out = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    g.render(scene, w, h, out.data_ptr(), depth=depth, mode=mode, timing=timing)
    return out.cpu().numpy()


@pytest.mark.parametrize("G", [1, 2, 3, 8])
@pytest.mark.parametrize("mode", ["parity", "fast"])
def test_sharded_small_goldens(G, mode, scenes, table):
    g = group([0] * G, "copy")
    assert g.size == G and g.transport == "copy"
    for name in SMALL:
        for d in (0, 4, 6):
            img = sharded(g, scenes[name], 256, 256, d, mode)
            key = golden_key(name, 256, 256, d, mode)
            assert p3_md5(img) == table[key]["md5"], f"{key} G={G}"


@pytest.mark.parametrize("key", ["quadric:4096x4096:d6:parity", "quadric:4096x4096:d6:fast",
                                 "reflection:2048x2048:d4:parity", "simple:1024x1024:d0:parity",
                                 "quadric:333x517:d6:parity", "quadric:1x4096:d6:parity"])
@pytest.mark.parametrize("G", [2, 8])
def test_sharded_configs(key, G, scenes, table):
    name, size, d, mode = key.split(":")
    w, h = map(int, size.split("x"))
    t = {}
    img = sharded(group([0] * G, "copy"), scenes[name], w, h, int(d[1:]), mode, t)
    assert p3_md5(img) == table[key]["md5"], f"{key} G={G}"
    if mode == "parity" and int(d[1:]) > 0:
        assert t["dep_pixels"] == table[key].get("dep_pixels", t["dep_pixels"])


def test_c5_eight_ranks(scenes, table):
    """BASELINE C5 as configured — quadric 8192^2 depth 6 over 8 row-sharded ranks (here on
    one GPU, device copies for the transfers) — md5-equal to the reference in both modes."""
    g8 = group([0] * 8, "copy")
    for mode in ("parity", "fast"):
        key = f"quadric:8192x8192:d6:{mode}"
        t = {}
        assert p3_md5(sharded(g8, scenes["quadric"], 8192, 8192, 6, mode, t)) == table[key]["md5"]
        if mode == "parity":
            assert t["dep_pixels"] == 11211976


def test_sharded_ragged_vs_oracle(scenes):
    """Images with fewer rows than ranks, single columns and odd sizes, against the oracle."""
    g5 = group([0] * 5, "copy")
    for name, w, h, d in [("quadric", 37, 29, 6), ("quadric", 50, 2, 6), ("reflection", 1, 41, 4),
                          ("simple", 3, 1, 6), ("quadric2", 64, 63, 6)]:
        for mode in ("parity", "fast"):
            want, st = oracle_render(scenes[name], w, h, d, mode)
            t = {}
            got = sharded(g5, scenes[name], w, h, d, mode, t)
            np.testing.assert_array_equal(got, want, err_msg=f"{name} {w}x{h} d{d} {mode}")
            assert t["zero_normalize"] == st["zero_normalize"]
            if mode == "parity" and d > 0:
                assert t["dep_pixels"] == st["dep_pixels"]


def test_sharded_phantom_lit(scenes):
    """Lit phantom (dep_fast off: phase C recomputes the whole pixel on its rank, from the
    image row of the rank-local pixel) against the reference's md5s."""
    tab = json.load(open(os.path.join(GOLDEN, "phantom_md5.json")))
    g3 = group([0] * 3, "copy")
    for key, want in sorted(tab.items()):
        name, size, d, mode = key.split(":")
        w, h = map(int, size.split("x"))
        assert p3_md5(sharded(g3, scenes[name], w, h, int(d[1:]), mode)) == want["md5"], key


@pytest.mark.parametrize("mode", ["parity", "fast"])
def test_sharded_rccl_one_rank(mode, scenes, table):
    """The RCCL transport: one communicator from ncclCommInitAll, and one rank of a
    multi-process job from ncclCommInitRank with a fresh unique id."""
    key = golden_key("quadric", 256, 256, 6, mode)
    g = group([0], "rccl")
    assert g.transport == "rccl"
    assert p3_md5(sharded(g, scenes["quadric"], 256, 256, 6, mode)) == table[key]["md5"]
    gr = rc.Group.rank(1, 0, rc.Group.unique_id(), 0)
    try:
        assert p3_md5(sharded(gr, scenes["quadric"], 256, 256, 6, mode)) == table[key]["md5"]
        big = "quadric:4096x4096:d6:" + mode
        assert p3_md5(sharded(gr, scenes["quadric"], 4096, 4096, 6, mode)) == table[big]["md5"]
        st = gr.stats()
        assert st["ranks"] == 1 and st["image_bytes"] == 4096 * 4096 * 3
    finally:
        gr.close()


@pytest.mark.parametrize("mode", ["parity", "fast"])
def test_sharded_rccl_one_rank_exchange(mode, scenes, table):
    """One-rank RCCL groups through the sharded exchange instead of the lone-frame bypass
    (rc_tuning.shard_lone = 0), on both group kinds: the row-block ncclGather, and in parity the
    exact-size exchange of a new key and the fixed-size one of repeated frames (both
    ncclSend/ncclRecv; the fixed-size one with padded per-rank blocks), the ncclAllReduce of the
    entry counts that bounds the next frame, and an overflowed bound (rendered again exactly).
    Every image md5-equal to the reference."""
    key = "quadric:1024x1024:d6:" + mode
    want = table[key]["md5"]
    with rc.tuned(shard_lone=0):
        gr = rc.Group.rank(1, 0, rc.Group.unique_id(), 0)
        try:
            for g in (group([0], "rccl"), gr):
                for i in range(3):   # exact (new key), then fixed twice
                    assert p3_md5(sharded(g, scenes["quadric"], 1024, 1024, 6, mode)) == want, i
                st = g.stats()
                assert st["ranks"] == 1
                if mode == "parity":
                    assert st["dep_pixels"] == table[key].get("dep_pixels", st["dep_pixels"])
                    assert st["resolve_ms"] > 0.0
                    g.debug_bound(16)   # the next frame's lists overflow the padded blocks
                    assert p3_md5(sharded(g, scenes["quadric"], 1024, 1024, 6, mode)) == want
                    assert p3_md5(sharded(g, scenes["quadric"], 1024, 1024, 6, mode)) == want
                    g.debug_bound(1 << 40)   # far above any count: clamped to the rank's pixels
                    assert p3_md5(sharded(g, scenes["quadric"], 1024, 1024, 6, mode)) == want
                    g.debug_bound(-1)
        finally:
            gr.close()


def test_sharded_repeat_and_stats(scenes, table):
    """Back-to-back sharded frames reuse every buffer (carry-in tags advance per frame); the
    exchange volumes follow the wire format (80 B per DEP entry of the other ranks in — the
    root's own entries are read in place — and nothing back: phase C runs on the root); every
    rank's own timeline is recorded (rc_group_rank_stats)."""
    key = "quadric:4096x4096:d6:parity"
    g4 = group([0] * 4, "copy")
    for _ in range(3):
        assert p3_md5(sharded(g4, scenes["quadric"], 4096, 4096, 6, "parity")) == table[key]["md5"]
    st = g4.stats()
    assert st["ranks"] == 4 and st["dep_pixels"] == 2804464
    ranks = [g4.rank_stats(r) for r in range(4)]
    assert st["entry_bytes"] == 80 * (st["dep_pixels"] - ranks[0]["dep_pixels"])
    assert st["carry_bytes"] == 0
    assert st["resolve_ms"] > 0.0 and st["device_ms"] >= st["resolve_ms"]
    assert [q["rank"] for q in ranks] == [0, 1, 2, 3] and sum(q["rows"] for q in ranks) == 4096
    assert sum(q["dep_pixels"] for q in ranks) == st["dep_pixels"]
    assert all(q["local_ms"] > 0.0 and q["total_ms"] >= q["local_ms"] for q in ranks)
    assert g4.rank_stats(4) is None


@pytest.mark.parametrize("G", [2, 5])
def test_sharded_cuda_mode(G, scenes):
    """RC_MODE_CUDA through the row-sharded path (pixel-parallel like fast mode) against its CPU
    restatement (oracle/rc_oracle_cuda.c)."""
    from helpers import oracle_render_cuda
    g = group([0] * G, "copy")
    for name in ("reflection", "quadric2"):
        for d in (6, 50):
            np.testing.assert_array_equal(sharded(g, scenes[name], 160, 97, d, "cuda"),
                                          oracle_render_cuda(scenes[name], 160, 97, d),
                                          err_msg=f"{name} d{d} G{G}")


@pytest.mark.parametrize("G", [1, 3, 8])
def test_sharded_fixed_exchange(G, scenes, table):
    """Repeated frames of one scene and size exchange the DEP entries in fixed-size per-rank
    blocks (no host synchronisation inside the frame, the bound from the previous frame); a
    frame whose entries overflow the bound is rendered again with exact sizes.  Every image
    md5-equal, for the exact, the fixed and the overflowed-then-exact frames."""
    g = group([0] * G, "copy")
    key = "quadric:1024x1024:d6:parity"
    want = table[key]["md5"]
    for i in range(3):   # exact (new key), then fixed twice
        assert p3_md5(sharded(g, scenes["quadric"], 1024, 1024, 6, "parity")) == want, i
    g.debug_bound(16)    # far below the real count: the next frame overflows, then renders exact
    assert p3_md5(sharded(g, scenes["quadric"], 1024, 1024, 6, "parity")) == want, "overflow"
    assert p3_md5(sharded(g, scenes["quadric"], 1024, 1024, 6, "parity")) == want, "after"
    g.debug_bound(-1)


@pytest.mark.parametrize("mode", ["parity", "fast"])
@pytest.mark.parametrize("G", [2, 8])
def test_render_num_gpus_shared_device(G, mode, scenes, table):
    """The drop-in's multi-GPU entry — rc_render (raycast()'s path, RAYCAST_GPUS) with num_gpus
    > 1 — through its cached local group, here with every rank on device 0
    (rc_tuning.share_device: device copies between the ranks) at C4, md5 vs the reference."""
    key = "quadric:4096x4096:d6:" + mode
    with rc.tuned(share_device=1):
        for _ in range(2):   # the group is built once, then reused
            t = {}
            img = rc.render(scenes["quadric"], 4096, 4096, depth=6, mode=mode, gpus=G, timing=t)
            assert p3_md5(img) == table[key]["md5"], f"G={G}"
            if mode == "parity":
                assert t["dep_pixels"] == 2804464


def test_render_num_gpus_clamped_warns(table):
    """More GPUs than the box has (one here, unless the box is bigger): rc_render renders on
    the devices there are and says so on stderr, md5 unchanged.  The warning is printed once
    per process, so the check runs in a fresh process (an earlier clamp in the test
    process would otherwise have used it up)."""
    import subprocess
    import sys
    tests = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import torch\n"
            "from helpers import p3_md5, rc, scene_path\n"
            "n = torch.cuda.device_count()\n"
            "s = rc.Scene.from_file(scene_path('quadric'))\n"
            "img = rc.render(s, 256, 256, depth=6, gpus=n + 3)\n"
            "print('RESULT', p3_md5(img), n, flush=True)\n" % tests)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    _, md5, n = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][-1].split()
    assert md5 == table["quadric:256x256:d6:parity"]["md5"]
    assert f"{int(n) + 3} GPUs requested" in r.stderr and f"rendering on {n}" in r.stderr, r.stderr
