"""CPU multi-process tests (gloo) of the row-shard protocol that rc_render_sharded runs over RCCL
(raytracing-programs_amd/csrc/rc_shard.hip), with the CPU oracle standing in
for the kernels (test infrastructure).

* fast mode: row-cyclic partition (row y -> rank y % G), every rank's padded row block
  gathered to rank 0 (a gather, as ncclGather does), de-interleaved there;
* parity mode: the carry chain's exchange, record for record as the device runs it —
  phase A on every rank (class, writer carry-outs, colours of the non-DEP pixels), the wire
  records (per DEP entry: image pixel, the last writer before it in its row and that writer's
  carry-out; per row: DEP count, segment starts inside the row, last writer / last DEP /
  first DEP's writer and the last writer's carry-out) and the row blocks gathered to rank 0,
  which rebuilds the image's scan order and segment table from the records alone
  (k_shard_rows / k_row_scan / k_shard_unpack), resolves the chain and shades every DEP entry
  into the de-interleaved image itself (phase C inside the root's resolver); nothing returns
  to the ranks.  Rank 0's own rows never travel (round 4): its phase A keeps its writer
  carry-outs at their image pixels — only the key writers of each 8-pixel tile row
  (k_phase_a writer_may_key) — and its entries are thin {image pixel, in-row writer} pairs whose
  carries the root looks up there; its row block is de-interleaved in place.  The image must
  equal the oracle's whole-image render."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import golden_key, golden_table, oracle_lib, oracle_render, p3_md5, rc, scene_path

IDENT, WRITER = 0, 1   # oracle classes; 2 / 3 = DEP (first reflection missed)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def pixels(scene, W, H, depth, mode, pix, cin=None):
    """Oracle per-pixel shade (rco_pixels): rgb, carry-out, class, zero-normalize events."""
    lib = oracle_lib()
    lib.rco_pixels.argtypes = [ctypes.POINTER(rc.JsonDataT)] + [ctypes.c_int] * 4 + [
        ctypes.c_int64] + [ctypes.c_void_p] * 6
    pix = np.ascontiguousarray(pix, dtype=np.int64)
    n = len(pix)
    rgb = np.zeros((n, 3), np.uint8)
    cout = np.zeros((n, 3), np.float32)
    cls = np.zeros(n, np.uint8)
    z = np.zeros(n, np.int64)
    cin_p = None
    if cin is not None:
        cin = np.ascontiguousarray(cin, dtype=np.float32)
        cin_p = cin.ctypes.data
    assert lib.rco_pixels(ctypes.byref(scene.js), W, H, depth + 1, rc.MODES[mode], n,
                          pix.ctypes.data, cin_p, rgb.ctypes.data, cout.ctypes.data,
                          cls.ctypes.data, z.ctypes.data) == 0
    return rgb, cout, cls, z


def key_writers(cls):
    """k_phase_a writer_may_key over one image row: a writer's carry-out is stored unless a
    later writer of its 8-pixel tile row follows with no DEP pixel between them."""
    W = len(cls)
    keep = np.zeros(W, bool)
    for x0 in range(0, W, 8):
        frag = [int(cls[x]) if x < W else -1 for x in range(x0, x0 + 8)]
        for l in range(8):
            if x0 + l < W and frag[l] == WRITER:
                nxt = [j for j in range(l + 1, 8) if frag[j] == WRITER]
                keep[x0 + l] = not nxt or any(frag[j] >= 2 for j in range(l + 1, nxt[0]))
    return keep


def rank_phase_a(scene, W, H, depth, rank, G):
    """A rank's phase A and wire records (k_phase_a + k_shard_pack).  Rank 0 (thin): entries
    are (image pixel, in-row writer) and its key writers' carry-outs stay in `carry` at their
    image pixels (the root resolver's own buffers)."""
    rows = list(range(rank, H, G))
    local = np.zeros((len(rows), W, 3), np.uint8)
    entries, summaries = [], []
    dep_pix = []
    carry = {}
    zero = 0
    for j, y in enumerate(rows):
        pix = np.arange(W, dtype=np.int64) + y * W
        rgb, cout, cls, z = pixels(scene, W, H, depth, "parity", pix)
        dep = cls >= 2
        local[j][~dep] = rgb[~dep]
        zero += int(z[~dep].sum())
        if rank == 0:
            for x in np.nonzero(key_writers(cls))[0]:
                carry[y * W + int(x)] = cout[x]
        lw = ld = wf = -1
        nst = 0
        first = True
        for x in range(W):
            if dep[x]:
                if first:
                    wf, first = lw, False
                elif lw > ld:
                    nst += 1   # a writer between the previous DEP and this one
                if rank == 0:   # thin: the carry is read at the writer's image pixel
                    entries.append((y * W + x, y * W + lw if lw >= 0 else -1))
                else:
                    kc = cout[lw] if lw >= 0 else np.zeros(3, np.float32)
                    entries.append((y * W + x, y * W + lw if lw >= 0 else -1, kc))
                dep_pix.append((j, x))
                ld = x
            elif cls[x] == WRITER:
                lw = x
        if rank == 0 and lw >= 0:   # the root reads its row-last writer's carry in place
            assert y * W + lw in carry, "a row's last writer is a key writer"
        summaries.append({"ndep": int(dep.sum()), "nstart": nst,
                          "lastw": y * W + lw if lw >= 0 else -1,
                          "lastd": y * W + ld if ld >= 0 else -1,
                          "wfirst": y * W + wf if wf >= 0 else -1,
                          "cw": (carry[y * W + lw] if rank == 0 else cout[lw]) if lw >= 0
                          else np.zeros(3, np.float32)})
    return local, entries, summaries, dep_pix, zero, carry


def root_resolve(scene, W, H, depth, G, entries_all, rows_all, root_carry):
    """Rank 0: the image's scan order from the wire records alone (its own thin entries
    with the carries its phase A kept), the segment table and the exact chain (every DEP
    pixel's carry-in, in each rank's entry order)."""
    row_off, pw, pd = {}, -1, -1
    starts = []          # (global entry index, initial carry)
    order = []           # (rank, local index) in image scan order
    for y in range(H):
        g, j = y % G, y // G
        r = rows_all[g][j]
        loff = sum(rows_all[g][q]["ndep"] for q in range(j))
        prev = pd
        for i in range(r["ndep"]):
            if g == 0:
                pix, kin = entries_all[0][loff + i]
                kc = root_carry[kin] if kin >= 0 else None   # KeyError: a key writer dropped
            else:
                pix, kin, kc = entries_all[g][loff + i]
            kw = kin if kin >= 0 else pw
            if prev < 0 or kw > prev:
                if kin >= 0:
                    c0 = kc
                elif pw >= 0:
                    yw = pw // W
                    c0 = rows_all[yw % G][yw // G]["cw"]
                else:
                    c0 = np.zeros(3, np.float32)
                starts.append((len(order), np.asarray(c0, np.float32)))
            order.append((g, loff + i))
            prev = pix
        if r["lastw"] >= 0:
            pw = r["lastw"]
        if r["lastd"] >= 0:
            pd = r["lastd"]
    cin = [np.zeros((len(e), 3), np.float32) for e in entries_all]
    bounds = [s for s, _ in starts] + [len(order)]
    for k, (s0, c0) in enumerate(starts):
        c = c0
        for idx in range(s0, bounds[k + 1]):   # the chain: one entry at a time
            g, li = order[idx]
            cin[g][li] = c
            _, cout, _, _ = pixels(scene, W, H, depth, "parity",
                                   [entries_all[g][li][0]], c[None, :])
            c = cout[0]
    return cin


def _worker(rank, world, port, name, W, H, depth, mode, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = rc.Scene.from_file(scene_path(name))
    row0, step, nrows = rc.row_shard(H, rank, world)
    rows_max = (H + world - 1) // world
    send = torch.zeros((rows_max, W, 3), dtype=torch.uint8)
    if mode == "fast":
        pix = np.concatenate([np.arange(W) + y * W for y in range(row0, H, step)] or [[]])
        rgb, _, _, z = pixels(scene, W, H, depth, "fast", pix.astype(np.int64))
        send[:nrows] = torch.from_numpy(rgb.reshape(nrows, W, 3))
        zero = int(z.sum())
    else:
        local, entries, summaries, dep_pix, zero, carry = rank_phase_a(scene, W, H, depth, rank,
                                                                       world)
        gathered = [None] * world if rank == 0 else None
        # rank 0's entries stay where they are: it contributes only its row summaries
        dist.gather_object((entries if rank else None, summaries), gathered, dst=0)
        if rank:
            send[:nrows] = torch.from_numpy(local)   # non-DEP pixels final after phase A
    blocks = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send, blocks, dst=0)
    zs = [None] * world if rank == 0 else None
    dist.gather_object(zero, zs, dst=0)
    if rank == 0:
        if mode == "parity":   # the root's own block is de-interleaved in place, never sent
            blocks[0][:nrows] = torch.from_numpy(local)
        img = rc.deinterleave(torch.stack(blocks), H).numpy()
        zero_all = sum(zs)
        if mode == "parity":   # the root: the chain, then phase C of every DEP entry into img
            ents = [entries] + [g[0] for g in gathered[1:]]
            cin = root_resolve(scene, W, H, depth, world, ents, [g[1] for g in gathered], carry)
            for g in range(world):
                if not len(ents[g]):
                    continue
                pix = [e[0] for e in ents[g]]
                rgb, _, _, z = pixels(scene, W, H, depth, "parity", pix, cin[g])
                flat = img.reshape(-1, 3)
                flat[np.asarray(pix)] = rgb
                zero_all += int(z.sum())
        np.save(result_path, img)
        np.save(result_path + ".zero.npy", np.array(zero_all))
    dist.destroy_process_group()


def run_world(tmp_path, world, name, W, H, depth, mode):
    out = str(tmp_path / f"img_{world}_{mode}.npy")
    mp.spawn(_worker, args=(world, _free_port(), name, W, H, depth, mode, out), nprocs=world,
             join=True)
    return np.load(out), int(np.load(out + ".zero.npy"))


@pytest.mark.parametrize("W,H", [(40, 31), (17, 2)])
def test_row_cyclic_gather_world2(tmp_path, W, H):
    scene = rc.Scene.from_file(scene_path("quadric"))
    img, zero = run_world(tmp_path, 2, "quadric", W, H, 6, "fast")
    want, st = oracle_render(scene, W, H, 6, "fast")
    np.testing.assert_array_equal(img, want)
    assert zero == st["zero_normalize"]


@pytest.mark.parametrize("world,name,W,H,depth", [(2, "quadric", 48, 40, 6),
                                                 (3, "reflection", 64, 64, 4),
                                                 (2, "simple", 64, 64, 6),
                                                 (3, "quadric", 23, 2, 6)])
def test_parity_shard_protocol(tmp_path, world, name, W, H, depth):
    """The parity exchange, modelled on CPU: byte-identical to the whole-image oracle (and to
    the reference's md5 where a golden exists)."""
    scene = rc.Scene.from_file(scene_path(name))
    img, zero = run_world(tmp_path, world, name, W, H, depth, "parity")
    want, st = oracle_render(scene, W, H, depth, "parity")
    assert st["dep_pixels"] > 0, "the case must exercise the carry chain"
    np.testing.assert_array_equal(img, want)
    assert zero == st["zero_normalize"]
    key = golden_key(name, W, H, depth, "parity")
    table = golden_table()
    if key in table:
        assert p3_md5(img) == table[key]["md5"]


def test_row_shard_partition():
    for H in (1, 2, 7, 4096):
        for world in (1, 2, 3, 8):
            rows = []
            for r in range(world):
                row0, step, n = rc.row_shard(H, r, world)
                rows += list(range(row0, H, step))[:n]
                assert n == len(range(row0, H, step))
            assert sorted(rows) == list(range(H))
