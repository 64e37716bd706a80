"""CPU multi-process test (gloo, world_size 2) of the multi-GPU row-shard path used by
bench.py in fast mode: row-cyclic partition -> per-rank row blocks -> all_gather ->
de-interleave.  Each rank "renders" its rows with the CPU oracle (test infrastructure), so the
collective logic is checked against a full-image render without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import oracle_render, rc, scene_path


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, W, H, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = rc.Scene.from_file(scene_path("quadric"))
    full, _ = oracle_render(scene, W, H, 6, "fast")
    row0, step, nrows = rc.row_shard(H, rank, world)
    rows_max = (H + world - 1) // world
    send = torch.zeros((rows_max, W, 3), dtype=torch.uint8)
    send[:nrows] = torch.from_numpy(full[row0::step])   # this rank's rows, as the GPU renders them
    gathered = torch.empty((world, rows_max, W, 3), dtype=torch.uint8)
    rc.gather_rows(send, gathered, dist)
    if rank == 0:
        img = rc.deinterleave(gathered, H).numpy()
        np.save(result_path, img)
        np.save(result_path + ".ref.npy", full)
    dist.destroy_process_group()


@pytest.mark.parametrize("W,H", [(40, 31), (17, 2)])
def test_row_cyclic_gather_world2(tmp_path, W, H):
    world = 2
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, out), nprocs=world, join=True)
    np.testing.assert_array_equal(np.load(out), np.load(out + ".ref.npy"))


def test_row_shard_partition():
    for H in (1, 2, 7, 4096):
        for world in (1, 2, 3, 8):
            rows = []
            for r in range(world):
                row0, step, n = rc.row_shard(H, r, world)
                rows += list(range(row0, H, step))[:n]
                assert n == len(range(row0, H, step))
            assert sorted(rows) == list(range(H))
