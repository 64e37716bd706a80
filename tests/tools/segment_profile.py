#!/usr/bin/env python3
"""Carry-chain profile of a parity render, from the CPU oracle (test tooling, not a test).

For every DEP pixel (first reflection missed, reads the stale carry) in scan
order: its segment (runs between pixels whose first reflection hit) and whether it is a
changer (its output carry differs bitwise from its input).  Writes an .npz with the DEP
sequence and prints the segment/changer summary the resolver is tuned against.

  python tests/tools/segment_profile.py [--size 4096] [--scene quadric] [--out prof.npz]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import helpers  # noqa: E402


def profile(scene_name, size, depth):
    rc = helpers.load_pkg()
    scene = rc.Scene.from_file(os.path.join(helpers.GOLDEN, "scenes", scene_name + ".scene"))
    lib = helpers.oracle_lib()
    lib.rco_render_cls.argtypes = lib.rco_render.argtypes + [ctypes.c_void_p]
    img = np.empty((size, size, 3), dtype=np.uint8)
    cin = np.zeros((size, size, 3), dtype=np.float32)
    cls = np.zeros((size, size), dtype=np.uint8)
    st = helpers.RcoStats()
    r = lib.rco_render_cls(ctypes.byref(scene.js), size, size, depth + 1, rc.MODES["parity"],
                           img.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st),
                           cin.ctypes.data_as(ctypes.c_void_p),
                           cls.ctypes.data_as(ctypes.c_void_p))
    assert r == 0
    cls = cls.reshape(-1)
    cinb = cin.reshape(-1, 3).view(np.uint32)
    dep = np.nonzero(cls >= 2)[0]
    # segment id of each DEP pixel: number of first-reflection writers before it
    writers = np.cumsum(cls == 1)
    seg = writers[dep]
    # changer: the next DEP pixel of the same segment reads a different carry
    same_seg = np.zeros(len(dep), dtype=bool)
    same_seg[:-1] = seg[1:] == seg[:-1]
    diff = np.zeros(len(dep), dtype=bool)
    diff[:-1] = np.any(cinb[dep[1:]] != cinb[dep[:-1]], axis=1)
    changer = same_seg & diff
    return dep, seg, changer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--scene", default="quadric")
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dep, seg, changer = profile(a.scene, a.size, a.depth)
    _, starts, lens = np.unique(seg, return_index=True, return_counts=True)
    order = np.argsort(-lens)
    print(f"dep pixels {len(dep)}, changers {int(changer.sum())}, segments {len(lens)}")
    for i in order[:10]:
        s, n = starts[i], lens[i]
        ch = np.nonzero(changer[s:s + n])[0]
        gaps = np.diff(ch) if len(ch) > 1 else np.array([0])
        print(f"  segment at {s}: {n} entries, {len(ch)} changers, gap median "
              f"{int(np.median(gaps))} p90 {int(np.percentile(gaps, 90))} max {int(gaps.max())}")
    if a.out:
        np.savez_compressed(a.out, dep=dep, seg=seg, changer=changer)


if __name__ == "__main__":
    main()
