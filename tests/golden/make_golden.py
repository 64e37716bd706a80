#!/usr/bin/env python3
"""Generate the golden fixtures from the reference itself (run in the build container).

Needs oracle/_ref/ (``make -C oracle ref``: the reference C/ sources compiled exactly as
C/Makefile:4, plus MAX_RECURSION depth variants and the break-on-miss "fast" variant of
C/raycast.c:359 — SURVEY.md Appendix B/B2).  Writes:

  tests/golden/md5.json     md5 + size of every golden P3 image, keyed
                            "<scene>:<W>x<H>:d<depth>:<parity|fast>"
  tests/golden/small.npz    the decoded RGB pixmaps of every 64x64 case (uint8 [64,64,3])

Usage: python tests/golden/make_golden.py [--big]   (--big adds C4/C5-sized images)
"""
import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.path.join(ROOT, "oracle", "_ref")
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
OUT = os.path.join(ROOT, "tests", "golden")

SMALL_SCENES = ["simple", "reflection", "quadric", "example2", "example3", "quadric2"]


def cases(big):
    cs = []
    for sc in SMALL_SCENES:
        for n in (64, 256):
            for d in (0, 4, 6):
                for mode in ("parity", "fast"):
                    cs.append((sc, n, n, d, mode))
    # BASELINE.json configs and the extra full-size rows of SURVEY Appendix B/B2
    cs += [("simple", 1024, 1024, 0, "parity"), ("reflection", 2048, 2048, 4, "parity"),
           ("reflection", 2048, 2048, 4, "fast"), ("simple", 1024, 1024, 6, "parity"),
           ("simple", 1024, 1024, 6, "fast"), ("reflection", 2048, 2048, 6, "parity"),
           ("reflection", 2048, 2048, 6, "fast"), ("quadric", 1024, 1024, 6, "parity"),
           ("quadric", 1024, 1024, 6, "fast"), ("quadric", 512, 384, 6, "parity"),
           ("quadric", 333, 517, 6, "parity"), ("reflection", 1, 1, 6, "parity"),
           ("quadric", 7, 3, 6, "parity"), ("quadric", 1, 4096, 6, "parity")]
    if big:
        cs += [("quadric", 4096, 4096, 6, "parity"), ("quadric", 4096, 4096, 6, "fast"),
               ("quadric", 8192, 8192, 6, "parity"), ("quadric", 8192, 8192, 6, "fast")]
    return cs


def key(sc, w, h, d, mode):
    return f"{sc}:{w}x{h}:d{d}:{mode}"


def decode_p3(data):
    toks = data.split()
    assert toks[0] == b"P3"
    w, h, mx = int(toks[1]), int(toks[2]), int(toks[3])
    assert mx == 255
    px = np.array([int(t) for t in toks[4:]], dtype=np.uint8)
    return px.reshape(h, w, 3)


def run(case):
    sc, w, h, d, mode = case
    exe = os.path.join(REF, ("raytrace_fast_d%d" if mode == "fast" else "raytrace_d%d") % d)
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        out = os.path.join(td, "o.ppm")
        subprocess.run([exe, str(w), str(h), os.path.join(SCENES, sc + ".scene"), out],
                       check=True, stdout=subprocess.DEVNULL, cwd=td)
        md5 = hashlib.md5()
        size = 0
        with open(out, "rb") as f:
            while True:
                b = f.read(1 << 24)
                if not b:
                    break
                md5.update(b)
                size += len(b)
        px = None
        if w * h <= 64 * 64:
            with open(out, "rb") as f:
                px = decode_p3(f.read())
        return case, md5.hexdigest(), size, px


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    ap.add_argument("-j", type=int, default=6)
    args = ap.parse_args()
    if not os.path.isdir(REF):
        sys.exit("oracle/_ref missing: run `make -C oracle ref` first")
    md5_path = os.path.join(OUT, "md5.json")
    table = json.load(open(md5_path)) if os.path.exists(md5_path) else {}
    small = {}
    with cf.ThreadPoolExecutor(args.j) as ex:
        for case, md5, size, px in ex.map(run, cases(args.big)):
            table[key(*case)] = {"md5": md5, "size": size}
            if px is not None and case[1] == 64 and case[2] == 64:
                small[key(*case)] = px
            print(key(*case), md5, size, flush=True)
    with open(md5_path, "w") as f:
        json.dump(dict(sorted(table.items())), f, indent=1)
        f.write("\n")
    if small:
        np.savez_compressed(os.path.join(OUT, "small.npz"), **small)


if __name__ == "__main__":
    main()
