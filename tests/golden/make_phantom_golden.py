#!/usr/bin/env python3
"""Golden fixtures for scenes whose phantom record is LIT, made by the
reference itself (oracle/_ref, run in the build container).

Writes tests/golden/scenes/phantom_<kind>.scene (quadric.scene with its point light replaced,
tests/helpers.py PHANTOM_LIT) and tests/golden/phantom_md5.json: md5 + size of the reference's
P3 output keyed "<scene>:<W>x<H>:d<depth>:parity".
Usage: python tests/golden/make_phantom_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import PHANTOM_LIT, phantom_lit_scene  # noqa: E402

SIZES = [(96, 96), (256, 200), (1024, 768)]
DEPTHS = [1, 4, 6]


def main():
    table = {}
    for kind in sorted(PHANTOM_LIT):
        name = "phantom_" + kind.split("-")[0]
        path = phantom_lit_scene(os.path.join(HERE, "scenes", name + ".scene"), kind)
        for w, h in SIZES:
            for d in DEPTHS:
                exe = os.path.join(ROOT, "oracle", "_ref", f"raytrace_d{d}")
                with tempfile.TemporaryDirectory(dir="/tmp") as td:
                    out = os.path.join(td, "o.ppm")
                    subprocess.run([exe, str(w), str(h), path, out], check=True,
                                   stdout=subprocess.DEVNULL, cwd=td)
                    data = open(out, "rb").read()
                table[f"{name}:{w}x{h}:d{d}:parity"] = {"md5": hashlib.md5(data).hexdigest(),
                                                        "bytes": len(data)}
    with open(os.path.join(HERE, "phantom_md5.json"), "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print(len(table), "entries")


if __name__ == "__main__":
    main()
