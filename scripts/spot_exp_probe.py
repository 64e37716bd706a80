"""Spot-light exponents outside the reference scenes (negative integers, non-integers): GPU
against the oracle (glibc pow), mismatching pixels per case.  Diagnostic for DESIGN.md §2."""
import os, sys, tempfile
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import oracle_render, rc, scene_path

base = open(scene_path("reflection")).read().splitlines()
for a0 in (-1, -2, -3, -5, -9, 2.5, 0.3, 7.25):
    for theta in (0.3, 0.9):
        spot = ("light, color: [1.5, 1.2, 1.0], radial-a2: 0.01, radial-a1: 0.0125, "
                f"radial-a0: 0.0125, position: [0, 2, 0], theta: {theta}, angular-a0: {a0}, "
                "direction: [0, -0.3, -1]")
        with tempfile.NamedTemporaryFile("w", suffix=".scene", delete=False) as f:
            f.write("\n".join(base + [spot]) + "\n")
        s = rc.Scene.from_file(f.name)
        for mode, d in (("fast", 4), ("parity", 4)):
            want, st = oracle_render(s, 256, 256, d, mode)
            got = rc.render(s, 256, 256, depth=d, mode=mode)
            bad = int((got != want).any(axis=2).sum())
            print(f"a0={a0} theta={theta} {mode} d{d}: {bad} of 65536 pixels differ, "
                  f"parity_defined={st['parity_defined']}", flush=True)
        os.unlink(f.name)
