"""rc_render's mapped-patch scatter (patch_host 2) against the device-patch path (patch_host 0)
on the same frames, in the order tests/test_gpu.py::test_parity_schedules renders them; prints
the differing pixels of each frame (count, first few, whether they are DEP pixels' phase-A
bytes).  Usage: python scripts/scatter_check.py [tuning=value ...]"""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location(
    "raytracing_programs_amd", os.path.join(ROOT, "raytracing-programs_amd", "__init__.py"))
pkg = importlib.util.module_from_spec(spec)
sys.modules["raytracing_programs_amd"] = pkg
spec.loader.exec_module(pkg)

tune = {k: int(v) for k, v in (a.split("=") for a in sys.argv[1:])}
scenes = {n: pkg.Scene.from_file(os.path.join(ROOT, "tests", "golden", "scenes", n + ".scene"))
          for n in ("quadric", "reflection")}
frames = [("quadric", 4096, 4096, 6), ("reflection", 2048, 2048, 4), ("quadric", 333, 517, 6)] * 3
want = {}
with pkg.tuned(patch_host=0, **tune):
    for f in frames[:3]:
        want[f] = pkg.render(scenes[f[0]], f[1], f[2], depth=f[3])
bad = 0
with pkg.tuned(**tune):
    for i, f in enumerate(frames):
        tim = {}
        img = pkg.render(scenes[f[0]], f[1], f[2], depth=f[3], timing=tim)
        d = np.argwhere(np.any(img != want[f], axis=2))
        bad += len(d)
        print(f"frame {i} {f}: dep {tim['dep_pixels']} differing {len(d)}"
              + ("" if not len(d) else f" first {d[:4].tolist()} got {img[tuple(d[0])].tolist()} "
                 f"want {want[f][tuple(d[0])].tolist()}"), flush=True)
sys.exit(1 if bad else 0)
