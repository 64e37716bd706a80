"""The drop-in rate: rc_render (upload + kernels + copy into a fresh pageable pixmap, as
raycast() runs it) at SIZE, median of REPS, md5-checked against the golden table."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import golden_table, p3_md5, rc, scene_path
n = int(os.environ.get("SIZE", "4096"))
scene, d, mode = os.environ.get("SCENE", "quadric"), int(os.environ.get("DEPTH", "6")), os.environ.get("MODE", "parity")
s = rc.Scene.from_file(scene_path(scene))
img = rc.render(s, n, n, depth=d, mode=mode)
key = f"{scene}:{n}x{n}:d{d}:{mode}"
ok = p3_md5(img) == golden_table()[key]["md5"]
ts, tims = [], []
for _ in range(int(os.environ.get("REPS", "7"))):
    tim = {}
    t0 = time.perf_counter()
    rc.render(s, n, n, depth=d, mode=mode, timing=tim)
    ts.append((time.perf_counter() - t0) * 1e3)
    tims.append(tim)
ts.sort()
print(os.environ.get("TAG", key), "md5", ok, "median ms %.3f" % ts[len(ts) // 2], "min %.3f" % ts[0],
      {k: round(v, 3) for k, v in tims[-1].items()}, flush=True)
