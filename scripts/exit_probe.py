"""Exit-time heap-abort bisection: one scenario per process (argv[1]); exit status tells."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import oracle_render, random_scene, rc, scene_path  # noqa: E402

what = sys.argv[1]
if what.startswith("shapes"):
    n = int(what.split(":")[1])
    mode = what.split(":")[2]
    rng = np.random.default_rng(1000 + n)
    path = f"/tmp/probe_m{n}.scene"
    random_scene(rng, path, n, 2)
    s = rc.Scene.from_file(path)
    if len(sys.argv) > 2:
        rc.set_tuning(**{k: int(v) for k, v in (a.split("=") for a in sys.argv[2:])})
    for d in (1, 4, 6):
        img = rc.render(s, 96, 72, depth=d, mode=mode)
elif what == "oracle":
    s = rc.Scene.from_file(scene_path("quadric"))
    oracle_render(s, 96, 72, 6, "parity")
elif what == "phantom":
    s = rc.Scene.from_file(scene_path("phantom_four"))
    rc.render(s, 200, 150, depth=6, mode="parity")
print("done", what, flush=True)
