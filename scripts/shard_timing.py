"""Sharded-path timings on one GPU: rc_render_sharded with G=1 over RCCL and
G=2/4/8 ranks sharing device 0 (RC_XFER_COPY: same kernels and wire records, device copies
instead of xGMI).  Prints one JSON line per case with the root's phase split."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import rc, scene_path  # noqa: E402

s = rc.Scene.from_file(scene_path("quadric"))
# the exchange path at every G (a one-rank group otherwise renders a lone frame)
rc.set_tuning(shard_lone=int(os.environ.get("SHARD_LONE", "0")))
for n in (4096, 8192):
    out = torch.empty((n, n, 3), dtype=torch.uint8, device="cuda")
    for G, tr in ((1, "rccl"), (2, "copy"), (4, "copy"), (8, "copy")):
        g = rc.Group.local([0] * G, tr)
        for mode in ("parity", "fast"):
            g.render(s, n, n, out.data_ptr(), depth=6, mode=mode)
            torch.cuda.synchronize()
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                g.render(s, n, n, out.data_ptr(), depth=6, mode=mode)
            ms = (time.perf_counter() - t0) * 1e3 / reps
            st = g.stats()
            print(json.dumps({"size": n, "G": G, "transport": tr, "mode": mode,
                              "ms": round(ms, 3), "rays_per_s": round(n * n / ms * 1e3, 1),
                              **{k: (round(v, 3) if isinstance(v, float) else v)
                                 for k, v in st.items()}}), flush=True)
        g.close()
    del out
