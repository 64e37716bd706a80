"""Early-team lone frames (rc_tuning.early_team): md5 of repeated lone renders (the first one
sets the band hint) against the reference's goldens, and forced bands (band_rows) that cut a
long segment or sit anywhere.  Measurement tooling; the GPU tests cover the same cases."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch
from helpers import golden_table, p3_md5, rc, scene_path
tab = golden_table()
cases = [("quadric", 4096, 6), ("simple", 1024, 6), ("reflection", 2048, 4), ("quadric", 1024, 6),
         ("quadric", 8192, 6), ("quadric", 333, 6)]
ok = True
for forced in (0, 204, 100, 1500):
    for name, n, d in cases:
        if forced and name == "quadric" and n in (8192, 333):
            continue
        key = f"{name}:{n}x{n}:d{d}:parity"
        if key not in tab:
            key = None
        s = rc.Scene.from_file(scene_path(name))
        out = torch.empty((n, n, 3), dtype=torch.uint8, device="cuda")
        res = []
        with rc.tuned(early_team=1, band_rows=forced):
            for i in range(3):
                torch.cuda.synchronize()
                t = time.perf_counter()
                rc.render_device(s, n, n, out.data_ptr(), depth=d, mode="parity")
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t) * 1e3
                m = p3_md5(out.cpu().numpy())
                good = key is None or m == tab[key]["md5"]
                ok &= good
                res.append(f"{ms:.2f}ms {'ok' if good else 'MISMATCH'}")
        chk = rc.lone_frames_check()
        print(f"forced {forced:5d} {name}:{n} d{d}: " + ", ".join(res), chk, flush=True)
print("ALL OK" if ok else "FAILURES")
sys.exit(0 if ok else 1)
