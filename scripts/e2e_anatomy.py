"""Where rc_render's end-to-end time goes beyond the device frame (quadric 4096^2 d6 parity).

For each tuning variant: rc_render into a fresh pageable pixmap (as bench.py's end_to_end leg),
median over reps of the caller's clock, the library's total_ms / kernel_ms / resolve_ms /
d2h_ms (rc_timing), next to rc_render_device's single-frame time on the same box.
Usage: [RC_E2E_TRACE=1] python scripts/e2e_anatomy.py [reps]
"""
import importlib.util
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location(
    "raytracing_programs_amd", os.path.join(ROOT, "raytracing-programs_amd", "__init__.py"))
pkg = importlib.util.module_from_spec(spec)
sys.modules["raytracing_programs_amd"] = pkg
spec.loader.exec_module(pkg)

W = H = 4096
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
scene = pkg.Scene.from_file(os.path.join(ROOT, "tests", "golden", "scenes", "quadric.scene"))
ref = None


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


def lone():
    d = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
    pkg.render_device(scene, W, H, d.data_ptr())
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        pkg.render_device(scene, W, H, d.data_ptr())
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return med(ts) * 1e3


def e2e(label, **tune):
    global ref
    base = pkg.get_tuning(default=True)
    pkg.set_tuning(**tune)
    try:
        pkg.render(scene, W, H)
        ts, fields = [], {}
        for _ in range(reps):
            out = np.empty((H, W, 3), dtype=np.uint8)
            tim = {}
            t0 = time.perf_counter()
            pkg.render(scene, W, H, timing=tim, out=out)
            ts.append(time.perf_counter() - t0)
            for k in ("total_ms", "kernel_ms", "resolve_ms", "d2h_ms"):
                fields.setdefault(k, []).append(tim[k])
            if ref is None:
                ref = out.copy()
            same = bool(np.array_equal(out, ref))
            del out
        row = {k: round(med(v), 3) for k, v in fields.items()}
        print(f"{label:28s} caller {med(ts) * 1e3:7.3f} ms  " +
              "  ".join(f"{k} {v:7.3f}" for k, v in row.items()) + f"  same {same}", flush=True)
    finally:
        pkg.set_tuning(**{k: base[k] for k in tune})


if os.environ.get("E2E_COPY_THREADS"):   # the host pool's size is fixed at its first use
    pkg.set_tuning(copy_threads=int(os.environ["E2E_COPY_THREADS"]))
    print(f"copy_threads {pkg.get_tuning()['copy_threads']}", flush=True)
print(f"lone rc_render_device {lone():.3f} ms", flush=True)
if os.environ.get("RC_E2E_TRACE"):   # host marks of each rep on stderr (rc_api.hip E2eTrace)
    e2e("default (traced)")
    e2e("patch_host=1 (traced)", patch_host=1)
    sys.exit(0)
e2e("default")
e2e("prefault=0", prefault=0)
e2e("patch_host=0", patch_host=0)
e2e("patch_host=1", patch_host=1)
e2e("overlap_d2h=0", overlap_d2h=0)
e2e("default again")
print(f"lone rc_render_device {lone():.3f} ms", flush=True)
