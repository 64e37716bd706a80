"""rc_render end to end (quadric 4096^2 d6 parity into a fresh pageable pixmap), a few warm
calls 20 ms apart, for a kernel + HIP API trace (rocprofv3 --kernel-trace --hip-trace): how
long the device waits for its first command after the call starts, and what follows the
frame's last kernel.  Prints each call's host start/end (time.monotonic_ns, the trace's clock
on Linux) so scripts/e2e_gaps.py can line them up with the trace.
Usage: python scripts/e2e_trace_run.py [calls]"""
import importlib.util
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location(
    "raytracing_programs_amd", os.path.join(ROOT, "raytracing-programs_amd", "__init__.py"))
pkg = importlib.util.module_from_spec(spec)
sys.modules["raytracing_programs_amd"] = pkg
spec.loader.exec_module(pkg)

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W = H = 4096
scene = pkg.Scene.from_file(os.path.join(ROOT, "tests", "golden", "scenes", "quadric.scene"))
pkg.render(scene, W, H)
pkg.render(scene, W, H)
for i in range(calls):
    out = np.empty((H, W, 3), dtype=np.uint8)
    tim = {}
    t0 = time.monotonic_ns()
    pkg.render(scene, W, H, timing=tim, out=out)
    t1 = time.monotonic_ns()
    print(f"call {i} start_ns {t0} end_ns {t1} ms {(t1 - t0) / 1e6:.3f} lib {tim['total_ms']:.3f} "
          f"kernel {tim['kernel_ms']:.3f}", flush=True)
    del out
    time.sleep(0.02)
