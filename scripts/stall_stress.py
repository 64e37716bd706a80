"""Repeated lone parity frames (rc_render_device, quadric 4096^2 d6) under a tuning, to
estimate how often a resolver hand-off times out (the frame then fails loudly).  Stops at the
first failure of each schedule.  With RC_STRESS_FLIGHT=1 the frames go in flight instead
(rc_frame_submit into 8 rotating buffers, rc_frames_wait every 40 frames; the last 8 frames'
bytes checked against the first frame's).
SCENE / SIZE / DEPTH pick another configuration (default quadric 4096 6); RC_STRESS_HOST=1
renders through rc_render (whose failure report includes the resolver's state).
Usage: [RC_STRESS_FLIGHT=1] python scripts/stall_stress.py FRAMES [name:k=v,k=v ...]"""
import importlib.util
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location(
    "raytracing_programs_amd", os.path.join(ROOT, "raytracing-programs_amd", "__init__.py"))
pkg = importlib.util.module_from_spec(spec)
sys.modules["raytracing_programs_amd"] = pkg
spec.loader.exec_module(pkg)

frames = int(sys.argv[1])
scheds = []
for a in sys.argv[2:] or ["default:"]:
    name, _, kv = a.partition(":")
    scheds.append((name, {k: int(v) for k, v in (p.split("=") for p in kv.split(",") if p)}))
scene = pkg.Scene.from_file(os.path.join(ROOT, "tests", "golden", "scenes",
                                        os.environ.get("SCENE", "quadric") + ".scene"))
W = H = int(os.environ.get("SIZE", "4096"))
D = int(os.environ.get("DEPTH", "6"))
out = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
flight = os.environ.get("RC_STRESS_FLIGHT") == "1"
bufs = [torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0") for _ in range(8 if flight else 0)]
for name, tune in scheds:
    t0 = time.time()
    done = 0
    with pkg.tuned(**tune):
        for i in range(frames):
            try:
                if flight:
                    pkg.frame_submit(scene, W, H, bufs[i % 8].data_ptr(), depth=D)
                    if i % 40 == 39 or i == frames - 1:
                        pkg.frames_wait()
                        if i == frames - 1:
                            ref = bufs[0]
                            same = sum(1 for b in bufs if torch.equal(b, ref))
                            if same != len(bufs):
                                raise RuntimeError(f"only {same} of {len(bufs)} buffers equal")
                elif os.environ.get("RC_STRESS_HOST") == "1":   # rc_render: a failure's details on stderr
                    pkg.render(scene, W, H, depth=D)
                else:
                    pkg.render_device(scene, W, H, out.data_ptr(), depth=D)
                    torch.cuda.synchronize()
                    if pkg.lone_frames_check()["failed"]:
                        raise RuntimeError("lone_frames_check reports a failed frame")
            except RuntimeError as e:
                print(f"{name}: FAILED at frame {i} after {time.time() - t0:.1f} s: {e}", flush=True)
                if flight:
                    try:
                        pkg.pipe_reset()
                    except RuntimeError:
                        pass
                break
            done += 1
            if i % 100 == 99:
                print(f"{name}: {i + 1} frames ok ({time.time() - t0:.1f} s)", flush=True)
        if flight:
            pkg.pipe_reset()   # the next schedule's pipeline is built from its own tuning
    print(f"{name} {tune}: {done}/{frames} frames ok", flush=True)
