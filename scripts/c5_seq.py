"""bench.py's parity sequence at one size: lone rc_render_device frames, then frames in flight,
then lone rc_render frames, each image checked against the golden md5."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

from helpers import golden_table, p3_md5, rc, scene_path  # noqa: E402

n = int(os.environ.get("SIZE", "8192"))
frames = int(os.environ.get("FRAMES", "43"))
want = golden_table()[f"quadric:{n}x{n}:d6:parity"]["md5"]
s = rc.Scene.from_file(scene_path("quadric"))
out = torch.empty((n, n, 3), dtype=torch.uint8, device="cuda")
for i in range(7):
    rc.render_device(s, n, n, out.data_ptr(), depth=6, mode="parity")
torch.cuda.synchronize()
print("lone device frames:", p3_md5(out.cpu().numpy()) == want, flush=True)
outs = [torch.empty((n, n, 3), dtype=torch.uint8, device="cuda") for _ in range(4)]
torch.cuda.synchronize()
for i in range(frames):
    rc.frame_submit(s, n, n, outs[i % 4].data_ptr(), depth=6, mode="parity")
rc.frames_wait()
print("in flight:", all(p3_md5(o.cpu().numpy()) == want for o in outs), flush=True)
for i in range(3):
    t0 = time.perf_counter()
    tim = {}
    img = rc.render(s, n, n, depth=6, mode="parity", timing=tim)
    print("lone rc_render", i, p3_md5(img) == want, f"{(time.perf_counter() - t0) * 1e3:.1f} ms",
          tim, flush=True)
