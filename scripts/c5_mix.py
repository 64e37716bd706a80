"""Lone 8192^2 parity renders after frames in flight of the same size (bench.py's order)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import torch
from helpers import rc, scene_path
s = rc.Scene.from_file(scene_path("quadric"))
n = int(os.environ.get("SIZE", "8192"))
ref = rc.render(s, n, n, depth=6, mode="parity")
print("lone before: ok", flush=True)
outs = [torch.empty((n, n, 3), dtype=torch.uint8, device="cuda") for _ in range(6)]
torch.cuda.synchronize()
for o in outs:
    rc.frame_submit(s, n, n, o.data_ptr(), depth=6, mode="parity")
rc.frames_wait()
print("in flight:", all(np.array_equal(o.cpu().numpy(), ref) for o in outs), flush=True)
for i in range(3):
    img = rc.render(s, n, n, depth=6, mode="parity")
    print("lone after", i, np.array_equal(img, ref), flush=True)
