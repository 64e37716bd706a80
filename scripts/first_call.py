# First-call latency: a fresh process's first lone frames (the raycast() situation).
import json, os, sys, time
sys.path.insert(0, "tests")
import torch
from helpers import golden_table, p3_md5, rc, scene_path
s = rc.Scene.from_file(scene_path("quadric"))
n = 4096
out = torch.empty((n, n, 3), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
for i in range(4):
    t = {}
    rc.render_device(s, n, n, out.data_ptr(), depth=6, mode="parity", timing=t)
    print("call", i, "kernel_ms", round(t["kernel_ms"], 3), "resolve_ms", round(t["resolve_ms"], 3), flush=True)
print("md5", p3_md5(out.cpu().numpy()) == golden_table()["quadric:4096x4096:d6:parity"]["md5"])
img = rc.render(s, n, n, depth=6, mode="parity", timing=t)
print("rc_render after: total_ms", round(t["total_ms"], 3))
