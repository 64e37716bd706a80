"""Lone parity frames (rc_render_device, the raycast() path) at SIZE: per-phase times."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch
from helpers import golden_table, p3_md5, rc, scene_path
n = int(os.environ.get("SIZE", "4096"))
D = int(os.environ.get("DEPTH", "6"))
s = rc.Scene.from_file(scene_path(os.environ.get("SCENE", "quadric")))
if os.environ.get("HELPERS"):   # schedule experiment (rc_set_tuning)
    rc.set_tuning(helpers=int(os.environ["HELPERS"]))
if os.environ.get("TUNE"):      # TUNE="field=v,field=v"
    rc.set_tuning(**{k: int(v) for k, v in (f.split("=") for f in os.environ["TUNE"].split(","))})
out = torch.empty((n, n, 3), dtype=torch.uint8, device="cuda")
for _ in range(2):
    rc.render_device(s, n, n, out.data_ptr(), depth=D, mode="parity")
torch.cuda.synchronize()
rc.profile_begin()
for _ in range(int(os.environ.get("REPS", "5"))):
    rc.render_device(s, n, n, out.data_ptr(), depth=D, mode="parity")
torch.cuda.synchronize()
ph = rc.profile_end()
key = f"{os.environ.get('SCENE', 'quadric')}:{n}x{n}:d{D}:parity"
ok = p3_md5(out.cpu().numpy()) == golden_table()[key]["md5"] if os.environ.get("CHECK") else None
print(os.environ.get("TAG", ""), json.dumps({k: round(v, 3) for k, v in ph.items()}), "md5", ok,
      flush=True)
