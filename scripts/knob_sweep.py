import json, os, sys, torch
sys.path.insert(0, "tests")
from helpers import golden_table, p3_md5, rc, scene_path
s = rc.Scene.from_file(scene_path("quadric"))
n = int(os.environ.get("SIZE", "4096"))
out = torch.empty((n, n, 3), dtype=torch.uint8, device="cuda")
base = rc.get_tuning()
import ast
cfgs = json.loads(os.environ["CFGS"]) if os.environ.get("CFGS") else [
    {}, dict(resolve_k=2), dict(resolve_k=3), dict(wave_k=1), dict(wave_k=3), dict(wave_k=4),
    dict(long_len=16384), dict(long_len=65536), dict(team_blocks=96), dict(team_blocks=160), {}]
for cfg in cfgs:
    rc.set_tuning(**dict(base, **cfg))
    for _ in range(2):
        rc.render_device(s, n, n, out.data_ptr(), depth=6, mode="parity")
    torch.cuda.synchronize()
    rc.profile_begin()
    for _ in range(5):
        rc.render_device(s, n, n, out.data_ptr(), depth=6, mode="parity")
    torch.cuda.synchronize()
    ph = rc.profile_end()
    ok = p3_md5(out.cpu().numpy()) == golden_table()[f"quadric:{n}x{n}:d6:parity"]["md5"]
    print(n, cfg, {k: round(v, 3) for k, v in ph.items() if k.endswith("_ms") and v}, "md5", ok, flush=True)
