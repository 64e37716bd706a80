"""Per-phase times of single renders (rc_render_device) under the current environment."""
import os, sys, json, importlib.util
root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
spec = importlib.util.spec_from_file_location("rc", os.path.join(root, "raytracing-programs_amd", "__init__.py"))
rc = importlib.util.module_from_spec(spec); sys.modules["rc"] = rc; spec.loader.exec_module(rc)
import torch
scene = sys.argv[1] if len(sys.argv) > 1 else "quadric"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
d = int(sys.argv[3]) if len(sys.argv) > 3 else 6
sc = rc.Scene.from_file(os.path.join(root, "tests/golden/scenes", scene + ".scene"))
out = torch.empty((n, n, 3), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    rc.render_device(sc, n, n, out.data_ptr(), st, depth=d)
torch.cuda.synchronize()
rc.profile_begin()
for _ in range(10):
    rc.render_device(sc, n, n, out.data_ptr(), st, depth=d)
torch.cuda.synchronize()
ph = rc.profile_end()
print(json.dumps({k: round(v, 4) for k, v in ph.items() if isinstance(v, float)}))
