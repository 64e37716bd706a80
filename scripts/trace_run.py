import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import importlib.util
root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
spec = importlib.util.spec_from_file_location("rc", os.path.join(root, "raytracing-programs_amd", "__init__.py"))
rc = importlib.util.module_from_spec(spec); sys.modules["rc"] = rc; spec.loader.exec_module(rc)
sc = rc.Scene.from_file(os.path.join(root, "tests/golden/scenes/quadric.scene"))
if os.environ.get("TUNE"):
    rc.set_tuning(**{k: int(v) for k, v in (f.split("=") for f in os.environ["TUNE"].split(","))})
n = int(os.environ.get("SIZE", "4096"))
for _ in range(3):
    tim = {}
    rc.render(sc, n, n, depth=6, mode="parity", timing=tim)
print("resolve_ms", round(tim["resolve_ms"], 3), "kernel_ms", round(tim["kernel_ms"], 3))
