"""Dump the CPU oracle's carry-in sequence of quadric.scene (scan-order DEP entries) and the
segment table to /tmp for scripts/pred_sim.py.   python3 scripts/pred_dump.py [SIZE]"""
import sys, os, numpy as np
sys.path.insert(0, "tests/tools"); sys.path.insert(0, "tests")
import segment_profile as sp, helpers, ctypes
rc = helpers.load_pkg()
scene = rc.Scene.from_file(os.path.join(helpers.GOLDEN, "scenes", "quadric.scene"))
lib = helpers.oracle_lib()
lib.rco_render_cls.argtypes = lib.rco_render.argtypes + [ctypes.c_void_p]
n=int(sys.argv[1]) if len(sys.argv)>1 else 4096
img = np.empty((n, n, 3), dtype=np.uint8); cin = np.zeros((n, n, 3), dtype=np.float32); cls = np.zeros((n, n), dtype=np.uint8)
st = helpers.RcoStats()
assert lib.rco_render_cls(ctypes.byref(scene.js), n, n, 7, rc.MODES["parity"], img.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st), cin.ctypes.data_as(ctypes.c_void_p), cls.ctypes.data_as(ctypes.c_void_p)) == 0
cls = cls.reshape(-1); cb = cin.reshape(-1,3).view(np.uint32).astype(np.int64)
dep = np.nonzero(cls >= 2)[0]; seg = np.cumsum(cls == 1)[dep]
_, starts, lens = np.unique(seg, return_index=True, return_counts=True)
np.save("/tmp/carries.npy", cb[dep]); np.save("/tmp/segs.npy", np.stack([starts, lens]))
print("saved", len(dep))
