"""Which scan-order carry segments cross a horizontal band boundary (the
dropped two-band lone-frame schedule changed simple 1024^2 d6's md5).  From the CPU oracle's
per-pixel classes: a segment is a run of DEP pixels between first-reflection writers; the
two-band schedule compacted band 0 (the first fifth of the rows) on its own.
  python scripts/band_segments.py"""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import helpers
rc = helpers.load_pkg()
lib = helpers.oracle_lib()
lib.rco_render_cls.argtypes = lib.rco_render.argtypes + [ctypes.c_void_p]
for name, size in [("simple", 1024), ("quadric", 4096), ("reflection", 2048), ("quadric", 2048)]:
    scene = rc.Scene.from_file(os.path.join(helpers.GOLDEN, "scenes", name + ".scene"))
    img = np.empty((size, size, 3), dtype=np.uint8); cin = np.zeros((size, size, 3), np.float32)
    cls = np.zeros((size, size), np.uint8); st = helpers.RcoStats()
    lib.rco_render_cls(ctypes.byref(scene.js), size, size, 7, rc.MODES["parity"], img.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st), cin.ctypes.data_as(ctypes.c_void_p), cls.ctypes.data_as(ctypes.c_void_p))
    c = cls.reshape(-1)
    dep = np.nonzero(c >= 2)[0]
    writers = np.cumsum(c == 1)
    seg = writers[dep]   # segment id = writers before
    # segments: first / last DEP pixel of each
    starts = np.r_[0, np.nonzero(np.diff(seg))[0] + 1]
    ends = np.r_[starts[1:] - 1, len(dep) - 1]
    first_row = dep[starts] // size; last_row = dep[ends] // size
    lens = ends - starts + 1
    for frac in (5,):
        b = size // frac
        cross = np.nonzero((first_row < b) & (last_row >= b))[0]
        print(f"{name} {size}^2: {len(starts)} segments; band boundary row {b}: {len(cross)} segment(s) cross it",
              [(int(lens[k]), int(first_row[k]), int(last_row[k])) for k in cross[:5]],
              "longest:", int(lens.max()), "rows", int(first_row[lens.argmax()]), "-", int(last_row[lens.argmax()]))
