#!/bin/bash
# Repeated lone 8192^2 parity renders against the golden md5 (hand-off / helper races).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
python - <<'PY'
import sys, os
sys.path.insert(0, "tests")
from helpers import rc, scene_path, p3_md5, golden_table
t = golden_table()
s = rc.Scene.from_file(scene_path("quadric"))
import numpy as np
first = rc.render(s, 8192, 8192, depth=6, mode="parity")
assert p3_md5(first) == t["quadric:8192x8192:d6:parity"]["md5"]
print("0 ok", flush=True)
for i in range(1, int(os.environ.get("N", "4"))):
    img = rc.render(s, 8192, 8192, depth=6, mode="parity")
    ok = np.array_equal(img, first)
    print(i, "ok" if ok else "MISMATCH", flush=True)
    assert ok
PY
