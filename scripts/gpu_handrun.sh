#!/bin/bash
# Helper hand-off threshold sweep: lone frames (4096^2, 8192^2) and frames in flight.
mkdir -p gpurun_out
cat > /tmp/hr.py <<'PY'
import json, os, sys, torch
sys.path.insert(0, "tests")
from helpers import golden_table, p3_md5, rc, scene_path
s = rc.Scene.from_file(scene_path("quadric"))
for n in (4096, 8192):
    out = torch.empty((n, n, 3), dtype=torch.uint8, device="cuda")
    for hr in (512, 256, 128, 64, 512, 128):
        rc.set_tuning(hand_run=hr)
        for _ in range(2):
            rc.render_device(s, n, n, out.data_ptr(), depth=6, mode="parity")
        torch.cuda.synchronize()
        rc.profile_begin()
        for _ in range(5):
            rc.render_device(s, n, n, out.data_ptr(), depth=6, mode="parity")
        torch.cuda.synchronize()
        ph = rc.profile_end()
        ok = p3_md5(out.cpu().numpy()) == golden_table()[f"quadric:{n}x{n}:d6:parity"]["md5"]
        print(n, "hand_run", hr, "resolve", round(ph["resolve_ms"], 3), "total", round(ph["total_ms"], 3), "md5", ok, flush=True)
    del out
PY
timeout -k 10 300 python -u /tmp/hr.py || exit 1
for hr in 512 128; do
  line=$(timeout -k 10 120 python -u bench.py --timed-only --steps 40 --tune hand_run=$hr 2>>gpurun_out/hr_err.log | grep '^{')
  echo "inflight hand_run $hr: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null)"
done
