#!/bin/bash
# Pipeline team size on the small configurations: 3/8 (default) vs half of the lane's grid.
mkdir -p gpurun_out
for cfg in "reflection 2048 4" "simple 1024 6"; do set -- $cfg
for t in -1 32 -1 32 28; do
  line=$(timeout -k 10 120 python -u bench.py --timed-only --scene $1 --size $2 --depth $3 --steps 60 --tune team_blocks=$t 2>>gpurun_out/team_err.log | grep '^{')
  rc=$?
  echo "$cfg team $t: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null) rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done; done
