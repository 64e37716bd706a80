#!/bin/bash
# Pipeline team-size sweep (frames in flight).
mkdir -p gpurun_out
for sz in 4096; do
for t in 64 72 80 88 64 80; do
  line=$(timeout -k 10 120 python -u bench.py --timed-only --size $sz --steps 30 --tune team_blocks=$t 2>>gpurun_out/team_err.log | grep '^{')
  rc=$?
  echo "size $sz team $t: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null) rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done; done
