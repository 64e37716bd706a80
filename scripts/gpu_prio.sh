#!/bin/bash
# Resolver issue-priority sweep (frames in flight, quadric 4096^2 and 8192^2).
mkdir -p gpurun_out
for sz in 4096 8192; do
for p in 0 1024 0 1024 256 4096; do
  line=$(timeout -k 10 120 python -u bench.py --timed-only --size $sz --steps 30 --tune resolve_prio_len=$p 2>>gpurun_out/prio_err.log | grep '^{')
  rc=$?
  echo "size $sz prio_len $p: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null) rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done; done
SIZE=4096 TAG="lone 4096" CHECK=1 timeout -k 10 120 python -u scripts/lone.py
