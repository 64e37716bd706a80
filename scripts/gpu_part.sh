#!/bin/bash
# Resolver-partition sweep with the half-grid team (quadric 4096^2, frames in flight).
mkdir -p gpurun_out
for cfg in 128 112 144 128 120 136; do
  line=$(timeout -k 10 120 python -u bench.py --timed-only --steps 40 --tune pipe_res_cus=$cfg 2>>gpurun_out/part_err.log | grep '^{')
  rc=$?
  echo "res_cus $cfg: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null) rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
for sl in 5 6; do
  line=$(timeout -k 10 120 python -u bench.py --timed-only --steps 40 --tune pipe_slots=$sl 2>>gpurun_out/part_err.log | grep '^{')
  echo "slots $sl: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,3), "e9 ms", d["ms_per_step"], "resolver", d["roofline"]["kernel_ms"])' 2>/dev/null)"
done
