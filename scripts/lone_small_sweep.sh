#!/bin/bash
# Lone-frame resolver knobs on the small configurations (bench.py --inflight 1 --timed-only).
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 150 python -u bench.py --timed-only --no-cpu-baseline --inflight 1 --steps 40 "$@" > gpurun_out/ls.log 2>&1 || { tail -n 5 gpurun_out/ls.log; exit 1; }
  tail -n 1 gpurun_out/ls.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms']; print('%.3e'%d['value'], d['ms_per_step'], 'resolve', p['resolve_ms'], 'phase_c', p['phase_c_ms'])"; }
for s in "--scene simple --size 1024" "--scene reflection --size 2048 --depth 4"; do
  run $s
  run $s --tune side=0
  run $s --tune single_res_cus=64
  run $s --tune single_res_cus=128
  run $s --tune team_blocks=32
  run $s --tune long_len=1000000
  run $s --tune wave_k=1
done
