#!/bin/bash
# Frames-in-flight partition sweep at quadric 4096^2 (bench.py --timed-only, 40 frames).
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 120 python -u bench.py --timed-only --steps 40 "$@" > gpurun_out/ps.log 2>&1 || { tail -n 5 gpurun_out/ps.log; exit 1; }
  tail -n 1 gpurun_out/ps.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3e'%d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
run
run --tune pipe_res_cus=136
run --tune pipe_res_cus=144
run --tune pipe_res_cus=160
run --tune pipe_resolvers=3 --tune pipe_res_cus=160 --tune pipe_slots=5
run --tune pipe_resolvers=3 --tune pipe_res_cus=192 --tune pipe_slots=5
run
# simple 1024^2 d6 (slower resolver than round 1's v10 line: 0.54 vs 0.41 ms)
run --scene simple --size 1024
run --scene simple --size 1024 --tune helpers=0
run --scene simple --size 1024 --tune team_blocks=0
run --scene simple --size 1024 --tune helpers=0 --tune team_blocks=0
