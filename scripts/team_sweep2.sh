#!/bin/bash
# Pipeline-lane team size without helpers (frames in flight, bench.py --timed-only).
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 150 python -u bench.py --timed-only --no-cpu-baseline "$@" > gpurun_out/ts.log 2>&1 || { tail -n 5 gpurun_out/ts.log; exit 1; }
  tail -n 1 gpurun_out/ts.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3e'%d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for t in -1 48 56 72 80; do run --steps 40 --tune team_blocks=$t; done
for t in -1 16 32 48; do run --steps 40 --scene reflection --size 2048 --depth 4 --tune team_blocks=$t; done
for t in -1 48 64; do run --steps 20 --size 8192 --tune team_blocks=$t; done
