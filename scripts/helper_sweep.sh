#!/bin/bash
# Helper workgroups on/off per image size (frames in flight, bench.py --timed-only), and lone
# frames (--inflight 1).
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 150 python -u bench.py --timed-only --no-cpu-baseline "$@" > gpurun_out/hs.log 2>&1 || { tail -n 5 gpurun_out/hs.log; exit 1; }
  tail -n 1 gpurun_out/hs.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3e'%d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for h in 8 0; do
  run --steps 40 --tune helpers=$h
  run --steps 40 --inflight 1 --tune helpers=$h
  run --steps 40 --scene reflection --size 2048 --depth 4 --tune helpers=$h
  run --steps 40 --scene reflection --size 2048 --depth 4 --inflight 1 --tune helpers=$h
  run --steps 40 --scene simple --size 1024 --inflight 1 --tune helpers=$h
  run --steps 20 --size 8192 --tune helpers=$h
  run --steps 10 --size 8192 --inflight 1 --tune helpers=$h
done
