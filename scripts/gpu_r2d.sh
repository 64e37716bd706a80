#!/bin/bash
# GPU suite, then the bench lines at every configuration (profile_round's bench part).
set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
b() { local n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > gpurun_out/prof/${TAG:-r02d}_$n.log 2>&1 || { echo "$n failed"; tail -n 5 gpurun_out/prof/${TAG:-r02d}_$n.log; exit 1; }
  tail -n 1 gpurun_out/prof/${TAG:-r02d}_$n.log | cut -c1-160; }
b bench_parity
b bench_c3p --scene reflection --size 2048 --depth 4 --no-cpu-baseline
b bench_c5p --size 8192 --steps 20 --no-cpu-baseline
b bench_s1024 --scene simple --size 1024 --no-cpu-baseline
b bench_c1p --scene simple --size 256 --no-cpu-baseline
