#!/bin/bash
# GPU suite, default bench (parity), fast bench, sharded-path timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python -u bench.py --mode fast --no-cpu-baseline > gpurun_out/bench_fast.log 2>&1 || { echo "bench fast failed"; tail -20 gpurun_out/bench_fast.log; exit 1; }
tail -1 gpurun_out/bench_fast.log
timeout -k 10 300 python -u scripts/shard_timing.py > gpurun_out/shard_timing.log 2>&1 || { echo "shard timing failed"; tail -20 gpurun_out/shard_timing.log; exit 1; }
cat gpurun_out/shard_timing.log
