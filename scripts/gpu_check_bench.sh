#!/bin/bash
# GPU suite, then the default parity bench line and the fast-mode line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -n 20 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --mode fast --no-cpu-baseline > gpurun_out/bench_fast.log 2>&1 || { echo "bench fast failed"; tail -n 20 gpurun_out/bench_fast.log; exit 1; }
tail -n 1 gpurun_out/bench_fast.log | cut -c1-400
