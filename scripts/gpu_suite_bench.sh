#!/bin/bash
# GPU suite (verbose log), then the default bench line and the fast-mode line, into gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_parity.log 2>&1 || { echo "bench failed"; tail -n 20 gpurun_out/bench_parity.log; exit 1; }
tail -n 1 gpurun_out/bench_parity.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("parity", d["value"], d["ms_per_step"], d["phases_ms"], d["single_frame"]["ms"], d["end_to_end"]["ms"], d["verified"], d["cpu_baseline"]["value"])'
timeout -k 10 300 python -u bench.py --mode fast --no-cpu-baseline > gpurun_out/bench_fast.log 2>&1 || { echo "bench fast failed"; tail -n 20 gpurun_out/bench_fast.log; exit 1; }
tail -n 1 gpurun_out/bench_fast.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("fast", d["value"], d["ms_per_step"])'
