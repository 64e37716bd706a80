#!/bin/bash
# GPU suite, the default bench line, then an A/B of a tuning field on frames in flight and
# lone frames:  scripts/gpu_ab_x0.sh FIELD   (FIELD=0 vs FIELD=1, two rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
F=${1:-x0}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -n 20 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("default", d["value"], d["ms_per_step"], d["phases_ms"], d["single_frame"]["ms"], d["end_to_end"]["ms"], d["verified"]["frames"])'
for r in 1 2; do for v in 0 1; do
  timeout -k 10 120 python -u bench.py --timed-only --steps 40 --warmup 3 --tune $F=$v > gpurun_out/ab.log 2>&1 || { echo "ab failed"; tail -n 20 gpurun_out/ab.log; exit 1; }
  tail -n 1 gpurun_out/ab.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$F=$v' inflight", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])'
  timeout -k 10 120 python -u bench.py --inflight 1 --timed-only --steps 20 --warmup 3 --tune $F=$v > gpurun_out/ab1.log 2>&1 || { echo "ab1 failed"; tail -n 20 gpurun_out/ab1.log; exit 1; }
  tail -n 1 gpurun_out/ab1.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$F=$v' lone", d["value"], d["ms_per_step"], d.get("phases_ms"))'
done; done
