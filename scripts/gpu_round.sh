#!/bin/bash
# One GPU round check into gpurun_out/<tag>_*: the -m gpu suite, smoke(), the default bench
# line (the driver's command), and the 2-rank gloo rehearsal of `bench.py --gpus 2` (two ranks
# self-launched on the one GPU, replicas).  Usage: scripts/gpu_round.sh TAG [skip-tests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r06}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" gpurun_out/${tag}_pytest_gpu.log | head -30; tail -5 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_smoke.log
fi
timeout -k 10 300 python -u bench.py --steps 20 > gpurun_out/${tag}_bench_20.log 2>&1 || { echo "bench failed"; tail -n 20 gpurun_out/${tag}_bench_20.log; exit 1; }
tail -n 1 gpurun_out/${tag}_bench_20.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("parity20", d["value"], d["ms_per_step"], d["single_frame"]["ms"], d["end_to_end"]["ms"], d["verified"]["frames"], d["cpu_baseline"]["value"])'
RC_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 > gpurun_out/${tag}_bench_gloo2.log 2>&1 || { echo "gloo rehearsal failed"; tail -n 20 gpurun_out/${tag}_bench_gloo2.log; exit 1; }
tail -n 1 gpurun_out/${tag}_bench_gloo2.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("gloo2", d["n_gpus"], d["config"]["parallelism"], d["value"], d["ms_per_step"], d["verified"]["frames"])'
