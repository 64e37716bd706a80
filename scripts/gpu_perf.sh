#!/bin/bash
# Quick perf iteration: parity subset, lone frames (4096^2, 8192^2), bench headline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "test_configs or test_parity_schedules or test_many_shapes or test_small_goldens or phantom" > gpurun_out/pytest_perf.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_perf.log; exit 1; }
tail -1 gpurun_out/pytest_perf.log
for sz in 4096 8192; do SIZE=$sz TAG="lone $sz" CHECK=1 timeout -k 10 120 python -u scripts/lone.py || exit 1; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_perf.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_perf.log; exit 1; }
python3 -c "
import json; l=json.loads(open('gpurun_out/bench_perf.log').read().strip().splitlines()[-1])
print('bench', l['value'], l['ms_per_step'], 'single', l['single_frame']['ms'], 'phases', l['phases_ms'], 'e2e', l['end_to_end']['ms'], 'res_inflight', l['single_frame']['resolve_ms_in_flight'])"
