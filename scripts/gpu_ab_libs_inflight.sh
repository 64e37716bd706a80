#!/bin/bash
# Same-box A/B of library builds (RC_HIP_LIB, raytracing-programs_amd/lib/) on frames in flight
# only, rounds interleaved.   scripts/gpu_ab_libs_inflight.sh lib1.so lib2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do for L in "$@"; do
  RC_HIP_LIB=$L timeout -k 10 120 python -u bench.py --timed-only --steps ${STEPS:-40} --warmup 3 ${BENCH_ARGS} > gpurun_out/abf.log 2>&1 || { echo "$L failed"; tail -n 20 gpurun_out/abf.log; exit 1; }
  tail -n 1 gpurun_out/abf.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$L'", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["verified"]["frame0_vs_reference"])'
done; done
