#!/bin/bash
# Same-box A/B of library builds (RC_HIP_LIB, raytracing-programs_amd/lib/): frames in flight and
# one frame at a time, two rounds, interleaved.   scripts/gpu_ab_libs.sh lib1.so lib2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do for L in "$@"; do
  RC_HIP_LIB=$L timeout -k 10 120 python -u bench.py --timed-only --steps 40 --warmup 3 > gpurun_out/ab.log 2>&1 || { echo "ab failed"; tail -n 20 gpurun_out/ab.log; exit 1; }
  tail -n 1 gpurun_out/ab.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$L' inflight", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["verified"]["frame0_vs_reference"])'
  RC_HIP_LIB=$L timeout -k 10 120 python -u bench.py --inflight 1 --timed-only --steps 20 --warmup 3 > gpurun_out/ab1.log 2>&1 || { echo "ab1 failed"; tail -n 20 gpurun_out/ab1.log; exit 1; }
  tail -n 1 gpurun_out/ab1.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); p=d.get("phases_ms",{}); print("'$L' lone", d["ms_per_step"], p.get("phase_a_ms"), p.get("resolve_ms"))'
done; done
