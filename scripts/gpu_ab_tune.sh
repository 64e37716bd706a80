#!/bin/bash
# Same-box A/B of schedule variants on frames in flight: each argument is one variant, a
# comma-separated list of rc_tuning FIELD=VALUE ("-" = the default), two rounds interleaved.
#   scripts/gpu_ab_tune.sh - comp_stream=1 pipe_res_cus=136
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do for v in "$@"; do
  args=()
  [ "$v" != "-" ] && for kv in ${v//,/ }; do args+=(--tune "$kv"); done
  timeout -k 10 120 python -u bench.py --timed-only --steps ${STEPS:-60} --warmup 3 "${args[@]}" > gpurun_out/abt.log 2>&1 || { echo "variant $v failed"; tail -n 20 gpurun_out/abt.log; exit 1; }
  tail -n 1 gpurun_out/abt.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'"$v"'", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["verified"]["frame0_vs_reference"])'
done; done
