#!/bin/bash
# Same-box A/B of schedule variants on lone frames (one frame at a time, bench.py --inflight 1):
# each argument is one variant, a comma-separated list of rc_tuning FIELD=VALUE ("-" = the
# default), rounds interleaved.   scripts/gpu_ab_lone_tune.sh - team_blocks=160
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do for v in "$@"; do
  args=()
  [ "$v" != "-" ] && for kv in ${v//,/ }; do args+=(--tune "$kv"); done
  timeout -k 10 120 python -u bench.py --inflight 1 --timed-only --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS} "${args[@]}" > gpurun_out/abl.log 2>&1 || { echo "variant $v failed"; tail -n 20 gpurun_out/abl.log; exit 1; }
  tail -n 1 gpurun_out/abl.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); p=d.get("phases_ms",{}); print("'"$v"'", d["ms_per_step"], p.get("phase_a_ms"), p.get("resolve_ms"), d["verified"]["frame0_vs_reference"])'
done; done
