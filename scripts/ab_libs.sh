#!/bin/bash
# Same-box A/B of library builds (scripts/build_variant.sh) on the driver's bench command,
# alternated: "" = the product library, NAME = libraycast_hip_NAME.so.
#   scripts/ab_libs.sh STEPS REPS "" NAME ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
steps=$1; reps=$2; shift 2
for r in $(seq $reps); do
  for v in "$@"; do
    lib=libraycast_hip.so; [ -n "$v" ] && lib=libraycast_hip_$v.so
    RC_HIP_LIB=$lib timeout -k 10 150 python3 -u bench.py --steps $steps --warmup 5 --no-cpu-baseline > /tmp/ab.log 2>&1 || { echo "run failed: $v"; tail -5 /tmp/ab.log; exit 1; }
    tail -n 1 /tmp/ab.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('${v:-product}', d['value'], d['ms_per_step'], d['verified']['frames'], d['single_frame']['ms'], d['phases_ms'], d['end_to_end']['ms'])"
  done
done
