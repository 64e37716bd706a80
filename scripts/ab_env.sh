#!/bin/bash
# A/B of environment settings on the driver's bench command (timed frames only), alternated.
#   scripts/ab_env.sh STEPS REPS "" "VAR=1" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
steps=$1; reps=$2; shift 2
for r in $(seq $reps); do
  for v in "$@"; do
    env $v timeout -k 10 120 python3 -u bench.py --steps $steps --warmup 5 --timed-only > /tmp/ab.log 2>&1 || { echo "run failed: $v"; tail -5 /tmp/ab.log; exit 1; }
    tail -n 1 /tmp/ab.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('${v:-default}', d['value'], d['ms_per_step'], d['verified']['frames'])"
  done
done
