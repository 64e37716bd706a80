#!/bin/bash
# Frames-in-flight partition sweep: one bench run per "lanes:res_cus:slots[:team]" config.
#   scripts/pipe_sweep.sh [bench args] -- cfg ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
args=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done
shift
for cfg in "$@"; do
  IFS=: read -r lanes res slots team <<< "$cfg"
  tune=(--tune pipe_resolvers="$lanes" --tune pipe_res_cus="$res" --tune pipe_slots="$slots")
  [ -n "$team" ] && tune+=(--tune team_blocks="$team")
  line=$(timeout -k 10 90 python bench.py --timed-only "${tune[@]}" "${args[@]}" \
         2>>gpurun_out/sweep_err.log | grep '^{')
  rc=$?
  echo "$cfg $(echo "$line" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"].get("kernel_ms"))' 2>/dev/null) rc=$rc"
  case $rc in 0|1) ;; *) echo "stop: rc $rc"; exit $rc ;; esac
done
