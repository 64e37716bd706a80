#!/bin/bash
# Run GPU steps in order, each under its own time limit, logging to gpurun_out/<name>.log.
# A plain failure (exit 1/2: test assertion, python error) moves on to the next step; a
# fault-type exit (timeout 124/137, abort 134, segfault 139, or any signal) stops the run.
#   scripts/gpu_steps.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name exit $rc after $(( $(date +%s) - start ))s"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then status=$rc; fi
  case $rc in
    0|1|2|3|4|5) ;;
    *) echo "== fault-type exit $rc: stopping"; exit $rc ;;
  esac
done
exit $status
