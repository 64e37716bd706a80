#!/bin/bash
# Same-box A/B of lone parity frames (scripts/lone.py, md5-checked): each argument is
# LIB[:TUNE] (RC_HIP_LIB name, optional rc_set_tuning fields "f=v;f=v"), ROUNDS interleaved.
#   scripts/gpu_ab_lone.sh libraycast_hip.so libraycast_hip_x.so libraycast_hip.so:resolve_clean=2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2 3}; do for a in "$@"; do
  L=${a%%:*}; T=""; [ "$a" != "$L" ] && T=${a#*:}
  RC_HIP_LIB=$L TUNE=${T//;/,} CHECK=1 REPS=${REPS:-8} TAG="$a" timeout -k 10 120 python -u scripts/lone.py > gpurun_out/abl.log 2>&1 || { echo "lone failed: $a"; tail -n 20 gpurun_out/abl.log; exit 1; }
  tail -n 1 gpurun_out/abl.log
done; done
