#!/bin/bash
# Same-box A/B of lone parity frames over several configurations (scripts/lone.py, md5-checked):
# CFGS = "scene:size:depth ..." ; each argument LIB[:TUNE] as in gpu_ab_lone.sh.
#   CFGS="quadric:8192:6 reflection:2048:4" scripts/gpu_ab_lone_cfgs.sh libraycast_hip.so "libraycast_hip.so:helpers=16"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for r in ${ROUNDS:-1}; do for cfg in ${CFGS:-quadric:4096:6}; do
  IFS=: read -r SC SZ DP <<< "$cfg"
  for a in "$@"; do
    L=${a%%:*}; T=""; [ "$a" != "$L" ] && T=${a#*:}
    SCENE=$SC SIZE=$SZ DEPTH=$DP RC_HIP_LIB=$L TUNE=${T//;/,} CHECK=1 REPS=${REPS:-6} TAG="$cfg $a" \
      timeout -k 10 120 python -u scripts/lone.py > gpurun_out/ablc.log 2>&1 || { echo "lone failed: $cfg $a"; tail -n 20 gpurun_out/ablc.log; exit 1; }
    tail -n 1 gpurun_out/ablc.log
  done
done; done
