#!/bin/bash
# Per-round team log of the long segment (diagnostic build `make stamps2`, RC_RESOLVE_TRACE):
# rounds, cycles and entries by kind (0 LANE SCAN, 1 RESOLVE, 2 cooperative SCAN), for a lone
# frame and for a lone frame sized like a pipeline lane (TUNE, e.g. single_res_cus=64).
#   scripts/gpu_team_rounds.sh TAG [TUNE]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-t}
out=gpurun_out/trace
mkdir -p $out
TUNE=$2 RC_HIP_LIB=libraycast_hip_stamps2.so RC_RESOLVE_TRACE=$out/${tag}.txt timeout -k 10 120 python3 -u scripts/trace_run.py || exit 1
python3 scripts/seg_trace.py $out/${tag}.txt | head -4
grep -v "^#" $out/${tag}.txt.team | awk '{n[$2]++; c[$2]+=$5; e[$2]+=$4-$3} END {for (m in n) printf "kind %s rounds %d cycles %d (%.3f ms at 2.4 GHz) entries %d\n", m, n[m], c[m], c[m]/2.4e6, e[m]}'
