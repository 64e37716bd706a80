#!/bin/bash
# Team-segment anatomy of a lone quadric 4096^2 frame from the diagnostic builds (make stamps
# stamps2): per-round team log (.team), eval/step/barrier-wait cycles of the leader's block
# windows (.cyc), per-segment trace.   scripts/gpu_trace_team.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-t}
out=gpurun_out/trace
mkdir -p $out
for v in stamps stamps2; do
  RC_HIP_LIB=libraycast_hip_$v.so RC_RESOLVE_TRACE=$out/${tag}_$v.txt timeout -k 10 120 python -u scripts/trace_run.py || exit 1
  python3 scripts/seg_trace.py $out/${tag}_$v.txt | head -12
  grep -v "^#" $out/${tag}_$v.txt.team | awk '{n[$2]++; c[$2]+=$5; l[$2]+=$6; k[$2]+=$7; ch[$2]+=$8} END {for (m in n) print "mode", m, "rounds", n[m], "cycles", c[m], "lane", l[m], "coop", k[m], "changers", ch[m]}'
  awk '/^round/ {e+=$4; s+=$6; w+=$8; n++} END {print "rounds", n, "eval", e, "step", s, "wait", w}' $out/${tag}_$v.txt.cyc
done
