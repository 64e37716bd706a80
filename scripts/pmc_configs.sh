#!/bin/bash
# Counter evidence for the bench configurations other than the default:
# kernel stats, VALU and HBM-traffic --pmc passes of lone parity frames at C3 (reflection
# 2048^2 depth 4) and C5 (quadric 8192^2 depth 6), one counter group per pass
# (MI355X_MICROARCH.md: at most 8 SQ / 4 TCC / 2 GRBM counters in one pass).
#   scripts/pmc_configs.sh TAG   -> gpurun_out/pmc_<cfg>/...  (scripts/pmc_summary.py reads them)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r03}
export TMPDIR=/tmp REPS=${REPS:-3}
step() {   # out name seconds cmd...
  local out=$1 name=$2 secs=$3; shift 3
  echo "== $out $name"
  timeout -s KILL "$secs" "$@" > "$out/${tag}_$name.log" 2>&1
  local rc=$?
  tail -n 1 "$out/${tag}_$name.log" | cut -c1-300
  [ $rc -eq 0 ] || { echo "stop: $name rc $rc"; exit $rc; }
}
for cfg in "c3 reflection 2048 4" "c5 quadric 8192 6"; do
  set -- $cfg
  out=gpurun_out/pmc_$1
  mkdir -p $out
  export SCENE=$2 SIZE=$3 DEPTH=$4
  L="python -u scripts/lone.py"
  step $out stats 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o s -- $L
  step $out sq1 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/sq1 -o p -- $L
  step $out fetch 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o p -- $L
  step $out write 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o p -- $L
done
echo done
