#!/bin/bash
# One consistent counter set for the headline: kernel stats and every PMC
# pass from the SAME command — the default bench's frames in flight at HEAD
# (bench.py --timed-only --steps 20 --warmup 3) — summarised into one JSON that bench.py reads
# for roofline.traffic / valu_busy.  One rocprofv3 run per counter group (MI355X_MICROARCH.md:
# at most 8 SQ, 4 TCC, 2 GRBM counters per pass).
#   scripts/pmc_headline.sh TAG      -> gpurun_out/pmch/<TAG>_*, gpurun_out/pmch/<TAG>_pmc.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r04}
out=gpurun_out/pmch
mkdir -p $out
export TMPDIR=/tmp
CMD="python -u bench.py --timed-only --steps 20 --warmup 3"
step() {   # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -s KILL "$secs" "$@" > "$out/${tag}_$name.log" 2>&1
  local rc=$?
  tail -n 1 "$out/${tag}_$name.log" | cut -c1-200
  [ $rc -eq 0 ] || { echo "stop: $name rc $rc"; exit $rc; }
}
step stats 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_stats -o s -- $CMD
step sq1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out/${tag}_pmc/sq1 -o p -- $CMD
step sq3 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/${tag}_pmc/sq3 -o p -- $CMD
step fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/${tag}_pmc/fetch -o p -- $CMD
step write 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/${tag}_pmc/write -o p -- $CMD
python3 scripts/pmc_summary.py $out/${tag}_pmc $out/${tag}_pmc.json "frames in flight: bench.py --timed-only --steps 20 --warmup 3, quadric 4096^2 depth 6, $tag; kernel stats $out/${tag}_stats"
echo done
