#!/bin/bash
# Counter evidence for fast mode's render kernel (its frac counts algorithmic
# flops): VALU busy / instruction counts and HBM bytes of k_render at quadric 4096^2, one
# --pmc pass per counter group.  -> gpurun_out/pmc_fast/{valu,fetch,write}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/pmc_fast
mkdir -p $out
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -s KILL "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "stop: $name rc $rc"; tail -5 "$out/$name.log"; exit $rc; }
}
B="python -u bench.py --mode fast --timed-only --steps 5 --warmup 1"
step stats 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o s -- $B
step valu 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/valu -o p -- $B
step fetch 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o p -- $B
step write 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o p -- $B
echo done
