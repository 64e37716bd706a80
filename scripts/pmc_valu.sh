#!/bin/bash
# Counter evidence for the parity frame's binding resource: rocprofv3
# --kernel-trace --stats of a lone-frame run and of the default bench's timed launches, then
# SQ instruction / cycle counters and the HBM traffic counters in separate --pmc passes
# (MI355X_MICROARCH.md: one pass holds at most 8 SQ / 4 TCC / 2 GRBM counters).
#   scripts/pmc_valu.sh TAG      -> gpurun_out/pmc/<TAG>_*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r02}
out=gpurun_out/pmc
mkdir -p $out
export TMPDIR=/tmp
export SIZE=${SIZE:-4096} REPS=${REPS:-3}
step() {   # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -s KILL "$secs" "$@" > "$out/${tag}_$name.log" 2>&1
  local rc=$?
  tail -n 2 "$out/${tag}_$name.log" | cut -c1-300
  [ $rc -eq 0 ] || { echo "stop: $name rc $rc"; exit $rc; }
}
step list 60 rocprofv3 -L
step stats_lone 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats_lone -o s -- python -u scripts/lone.py
step stats_bench 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats_bench -o s -- python -u bench.py --timed-only --steps 20 --warmup 3
step sq1 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $out/sq1 -o p -- python -u scripts/lone.py
step sq2 90 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d $out/sq2 -o p -- python -u scripts/lone.py
step sq3 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/sq3 -o p -- python -u scripts/lone.py
step fetch 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o p -- python -u scripts/lone.py
step write 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o p -- python -u scripts/lone.py
echo done
