#!/bin/bash
# Every counter file bench.py reads, from HEAD in one call: per
# configuration a rocprofv3 --kernel-trace --stats run and one --pmc pass per counter group
# (MI355X_MICROARCH.md: at most 8 SQ, 4 TCC, 2 GRBM counters per pass; FETCH_SIZE and
# WRITE_SIZE in passes of their own), summarised by scripts/pmc_summary.py into
# gpurun_out/pmca/<TAG>_<cfg>.json.  Configurations:
#   headline  the driver's command, frames in flight (bench.py --timed-only --steps 20 --warmup 5)
#   c4        lone quadric 4096^2 d6 parity frames (scripts/lone.py)
#   c3        lone reflection 2048^2 d4 parity frames
#   c5        lone quadric 8192^2 d6 parity frames
#   fast      quadric 4096^2 fast mode (bench.py --mode fast --timed-only)
#   scripts/pmc_all.sh TAG [cfg ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r06}; shift
cfgs=${*:-headline c4 c3 c5 fast}
export TMPDIR=/tmp REPS=${REPS:-3}
base=gpurun_out/pmca
mkdir -p $base
step() {   # dir name seconds cmd...
  local d=$1 name=$2 secs=$3; shift 3
  timeout -s KILL "$secs" "$@" > "$d/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "stop: $d $name rc $rc"; tail -n 3 "$d/$name.log"; exit $rc; }
}
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
SQ3="SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
for cfg in $cfgs; do
  case $cfg in
    headline) C="python3 -u bench.py --timed-only --steps 20 --warmup 5"; E="" ;;
    c4) C="python3 -u scripts/lone.py"; E="SCENE=quadric SIZE=4096 DEPTH=6" ;;
    c3) C="python3 -u scripts/lone.py"; E="SCENE=reflection SIZE=2048 DEPTH=4" ;;
    c5) C="python3 -u scripts/lone.py"; E="SCENE=quadric SIZE=8192 DEPTH=6" ;;
    fast) C="python3 -u bench.py --mode fast --timed-only --steps 5 --warmup 1"; E="" ;;
    *) echo "unknown cfg $cfg"; exit 2 ;;
  esac
  d=$base/${tag}_$cfg
  mkdir -p $d/pmc
  export SCENE=quadric SIZE=4096 DEPTH=6
  [ -n "$E" ] && export $E
  echo "== $cfg: $C ($E)"
  step $d stats 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d/stats -o s -- $C
  step $d sq1 150 rocprofv3 --pmc $SQ1 --kernel-trace --output-format csv -d $d/pmc/sq1 -o p -- $C
  step $d sq3 150 rocprofv3 --pmc $SQ3 --kernel-trace --output-format csv -d $d/pmc/sq3 -o p -- $C
  step $d fetch 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $d/pmc/fetch -o p -- $C
  step $d write 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $d/pmc/write -o p -- $C
  python3 scripts/pmc_summary.py $d/pmc $base/${tag}_$cfg.json "$cfg: $C ($E) at HEAD $(cat .git_head 2>/dev/null); kernel stats $d/stats" || exit 1
  python3 - $base/${tag}_$cfg.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    n = k.split("::")[-1].split("<")[0]
    if n in ("k_resolve", "k_phase_a", "k_render", "k_dep_chunks", "k_render_cuda"):
        print(f"  {n:14s} valu_busy {v.get('valu_busy')} hbm_bytes {v.get('hbm_bytes')} wait_any {v.get('frac_wait_any')}")
PY
done
echo done
