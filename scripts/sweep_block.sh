#!/bin/bash
# Lone-frame and frames-in-flight sweep of rc_tuning.block_min (long regular carry segments
# on whole resolver workgroups), md5-checked; then the resolver traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for t in ${LONE:-block_min=0 block_min=1536 block_min=2048 block_min=3072}; do
  TAG="lone4096 $t" TUNE="$t" CHECK=1 REPS=10 timeout -k 10 120 python -u scripts/lone.py || exit 1
done
for t in ${LONE8K:-}; do
  TAG="lone8192 $t" SIZE=8192 TUNE="$t" CHECK=1 REPS=5 timeout -k 10 120 python -u scripts/lone.py || exit 1
done
for t in ${PIPE:-}; do
  echo "bench $t"; timeout -k 10 200 python -u bench.py --timed-only --steps 30 --warmup 3 --tune ${t//,/ --tune } | python3 -c "import json,sys; l=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(l['value'], l['ms_per_step'], l['verified']['frames'], l['roofline']['kernel_ms'])" || exit 1
done
for t in ${TRACE:-}; do
  RC_HIP_LIB=${STAMPLIB:-libraycast_hip_stamps2.so} RC_RESOLVE_TRACE=gpurun_out/trace_$t.txt TUNE=$t timeout -k 10 120 python -u scripts/trace_run.py && python3 scripts/seg_trace.py gpurun_out/trace_$t.txt | grep -v "^  " || exit 1
  tail -8 gpurun_out/trace_$t.txt.cyc
done
