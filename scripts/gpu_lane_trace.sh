#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace, CSV with queue ids) of the driver's bench command at
# frames in flight, for scripts/lane_gaps.py; with "hip" also the HIP API trace (host enqueue
# times).   scripts/gpu_lane_trace.sh TAG [hip] [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r06}; shift
extra=""
if [ "$1" = "hip" ]; then extra="--hip-trace"; shift; fi
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace $extra --stats --output-format csv -d gpurun_out/${tag}_trace -o k -- python3 -u bench.py --timed-only --steps 20 --warmup 5 "$@" > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/${tag}_trace.log; exit 1; }
tail -n 1 gpurun_out/${tag}_trace.log | cut -c1-200
f=$(find gpurun_out/${tag}_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/lane_gaps.py "$f" 20 | tail -3
