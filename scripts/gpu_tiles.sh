#!/bin/bash
# Framebuffer-store variants: lane stores (default, 16x16), 16x16 staged, 32x8 staged (coalesced).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for v in libraycast_hip.so libraycast_hip_t16.so libraycast_hip_coalesced.so; do
  export RC_HIP_LIB=$v
  SIZE=4096 TAG="$v lone" timeout -k 10 120 python -u scripts/lone.py 2>/dev/null || exit 1
  timeout -k 10 120 python -u bench.py --mode fast --no-cpu-baseline --timed-only 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v fast', d['roofline_render']['kernel_ms'])" || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/tiles_$v -o p -- python -u bench.py --mode fast --no-cpu-baseline --timed-only --steps 3 > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/tilesp_$v -o p -- python -u scripts/lone.py > /dev/null 2>&1 || exit 1
done
