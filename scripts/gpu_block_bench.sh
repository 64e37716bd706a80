#!/bin/bash
# The team leader's block step in isolation (scripts/block_bench.hip): entries of quadric
# 4096^2's team segment from the CPU oracle (scripts/dump_entries.c, written on the box's CPU),
# then each variant given (0 = the product step, 2 = split by shape class), every carry-in
# checked bit for bit.  Build first: hipcc ... scripts/block_bench.hip -o scripts/bin/block_bench
#   scripts/gpu_block_bench.sh TAG "0 2 0 2"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r06}
mkdir -p gpurun_out
ent=/tmp/team_entries.bin
timeout -k 10 120 scripts/bin/dump_entries tests/golden/scenes/quadric.scene 4096 7 team $ent > gpurun_out/${tag}_dump.log 2>&1 || { echo "dump failed"; tail gpurun_out/${tag}_dump.log; exit 1; }
tail -n 2 gpurun_out/${tag}_dump.log
for v in ${2:-0 2}; do
  timeout -k 10 120 scripts/bin/block_bench $ent 64 $v >> gpurun_out/${tag}_block_bench.log 2>&1 || { echo "block_bench $v failed"; tail gpurun_out/${tag}_block_bench.log; exit 1; }
done
cat gpurun_out/${tag}_block_bench.log
