#!/bin/bash
# Bench lines at every BASELINE config (roofline + cpu_baseline): C2, C3 (parity, fast), C5 (parity, fast).
set -o pipefail
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$tag.log 2>&1 || { echo "bench $tag failed"; tail -20 gpurun_out/bench_$tag.log; exit 1; }; tail -1 gpurun_out/bench_$tag.log | cut -c1-400; }
run c2 --scene simple --size 1024 --depth 0
run c3p --scene reflection --size 2048 --depth 4
run c3f --scene reflection --size 2048 --depth 4 --mode fast
run c5p --scene quadric --size 8192 --depth 6 --steps 20
run c5f --scene quadric --size 8192 --depth 6 --mode fast --no-cpu-baseline
run c1p --scene simple --size 256 --depth 6
