#!/bin/bash
# Sharded-path GPU tests, then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_shard.log 2>&1 || { echo "shard tests failed"; tail -40 gpurun_out/pytest_shard.log; exit 1; }
tail -3 gpurun_out/pytest_shard.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
