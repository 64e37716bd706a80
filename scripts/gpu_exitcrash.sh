#!/bin/bash
# The subset that aborted at exit (two HIP runtimes), now with torch loaded first by the binding.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "test_many_shapes or phantom" > gpurun_out/exit2.log 2>&1; echo "shapes+phantom rc=$?"; tail -3 gpurun_out/exit2.log
