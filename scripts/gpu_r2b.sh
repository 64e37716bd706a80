set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r2b.log 2>&1
SIZE=4096 timeout -k 10 120 python -u scripts/lone.py > gpurun_out/r2b_lone.log 2>&1
SIZE=4096 timeout -k 10 120 python -u scripts/e2e.py > gpurun_out/r2b_e2e.log 2>&1
timeout -k 10 120 python -u bench.py --mode fast --no-cpu-baseline > gpurun_out/r2b_fast.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw -o p -- python -u scripts/lone.py > gpurun_out/r2b_pmcw.log 2>&1
MODE=fast DEPTH=6 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcwf -o p -- python -u scripts/e2e.py > gpurun_out/r2b_pmcwf.log 2>&1
