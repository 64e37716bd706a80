mkdir -p gpurun_out
SIZE=4096 CHECK=1 TAG="lone4096" REPS=10 timeout -k 10 60 python -u scripts/lone.py || exit 1
timeout -k 10 200 python -u bench.py --timed-only --no-cpu-baseline --steps 40 --warmup 3 > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified']['frames'], d['verified']['frame0_vs_reference'])"
timeout -k 10 200 python -u bench.py --mode fast --timed-only --no-cpu-baseline --steps 40 --warmup 3 > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fast', d['value'], d['ms_per_step'], d['verified'])"
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu.py -m gpu > gpurun_out/tg.log 2>&1; rc=$?; tail -2 gpurun_out/tg.log; exit $rc
