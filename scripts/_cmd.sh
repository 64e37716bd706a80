mkdir -p gpurun_out
SIZE=4096 CHECK=1 TAG=lone4096 REPS=10 timeout -k 10 120 python -u scripts/lone.py || exit 1
timeout -k 10 300 python -u bench.py --force-group --no-cpu-baseline > gpurun_out/fg.log 2>&1 || { tail -5 gpurun_out/fg.log; exit 1; }
tail -1 gpurun_out/fg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['single_frame']['ms'], json.dumps(d['sharded_single_image'])[:400])"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/tg.log 2>&1; rc=$?; tail -3 gpurun_out/tg.log; exit $rc
