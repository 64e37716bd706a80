mkdir -p gpurun_out
for t in side=3 side=5; do
  SIZE=4096 CHECK=1 TAG="lone4096 $t" TUNE=$t REPS=10 timeout -k 10 120 python -u scripts/lone.py || exit 1
done
for t in side=3 side=5; do
  SIZE=8192 CHECK=1 TAG="lone8192 $t" TUNE=$t REPS=5 timeout -k 10 120 python -u scripts/lone.py || exit 1
done
for cfg in "reflection 2048 4" "simple 1024 6"; do set -- $cfg
for t in side=3 side=5; do
  SCENE=$1 SIZE=$2 DEPTH=$3 CHECK=1 TAG="$cfg $t" TUNE=$t REPS=10 timeout -k 10 120 python -u scripts/lone.py || exit 1
done; done
timeout -k 10 200 python -u bench.py --timed-only --no-cpu-baseline --steps 40 --warmup 3 > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified']['frames'])"
