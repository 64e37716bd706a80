mkdir -p gpurun_out
for i in 1 2; do for lib in libraycast_hip_prev.so libraycast_hip.so; do
  echo "== $lib"; RC_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --timed-only --no-cpu-baseline --steps 40 --warmup 3 --tune block_min=0 > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified']['frames'])"
done; done
