mkdir -p gpurun_out
for i in 1 2; do for t in "" "--tune comp_stream=1"; do
  echo "== $t"; timeout -k 10 200 python -u bench.py --timed-only --no-cpu-baseline --steps 40 --warmup 3 $t > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified']['frames'], d['roofline']['traffic'], d['roofline']['pmc_source'])"
done; done
