mkdir -p gpurun_out
for t in block_min=0 block_min=3000; do
  SIZE=4096 CHECK=1 TAG="lone4096 $t" TUNE=$t REPS=10 timeout -k 10 120 python -u scripts/lone.py || exit 1
done
RC_HIP_LIB=libraycast_hip_stamps2.so RC_RESOLVE_TRACE=gpurun_out/trace_pf.txt TUNE=block_min=3000 timeout -k 10 120 python -u scripts/trace_run.py && python3 scripts/seg_trace.py gpurun_out/trace_pf.txt > gpurun_out/seg_pf.txt || exit 1
head -6 gpurun_out/seg_pf.txt
awk '$2==0 {s+=$5; n++} $2==1 {r+=$5; m++} END {print "scan", n, s, "resolve", m, r}' gpurun_out/trace_pf.txt.team
timeout -k 10 200 python -u bench.py --timed-only --no-cpu-baseline --steps 30 --warmup 3 > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('verified')['frames'])"
