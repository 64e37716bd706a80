#!/bin/bash
# The bench line at every BASELINE configuration at HEAD (and the other modes), plus the N = 2
# rehearsal under the driver's own launcher form (torchrun, gloo: two ranks on the one GPU).
# Output: gpurun_out/<TAG>_bench_*.log.   scripts/bench_configs.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r06}
mkdir -p gpurun_out
run() {   # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_bench_$name.log" 2>&1
  local rc=$?
  tail -n 1 "gpurun_out/${tag}_bench_$name.log" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d['verified']['frames'], d['verified']['frame0_vs_reference'], (d.get('single_frame') or {}).get('ms'), (d.get('end_to_end') or {}).get('ms'))" 2>/dev/null || echo "$name: no line"
  [ $rc -eq 0 ] || { echo "stop: $name rc $rc"; exit $rc; }
}
run parity40 200 python3 -u bench.py --steps 40 --no-cpu-baseline
run parity_serial 120 python3 -u bench.py --inflight 1 --no-cpu-baseline
run c2 120 python3 -u bench.py --scene simple --size 1024 --depth 0 --no-cpu-baseline
run c3p 120 python3 -u bench.py --scene reflection --size 2048 --depth 4 --no-cpu-baseline
run c5p 200 python3 -u bench.py --size 8192 --steps 20 --no-cpu-baseline
run s1024 120 python3 -u bench.py --scene simple --size 1024 --no-cpu-baseline
run fast 120 python3 -u bench.py --mode fast --no-cpu-baseline
run cuda50 120 python3 -u bench.py --mode cuda --depth 50
run force_group 200 python3 -u bench.py --force-group --no-cpu-baseline
RC_BENCH_BACKEND=gloo run torchrun_gloo2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5
