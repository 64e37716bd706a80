#!/bin/bash
# Refresh the committed measurements: bench lines for every BASELINE config, a rocprofv3
# kernel-trace --stats summary of the default bench's timed launches, and the PMC HBM traffic
# (FETCH_SIZE / WRITE_SIZE in separate passes).  Output: gpurun_out/prof/<tag>_*.
#   scripts/profile_round.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-v}
out=gpurun_out/prof
mkdir -p $out
export TMPDIR=/tmp
run() {   # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$out/${tag}_$name.log" 2>&1
  local rc=$?
  tail -n 1 "$out/${tag}_$name.log" | cut -c1-300
  case $rc in 0|1|2) ;; *) echo "stop: $name rc $rc"; exit $rc ;; esac
}
run bench_parity 200 python -u bench.py
run bench_parity_serial 120 python -u bench.py --inflight 1 --no-cpu-baseline
run bench_c2 120 python -u bench.py --scene simple --size 1024 --depth 0 --no-cpu-baseline
run bench_c3p 120 python -u bench.py --scene reflection --size 2048 --depth 4 --no-cpu-baseline
run bench_c5p 200 python -u bench.py --size 8192 --steps 20 --no-cpu-baseline
run bench_s1024 120 python -u bench.py --scene simple --size 1024 --no-cpu-baseline
run bench_fast 120 python -u bench.py --mode fast --no-cpu-baseline
run bench_force_group 200 python -u bench.py --force-group --no-cpu-baseline
run rocprof_stats 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o stats -- python -u bench.py --timed-only --steps 20 --warmup 3
run pmc_fetch 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -o fetch -- python -u bench.py --timed-only --steps 3 --warmup 1
run pmc_write 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -o write -- python -u bench.py --timed-only --steps 3 --warmup 1
echo done
