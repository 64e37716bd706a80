#!/bin/bash
# Round-4 measurement set at HEAD: the bench line at every BASELINE configuration (C2-C5,
# fast), the forced one-rank sharded exchange, the GPU suite, then the headline's counter set
# from one command (scripts/pmc_headline.sh).  Output under gpurun_out/prof/<TAG>_*.
#   scripts/profile_r04.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r04}
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
run bench_parity 240 python -u bench.py
run bench_parity_serial 120 python -u bench.py --inflight 1 --no-cpu-baseline
run bench_c2 120 python -u bench.py --scene simple --size 1024 --depth 0 --no-cpu-baseline
run bench_c3p 120 python -u bench.py --scene reflection --size 2048 --depth 4 --no-cpu-baseline
run bench_c5p 240 python -u bench.py --size 8192 --steps 20 --no-cpu-baseline
run bench_s1024 120 python -u bench.py --scene simple --size 1024 --no-cpu-baseline
run bench_fast 120 python -u bench.py --mode fast --no-cpu-baseline
run bench_force_group_x 240 python -u bench.py --force-group --tune shard_lone=0 --no-cpu-baseline
echo done
