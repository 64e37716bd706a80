set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in copy_threads=8 copy_threads=16 prefault=0; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --tune $v > gpurun_out/e2e.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/e2e.log; exit 1; }
  tail -n 1 gpurun_out/e2e.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); e=d["end_to_end"]; print("'$v'", e["ms"], e.get("lib_total_ms"), d["single_frame"]["ms"])'
done; done
