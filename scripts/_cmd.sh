mkdir -p gpurun_out
for cfg in "simple 1024 6" "reflection 2048 4" "simple 1024 1" "quadric 2048 6"; do set -- $cfg
 for t in side=0 side=3; do
  SCENE=$1 SIZE=$2 DEPTH=$3 TUNE=$t TAG="$cfg $t" timeout -k 10 120 python -u scripts/lone.py || exit 1
 done; done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/tg.log 2>&1; rc=$?; tail -3 gpurun_out/tg.log; exit $rc
