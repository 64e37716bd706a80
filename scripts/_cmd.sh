mkdir -p gpurun_out
SIZE=4096 CHECK=1 TAG="lone4096 default" REPS=10 timeout -k 10 60 python -u scripts/lone.py || exit 1
SIZE=4096 CHECK=1 TAG="lone4096 bands" TUNE=bands=1 REPS=10 timeout -k 10 60 python -u scripts/lone.py || exit 1
SIZE=4096 CHECK=1 TAG="lone4096 bands1024" TUNE=bands=1024 REPS=10 timeout -k 10 60 python -u scripts/lone.py || exit 1
for cfg in "reflection 2048 4" "simple 1024 6" "quadric 2048 6"; do set -- $cfg
  SCENE=$1 SIZE=$2 DEPTH=$3 CHECK=1 TAG="$cfg bands" TUNE=bands=1 REPS=10 timeout -k 10 60 python -u scripts/lone.py || exit 1
done
SIZE=8192 CHECK=1 TAG="lone8192 bands" TUNE=bands=1 REPS=3 timeout -k 10 90 python -u scripts/lone.py || exit 1
