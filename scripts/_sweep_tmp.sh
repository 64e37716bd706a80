for cfg in "8 512" "8 384" "16 256" "32 128" "0 512"; do set -- $cfg
  echo "helpers $1 run $2 single $(RC_HELPERS=$1 RC_HAND_RUN=$2 python scripts/phase_probe.py 2>/dev/null | tail -1 | cut -c1-80)"
  echo "helpers $1 run $2 pipe $(RC_HELPERS=$1 RC_HAND_RUN=$2 timeout -k 5 60 python bench.py --timed-only --steps 60 2>/dev/null | tail -1 | cut -c60-110)"
done
RC_HELPERS=8 RC_HAND_RUN=512 RC_RESOLVE_TRACE=gpurun_out/trh8.txt timeout -k 5 60 python scripts/trace_run.py > /dev/null 2>&1
