for v in libraycast_hip.so var/libraycast_hip_p0.so; do
  echo "$v single $(RC_HIP_LIB=$v python scripts/phase_probe.py 2>/dev/null | tail -1)"
  RC_HIP_LIB=$v RC_RESOLVE_TRACE=gpurun_out/trp_$(basename $v .so).txt python scripts/trace_run.py > /dev/null 2>&1
  echo "$v pipe $(RC_HIP_LIB=$v python bench.py --timed-only --steps 60 2>/dev/null | tail -1 | cut -c1-130)"
done
