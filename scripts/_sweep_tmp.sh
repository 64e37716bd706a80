scripts/pipe_sweep.sh --steps 60 -- 2:128:4 2:112:4 2:96:4 2:144:4 > gpurun_out/sweep23.log 2>&1
cat gpurun_out/sweep23.log
