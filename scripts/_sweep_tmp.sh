scripts/pipe_sweep.sh --steps 60 -- 2:128:4 2:128:4 2:128:4 2:120:4 2:120:4 > gpurun_out/sweep10.log 2>&1
cat gpurun_out/sweep10.log
