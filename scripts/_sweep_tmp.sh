scripts/pipe_sweep.sh --steps 16 --size 8192 -- 2:96:4 2:80:4 2:64:4 > gpurun_out/sweep22.log 2>&1
cat gpurun_out/sweep22.log
