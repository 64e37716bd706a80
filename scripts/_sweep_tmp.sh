scripts/pipe_sweep.sh --steps 60 -- 2:128:4 2:112:4 2:96:4 > gpurun_out/sweep24.log 2>&1
RC_HELPERS=16 RC_HAND_RUN=256 scripts/pipe_sweep.sh --steps 60 -- 2:112:4 2:96:4 >> gpurun_out/sweep24.log 2>&1
cat gpurun_out/sweep24.log
