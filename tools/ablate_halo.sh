cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_conv.py 32 0,11,12,13,30 "64,64,64,0;64,32,128,0;32,64,128,0" > gpurun_out/ablate_halo.log 2>&1
