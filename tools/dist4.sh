#!/bin/bash
# bench.py's G=4 round (default: c4 strong plus the sharded c5) on a one-GPU box (four ranks share the GPU; the reduce-scatter
# runs over gloo on host copies because RCCL refuses duplicate devices).  Full c4 sizes per rank:
# checks the G=4 window planning and the out == |U| invariant across ranks, not the timing.
mkdir -p gpurun_out
export HIP_VISIBLE_DEVICES=0
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo > gpurun_out/bench_g4_gloo.log 2>&1
