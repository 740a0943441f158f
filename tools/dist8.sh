#!/bin/bash
# bench.py's G=8 round (default: c4 strong, n=1024 in total, plus the sharded c5) on a one-GPU box (eight ranks share the GPU; the reduce-scatter
# runs over gloo on host copies because RCCL refuses duplicate devices).  Full c4 sizes per rank
# (N = 8192 clients, 4 GiB of rows per rank): checks the G=8 client/slot sharding, the N=8192 seed
# table and the out == |U| invariant across ranks, not the timing.
mkdir -p gpurun_out
export HIP_VISIBLE_DEVICES=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --steps 3 --warmup 1 --dist-backend gloo > gpurun_out/bench_g8_gloo.log 2>&1
