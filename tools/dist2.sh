#!/bin/bash
# Multi-rank paths on a one-GPU box: RCCL refuses two ranks on one device, so the
# collectives run over gloo on host copies (ShardedRound's / ShardedReconstruction's test
# path); everything else (client sharding, shard windows in the kernel, bench's G>1 flow with
# the c4 strong round and the sharded c5 reconstruction) is the real code.
mkdir -p gpurun_out
export HIP_VISIBLE_DEVICES=0 FLM_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dist_smoke.py > gpurun_out/dist2.log 2>&1 || exit $?
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > gpurun_out/bench_g2_gloo.log 2>&1 || exit $?
