#!/bin/bash
# The default bench with the strided-EC queue schedule measured beside the first-pick one (other_configs.c5).
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu --no-copy > gpurun_out/bench_stride.json 2> gpurun_out/bench_stride.err || exit $?
