#!/bin/bash
# Late round-2 session: wrapper-check / group / reconstruction GPU tests, then the 2-rank bench rehearsal
# (gloo on one GPU) that now includes the sharded with-copy leg.
mkdir -p gpurun_out
bash tools/gpu_checks.sh || exit $?
bash tools/dist2.sh
