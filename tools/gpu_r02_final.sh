#!/bin/bash
# Round-2 evidence session: profile set (tools/gpu_prof.sh r02), clock/CPI passes, 2-rank rehearsal.
bash tools/gpu_prof.sh r02 || exit $?
cd $GRAFT_REPO_ROOT
bash tools/gpu_clock.sh r02 > gpurun_out/clock_run.log 2>&1 || exit $?
bash tools/dist2.sh
