#!/bin/bash
# Round-2 check: GPU tests, smoke, full bench (driver's flags), then the 2-rank gloo rehearsal.
bash tools/gpu_round.sh --steps 20 --warmup 5 || exit $?
grep -q "pytest rc=0" gpurun_out/pytest_gpu.log || exit 1
bash tools/dist2.sh
