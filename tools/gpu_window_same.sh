#!/bin/bash
# Same-tile window items (pairing 2) vs dual-tile items (pairing 1) for one rank of the strong-scaled c4 round.
mkdir -p gpurun_out
SWEEP=1 timeout -k 10 300 python -u tools/window_same_probe.py > gpurun_out/window_same.log 2>&1
