#!/bin/bash
# A/B of the c4 kernel's row-load cache policy (flamingo_amd/lib_v/aux*: FLM_ROW_AUX=1 sc0, 16 sc1,
# 17 sc0 sc1, 18 sc1 nt) against the default build on the full and rows-only launch shapes.
mkdir -p gpurun_out
bash tools/ab_variants.sh gpurun_out/ab_aux.log 3 "full rows" aux1 aux16 aux17 aux18
