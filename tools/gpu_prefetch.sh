#!/bin/bash
# A/B: seed-record prefetch (lib_v/pf2) vs the default build on the c4 mask-only, c4 full and
# client-masking launch shapes (tools/ab_variants.sh, alternating processes).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && bash tools/ab_variants.sh gpurun_out/ab_prefetch.log 3 "mask full client" pf2
