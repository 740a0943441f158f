cd $GRAFT_REPO_ROOT
for g in 4 2; do timeout -k 10 300 python -u tools/probes/rank8_overlap_probe.py --shapes --G=$g > gpurun_out/r03_rank_overlap_G$g.log 2>&1 || exit 1; done
