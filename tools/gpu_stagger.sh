R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && bash tools/ab_variants.sh gpurun_out/ab_stagger.log 3 "mask full" stag4 stag16 stag64 && \
timeout -k 10 300 python3 -u tools/ab_items.py --workloads mask,full --variants auto --subtiles 1 --min-items 1024,4096,16384 --rounds 3 --reps 5 > gpurun_out/ab_min_items.log 2>&1
