set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash tools/gpu.sh r05g "tests:ec_ or h2c or teardown"
for g in 1 2 4; do
  timeout -k 10 120 python tools/ec_bench.py --D 121 --T 20 --scalars lagrange --coop 2 --row-terms $g --reps 20 --cpu-sample 10 > $O/r05g_ecbench_row$g.log 2>&1
  tail -1 $O/r05g_ecbench_row$g.log | cut -c1-300
done
timeout -k 10 300 python -u tools/probes/rank8_overlap_probe.py --straus > $O/r05g_rank8_straus.log 2>&1
cat $O/r05g_rank8_straus.log | grep -v amdgpu.ids
