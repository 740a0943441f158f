R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for S in pow2 lagrange; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ecsplit_$S -o run -- python3 $R/tools/ec_bench.py --D 120 --T 20 --reps 10 --cpu-sample 1 --scalars $S --coop 1 > $R/gpurun_out/ecsplit_$S.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d $R/gpurun_out/ecsplit_pmc -o run -- python3 $R/tools/ec_bench.py --D 120 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop 1 > $R/gpurun_out/ecsplit_pmc.log 2>&1 || exit $?
