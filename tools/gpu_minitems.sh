mkdir -p gpurun_out
for mi in 1024 2048 4096; do
  echo "MIN_ITEMS=$mi" >> gpurun_out/q_minitems.log
  MIN_ITEMS=$mi EC_CUS=24,32 SPLIT=0,q CU_PICK=first timeout -k 10 200 python -u tools/recon_split_sweep.py >> gpurun_out/q_minitems.log 2>&1 || exit $?
done
