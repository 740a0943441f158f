# kernel timeline of the pair_queue reconstruction (tools/recon_trace.py QUEUE=1)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
QUEUE=1 EC_CUS=${EC_CUS:-24} EC_TERMS=${EC_TERMS:-2} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/qtrace -o run -- python3 $R/tools/recon_trace.py > $R/gpurun_out/qtrace.log 2>&1
