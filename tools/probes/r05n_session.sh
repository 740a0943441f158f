# kernel trace of the c5 agent simulation (4 iterations): are the slow "unmask + D2H" walls GPU time?
set -e
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/r05n_simtrace -o run -- python3 -u -m flamingo_amd.abides -c flamingo -n 4096 --vector_len 1048576 -i 4 --dropout 0.01 --latency deterministic -k -s 5 > $O/r05n_simtrace.log 2>&1
grep "iteration [0-9]*:" $O/r05n_simtrace.log
