"""Run a module (``python tools/probes/mempolicy_run.py [--thp-off] [--no-mpol] MODULE ARGS...``)
with the process's memory policy set to MPOL_LOCAL first (set_mempolicy(2), x86-64 syscall 238),
and optionally transparent huge pages off for it (prctl(PR_SET_THP_DISABLE)), before anything
allocates.

Why (the agent run's unmask stall): an explicit task policy carries no
MPOL_F_MOF flag, so the kernel's automatic NUMA balancing (task_numa_work) skips this process's
VMAs.  Its scans change page protections (PROT_NONE hinting faults); an MMU-notifier invalidation
over a HIP pinned host buffer (a KFD userptr allocation) makes KFD evict the process's GPU queues
until the buffer is validated again.  khugepaged collapsing pages under such a buffer does the same;
--thp-off keeps the process's memory out of its reach."""
import ctypes
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
MPOL_LOCAL = 4
SYS_set_mempolicy = 238  # x86-64
PR_SET_THP_DISABLE = 41

libc = ctypes.CDLL(None, use_errno=True)
args = sys.argv[1:]
thp_off = "--thp-off" in args
mpol = "--no-mpol" not in args
args = [a for a in args if a not in ("--thp-off", "--no-mpol")]
if mpol:
    if libc.syscall(SYS_set_mempolicy, MPOL_LOCAL, None, 0) != 0:
        print(f"mempolicy_run: set_mempolicy(MPOL_LOCAL) failed, errno {ctypes.get_errno()}", file=sys.stderr)
        sys.exit(3)
if thp_off:
    if libc.prctl(PR_SET_THP_DISABLE, 1, 0, 0, 0) != 0:
        print(f"mempolicy_run: prctl(PR_SET_THP_DISABLE) failed, errno {ctypes.get_errno()}", file=sys.stderr)
        sys.exit(3)
print(f"mempolicy_run: pid {os.getpid()} MPOL_LOCAL {mpol} THP off {thp_off}", flush=True)
mod = args[0]
sys.argv = [mod] + args[1:]
runpy.run_module(mod, run_name="__main__", alter_sys=True)
