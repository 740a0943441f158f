"""Run a module (``python tools/probes/mempolicy_run.py MODULE ARGS...``) with the process's memory
policy set to MPOL_LOCAL first (set_mempolicy(2), x86-64 syscall 238), before anything allocates.

Why (the agent run's unmask stall): an explicit task policy carries no
MPOL_F_MOF flag, so the kernel's automatic NUMA balancing (task_numa_work) skips this process's
VMAs.  Its scans change page protections (PROT_NONE hinting faults); an MMU-notifier invalidation
over a HIP pinned host buffer (a KFD userptr allocation) makes KFD evict the process's GPU queues
until the buffer is validated again.  If the stall is that, this run does not stall."""
import ctypes
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
MPOL_LOCAL = 4
SYS_set_mempolicy = 238  # x86-64

libc = ctypes.CDLL(None, use_errno=True)
rc = libc.syscall(SYS_set_mempolicy, MPOL_LOCAL, None, 0)
if rc != 0:
    print(f"mempolicy_run: set_mempolicy(MPOL_LOCAL) failed, errno {ctypes.get_errno()}", file=sys.stderr)
    sys.exit(3)
print(f"mempolicy_run: MPOL_LOCAL set for pid {os.getpid()}", flush=True)
mod = sys.argv[1]
sys.argv = [mod] + sys.argv[2:]
runpy.run_module(mod, run_name="__main__", alter_sys=True)
