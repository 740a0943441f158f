"""Run the agent simulation (``python tools/probes/evict_probe_run.py ARGS...`` = ``python -m
flamingo_amd.abides ARGS...``) and read KFD's per-process queue-eviction counter around every
server unmask: /sys/class/kfd/kfd/proc/<pid>/stats_<gpuid>/evicted_ms is the cumulative time this
process's GPU queues have spent evicted (unmapped by the kernel driver).  If the agent run's
unmask stall (commands enqueued, the GPU idle for 15-45 ms before the first
starts) is a queue eviction, the counter grows by about the stall during that unmask.

Prints one line per unmask: wall ms, the store's device ms, evicted_ms before / after / delta
for every GPU of the process, plus the counter at the start and end of the run."""
import glob
import os
import runpy
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
PID = os.getpid()
if "--thp-off" in sys.argv:  # transparent huge pages off for this process (prctl PR_SET_THP_DISABLE), first thing
    import ctypes
    sys.argv.remove("--thp-off")
    if ctypes.CDLL(None, use_errno=True).prctl(41, 1, 0, 0, 0) != 0:
        sys.exit(f"evict_probe_run: prctl(PR_SET_THP_DISABLE) failed, errno {ctypes.get_errno()}")
    print("[evict_probe] THP disabled for this process", flush=True)


def evicted():
    """evicted_ms of every KFD process directory visible (sysfs names them by the HOST pid, which a
    container's getpid() does not give: on the box this process is the only GPU user)."""
    out = {}
    for f in sorted(glob.glob("/sys/class/kfd/kfd/proc/*/stats_*/evicted_ms")):
        key = f.split("/")[-3] + "/" + f.split("/")[-2]
        try:
            with open(f) as fh:
                out[key] = int(fh.read().strip() or 0)
        except OSError as e:
            out[key] = f"error {e}"
    return out


from flamingo_amd import ingest  # noqa: E402

_unmask = ingest.VectorStore.unmask
_n = [0]


def unmask(self, seeds, signs):
    e0 = evicted()
    t0 = time.perf_counter()
    out = _unmask(self, seeds, signs)
    wall = (time.perf_counter() - t0) * 1e3
    e1 = evicted()
    try:
        gpu = self.unmask_ms()
    except Exception:
        gpu = float("nan")
    _n[0] += 1
    delta = {k: (e1.get(k, 0) - v) if isinstance(v, int) and isinstance(e1.get(k), int) else None
             for k, v in e0.items()}
    print(f"[evict_probe] unmask {_n[0]}: wall {wall:.3f} ms, GPU {gpu:.3f} ms, evicted_ms before {e0} after {e1} "
          f"delta {delta}", flush=True)
    return out


ingest.VectorStore.unmask = unmask
print(f"[evict_probe] pid {PID}; kfd proc dirs: {glob.glob('/sys/class/kfd/kfd/proc/*')}; "
      f"start {evicted()}", flush=True)
sys.argv = ["flamingo_amd.abides"] + sys.argv[1:]
try:
    runpy.run_module("flamingo_amd.abides", run_name="__main__", alter_sys=True)
finally:
    dirs = glob.glob("/sys/class/kfd/kfd/proc/*")
    print(f"[evict_probe] end {evicted()}; kfd proc dirs {dirs}; files of the first "
          f"{sorted(os.listdir(dirs[0])) if dirs else None}", flush=True)
