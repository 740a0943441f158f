"""Build libflamingo_hip.so in-tree for gfx950 (hipcc, no JIT cache).

``python -m flamingo_amd.build`` or ``flamingo_amd.build.build()``.  The .so
lands in flamingo_amd/lib/ (git-ignored, shipped to the GPU box with the tree).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = [os.path.join(HERE, "csrc", f) for f in ("flm_kernels.hip", "flm_runtime.hip", "flm_p256.hip", "flm_comm.hip",
                                                        "flm_store.hip")]
HDRS = [os.path.join(HERE, "csrc", "flm_internal.h"),
        os.path.join(os.path.dirname(HERE), "include", "flamingo_hip.h")]
OUT = os.path.join(HERE, "lib", "libflamingo_hip.so")
ARCH = os.environ.get("FLM_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in SRC + HDRS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    # one hipcc per source, in parallel, then one link (the P-256 and kernel files dominate)
    objs = [os.path.join(os.path.dirname(OUT), os.path.basename(s) + ".o") for s in SRC]
    procs = []
    for s, o in zip(SRC, objs):
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-c", "-o", o, s]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), cmd))
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", OUT + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
