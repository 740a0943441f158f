"""Summarise the kernel launches of a HIP runtime log (AMD_LOG_LEVEL=4, stderr of the traced run):
each dispatched kernel's name and how many times it ran.  Used by tools/gpu.sh step `rccl` to show
which RCCL kernels tools/rccl_clique_smoke.py launched (the rocprofv3 trace of the same script
crashes at process exit, after every check has passed, when RCCL was loaded).
Usage: python tools/kernel_log_summary.py LOG [OUT.json]"""
import collections
import json
import re
import sys

src = sys.argv[1]
names = collections.Counter()
pat = re.compile(r"ShaderName\s*:\s*(\S+)")
with open(src, errors="replace") as f:
    for line in f:
        m = pat.search(line)
        if m:
            names[m.group(1)] += 1
rccl = {k: v for k, v in names.items() if "nccl" in k.lower() or "rccl" in k.lower()}
res = {"log": src, "kernels_launched": sum(names.values()), "distinct": len(names),
       "rccl_kernels": rccl, "all": dict(names.most_common())}
out = json.dumps(res, indent=1)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out + "\n")
print(json.dumps({"kernels_launched": res["kernels_launched"], "rccl_kernels": rccl}))
