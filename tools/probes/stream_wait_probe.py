"""Debug probe: does a stream wait made through torch order a library launch after torch's
default-stream work?  x is written on the default stream behind a long kernel; then
  A: torch clone on an ExternalStream(flm_ctx_stream) after ext.wait_stream(default)
  B: the library's rows-only round on that ExternalStream after the same wait
  C: the library's round on a torch.cuda.Stream() after wait_stream(default)
  D: the library's round on the default stream itself (stream=None)
and each result is compared with the expected value."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

dev = torch.device("cuda", 0)
eng = MaskEngine(0)
h = eng.lib.flm_ctx_stream(eng.ctx)
ext = torch.cuda.ExternalStream(h, device=dev)
print("ctx stream", hex(h), "default stream", torch.cuda.current_stream().cuda_stream, flush=True)
L = 1 << 22


def long_kernel(n=8192, reps=12):
    a = torch.ones((n, n), device=dev)
    for _ in range(reps):
        a = a @ a * 1e-4
    return a


for trial in range(2):
    for name in ("A", "B", "C", "D"):
        x = torch.zeros((1, L), dtype=torch.int32, device=dev)
        y = torch.zeros(L, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        keep = long_kernel()
        x.fill_(5 + trial)
        if name == "A":
            ext.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(ext):
                y.copy_(x[0])
            torch.cuda.current_stream().wait_stream(ext)
        elif name == "B":
            ext.wait_stream(torch.cuda.current_stream())
            eng.aggregate_unmask_dev(x, None, None, y, L=L, stream=ext)
            torch.cuda.current_stream().wait_stream(ext)
        elif name == "C":
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            eng.aggregate_unmask_dev(x, None, None, y, L=L, stream=s)
            torch.cuda.current_stream().wait_stream(s)
        else:
            eng.aggregate_unmask_dev(x, None, None, y, L=L)
        torch.cuda.synchronize()
        bad = int((y != 5 + trial).sum().item())
        print(f"trial {trial} {name}: {bad} of {L} slots wrong", flush=True)
        del keep
eng.close()
