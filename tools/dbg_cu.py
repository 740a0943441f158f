import sys, os, faulthandler
faulthandler.enable()
sys.path.insert(0, os.getcwd())
import torch, numpy as np
from flamingo_amd import MaskEngine
eng = MaskEngine(0)
print("cu_count", eng.cu_count(), flush=True)
s = eng.cu_stream(list(range(0, 256, 16)))
print("stream", hex(s.cuda_stream), flush=True)
x = torch.zeros(1 << 20, dtype=torch.int32, device="cuda")
ev0 = torch.cuda.Event(); ev0.record(); s.wait_event(ev0)
x += 1
torch.cuda.synchronize()
print("add on masked stream ok", int(x.sum()), flush=True)
seeds = torch.zeros((4, 32), dtype=torch.uint8, device="cuda")
signs = torch.ones(4, dtype=torch.int8, device="cuda")
rows = torch.zeros((2, 4096), dtype=torch.int32, device="cuda")
out = torch.empty(4096, dtype=torch.int32, device="cuda")
eng.aggregate_unmask_dev(rows, seeds, signs, out, L=4096, stream=s)
s.synchronize()
print("aggregate on masked stream ok", flush=True)
ev = torch.cuda.Event(); ev.record(torch.cuda.current_stream()); s.wait_event(ev)
del x
torch.cuda.synchronize()
eng.close()
print("closed", flush=True)
