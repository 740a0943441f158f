"""The hash-to-curve table launch alone (bench.measure_h2c), for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace --stats -d gpurun_out/h2c -o run -- python3 tools/h2c_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch
    import bench
    from flamingo_amd import MaskEngine
    torch.cuda.set_device(0)
    eng = MaskEngine(0)
    print(json.dumps(bench.measure_h2c(eng, torch, reps=10, cpu_sample=int(sys.argv[1]) if len(sys.argv) > 1 else 512)),
          flush=True)
    eng.close()
