"""c5 seed recovery alone (bench.measure_recovery), for rocprofv3 runs.  Prints one JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from flamingo_amd import MaskEngine  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--D", type=int, default=962)
    ap.add_argument("--M", type=int, default=4055)
    ap.add_argument("--T", type=int, default=20)
    a = ap.parse_args()
    eng = MaskEngine(0)
    print(json.dumps(bench.measure_recovery(eng, torch, D=a.D, M=a.M, T=a.T, cpu_pool=True)))
