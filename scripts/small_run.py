"""BASELINE config 4's hashing alone (bench.py small_blobs), for profiling:
python scripts/small_run.py [reps] -> one JSON line"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch
    from glfs_amd import _native as N
    import bench
    N.set_device(0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    s = torch.cuda.Stream()
    print(json.dumps(bench.small_blobs(torch, N, s, ctypes.c_void_p(s.cuda_stream), reps=reps)),
          flush=True)
