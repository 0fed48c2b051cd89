import ctypes, json, sys
sys.path.insert(0, '.')
import torch
from glfs_amd import _native as N
import bench
N.set_device(0)
s = torch.cuda.Stream()
for n in (1 << 20, 1 << 22, 1 << 24):
    r = bench.small_blobs(torch, N, s, ctypes.c_void_p(s.cuda_stream), n=n, reps=3)
    print(n, r["value"], r["ms"], flush=True)
    torch.cuda.empty_cache()
