"""Diagnostic (round 3): how many k_small_q fine items took the dense path vs
the one-lane-per-blob fallback (needs a -DGLFSX_SFINE_CNT=1 build of the
fine-item experiment)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from glfs_amd import _native as N
    N.set_device(0)
    s = torch.cuda.Stream()
    r = bench.small_blobs(torch, N, s, ctypes.c_void_p(s.cuda_stream), n=1 << 20, reps=1)
    lib = ctypes.CDLL(os.environ["GLFSX_LIB"])
    out = (ctypes.c_uint32 * 2)()
    lib.glfsx_debug_sfine(out)
    print("value", r["value"], "dense items", out[0], "fallback items", out[1])


if __name__ == "__main__":
    main()
