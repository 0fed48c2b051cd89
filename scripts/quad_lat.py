"""Latency-mode kernels of one message (glfsx_post_batch_device, n = 1) for a
range of message sizes, to time the index node's dependent chain: run under
rocprofv3 --kernel-trace and read k_quad / k_decrypt_lines durations per
size (the sizes run in order, REPS posts each, with a marker k_fill between).
usage: rocprofv3 --kernel-trace -d OUT -o run -- python scripts/quad_lat.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = [64, 1024, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20]
REPS = 20


def main():
    import torch
    from glfs_amd import _native as N
    N.set_device(0)
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    mx = max(SIZES)
    data = torch.empty(mx, dtype=torch.uint8, device="cuda")
    ct = torch.empty(mx, dtype=torch.uint8, device="cuda")
    refs = torch.empty(64, dtype=torch.uint8, device="cuda")
    salt = bytes(32)
    for L in SIZES:
        # marker between sizes: a fill of the buffer
        N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, mx, L, sp))
        for _ in range(REPS):
            N.check(N.lib.glfsx_post_batch_device(salt, data.data_ptr(), L, L, ct.data_ptr(),
                                                  refs.data_ptr(), None, sp))
        s.synchronize()
    print("sizes", SIZES, "reps", REPS)


if __name__ == "__main__":
    main()
