"""Time glfsx_tree_encode_device alone on config 4's tree (1,048,576 entries,
"%07d" names, type "blob", random roots): HIP events on the launch stream,
min / median over reps.  usage: python scripts/tree_enc_time.py [reps]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import numpy as np
    import torch
    from glfs_amd import _native as N
    torch.cuda.set_device(0)
    N.set_device(0)
    n = 1 << 20
    cuda = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    names = cuda(np.frombuffer("".join("%07d" % i for i in range(n)).encode(), dtype=np.uint8))
    name_offs = cuda((np.arange(n + 1, dtype=np.int64) * 7))
    types = cuda(np.frombuffer(b"blob" * n, dtype=np.uint8))
    type_offs = cuda(np.arange(n + 1, dtype=np.int64) * 4)
    modes = cuda(np.full(n, 0o644, dtype=np.int32))
    sizes = cuda(np.full(n, 4096, dtype=np.int64))
    bss = cuda(np.full(n, 2 << 20, dtype=np.int64))
    roots = torch.randint(0, 256, (64 * n,), dtype=torch.uint8, device="cuda")
    lines = torch.empty(260 * n, dtype=torch.uint8, device="cuda")
    total = ctypes.c_uint64()
    stream = torch.cuda.current_stream()

    def run():
        N.check(N.lib.glfsx_tree_encode_device(n, names.data_ptr(), name_offs.data_ptr(),
                                               modes.data_ptr(), types.data_ptr(),
                                               type_offs.data_ptr(), roots.data_ptr(),
                                               sizes.data_ptr(), bss.data_ptr(),
                                               lines.data_ptr(), lines.numel(), None,
                                               ctypes.byref(total), None))
    run()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run()
        e1.record(stream)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    print(json.dumps({"lib": os.environ.get("GLFSX_LIB", "libglfsx.so"), "bytes": total.value,
                      "us_min": round(ts[0], 1), "us_med": round(ts[len(ts) // 2], 1)}))


if __name__ == "__main__":
    main()
