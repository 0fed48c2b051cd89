"""Refs and ctext digests of one device-resident batch post through whichever
library GLFSX_LIB names (tests/test_gpu_variants.py runs it once per variant
build in a child process and compares with the shipped library and the
oracle).  usage: GLFSX_LIB=... python scripts/variant_refs.py TOTAL BS SEED"""
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def digests(total, bs, seed):
    import torch
    from glfs_amd import _native as N
    N.set_device(0)
    n = (total + bs - 1) // bs
    data = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    ct = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    refs = torch.empty(64 * n, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, total, seed, None))
    salt = bytes(range(32))
    N.check(N.lib.glfsx_post_batch_device(salt, data.data_ptr(), total, bs, ct.data_ptr(),
                                          refs.data_ptr(), None, None))
    torch.cuda.synchronize()
    r = refs.cpu().numpy().tobytes()
    c = ct[:total].cpu().numpy().tobytes()
    return {"refs": hashlib.sha256(r).hexdigest(), "ctext": hashlib.sha256(c).hexdigest(),
            "lib": os.path.basename(N.LIB_PATH)}


if __name__ == "__main__":
    total, bs, seed = (int(x) for x in sys.argv[1:4])
    print(json.dumps(digests(total, bs, seed)), flush=True)
