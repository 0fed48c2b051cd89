import sys, ctypes, torch
sys.path.insert(0, '.')
from glfs_amd import _native as N
from oracle import oracle as O
torch.cuda.init()
def run(bs, total, salt=bytes(32)):
    data = O.fill_splitmix(total, total)
    n = (total + bs - 1)//bs
    t = torch.empty(total + 64, dtype=torch.uint8, device='cuda'); t[:total].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    refs = torch.zeros(64*n, dtype=torch.uint8, device='cuda'); torch.cuda.synchronize()
    N.check(N.lib.glfsx_dek_batch_device(salt, t.data_ptr(), total, bs, refs.data_ptr(), None)); torch.cuda.synchronize()
    dek_only = bytes(refs.cpu().numpy().tobytes())
    N.check(N.lib.glfsx_cid_batch_device(t.data_ptr(), total, bs, None, refs.data_ptr(), None, None)); torch.cuda.synchronize()
    full = bytes(refs.cpu().numpy().tobytes())
    out = []
    for j in range(n):
        blk = data[j*bs:(j+1)*bs]
        r, c = O.post(salt, blk)
        out.append((j, len(blk), dek_only[64*j+32:64*j+64] == r[32:], full[64*j+32:64*j+64]==r[32:], full[64*j:64*j+32]==r[:32]))
    print(bs, total, out)
for bs, total in [(300000, 300001), (300000, 300000+5), (300000, 2*300000+1), (4096, 4097), (2048*256, 2048*256+1), (1<<20, (1<<20)+1), (1<<20, (1<<20)+3000), (300000, 300001+3000)]:
    run(bs, total)
