import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
import oracle_lib as O
from firedancer_amd import Verifier
from firedancer_amd import workload as W
dev = torch.device("cuda", 0)
for chunk, n in ((1 << 18, 1 << 22), (1 << 20, 1 << 22), (1 << 18, 1 << 20)):
    v = Verifier(device=0, chunk_sigs=chunk)
    b = W.make_batch_gpu(v, n, msg_sz=32, seed=0xc3, mix="c1", shared_msg=True)
    torch.cuda.synchronize()
    codes = torch.full((n,), 9, dtype=torch.int8, device=dev)
    v.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes)
    torch.cuda.synchronize()
    c = codes.cpu().numpy()
    bad = np.nonzero(c != 0)[0]
    print(chunk, n, "bad", bad.size, "codes", np.unique(c[bad], return_counts=True) if bad.size else "")
    if bad.size:
        per_chunk = np.bincount(bad // chunk, minlength=n // chunk)
        print(" per chunk", per_chunk.tolist()[:32])
        idx = bad[:200]
        pool = b.pool.cpu().numpy()
        sigs = b.sigs[torch.from_numpy(idx).to(dev)].cpu().numpy(); pubs = b.pubs[torch.from_numpy(idx).to(dev)].cpu().numpy()
        moff = np.zeros(idx.size, np.uint32); msz = np.full(idx.size, 32, np.uint32)
        exp = O.verify_many(sigs, pubs, pool, moff, msz)
        print(" oracle on first 200 bad:", np.unique(exp, return_counts=True))
        codes2 = torch.full((n,), 9, dtype=torch.int8, device=dev)
        v.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes2, stream="ctx")
        v.sync()
        c2 = codes2.cpu().numpy()
        print(" rerun on ctx stream bad:", int((c2 != 0).sum()), "same as first:", bool(np.array_equal(c, c2)))
        v.set_halfsize(0)
        codes3 = torch.full((n,), 9, dtype=torch.int8, device=dev)
        v.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes3)
        torch.cuda.synchronize()
        print(" full-length scalars bad:", int((codes3.cpu().numpy() != 0).sum()))
    v.close()
