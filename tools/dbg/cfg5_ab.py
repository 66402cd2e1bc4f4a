"""cfg5 (1B, 15 Gbp, repeat-rich): record vs generic pipeline on one GPU -- time,
fallback reason, and whether the two outputs are identical."""
import hashlib, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import repkiller_amd as rk
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
L = 15_000_000_000
f = rk.synth(n, L, seed=5, family_frac=0.95, copies=(100, 600), with_ident=False)
dev = torch.device("cuda", 0)
x = torch.from_numpy(f.x_start.view(np.int64)).to(dev); y = torch.from_numpy(f.y_start.view(np.int64)).to(dev)
ln = torch.from_numpy(f.length.view(np.int64)).to(dev); s = torch.from_numpy(f.strand).to(dev)
del f
digests = {}
for mode in sys.argv[2:] or ["auto", "generic"]:
    gid = torch.empty(n, dtype=torch.int32, device=dev); rep = torch.empty(n, dtype=torch.uint8, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    ctx = rk.Context(0)
    if mode == "generic":
        ctx.set_pipeline("generic")
    for i in range(2):
        torch.cuda.synchronize(); t = time.time()
        n_out, ng = ctx.classify_device(x, y, ln, s, gid, rep, order, L, L)
        torch.cuda.synchronize()
        print(mode, "run", i, round((time.time() - t) * 1e3, 1), "ms", ng, ctx.stats(), flush=True)
    ctx.close()
    h = hashlib.sha256()
    for a in (order[:n_out], gid[:n_out], rep[:n_out]):
        h.update(a.cpu().numpy().tobytes())
    digests[mode] = (ng, h.hexdigest())
    print(mode, digests[mode], flush=True)
    del gid, rep, order
    torch.cuda.empty_cache()
print("identical:", len(set(digests.values())) == 1, flush=True)
