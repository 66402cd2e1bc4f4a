"""Debug/timing: cfg5 (1B, 15 Gbp, repeat-rich) through classify_device: pipeline, time."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import repkiller_amd as rk
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
L = 15_000_000_000
t0 = time.time()
f = rk.synth(n, L, seed=5, family_frac=0.95, copies=(100, 600), with_ident=False)
print("synth", round(time.time() - t0, 1), flush=True)
dev = torch.device("cuda", 0)
x = torch.from_numpy(f.x_start.view(np.int64)).to(dev); y = torch.from_numpy(f.y_start.view(np.int64)).to(dev)
ln = torch.from_numpy(f.length.view(np.int64)).to(dev); s = torch.from_numpy(f.strand).to(dev)
del f
gid = torch.empty(n, dtype=torch.int32, device=dev); rep = torch.empty(n, dtype=torch.uint8, device=dev)
order = torch.empty(n, dtype=torch.int32, device=dev)
ctx = rk.Context(0)
for i in range(3):
    torch.cuda.synchronize(); t = time.time()
    n_out, ng = ctx.classify_device(x, y, ln, s, gid, rep, order, L, L)
    torch.cuda.synchronize()
    print("run", i, round((time.time() - t) * 1e3, 1), "ms", ng, ctx.stats(), flush=True)
