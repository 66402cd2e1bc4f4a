"""Probe: torch + librepkiller_amd in one process (HIP runtime sharing) and a first timing."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1]
if order == "torch_first":
    import torch
    torch.cuda.init()
    print("torch devices", torch.cuda.device_count(), flush=True)
import numpy as np
import repkiller_amd as rk
from oracle import rk_oracle as ro
ctx = rk.Context(0)
f = rk.synth(100_000, 5_000_000, seed=7)
r = ctx.classify(f, 5_000_000, 5_000_000)
rc, g2, r2, o2, ng2 = ro.classify(f.x_start, f.y_start, f.length, f.strand, 5_000_000, 5_000_000)
print("host path ok", np.array_equal(r.out_order, o2), flush=True)
if order == "torch_first":
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(f.x_start.view(np.int64)).to(dev)
    y = torch.from_numpy(f.y_start.view(np.int64)).to(dev)
    ln = torch.from_numpy(f.length.view(np.int64)).to(dev)
    s = torch.from_numpy(f.strand).to(dev)
    gid = torch.empty(f.n, dtype=torch.int32, device=dev)
    rep = torch.empty(f.n, dtype=torch.uint8, device=dev)
    order_t = torch.empty(f.n, dtype=torch.int32, device=dev)
    n_out, ng = ctx.classify_device(x, y, ln, s, gid, rep, order_t, 5_000_000, 5_000_000)
    print("device path ok", np.array_equal(order_t[:n_out].cpu().numpy().view(np.uint32), o2), flush=True)
for n, L in ((1_000_000, 100_000_000), (10_000_000, 600_000_000), (50_000_000, 3_000_000_000)):
    t = time.time(); f = rk.synth(n, L, seed=3); tg = time.time() - t
    for it in range(3):
        t = time.time(); r = ctx.classify(f, L, L); dt = time.time() - t
        st = ctx.stats()
        print(f"n={n} L={L} gen={tg:.2f}s classify={dt*1e3:.1f}ms device={st['device_ms']:.1f}ms "
              f"xs={st['x_sweeps']} ys={st['y_sweeps']} jr={st['jump_rounds']} groups={st['n_groups']}", flush=True)
