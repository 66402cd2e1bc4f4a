#!/usr/bin/env python3
"""Full-size check of the sharded path on ONE GPU: cfg4 (200M fragments, 3 Gbp).

P ranks (default 4) share the box's GPU and exchange through gloo host
callbacks; rank r holds rows [r*n, (r+1)*n) of ONE 200M-fragment set
(block r = synth(n, L, seed=3+r), as bench.py's sharded leg builds it).  The
concatenated shares are compared bit for bit with the single-device path on
the concatenated input.  Prints one JSON line (timings, equality).

  python tools/shard_scale_check.py [--ranks 4] [--n 50000000] [--lead-in -1]
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def worker(rank, world, port, n, L, lead_in, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import repkiller_amd as rk
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = rk.Context(0)
    comm = rk.Comm.torch_host(rank, world)
    f = rk.synth(n, L, seed=3 + rank)
    dev = torch.device("cuda", 0)
    t = [torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(dev)
         for a in (f.x_start, f.y_start, f.length, f.strand)]
    dist.barrier()
    t0 = time.perf_counter()
    out = rk.classify_sharded(ctx, comm, *t, L, L, 0.3, 0.3, lead_in)
    dt = time.perf_counter() - t0
    r = out.result
    np.save(os.path.join(outdir, f"order{rank}.npy"), r.out_order)
    np.save(os.path.join(outdir, f"gid{rank}.npy"), r.gid)
    np.save(os.path.join(outdir, f"rep{rank}.npy"), r.repval)
    with open(os.path.join(outdir, f"meta{rank}.json"), "w") as fh:
        json.dump({"offset": out.out_offset, "total": out.n_out_total, "groups": out.n_groups,
                   "seconds": dt, "stats": rk.shard_stats(ctx)}, fh)
    comm.close()
    ctx.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--n", type=int, default=50_000_000)
    ap.add_argument("--genome", type=int, default=3_000_000_000)
    ap.add_argument("--lead-in", type=int, default=-1)
    args = ap.parse_args()
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=worker, args=(r, args.ranks, port, args.n, args.genome,
                                                  args.lead_in, d)) for r in range(args.ranks)]
        t0 = time.perf_counter()
        for p in procs:
            p.start()
        for p in procs:
            p.join()
            assert p.exitcode == 0, p.exitcode
        wall = time.perf_counter() - t0
        metas = [json.load(open(os.path.join(d, f"meta{r}.json"))) for r in range(args.ranks)]
        parts = sorted(range(args.ranks), key=lambda r: metas[r]["offset"])
        cat = lambda nm: np.concatenate([np.load(os.path.join(d, f"{nm}{r}.npy")) for r in parts])  # noqa: E731
        order, gid, rep = cat("order"), cat("gid"), cat("rep")

    import torch
    import repkiller_amd as rk
    blocks = [rk.synth(args.n, args.genome, seed=3 + r) for r in range(args.ranks)]
    full = rk.Frags(*[np.concatenate([getattr(b, k) for b in blocks])
                      for k in ("x_start", "y_start", "length", "strand")])
    del blocks
    ctx = rk.Context(0)
    dev = torch.device("cuda", 0)
    N = full.n
    t = [torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(dev)
         for a in (full.x_start, full.y_start, full.length, full.strand)]
    g = torch.empty(N, dtype=torch.int32, device=dev)
    rp = torch.empty(N, dtype=torch.uint8, device=dev)
    od = torch.empty(N, dtype=torch.int32, device=dev)
    ctx.classify_device(*t, g, rp, od, args.genome, args.genome)  # sizes the workspace
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    n_out, ng = ctx.classify_device(*t, g, rp, od, args.genome, args.genome)
    torch.cuda.synchronize()
    single_s = time.perf_counter() - t1
    same = (n_out == order.shape[0] and ng == metas[0]["groups"]
            and np.array_equal(od[:n_out].cpu().numpy().view(np.uint32), order)
            and np.array_equal(g[:n_out].cpu().numpy().view(np.uint32), gid)
            and np.array_equal(rp[:n_out].cpu().numpy(), rep))
    print(json.dumps({
        "check": "sharded vs single-device, bit-exact", "identical": bool(same),
        "fragments": N, "genome_bp": args.genome, "ranks": args.ranks,
        "comm": "gloo host callbacks (ranks share one GPU)", "groups": ng, "rows": n_out,
        "single_device_s": round(single_s, 4),
        "sharded_s_per_rank": [round(m["seconds"], 3) for m in metas],
        "sharded_wall_s_incl_startup": round(wall, 1),
        "shard_stats": [m["stats"] for m in metas],
    }), flush=True)
    assert same


if __name__ == "__main__":
    main()
