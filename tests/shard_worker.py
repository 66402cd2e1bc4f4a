"""Rank body of the sharded-classification tests (tests/test_sharded.py).

Every rank rebuilds the same global fragment set, keeps its block of input rows
(rank r: rows [r*n//P, (r+1)*n//P), the file-order blocks rk_classify_sharded
expects), runs rk_classify_sharded on cuda:0 (several ranks share the one GPU
of the test box; collectives are torch.distributed gloo host callbacks) and
reports its share of the output to the parent.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def load_case(case):
    import repkiller_amd as rk
    if case["kind"] == "synth" and case["n"] == 0:
        import numpy as np
        e = np.empty(0, np.uint64)
        return rk.Frags(e, e.copy(), e.copy(), np.empty(0, np.uint8)), case["L"], case["L"]
    if case["kind"] == "long_runs":
        from long_runs import long_run_set
        return long_run_set(case["runs_len"], case["seed"]), case["L"], case["L"]
    if case["kind"] == "synth":
        f = rk.synth(case["n"], case["L"], seed=case["seed"], family_frac=case.get("ff", 0.8),
                     copies=tuple(case.get("copies", (2, 30))))
        if "long_row" in case:  # one row outside the 16-B record (length >= 2^24)
            k = case["long_row"]
            f.x_start[k], f.y_start[k], f.length[k] = 1000, 1000, (1 << 24) + 5
        return f, case["L"], case["L"]
    db = rk.FragmentsDatabase(case["path"])
    return db.frags, db.len_x_hdr, db.len_y_hdr


def worker(rank, world, port, cases, q, comm_kind="host", env=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.update(env or {})  # read once by the library (e.g. RK_SHARD_GENERIC)
    import numpy as np
    import torch
    import torch.distributed as dist
    import repkiller_amd as rk
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = rk.Context(0)
        comm = (rk.Comm.rccl(rank, world, 0) if comm_kind == "rccl"
                else rk.Comm.torch_host(rank, world))
        for ci, case in enumerate(cases):
            f, lx, ly = load_case(case)
            n = f.n
            a, b = rank * n // world, (rank + 1) * n // world
            dev = torch.device("cuda:0")

            def t(arr, dt):
                return torch.from_numpy(arr[a:b].astype(dt, copy=True)).to(dev)
            x, y = t(f.x_start, "int64"), t(f.y_start, "int64")
            ln, s = t(f.length, "int64"), t(f.strand, "uint8")
            lr = case.get("lr", 0.3)
            if case.get("bad_rank") == rank:
                lr = -1.0  # this rank alone fails its argument check
            if case.get("fault_rank") == rank:  # rk_shard.hip fault_here(): fail at that stage
                os.environ["RK_TEST_FAULT"] = case["fault"]
            # repeat: the same call again on the same context (the second finds
            # every stage's sizes known: the fast path's no-agreement stages);
            # every repetition must give the same share, the last one's
            # statistics are reported with the list of all
            reps, first, stats = case.get("repeat", 1), None, []
            try:
                for _ in range(reps):
                    out = rk.classify_sharded(ctx, comm, x, y, ln, s, lx, ly, lr,
                                              case.get("pr", 0.3), case.get("lead_in", -1))
                    stats.append(rk.shard_stats(ctx))
                    r = out.result
                    share = (out.out_offset, out.n_out_total, out.n_groups, r.out_order, r.gid,
                             r.repval)
                    if first is None:
                        first = share
                    else:
                        assert share[:3] == first[:3], (share[:3], first[:3])
                        for a, b in zip(share[3:], first[3:]):
                            assert np.array_equal(a, b), "repeated call differs"
            except rk.RkError as e:
                q.put((ci, rank, "error", e.code))
                continue
            finally:
                os.environ.pop("RK_TEST_FAULT", None)
            st = dict(stats[-1])
            st["calls"] = stats
            q.put((ci, rank, "ok", first + (st,)))
        comm.close()
        ctx.close()
    except Exception:  # noqa: BLE001 -- surfaced to the parent
        import traceback
        q.put((-1, rank, "crash", traceback.format_exc()))
    finally:
        dist.destroy_process_group()
