"""Debug: the 64-bit long-run path (long_run_set + lengths >= 2^31), per pipeline."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import repkiller_amd as rk
from long_runs import long_run_set
from oracle import rk_oracle as ro

def case():
    f = long_run_set(2500, seed=77)
    k = 8
    rng = np.random.default_rng(77)
    return rk.Frags(np.concatenate([f.x_start, rng.integers(1, 1_000_000, k).astype(np.uint64)]),
                    np.concatenate([f.y_start, rng.integers(1, 1_000_000, k).astype(np.uint64)]),
                    np.concatenate([f.length, np.full(k, 2**31 + 5, np.uint64)]),
                    np.concatenate([f.strand, np.full(k, ord('r'), np.uint8)]))

if __name__ == "__main__":
  for mode in sys.argv[1:]:
      ctx = rk.Context(0)
      if mode == "generic":
          ctx.set_pipeline("generic")
      g = case()
      L = 5_000_000_000
      try:
          r = ctx.classify(g, L, L, 0.05, 0.05)
          rc, gid, rep, order, ng = ro.classify(g.x_start, g.y_start, g.length, g.strand, L, L, 0.05, 0.05)
          print(mode, "ok", r.n_groups == ng and np.array_equal(r.out_order, order), ctx.stats(), flush=True)
      except rk.RkError as e:
          print(mode, "ERROR", e, flush=True)
      ctx.close()
