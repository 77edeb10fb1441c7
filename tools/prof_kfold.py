"""Config-3 dg_apply_deltas loop for rocprofv3 (tools/prof_kfold.sh): 10M-key state,
64 keyed deltas, `reps` one-pass folds."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from delta_crdt_ex_amd import workloads as W  # noqa: E402
from delta_crdt_ex_amd.store import Context, Engine, Store  # noqa: E402

n_keys = int(os.environ.get("KF_KEYS", 10_000_000))
reps = int(os.environ.get("KF_REPS", 10))
dev = "cuda:0"
base, deltas = W.config3(n_keys=n_keys, n_replicas=64, touch=0.01, seed=3)
sb = Store.from_numpy(*base["rows"], device=dev)
cb = Context.from_numpy(*base["ctx"], dev)
ds = [Store.from_numpy(*d["rows"], device=dev) for d in deltas]
dc = [Context.from_numpy(*d["ctx"], dev) for d in deltas]
ks = [torch.from_numpy(d["keys"].view(np.int64)).to(dev) for d in deltas]
out = Store.empty(sb.n + sum(d.n for d in ds), dev)
octx = Context.empty(0, cb.n + sum(c.n for c in dc), dev)
eng = Engine(0)
import time  # noqa: E402
for i in range(reps):
    t0 = time.perf_counter()
    o, c = eng.apply_deltas(sb, cb, ds, dc, ks, out=out, out_ctx=octx)
    print(f"rep {i}: {(time.perf_counter() - t0) * 1e3:.3f} ms, {o.n} rows", flush=True)
eng.close()
