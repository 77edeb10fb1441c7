"""Config-5 full-state join loop for rocprofv3 / PMC passes / stamps (12.5M keys per GPU,
remove-heavy, 64 nodes, LWW ties): `C5_REPS` back-to-back dg_join2_async launches, then
one sync.  C5_KEYS overrides the size; C5_CONFIG=2 joins the config-2 replicas instead."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from delta_crdt_ex_amd import workloads as W  # noqa: E402
from delta_crdt_ex_amd.store import Context, Engine, Store  # noqa: E402

n_keys = int(os.environ.get("C5_KEYS", 12_500_000))
reps = int(os.environ.get("C5_REPS", 20))
dev = "cuda:0"
if os.environ.get("C5_CONFIG") == "2":
    a, b = W.config2()
else:
    a, b = W.config5(n_keys=n_keys, n_nodes=64, seed=5)
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
out = Store.empty(sa.n + sb.n, dev)
octx = Context.empty(0, ca.n + cb.n, dev)
eng = Engine(0)
d_counts = torch.zeros(8, dtype=torch.int64, device=dev)
launch = eng.prepare_join2(sa, ca, sb, cb, out, octx, d_counts)
launch()
eng.sync()
t0 = time.perf_counter()
for _ in range(reps):
    launch()
eng.sync()
dt = (time.perf_counter() - t0) / reps
n_out = int(d_counts[0].item())
print(f"config5 rows_in={sa.n + sb.n} rows_out={n_out} {dt * 1e3:.3f} ms/join "
      f"{36 * (sa.n + sb.n + n_out) / dt / 1e12:.2f} TB/s", flush=True)
if os.environ.get("C5_STAMPS"):
    import ctypes as C

    import numpy as np
    lib = eng.lib
    buf = np.zeros(65536 * 16, np.uint64)
    lib.dg_debug_join_stamps.argtypes = [C.c_void_p, C.c_size_t]
    assert lib.dg_debug_join_stamps(buf.ctypes.data, len(buf)) == 0
    np.save(os.environ["C5_STAMPS"], buf)
eng.close()
