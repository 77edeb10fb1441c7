"""read/1 on config 5's joined state and a Merkle build + diff (config-4 shape) for
rocprofv3: kernel times of segred_kernel<Read>, the Merkle kernels."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from delta_crdt_ex_amd import workloads as W  # noqa: E402
from delta_crdt_ex_amd.store import Context, Engine, Store  # noqa: E402

dev = "cuda:0"
eng = Engine(0)
a, b = W.config5(n_keys=int(os.environ.get("RD_KEYS", 12_500_000)), n_nodes=64, seed=5)
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
out, octx = eng.join2(sa, ca, sb, cb)
for _ in range(10):
    k, v = eng.read_lww(out)
print("read", out.n, "rows ->", k.numel(), "keys", flush=True)
m1, m2 = W.merkle_pair(n_keys=1_000_000, diff_frac=0.01, seed=4)
s1, s2 = Store.from_numpy(*m1["rows"], device=dev), Store.from_numpy(*m2["rows"], device=dev)
t1, t2 = eng.merkle_build(s1, 18), eng.merkle_build(s2, 18)
for _ in range(10):
    eng.merkle_build(s1, 18, t1)
    eng.merkle_build(s2, 18, t2)
    d = eng.merkle_diff(t1, t2)
print("merkle diff", d.numel(), flush=True)
eng.close()
