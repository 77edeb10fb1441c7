"""Host cost of one dg_join2_async launch (prepared, config 2) vs the wall time per join."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.store import Context, Engine, Store
dev = "cuda:0"
a, b = W.config2()
eng = Engine(0)
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
out = Store.empty(sa.n + sb.n, dev); octx = Context.empty(0, 8, dev)
d = torch.zeros(8, dtype=torch.int64, device=dev)
f = eng.prepare_join2(sa, ca, sb, cb, out, octx, d)
for _ in range(20): f()
eng.sync()
t0 = time.perf_counter()
for _ in range(200): f()
t1 = time.perf_counter()
eng.sync()
t2 = time.perf_counter()
print(f"host enqueue {((t1-t0)/200)*1e6:.1f} us/launch, wall {((t2-t0)/200)*1e6:.1f} us/launch")
