"""dg_join2_changes vs dg_join2 on config 2 for rocprofv3 (kernel times of both)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from delta_crdt_ex_amd import workloads as W  # noqa: E402
from delta_crdt_ex_amd.store import Context, Engine, Store  # noqa: E402

dev = "cuda:0"
a, b = W.config2()
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
out = Store.empty(sa.n + sb.n, dev)
octx = Context.empty(0, ca.n + cb.n, dev)
eng = Engine(0)
for name, fn in (("join2", lambda: eng.join2(sa, ca, sb, cb, out=out, out_ctx=octx)),
                 ("changes", lambda: eng.join2_changes(sa, ca, sb, cb, out=out, out_ctx=octx))):
    fn()
    t0 = time.perf_counter()
    for _ in range(20):
        fn()
    print(f"{name}: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us/call", flush=True)
eng.close()
