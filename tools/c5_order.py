"""Config-5 join launch time (HIP events, 20 back-to-back launches) with the engine
created before (C5_ORDER=engine_first) or after (data_first) the stores: tools/prof_c5.py
(data first) measured the stream kernel ~10 % slower than bench.py's config5_rate (engine
first) on the same box and data.  Prints the columns' device addresses modulo 2 MB too.
C5_WARM=n: n synchronous joins first (bench.py's _timed does 6); C5_DEL=1: the host
arrays freed once uploaded (bench.py's `del a, b`)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from delta_crdt_ex_amd import workloads as W  # noqa: E402
from delta_crdt_ex_amd.store import Context, Engine, Store  # noqa: E402

order = os.environ.get("C5_ORDER", "engine_first")
dev = "cuda:0"
a, b = W.config5_shard(0, 1, keys_per_rank=12_500_000)
eng = Engine(0) if order == "engine_first" else None
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
out = Store.empty(sa.n + sb.n, dev)
octx = Context.empty(0, ca.n + cb.n, dev)
if eng is None:
    eng = Engine(0)
if os.environ.get("C5_DEL") == "1":
    del a, b
d_counts = torch.zeros(8, dtype=torch.int64, device=dev)
launch = eng.prepare_join2(sa, ca, sb, cb, out, octx, d_counts)
for _ in range(int(os.environ.get("C5_WARM", "0"))):
    launch()
    eng.sync()
res = []
for rep in range(3):
    launch()
    eng.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(eng.stream)
    for _ in range(20):
        launch()
    e1.record(eng.stream)
    eng.sync()
    res.append(e0.elapsed_time(e1) * 1e3 / 20)
mods = {n: [(t.data_ptr() % (2 << 20)) >> 12 for t in (s.key, s.val, s.ts, s.node, s.cnt)]
        for n, s in (("a", sa), ("b", sb), ("out", out))}
print(f"{order} warm={os.environ.get('C5_WARM', '0')} del={os.environ.get('C5_DEL', '0')}: us per launch {' '.join(f'{x:.1f}' for x in res)}  addr%2MB (4K pages) {mods}", flush=True)
eng.close()
