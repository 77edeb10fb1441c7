"""Wall time of one SYNCHRONOUS dg_join2 call on config 2, as a NIF would pay it: the C-ABI
called directly with pre-marshalled arguments (no Python wrapper work per call), next to the
asynchronous launch rate and the stream kernel's own time.  DG_LIB_PATH picks the build."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.store import Context, Engine, Store

dev = "cuda:0"
a, b = W.config2()
eng = Engine(0)
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
out = Store.empty(sa.n + sb.n, dev)
octx = Context.empty(0, ca.n + cb.n, dev)
torch.cuda.synchronize()
args = [sa.abi(), ca.abi(), sb.abi(), cb.abi(), out.abi(), octx.abi()]
refs = [C.byref(x) for x in args]
nk = C.c_uint64(0)
kp = eng._keys(None)[0]
lib, h = eng.lib, eng.h


def sync_join():
    rc = lib.dg_join2(h, refs[0], refs[1], refs[2], refs[3], kp, 0, refs[4], refs[5])
    assert rc == 0, rc


def timed(fn, reps=200):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


us_sync = timed(sync_join)
assert args[4].n == 1100011, args[4].n
d = torch.zeros(8, dtype=torch.int64, device=dev)
f = eng.prepare_join2(sa, ca, sb, cb, out, octx, d)
for _ in range(20):
    f()
eng.sync()
t0 = time.perf_counter()
for _ in range(200):
    f()
eng.sync()
us_async = (time.perf_counter() - t0) / 200 * 1e6
print(f"{os.path.basename(eng.lib._name)}: sync dg_join2 {us_sync:.1f} us/call (median), "
      f"async back-to-back {us_async:.1f} us/join")


def py_join():
    eng.join2(sa, ca, sb, cb, out=out, out_ctx=octx)


us_py = timed(py_join)
print(f"{os.path.basename(eng.lib._name)}: sync Engine.join2 (Python mirror) {us_py:.1f} us/call (median)")
