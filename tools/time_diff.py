"""Where the synchronous merkle_diff's Python wall time goes (config-4 shard trees): the
binding's steps timed one by one, beside the C-ABI call alone.  Usage: python tools/time_diff.py"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_crdt_ex_amd import _abi  # noqa: E402
from delta_crdt_ex_amd import workloads as W  # noqa: E402
from delta_crdt_ex_amd.store import Engine, MerkleTree, Store, TermHashes, _ptr, check  # noqa: E402

a, b = W.config4_shard(0, 1, keys_per_rank=12_500_000, diff_frac=0.01)
dev = "cuda:0"
eng = Engine(0)
terms = TermHashes(*a["nodes"].universe.term_tables(), dev)
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
ta = eng.merkle_build(sa, 22, MerkleTree.empty(22, dev, 0, 0, terms), 0, 0)
tb = eng.merkle_build(sb, 22, MerkleTree.empty(22, dev, 0, 0, terms), 0, 0)
cap = ta.n_keys + tb.n_keys
res = {k: [] for k in ("order", "abi", "c_call", "clone", "python_total", "python_total_idle")}
with torch.cuda.stream(eng.stream):
    for rep in range(12):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng._order()
        t1 = time.perf_counter()
        out = eng._diff_out if getattr(eng, "_diff_out", None) is not None else torch.empty(cap, dtype=torch.int64, device=dev)
        eng._diff_out = out
        n, tot = C.c_uint64(), C.c_uint64()
        xa, xb, ya, yb = ta.abi(), tb.abi(), ta.store.abi(), tb.store.abi()
        t2 = time.perf_counter()
        check(eng.lib.dg_merkle_diff(eng.h, C.byref(xa), C.byref(ya), C.byref(xb), C.byref(yb),
                                     _ptr(out, _abi.P64), cap, C.byref(n), C.byref(tot)))
        t3 = time.perf_counter()
        keys = out[: n.value].clone()
        t4 = time.perf_counter()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        k2 = eng.merkle_diff(ta, tb, cap=cap)
        t6 = time.perf_counter()
        torch.cuda.synchronize()
        time.sleep(0.002)  # an idle GPU before the call, as in the bench's round
        t7 = time.perf_counter()
        k3 = eng.merkle_diff(ta, tb, cap=cap)
        t8 = time.perf_counter()
        if rep >= 2:
            for k, v in (("order", t1 - t0), ("abi", t2 - t1), ("c_call", t3 - t2), ("clone", t4 - t3),
                         ("python_total", t6 - t5), ("python_total_idle", t8 - t7)):
                res[k].append(v * 1e6)
print({k: round(float(np.median(v)), 1) for k, v in res.items()}, "(median us)")
