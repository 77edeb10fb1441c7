"""The config-4 round's take (Map.take(B.value, keys), dg_take_keys) through the Python
binding: the default output sizing against a store-sized output allocated per call (the
previous binding) and the C-ABI call alone.  Usage: python tools/time_take.py"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_crdt_ex_amd import _abi  # noqa: E402
from delta_crdt_ex_amd import workloads as W  # noqa: E402
from delta_crdt_ex_amd.store import Engine, MerkleTree, Store, TermHashes  # noqa: E402

a, b = W.config4_shard(0, 1, keys_per_rank=12_500_000, diff_frac=0.01)
dev = "cuda:0"
eng = Engine(0)
terms = TermHashes(*a["nodes"].universe.term_tables(), dev)
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
depth = 22
ta = eng.merkle_build(sa, depth, MerkleTree.empty(depth, dev, 0, 0, terms), 0, 0)
tb = eng.merkle_build(sb, depth, MerkleTree.empty(depth, dev, 0, 0, terms), 0, 0)
keys = eng.merkle_diff(ta, tb)
res = {"default": [], "store_sized_per_call": [], "c_abi": []}
with torch.cuda.stream(eng.stream):
    for rep in range(12):
        for mode in res:
            torch.cuda.synchronize()
            if mode == "default":
                t0 = time.perf_counter()
                d = eng.take_keys(sb, keys)
            elif mode == "store_sized_per_call":
                t0 = time.perf_counter()
                d = eng.take_keys(sb, keys, out=Store.empty(max(sb.n, 1), dev))
            else:
                out = Store.empty(4 * keys.numel(), dev)
                so, ss = out.abi(), sb.abi()
                kp, nk = eng._keys(keys)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rc = eng.lib.dg_take_keys(eng.h, C.byref(ss), kp, nk, C.byref(so))
                assert rc == 0
            dt = time.perf_counter() - t0
            if rep >= 2:
                res[mode].append(dt * 1e6)
print({k: (round(float(np.median(v)), 1), round(float(min(v)), 1)) for k, v in res.items()}, "(median, min us)")
