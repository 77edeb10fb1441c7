"""Where the config-4 round's join_delta wall time goes (bench.py config4_round's call):
the Python wrapper as the bench calls it, the same inside the engine's stream context (no
cross-stream ordering), and the C-ABI call alone (ctypes arguments built beforehand: what
the NIF pays).  Usage: python tools/time_join_delta.py [keys_per_gpu]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_crdt_ex_amd import _abi  # noqa: E402
from delta_crdt_ex_amd import workloads as W  # noqa: E402
from delta_crdt_ex_amd.store import Context, Engine, MerkleTree, Store, TermHashes, _ptr, check  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
a, b = W.config4_shard(0, 1, keys_per_rank=n, diff_frac=0.01)
dev = "cuda:0"
eng = Engine(0)
terms = TermHashes(*a["nodes"].universe.term_tables(), dev)
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
depth = max(8, min(28, int(np.ceil(np.log2(max(len(a["rows"][0]), 2) / 3)))))
ta = eng.merkle_build(sa, depth, MerkleTree.empty(depth, dev, 0, 0, terms), 0, 0)
tb = eng.merkle_build(sb, depth, MerkleTree.empty(depth, dev, 0, 0, terms), 0, 0)
st = Store.empty(sa.n + sb.n, dev)
spare = Store.empty(sa.n + sb.n, dev)
sc = Context.empty(ca.kind, ca.n + cb.n, dev)
keys = eng.merkle_diff(ta, tb)
delta = eng.take_keys(sb, keys)
changed = torch.empty(max(int(keys.numel()), 1), dtype=torch.int64, device=dev)


def restore():
    for f in ("key", "val", "ts", "node", "cnt"):
        getattr(st, f)[: sa.n].copy_(getattr(sa, f)[: sa.n])
    st.n = sa.n
    sc.node[: ca.n].copy_(ca.node[: ca.n])
    sc.cnt[: ca.n].copy_(ca.cnt[: ca.n])
    sc.n, sc.kind = ca.n, ca.kind
    t = ta.clone()
    t.store = st
    torch.cuda.synchronize()
    return t


res = {"python": [], "python_engine_stream": [], "c_abi_call": [], "device_events": []}
for rep in range(9):
    for mode in ("python", "python_engine_stream", "c_abi_call"):
        t = restore()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if mode == "python":
            t0 = time.perf_counter()
            e0.record(eng.stream)
            eng.join_delta(st, sc, delta, cb, keys, spare, t)
            e1.record(eng.stream)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res["device_events"].append(e0.elapsed_time(e1) * 1e3)
        elif mode == "python_engine_stream":
            with torch.cuda.stream(eng.stream):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eng.join_delta(st, sc, delta, cb, keys, spare, t, changed=changed)
                dt = time.perf_counter() - t0
        else:
            ss, scc, sd, cd, sp, tt = st.abi(), sc.abi(), delta.abi(), cb.abi(), spare.abi(), t.abi()
            kp, nk = eng._keys(keys)
            nn, sw = C.c_uint64(0), C.c_int(0)
            args = (eng.h, C.byref(ss), C.byref(scc), C.byref(sd), C.byref(cd), kp, nk, C.byref(sp),
                    C.byref(tt), _ptr(changed, _abi.P64), int(changed.numel()), C.byref(nn), C.byref(sw))
            f = eng.lib.dg_join_delta
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc = f(*args)
            dt = time.perf_counter() - t0
            check(rc)
        if rep >= 2:
            res[mode].append(dt * 1e6)
print({k: (round(float(np.median(v)), 1), round(float(min(v)), 1)) for k, v in res.items()}, "(median, min us)")
