"""Phase breakdown of kfold_kernel (dg_apply_deltas' one-pass fold) from the DG_STAMPS
diagnostic build, on config 3 (KF_KEYS keys, 64 keyed deltas).

    DG_STAMPS=1 python -m delta_crdt_ex_amd.build   # on the CPU host
    python tools/kfold_stamps.py                       # on the GPU box

Stamps (s_memrealtime, 100 MHz) by lane 0 of every bucket at: 0 start (after the
ticket)  1 slices staged in LDS  13 keyset entries folded into rows + sub-bucket histogram  2 delta items sorted  7 key masks built  3 candidates
evaluated (VV tables)  4 survivor scans done  5 survivors ranked  6 offset looked up and
rows written; 12 run offsets scanned, 9 sub-bucket scan, 10 scatter.  Only SHARES are meaningful
(stamps add barriers)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from delta_crdt_ex_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.environ.get("KF_STAMPS_LIB") or os.path.join(ROOT, "delta_crdt_ex_amd", "ab", "libdeltagpu_stamps.so")


def main():
    import torch
    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Context, Engine, Store
    lib = _abi.load(_abi.LIB_PATH)
    dev = "cuda:0"
    base, deltas = W.config3(n_keys=int(os.environ.get("KF_KEYS", 10_000_000)), n_replicas=64,
                             touch=0.01, seed=3)
    sb = Store.from_numpy(*base["rows"], device=dev)
    cb = Context.from_numpy(*base["ctx"], dev)
    ds = [Store.from_numpy(*d["rows"], device=dev) for d in deltas]
    dc = [Context.from_numpy(*d["ctx"], dev) for d in deltas]
    ks = [torch.from_numpy(d["keys"].view(np.int64)).to(dev) for d in deltas]
    eng = Engine(0)
    for _ in range(3):
        o, c = eng.apply_deltas(sb, cb, ds, dc, ks)
    buf = np.zeros(65536 * 16, np.uint64)
    lib.dg_debug_kfold_stamps.argtypes = [C.c_void_p, C.c_size_t]
    assert lib.dg_debug_kfold_stamps(buf.ctypes.data, len(buf)) == 0
    st = buf.reshape(65536, 16).astype(np.int64)
    nb = int(np.nonzero(st[:, 0])[0].max()) + 1
    st = st[:nb]
    t0 = st[:, 0].min()
    names = ["stage:meta+scan", "stage:rows", "keyset-drop+histogram", "sort:scan",
             "sort:scatter", "sort:rank+move", "masks", "vv-tables", "scans", "rank", "lookback+write"]
    d = np.diff(st[:, [0, 12, 1, 13, 9, 10, 2, 7, 3, 4, 5, 6]], axis=1) * 10 / 1000.0  # us
    print(f"buckets={nb} kernel span={(st[:, 6].max() - t0) * 10 / 1000:.1f} us")
    for i, nm in enumerate(names):
        print(f"{nm:16s} median {np.median(d[:, i]):7.2f} us  p90 {np.percentile(d[:, i], 90):7.2f}"
              f"  mean {d[:, i].mean():7.2f}")
    tot = (st[:, 6] - st[:, 0]) * 10 / 1000
    print(f"per-bucket total median {np.median(tot):.2f} us  mean {tot.mean():.2f}")
    starts = (st[:, 0] - t0) * 10 / 1000
    print("bucket start times (us) at deciles:", np.percentile(starts, np.arange(0, 101, 10)).round(1))


if __name__ == "__main__":
    main()
