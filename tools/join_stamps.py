"""Phase breakdown of the join kernel from the DG_STAMPS diagnostic build.

    DG_STAMPS=1 python -m delta_crdt_ex_amd.build   # on the CPU host
    python tools/join_stamps.py                        # on the GPU box

Stamps are s_memrealtime (100 MHz) taken by lane 0 of every tile at:
0 tile start (after the ticket)  1 VV tables filled  2 rows staged in LDS
3 per-thread merge done          4 block scan + compaction list done
5 look-back done (single pass) / count written (two pass)   6 output written.
Only SHARES are meaningful (stamps add barriers).
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from delta_crdt_ex_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.path.join(ROOT, "delta_crdt_ex_amd", "libdeltagpu_stamps.so")


def main():
    import torch
    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Context, Engine, Store
    lib = _abi.load(_abi.LIB_PATH)
    dev = "cuda:0"
    a, b = W.config2()
    eng = Engine(0)
    sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
    ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
    out = Store.empty(sa.n + sb.n, dev)
    octx = Context.empty(0, 8, dev)
    for _ in range(5):
        eng.join2(sa, ca, sb, cb, out=out, out_ctx=octx)
    buf = np.zeros(65536 * 8, np.uint64)
    lib.dg_debug_join_stamps.argtypes = [C.c_void_p, C.c_size_t]
    assert lib.dg_debug_join_stamps(buf.ctypes.data, len(buf)) == 0
    st = buf.reshape(65536, 8).astype(np.int64)
    ntiles = int(np.nonzero(st[:, 0])[0].max()) + 1  # tiles of the last launch stamp slot 0
    st = st[:ntiles]
    t0 = st[:, 0].min()
    order = [0, 1, 2, 3, 4, 5, 6]
    names = ["tables", "stage", "merge", "scan", "lookback", "write"]
    d = np.diff(st[:, order], axis=1) * 10 / 1000.0  # us
    print(f"tiles={ntiles} kernel span={(st[:, 6].max() - t0) * 10 / 1000:.1f} us")
    for i, nm in enumerate(names):
        print(f"{nm:9s} median {np.median(d[:, i]):6.2f} us  p90 {np.percentile(d[:, i], 90):6.2f}"
              f"  mean {d[:, i].mean():6.2f}")
    tot = (st[:, 6] - st[:, 0]) * 10 / 1000  # 0 -> 6
    print(f"per-tile total median {np.median(tot):.2f} us  mean {tot.mean():.2f}")
    starts = (st[:, 0] - t0) * 10 / 1000
    print("tile start times (us) at deciles:", np.percentile(starts, np.arange(0, 101, 10)).round(1))


if __name__ == "__main__":
    main()
