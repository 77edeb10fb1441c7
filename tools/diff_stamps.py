"""Phase breakdown of merkle_diff_count_kernel from the DG_STAMPS diagnostic build, on the
config-4 shard (tools/prof_merkle.py's trees).

    DG_STAMPS=1 python -m delta_crdt_ex_amd.build     # on the CPU host
    python tools/diff_stamps.py                          # on the GPU box

Stamps (s_memrealtime, 100 MHz) by thread 0 of every subtree workgroup at: 0 start,
1 subtree root compared (the first round trip: roots, ancestors, counts, bounds),
2 the four prefixes scanned (the leaf nodes' round trip), 3 the differing buckets listed,
4 their rows loaded and hashed, 5 keys merged and counted, 6 keys written.  Every stamp
is behind a barrier: shares are meaningful, absolute times are inflated."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from delta_crdt_ex_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.environ.get("DF_STAMPS_LIB") or os.path.join(ROOT, "delta_crdt_ex_amd", "ab", "libdeltagpu_stamps.so")
NAMES = ["root compared (round trip 1)", "prefixes (leaf nodes)", "buckets listed",
         "rows loaded + hashed", "keys merged + counted", "keys written"]


def main():
    import torch
    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Engine, MerkleTree, Store, TermHashes
    lib = _abi.load(_abi.LIB_PATH)
    lib.dg_debug_diff_stamps.argtypes = [C.c_void_p, C.c_size_t]
    n = 12_500_000
    a, b = W.config4_shard(0, 8, keys_per_rank=n, diff_frac=0.01)
    dev = "cuda:0"
    eng = Engine(0)
    terms = TermHashes(*a["nodes"].universe.term_tables(), dev)
    sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
    depth = int(np.ceil(np.log2(len(a["rows"][0]) / 3)))
    ta = eng.merkle_build(sa, depth, MerkleTree.empty(depth, dev, 3, 0, terms), 3, 0)
    tb = eng.merkle_build(sb, depth, MerkleTree.empty(depth, dev, 3, 0, terms), 3, 0)
    for _ in range(3):
        keys = eng.merkle_diff(ta, tb)
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8, np.uint64)
    assert lib.dg_debug_diff_stamps(buf.ctypes.data, len(buf)) == 0
    s = buf.reshape(4096, 8).astype(np.int64)
    live = s[:, 0] > 0
    full = live & (s[:, 6] > 0)
    t0 = s[live, 0].min()
    us = lambda x: x / 100.0  # 100 MHz ticks -> us
    print(f"depth {depth}, diff keys {keys.numel()}, subtrees {live.sum()}, merged in LDS {full.sum()}")
    print(f"kernel span (first start -> last stamp) {us(s[live].max() - t0):.1f} us")
    ends = np.where(full, s[:, 6], s[:, 1])[live]
    print("start at deciles (us):", np.round(us(np.percentile(s[live, 0] - t0, range(0, 101, 10))), 1))
    print("end at deciles (us):  ", np.round(us(np.percentile(ends - t0, range(0, 101, 10))), 1))
    f = s[full]
    for k in range(1, 7):
        d = us(f[:, k] - f[:, k - 1])
        print(f"{NAMES[k - 1]:32s} median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f}  mean {d.mean():6.2f}")
    tot = us(f[:, 6] - f[:, 0])
    print(f"{'per-subtree total':32s} median {np.median(tot):6.2f} us  p90 {np.percentile(tot, 90):6.2f}")
    where = buf.reshape(4096, 8)[:, 7]
    if full.any() and where[full].any():  # a build that records CU and XCC (slot 7)
        cu, xcc = (where & 0xFFFFFFFF).astype(np.int64), (where >> np.uint64(32)).astype(np.int64)
        leaf = us(s[:, 2] - s[:, 1])
        idx = np.flatnonzero(full)
        print("leaf phase by XCC (median us):",
              {int(x): round(float(np.median(leaf[idx][xcc[idx] == x])), 2) for x in np.unique(xcc[idx])})
        rank = np.zeros(4096, np.int64)  # order of arrival of the subtrees sharing a CU
        for key in np.unique(xcc[idx] * 65536 + cu[idx]):
            m = idx[(xcc[idx] * 65536 + cu[idx]) == key]
            rank[m[np.argsort(s[m, 0])]] = np.arange(len(m))
        print("leaf phase by arrival rank on its CU (median, p90 us):",
              {int(r): (round(float(np.median(leaf[idx][rank[idx] == r])), 2),
                        round(float(np.percentile(leaf[idx][rank[idx] == r], 90)), 2))
               for r in np.unique(rank[idx])})
        print("per-subtree total by rank (median us):",
              {int(r): round(float(np.median(tot[rank[idx] == r])), 2) for r in np.unique(rank[idx])})
    eng.close()


if __name__ == "__main__":
    main()
