"""Phase breakdown of kd_count_kernel (dg_join_delta's one-wait path) from the DG_STAMPS
diagnostic build, on the config-4 round (tools/prof_merkle.py's shard).

    DG_STAMPS=1 python -m delta_crdt_ex_amd.build     # on the CPU host
    python tools/kd_stamps.py                            # on the GPU box

Stamps (s_memrealtime, 100 MHz) per key workgroup, no barriers added: 0 entry (thread 2),
1 the workgroup's delta range searched (thread 0), 2 thread 2's state search done,
3 past the barrier (tables, staged delta keys), 4 thread 2's per-key join done, 5 its tree
put done, 6 arrival (thread 0), 7 the last workgroup's totals written."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from delta_crdt_ex_amd import _abi  # noqa: E402

LIB = os.environ.get("KD_STAMPS_LIB") or os.path.join(ROOT, "delta_crdt_ex_amd", "ab", "libdeltagpu_stamps.so")


def main():
    import ctypes as C

    import torch
    os.environ["DG_LIB_PATH"] = LIB
    os.environ["DG_LIB_ANY_DIGEST"] = "1"
    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Context, Engine, MerkleTree, Store, TermHashes
    lib = _abi.load(LIB)
    lib.dg_debug_kd_stamps.argtypes = [C.c_void_p, C.c_size_t]
    a, b = W.config4_shard(0, 8, keys_per_rank=12_500_000, diff_frac=0.01)
    dev = "cuda:0"
    eng = Engine(0)
    terms = TermHashes(*a["nodes"].universe.term_tables(), dev)
    sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
    ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
    depth = int(np.ceil(np.log2(len(a["rows"][0]) / 3)))
    ta = eng.merkle_build(sa, depth, MerkleTree.empty(depth, dev, 3, 0, terms), 3, 0)
    tb = eng.merkle_build(sb, depth, MerkleTree.empty(depth, dev, 3, 0, terms), 3, 0)
    st, spare = Store.empty(sa.n + sb.n, dev), Store.empty(sa.n + sb.n, dev)
    sc = Context.empty(ca.kind, ca.n + cb.n, dev)
    rows = []
    for rep in range(4):
        for f in ("key", "val", "ts", "node", "cnt"):
            getattr(st, f)[: sa.n].copy_(getattr(sa, f)[: sa.n])
        st.n = sa.n
        sc.node[: ca.n].copy_(ca.node[: ca.n])
        sc.cnt[: ca.n].copy_(ca.cnt[: ca.n])
        sc.n, sc.kind = ca.n, ca.kind
        t = ta.clone()
        t.store = st
        keys = eng.merkle_diff(ta, tb)
        delta = eng.take_keys(sb, keys)
        torch.cuda.synchronize()
        eng.join_delta(st, sc, delta, cb, keys, spare, t)
        torch.cuda.synchronize()
        nt = (int(keys.numel()) + 255) // 256
        buf = np.zeros(4096 * 8, np.uint64)
        assert lib.dg_debug_kd_stamps(buf.ctypes.data, len(buf)) == 0
        s = buf[: nt * 8].reshape(nt, 8).astype(np.float64) / 100.0  # us
        if rep > 0:
            rows.append(s)
    for s in rows:
        t0 = s[:, 0].min()
        rel = s - t0
        med = lambda x: float(np.median(x))  # noqa: E731
        print("workgroups %d: entry spread %.1f us; delta range +%.1f; state search +%.1f; barrier +%.1f; "
              "join %.1f; tree put %.1f; to arrival %.1f (medians from the workgroup's entry)" % (
                  len(s), med(rel[:, 0]) * 0 + (rel[:, 0].max()), med(s[:, 1] - s[:, 0]), med(s[:, 2] - s[:, 0]),
                  med(s[:, 3] - s[:, 0]), med(s[:, 4] - s[:, 3]), med(s[:, 5] - s[:, 4]), med(s[:, 6] - s[:, 5])))
        last = s[:, 7].max() - t0
        arr = np.sort(rel[:, 6])
        print("  arrivals at deciles (us from the first entry):", np.round(arr[np.linspace(0, len(arr) - 1, 11).astype(int)], 1),
              " last workgroup's totals at %.1f us" % last)
        p90 = lambda x: float(np.percentile(x, 90))  # noqa: E731
        print("  p90: delta range %.1f, state search %.1f, barrier %.1f, join %.1f, tree put %.1f" % (
            p90(s[:, 1] - s[:, 0]), p90(s[:, 2] - s[:, 0]), p90(s[:, 3] - s[:, 0]), p90(s[:, 4] - s[:, 3]), p90(s[:, 5] - s[:, 4])))


if __name__ == "__main__":
    main()
