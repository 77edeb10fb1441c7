"""The config-4 anti-entropy round at the bench's shard shape (rocprofv3 target), as
bench.py's config4_round runs it on the receiving replica: trees over node terms
(dg_term_hashes), builds, the diff, the sync delta (dg_take_keys) and dg_join_delta_rows
on A's device-resident state (the keyed join in place, its changed keys, the MerkleMap
update, the changed keys' rows).  Usage: python tools/prof_merkle.py [keys_per_gpu]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from delta_crdt_ex_amd import workloads as W  # noqa: E402
from delta_crdt_ex_amd.store import Context, Engine, MerkleTree, Store, TermHashes  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
a, b = W.config4_shard(0, 8, keys_per_rank=n, diff_frac=0.01)
dev = "cuda:0"
eng = Engine(0)
terms = TermHashes(*a["nodes"].universe.term_tables(), dev)
sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
depth = int(np.ceil(np.log2(len(a["rows"][0]) / 3)))
# shard 0 of 8: the shard trees cover the shard's key range (shard_bits 3)
ta = eng.merkle_build(sa, depth, MerkleTree.empty(depth, dev, 3, 0, terms), 3, 0)
tb = eng.merkle_build(sb, depth, MerkleTree.empty(depth, dev, 3, 0, terms), 3, 0)
for _ in range(3):
    eng.merkle_build(sa, depth, ta, 3, 0)
    eng.merkle_build(sb, depth, tb, 3, 0)
st = Store.empty(sa.n + sb.n, dev)
spare = Store.empty(sa.n + sb.n, dev)
sc = Context.empty(ca.kind, ca.n + cb.n, dev)
rows = Store.empty(sa.n + sb.n, dev)
for _ in range(5):
    for f in ("key", "val", "ts", "node", "cnt"):  # A's pristine state (outside the round)
        getattr(st, f)[: sa.n].copy_(getattr(sa, f)[: sa.n])
    st.n = sa.n
    sc.node[: ca.n].copy_(ca.node[: ca.n])
    sc.cnt[: ca.n].copy_(ca.cnt[: ca.n])
    sc.n, sc.kind = ca.n, ca.kind
    t = ta.clone()
    t.store = st
    torch.cuda.synchronize()
    keys = eng.merkle_diff(ta, tb)
    delta = eng.take_keys(sb, keys)
    changed, swapped = eng.join_delta(st, sc, delta, cb, keys, spare, t, rows=rows)
torch.cuda.synchronize()
print("depth", depth, "diff keys", keys.numel(), "changed", changed.numel(), "in place", not swapped,
      flush=True)
