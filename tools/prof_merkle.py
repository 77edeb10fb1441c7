"""The config-4 anti-entropy round at the bench's shard shape (rocprofv3 target): trees
over node terms (dg_term_hashes, as bench.py builds them), builds, diffs, the sync delta
(dg_take_keys), the keyed join with its changed keys (the splice), and the incremental
tree update.  Usage: python tools/prof_merkle.py [keys_per_gpu]"""
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
for _ in range(5):
    torch.cuda.synchronize()
    keys = eng.merkle_diff(ta, tb)
    delta = eng.take_keys(sb, keys)
    out, octx, changed = eng.join2_changes(sa, ca, delta, cb, keys=keys)
    t = ta.clone()
    eng.merkle_update(t, out, changed)
torch.cuda.synchronize()
print("depth", depth, "diff keys", keys.numel(), "changed", changed.numel(), flush=True)
