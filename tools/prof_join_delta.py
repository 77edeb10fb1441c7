"""dg_join_delta on the config-4 shard (rocprofv3 target): a sync delta of the 1 % differing
keys applied in place to a 12.5M-key state, with the tree update; 5 reps, the state
restored between them."""
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
depth = int(np.ceil(np.log2(len(a["rows"][0]) / 3)))
sa = Store.from_numpy(*a["rows"], device=dev)
sb = Store.from_numpy(*b["rows"], device=dev)
ta = eng.merkle_build(sa, depth, MerkleTree.empty(depth, dev, 3, 0, terms), 3, 0)
tb = eng.merkle_build(sb, depth, MerkleTree.empty(depth, dev, 3, 0, terms), 3, 0)
keys = eng.merkle_diff(ta, tb)
d = W.sync_delta(b, keys.cpu().numpy().view(np.uint64))
sd = Store.from_numpy(*d["rows"], device=dev)
cd = Context.from_numpy(*d["ctx"], dev)
st = Store.empty(sa.n + sd.n, dev)
spare = Store.empty(sa.n + sd.n, dev)
ca = a["ctx"]
sc = Context.empty(ca[0], len(ca[1]) + len(d["ctx"][1]), dev)
for _ in range(6):
    for f in ("key", "val", "ts", "node", "cnt"):
        getattr(st, f)[: sa.n].copy_(getattr(sa, f)[: sa.n])
    st.n = sa.n
    sc.node[: len(ca[1])].copy_(torch.from_numpy(ca[1].view(np.int32)))
    sc.cnt[: len(ca[1])].copy_(torch.from_numpy(ca[2].view(np.int64)))
    sc.n = len(ca[1])
    t = ta.clone()
    t.store = st
    torch.cuda.synchronize()
    ch, sw = eng.join_delta(st, sc, sd, cd, keys, spare, t)
torch.cuda.synchronize()
print("changed", ch.numel(), "swapped", sw, flush=True)
