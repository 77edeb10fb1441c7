"""dg_mutate_batch on cuda:0: the batch delta's rows, dot-list context
and touched keys equal the oracle's (ref.mutate_batch, which tests/test_configs.py pins
to the term oracle's op-by-op fold), and the mirror's apply_ops equals applying the
same ops one at a time through add/4, remove/3 and join/3."""
import numpy as np
import pytest
import torch

from delta_crdt_ex_amd import aw_lww_map as M
from delta_crdt_ex_amd import causal_crdt as CC
from delta_crdt_ex_amd._abi import DeltaGpuError
from delta_crdt_ex_amd.store import u64
from kfold_cases import random_fold
from oracle import ref as R
from test_gpu_parity import DEV, ctx_eq, rows_eq, up

pytestmark = pytest.mark.gpu


def dev(a, dt):
    return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(DEV)


def run(engine, st, node, ops):
    m = len(ops)
    kind = np.array([1 if o[0] == "add" else 0 for o in ops], np.uint8)
    key = np.array([o[1] for o in ops], np.uint64)
    val = np.array([o[2] for o in ops], np.uint64)
    ts = np.array([o[3] for o in ops], np.int64)
    rank = (np.cumsum(kind, dtype=np.uint64) - kind).astype(np.uint64)
    order = np.argsort(key, kind="stable")
    s, c = up(st)
    kt = torch.from_numpy(kind[order]).to(DEV) if m else torch.zeros(1, dtype=torch.uint8, device=DEV)
    return engine.mutate_batch(s, c, node, kt, dev(key[order], np.int64), dev(val[order], np.int64),
                               dev(ts[order], np.int64), dev(rank[order], np.int64), int(kind.sum()))


def random_ops(rng, keys, n):
    ops = []
    for _ in range(n):
        k = int(keys[rng.integers(0, len(keys))]) if rng.random() < 0.8 else int(rng.integers(1, 1 << 63))
        if rng.random() < 0.7:
            ops.append(("add", k, int(rng.integers(0, 9)) + (1 << 62), int(rng.integers(0, 1 << 40))))
        else:
            ops.append(("remove", k, 0, 0))
    return ops


@pytest.mark.parametrize("seed,n_ops", [(0, 1), (1, 50), (2, 3000), (3, 20000)])
def test_mutate_batch_parity(engine, seed, n_ops):
    rng = np.random.default_rng(seed)
    st, _ = random_fold(70 + seed, n_keys=5000, k=0, n_nodes=6, rows_per_key=3)
    ops = random_ops(rng, np.unique(st["rows"][0]), n_ops)
    drows, dctx, dkeys = run(engine, st, 9, ops)
    wr, wc, wk = R.mutate_batch(st["rows"], st["ctx"], 9, ops)
    rows_eq(drows, wr)
    ctx_eq(dctx, wc)
    assert np.array_equal(u64(dkeys), wk)
    # joined with the touched keys: the op-by-op result (oracle fold of the same ops)
    s, c = up(st)
    out, octx = engine.join2(s, c, drows, dctx, keys=dkeys)
    jr, jc = R.join2(st["rows"], st["ctx"], wr, wc, wk)
    rows_eq(out, jr)
    ctx_eq(octx, jc)


def test_mutate_batch_errors(engine):
    st, _ = random_fold(80, n_keys=200, k=0)
    s, c = up(st)
    # unsorted ops are refused
    key = dev(np.array([5, 3], np.uint64), np.int64)
    z = dev(np.zeros(2, np.uint64), np.int64)
    with pytest.raises(DeltaGpuError, match="sorted"):
        engine.mutate_batch(s, c, 1, torch.ones(2, dtype=torch.uint8, device=DEV), key, z, z, z, 2)
    # an empty batch is an empty delta
    e = torch.zeros(0, dtype=torch.int64, device=DEV)
    d, dc, k = engine.mutate_batch(s, c, 1, torch.zeros(0, dtype=torch.uint8, device=DEV), e, e, e,
                                   e, 0)
    assert d.n == 0 and dc.n == 0 and k.numel() == 0


def test_apply_ops_equals_one_by_one():
    st = M.compress_dots(M.new())
    for i in range(20):
        st = M.join(st, M.add(i, i * 10, "n1", st, ts=i), [i])
    ops = [("add", 3, 33, 100), ("remove", 4), ("add", 4, 44, 101), ("add", 3, 333, 102),
           ("remove", 5), ("add", 99, 9, 103), ("remove", 99), ("add", 7, 70, 104)]
    one = st
    for op in ops:
        d = M.add(op[1], op[2], "n2", one, ts=op[3]) if op[0] == "add" else M.remove(op[1], "n2", one)
        one = M.join(one, d, [op[1]])
    batch, diffs = CC.apply_ops(st, ops, "n2")
    for x, y in zip(one.rows.to_numpy(), batch.rows.to_numpy()):
        assert np.array_equal(x, y)
    for x, y in zip(one.ctx.to_numpy(), batch.ctx.to_numpy()):
        assert np.array_equal(x, y)
    assert M.read(batch) == M.read(one)
    assert sorted(diffs, key=repr) == sorted([("add", 3, 333), ("add", 4, 44), ("remove", 5)],
                                             key=repr)
