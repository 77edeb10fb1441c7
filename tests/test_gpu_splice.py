"""The sparse keyed join as a splice (csrc/splice.hip; api.hip splice_join): a sync delta
Map.take(B, K) joined into a large state with its keyset K (causal_crdt.ex:383-384),
bit-exact against the C oracle's keyed join and CausalCrdt's changed keys, and equal to
the full-merge join (DG_SPLICE=0) -- including the inputs on which the splice hands over
to the full join (a delta key outside K, more taken rows than the splice's bound)."""
import os

import numpy as np
import pytest
import torch

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.store import Engine, Store, u64
from oracle import ref as R
from test_gpu_parity import DEV, ctx_eq, rows_eq, up

pytestmark = pytest.mark.gpu


def kdev(keys):
    return torch.from_numpy(np.ascontiguousarray(keys, np.uint64).view(np.int64)).to(DEV)


@pytest.fixture(scope="module")
def full_engine():
    """An engine whose keyed joins always merge the whole state (the reference path)."""
    os.environ["DG_SPLICE"] = "0"
    try:
        e = Engine(0)
    finally:
        del os.environ["DG_SPLICE"]
    yield e
    e.close()


def check(engine, full_engine, a, b, keys, changes=True):
    keys = np.unique(np.asarray(keys, np.uint64))
    sa, ca = up(a)
    sb, cb = up(b)
    wr, wc = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"], keys=keys)
    if changes:
        out, octx, ch = engine.join2_changes(sa, ca, sb, cb, keys=kdev(keys))
        assert np.array_equal(u64(ch), R.changed_keys(a["rows"], wr, keys))
    else:
        out, octx = engine.join2(sa, ca, sb, cb, keys=kdev(keys))
    rows_eq(out, wr)
    ctx_eq(octx, wc)
    fo, fc = full_engine.join2(sa, ca, sb, cb, keys=kdev(keys))
    x, y = out.to_numpy(), fo.to_numpy()
    assert out.n == fo.n and all(np.array_equal(p, q) for p, q in zip(x, y))
    return out


@pytest.fixture(scope="module")
def pair():
    return W.random_pair(np.random.default_rng(11), 40_000, n_nodes=6, ts_range=1 << 20,
                         dense_ctx=False)


@pytest.mark.parametrize("frac", [0.001, 0.01, 0.05])
def test_sync_delta_splice(engine, full_engine, pair, frac):
    a, b = pair
    rng = np.random.default_rng(int(frac * 1e4))
    kb = np.unique(np.concatenate([a["rows"][0], b["rows"][0]]))
    keys = np.sort(rng.choice(kb, max(1, int(frac * len(kb))), replace=False))
    check(engine, full_engine, a, W.sync_delta(b, keys), keys)
    check(engine, full_engine, a, W.sync_delta(b, keys), keys, changes=False)


def test_splice_edges(engine, full_engine, pair):
    a, b = pair
    ak = a["rows"][0]
    rng = np.random.default_rng(5)
    absent = rng.integers(0, 2**64, 50, dtype=np.uint64)          # keys no replica holds
    ends = np.concatenate([ak[:3], ak[-3:]])                       # the state's first/last keys
    below_above = np.array([0, 2**64 - 1], np.uint64)
    for keys in (ends, np.concatenate([ends, absent, below_above]), absent, ak[:1], ak[-1:]):
        check(engine, full_engine, a, W.sync_delta(b, keys), keys)
    # a delta without rows (every key of K removed at B): E holds only the state's rows
    # that B's context does not cover
    keys = np.unique(ak[::97])
    empty = {"rows": tuple(c[:0] for c in b["rows"]), "ctx": b["ctx"]}
    check(engine, full_engine, a, empty, keys)


def test_splice_dense_keyset_in_one_tile(engine, full_engine, pair):
    """3000 keyset keys between two neighbouring state keys (one copy tile holds more
    keyset entries than it stages in LDS), plus a spread of real keys."""
    a, b = pair
    ak = np.unique(a["rows"][0])
    i = len(ak) // 2
    gap_keys = ak[i] + np.arange(1, 3001, dtype=np.uint64)
    assert gap_keys[-1] < ak[i + 1]
    keys = np.concatenate([gap_keys, ak[::400]])
    check(engine, full_engine, a, W.sync_delta(b, keys), keys)


def test_splice_hands_over_to_the_full_join(engine, full_engine, pair):
    a, b = pair
    kb = np.unique(b["rows"][0])
    keys = kb[::200]
    # the delta carries a key outside K: its rows replace the state's (the carry)
    extra = kb[101:102]
    d = W.sync_delta(b, np.union1d(keys, extra))
    check(engine, full_engine, a, d, keys)
    # a keyset key with more state rows than the splice's bound (16 per key + 4096)
    n_hot = 6000
    hot = np.full(n_hot, a["rows"][0][0], np.uint64)
    rows = tuple(np.concatenate([c, h]) for c, h in zip(
        a["rows"], (hot, np.arange(n_hot, dtype=np.uint64) + (1 << 62),
                    np.zeros(n_hot, np.int64), np.zeros(n_hot, np.uint32),
                    np.arange(1, n_hot + 1, dtype=np.uint64) + (1 << 40))))
    a2 = {"rows": W.sort_rows(*rows), "ctx": a["ctx"]}
    k5 = np.union1d(keys[:5], hot[:1])
    check(engine, full_engine, a2, W.sync_delta(b, k5), k5)


@pytest.mark.parametrize("rank", [0, 7])
def test_config4_round_splice_vs_full(engine, full_engine, rank):
    """The config-4 shard round's keyed join (80k keys per shard, 1 % differing): the
    splice equals the oracle's full-state join and the full-merge keyed join."""
    a, b = W.config4_shard(rank, 8, keys_per_rank=80_000, diff_frac=0.01)
    want = R.store_diff(a["rows"], b["rows"])
    out = check(engine, full_engine, a, W.sync_delta(b, want), want)
    wr, _ = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    rows_eq(out, wr)


def test_splice_unaligned_columns_take_the_full_join(engine, full_engine, pair):
    """A state whose columns are 8-byte offset views (not 16-byte aligned) is joined by
    the full merge; the result is the same."""
    a, b = pair
    keys = np.unique(a["rows"][0][::150])
    sa, ca = up(a)
    n = sa.n
    cols = []
    for c in (sa.key, sa.val, sa.ts, sa.node, sa.cnt):
        buf = torch.empty(n + 1, dtype=c.dtype, device=DEV)
        buf[1:].copy_(c[:n])
        cols.append(buf[1:])
    su = Store(*cols, n)
    d = W.sync_delta(b, keys)
    sd, cd = up(d)
    out, octx = engine.join2(su, ca, sd, cd, keys=kdev(keys))
    wr, wc = R.join2(a["rows"], a["ctx"], d["rows"], d["ctx"], keys=keys)
    rows_eq(out, wr)
    ctx_eq(octx, wc)
