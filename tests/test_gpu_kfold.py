"""dg_apply_deltas' one-pass keyed fold (csrc/kfold.hip) on cuda:0, bit-exact against the
C oracle's delta-by-delta fold of join/3 (causal_crdt.ex:383-384; tests/test_configs.py
pins that fold to the term oracle on the same generator).  The `strict` engine runs with
DG_APPLY_MODE=onepass, so a test that passes on it proves the one-pass kernels produced
the result (that engine errors instead of falling back to the step-by-step fold).  The
default engine covers the inputs the one-pass fold hands to the step-by-step fold."""
import os

import numpy as np
import pytest

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd._abi import DeltaGpuError
from delta_crdt_ex_amd.store import Engine
from kfold_cases import mutation_fold, random_fold
from oracle import ref as R
from test_gpu_configs import keys_dev
from test_gpu_parity import DEV, ctx_eq, rows_eq, up

pytestmark = pytest.mark.gpu


def _engine(mode):
    os.environ["DG_APPLY_MODE"] = mode
    try:
        return Engine(0)
    finally:
        del os.environ["DG_APPLY_MODE"]


@pytest.fixture(scope="module")
def strict():
    e = _engine("onepass")
    yield e
    e.close()


@pytest.fixture(scope="module")
def stepwise():
    e = _engine("fold")
    yield e
    e.close()


def run(engine, st, ds, keys=True):
    s, c = up(st)
    dd = [up(d) for d in ds]
    ks = None
    if keys:
        ks = [None if d["keys"] is None else keys_dev(d["keys"]) for d in ds]
    return engine.apply_deltas(s, c, [x[0] for x in dd], [x[1] for x in dd], ks)


def want(st, ds, keys=True):
    return R.apply_deltas(st["rows"], st["ctx"], [d["rows"] for d in ds],
                          [d["ctx"] for d in ds], [d["keys"] for d in ds] if keys else None)


def check(engine, st, ds, keys=True):
    out, octx = run(engine, st, ds, keys)
    wr, wc = want(st, ds, keys)
    rows_eq(out, wr)
    ctx_eq(octx, wc)


@pytest.mark.parametrize("seed,k", [(0, 1), (1, 3), (2, 8), (3, 17), (4, 64)])
def test_onepass_random(strict, seed, k):
    st, ds = random_fold(seed, n_keys=3000, k=k)
    check(strict, st, ds)


@pytest.mark.parametrize("seed", range(3))
def test_onepass_crowded_keys(strict, seed):
    """Many deltas touching the same keys with the same tuples: big key groups, tuples
    held by the state and several deltas, adds and removes interleaved."""
    st, ds = random_fold(10 + seed, n_keys=400, k=24, rows_per_key=8, p_keys=0.4, p_take=0.8,
                         p_outside=0.05)
    check(strict, st, ds)


def test_onepass_full_state_deltas(strict):
    """keys_i NULL (a full-state join of that delta) mixed with keyed deltas, and
    keys=None for every delta."""
    st, ds = random_fold(20, n_keys=2000, k=12, p_full=0.3)
    assert any(d["keys"] is None for d in ds) and any(d["keys"] is not None for d in ds)
    check(strict, st, ds)
    check(strict, st, ds, keys=False)


def test_onepass_empty_inputs(strict):
    st, ds = random_fold(21, n_keys=1500, k=6)
    # empty keysets: every delta row is carried right-biased
    d0 = dict(ds[0], keys=np.zeros(0, np.uint64))
    # an empty delta (no rows) with a keyset: removals only
    e = tuple(c[:0] for c in ds[1]["rows"])
    d1 = dict(ds[1], rows=e)
    check(strict, st, [d0, d1] + ds[2:])
    # an empty state
    es = {"rows": tuple(c[:0] for c in st["rows"]), "ctx": st["ctx"]}
    check(strict, es, ds)


@pytest.mark.parametrize("n_keys,keep", [(40, None), (65, None), (130, None), (3000, 1),
                                         (3000, 63), (3000, 64), (3000, 65)])
def test_onepass_small_states(strict, n_keys, keep):
    """States of 0-130 rows: the per-bucket wave search for the state's bucket starts
    (kfold_fill_kernel) below, at and just above one wave's width, and many buckets with no
    state row at all."""
    st, ds = random_fold(30 + n_keys + (keep or 0), n_keys=n_keys, k=5)
    if keep is not None:
        st = {"rows": tuple(c[:keep] for c in st["rows"]), "ctx": st["ctx"]}
    check(strict, st, ds)


@pytest.mark.parametrize("seed", range(2))
def test_onepass_unequal_runs(strict, seed):
    """Runs of very unequal lengths: one delta with rows of most keys (its run is cut into
    more than 8 slices by the fill, P > 8) beside deltas of a few hundred rows, an empty delta and
    an empty keyset -- most (run, slice) pairs of the fill are empty, and slice i of a long
    run and of a short one cover different bucket ranges."""
    n = 30_000
    st, ds = random_fold(50 + seed, n_keys=n, k=9, p_keys=0.002)
    _, big = random_fold(50 + seed, n_keys=n, k=1, p_keys=0.9, p_take=0.9)
    assert len(big[0]["rows"][0]) > 8 * 2048
    empty = dict(ds[1], rows=tuple(c[:0] for c in ds[1]["rows"]))
    nokeys = dict(ds[2], keys=np.zeros(0, np.uint64))
    check(strict, st, ds[:1] + [empty, nokeys] + ds[3:5] + big + ds[5:])


def test_onepass_large_node_ids_in_rows(strict):
    """Row node ids >= the VV table width that no context names: never covered."""
    st, ds = random_fold(22, n_keys=2000, k=8, n_nodes=40, node_base=1000, ctx_node_max=1024)
    assert st["rows"][3].max() >= 1024
    check(strict, st, ds)


def test_onepass_two_passes(strict):
    """70 deltas: two one-pass folds of 64 and 6 deltas."""
    st, ds = random_fold(23, n_keys=3000, k=70, p_keys=0.02)
    check(strict, st, ds)


@pytest.mark.parametrize("case", ["context node ids", "unhashed keys", "dot-set contexts"])
def test_stepwise_fallback(engine, strict, case):
    """Inputs the one-pass fold does not take: the strict engine refuses them, the
    default engine folds them delta by delta, bit-exact."""
    if case == "context node ids":
        st, ds = random_fold(30, n_keys=2000, k=6, n_nodes=40, node_base=1000)
    elif case == "unhashed keys":  # every key in bucket 0: over the LDS capacity
        st, ds = random_fold(31, n_keys=3000, k=6, hashed=False)
    else:
        st, ds = random_fold(32, n_keys=800, k=5, dots_ctx=True)
    with pytest.raises(DeltaGpuError, match="one-pass fold not applicable"):
        run(strict, st, ds)
    check(engine, st, ds)


@pytest.mark.parametrize("seed,k", [(40, 1), (41, 5), (42, 16), (43, 64)])
def test_onepass_dot_set_contexts(strict, seed, k):
    """Mutation deltas (MapSet contexts, aw_lww_map.ex:124-146) folded in ONE pass (the
    strict engine refuses the stepwise fold): their dots go to the device hash set, their
    per-node maxima into the VV prefix unions (they used to fall back)."""
    st, ds = mutation_fold(seed, n_keys=20_000, k=k, ops=400)
    assert all(d["ctx"][0] == 1 for d in ds)
    check(strict, st, ds)


@pytest.mark.parametrize("seed", range(3))
def test_onepass_mixed_contexts(strict, seed):
    """Random folds whose deltas carry dot sets, and dot sets mixed with version vectors
    (sync deltas and mutation deltas in one batch), crowded keys included."""
    st, ds = random_fold(50 + seed, n_keys=2000, k=12, delta_dots=True)
    check(strict, st, ds)
    st2, ds2 = random_fold(60 + seed, n_keys=600, k=20, rows_per_key=6, p_keys=0.3, p_take=0.7)
    _, dd = random_fold(70 + seed, n_keys=600, k=20, rows_per_key=6, p_keys=0.3, p_take=0.7,
                        delta_dots=True)
    mixed = [ds2[i] if i % 2 else dict(ds2[i], ctx=dd[i]["ctx"]) for i in range(20)]
    check(strict, st2, mixed)


def test_config3_onepass(strict):
    base, deltas = W.config3(n_keys=200_000, n_replicas=64, touch=0.01, seed=5)
    check(strict, base, deltas)


def test_config3_onepass_equals_stepwise_large(strict, stepwise):
    """2M keys x 64 deltas: the one-pass fold and the step-by-step fold of join/3 agree
    row for row."""
    base, deltas = W.config3(n_keys=2_000_000, n_replicas=64, touch=0.01, seed=6)
    a, ac = run(strict, base, deltas)
    b, bc = run(stepwise, base, deltas)
    x, y = a.to_numpy(), b.to_numpy()
    assert a.n == b.n and all(np.array_equal(p, q) for p, q in zip(x, y))
    assert all(np.array_equal(p, q) for p, q in zip(ac.to_numpy(), bc.to_numpy()))


def test_prepared_apply_deltas(engine):
    """prepare_apply_deltas (arguments marshalled once, called repeatedly) == apply_deltas."""
    from delta_crdt_ex_amd.store import Context, Store
    st, ds = random_fold(24, n_keys=3000, k=10, p_full=0.2)
    s, c = up(st)
    dd = [up(d) for d in ds]
    ks = [None if d["keys"] is None else keys_dev(d["keys"]) for d in ds]
    a, ac = engine.apply_deltas(s, c, [x[0] for x in dd], [x[1] for x in dd], ks)
    out = Store.empty(s.n + sum(x[0].n for x in dd), DEV)
    octx = Context.empty(0, c.n + sum(x[1].n for x in dd), DEV)
    call = engine.prepare_apply_deltas(s, c, [x[0] for x in dd], [x[1] for x in dd], ks, out, octx)
    for _ in range(2):
        b, bc = call()
        assert a.n == b.n and all(np.array_equal(x, y) for x, y in zip(a.to_numpy(), b.to_numpy()))
        assert all(np.array_equal(x, y) for x, y in zip(ac.to_numpy(), bc.to_numpy()))
