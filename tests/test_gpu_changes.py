"""dg_join2_changes on cuda:0: the join's rows and context equal
dg_join2's, and its changed keys equal the C oracle's exact per-key row-set diff
restricted to `keys` (ref.changed_keys; tests/test_configs.py pins that to the term
oracle's diff/3 of causal_crdt.ex:343-351).  Plus delta_subscriber_test.exs:20-27
restated step for step through the CausalCrdt mirror, and op histories with nil values
against the oracle's diffs_to_callback/3."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as hst

from delta_crdt_ex_amd import aw_lww_map as M
from delta_crdt_ex_amd import causal_crdt as CC
from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.store import u64
from delta_crdt_ex_amd.terms import Atom
from kfold_cases import random_fold
from oracle import awlww_term as T
from oracle import ref as R
from oracle.erlterm import tg
from test_gpu_configs import keys_dev
from test_gpu_parity import ctx_eq, rows_eq, up

pytestmark = pytest.mark.gpu


def check(engine, a, b, keys=None):
    sa, ca = up(a)
    sb, cb = up(b)
    kt = None if keys is None else keys_dev(keys)
    out, octx, ch = engine.join2_changes(sa, ca, sb, cb, keys=kt)
    wr, wc = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"], keys)
    rows_eq(out, wr)
    ctx_eq(octx, wc)
    want = R.changed_keys(a["rows"], wr, keys)
    assert np.array_equal(u64(ch), want), (len(u64(ch)), len(want))
    return len(want)


def test_changes_config2(engine):
    a, b = W.config2(n_keys=300_000, seed=2)
    assert check(engine, a, b) > 1000


def test_changes_config5(engine):
    a, b = W.config5(n_keys=100_000, n_nodes=64, seed=3)
    assert check(engine, a, b) > 1000


@pytest.mark.parametrize("seed", range(4))
def test_changes_keyed(engine, seed):
    """Keyed joins: removals, adds, rows outside `keys` (carried, never reported)."""
    st, ds = random_fold(50 + seed, n_keys=4000, k=1, rows_per_key=4, p_keys=0.2, p_take=0.6,
                         p_outside=0.05)
    d = ds[0]
    assert check(engine, st, d, d["keys"]) > 10


def test_changes_edges(engine):
    a, b = W.config2(n_keys=5000, seed=4)
    # joining a state with itself changes nothing
    assert check(engine, a, a) == 0
    # an empty keyset: nothing joined, nothing reported
    assert check(engine, a, b, np.zeros(0, np.uint64)) == 0
    # empty sides
    e = {"rows": tuple(c[:0] for c in a["rows"]), "ctx": a["ctx"]}
    assert check(engine, e, b) > 0
    check(engine, a, e)
    check(engine, e, e)


def test_changes_large_properties(engine):
    """2M keys: the changed set is large, ascending and unique, and joining the same
    delta into the result again changes nothing (join is idempotent)."""
    a, b = W.config2(n_keys=2_000_000, seed=8)
    sa, ca = up(a)
    sb, cb = up(b)
    out, octx, ch = engine.join2_changes(sa, ca, sb, cb)
    c = u64(ch)
    assert len(c) > 100_000 and np.all(c[1:] > c[:-1])
    _, _, again = engine.join2_changes(out, octx, sb, cb)
    assert again.numel() == 0


def test_delta_subscriber_scenario():
    """delta_subscriber_test.exs:20-27 step for step: the first add reports {:add, k, v};
    adding the same value again changes the key's dots but not its value, so on_diffs
    receives []; `add "Derek" nil` reports {:remove, "Derek"} (H9: Map.get of a nil value
    is nil); removing the nil value then reports [] ({nil, nil} matches {old, old})."""
    st = M.compress_dots(M.new())
    st, diffs = CC.update_state_with_delta(st, M.add("Derek", "Kraan", 1, st), ["Derek"])
    assert diffs == [("add", "Derek", "Kraan")]
    st, diffs = CC.update_state_with_delta(st, M.add("Derek", "Kraan", 1, st), ["Derek"])
    assert diffs == []
    st, diffs = CC.update_state_with_delta(st, M.add("Derek", None, 1, st), ["Derek"])
    assert diffs == [("remove", "Derek")]
    assert M.read(st) == {"Derek": None}
    st, diffs = CC.update_state_with_delta(st, M.remove("Derek", 1, st), ["Derek"])
    assert diffs == []
    # removing an absent key changes no raw value map: on_diffs is not called
    st, diffs = CC.update_state_with_delta(st, M.remove("Derek", 1, st), ["Derek"])
    assert diffs is None
    # a key the delta does not touch: no diff at all
    st, diffs = CC.update_state_with_delta(st, M.add("Other", 1, 1, st), ["Nope"])
    assert diffs is None


_VALS = [None, 0, 1, 1.0, -0.0, True, Atom("nil_not"), "Kraan", b"x", (1, None)]


@settings(max_examples=40, deadline=None, suppress_health_check=list(HealthCheck))
@given(hst.lists(hst.tuples(hst.sampled_from(["add", "remove"]), hst.integers(0, 3),
                            hst.integers(0, len(_VALS) - 1), hst.integers(0, 2)),
                 min_size=1, max_size=14))
def test_on_diffs_histories_match_oracle(ops):
    """Op histories with nil values (and 1 / 1.0 / true, which BEAM keeps apart) through
    the mirror's update_state_with_delta equal the term oracle's diffs_to_callback
    (causal_crdt.ex:361-404) call for call."""
    st = M.compress_dots(M.new())
    ref = T.compress_dots(T.new())
    t = 1000
    for op, k, v, node in ops:
        key, val = f"k{k}", _VALS[v]
        t += 1
        if op == "add":
            d, rd = M.add(key, val, node, st, ts=t), T.add(tg(key), tg(val), node, ref, t)
        else:
            d, rd = M.remove(key, node, st), T.remove(tg(key), node, ref)
        st, got = CC.update_state_with_delta(st, d, [key])
        ref, want = T.update_state_with_delta(ref, rd, [tg(key)])
        norm = None if got is None else [(g[0],) + tuple(tg(x) for x in g[1:]) for g in got]
        wnorm = None if want is None else [(w[0],) + tuple(tg(x) for x in w[1:]) for w in want]
        assert norm == wnorm, (op, key, val)
    assert {tg(k): tg(v) for k, v in M.read(st).items()} == T.read(ref)


def test_changes_sparse_keyed_multichunk(engine):
    """A keyed join touching a few dozen keys of a 4.3M-key state: ~4200 tiles, almost all
    without change events, so an event tile's nearest non-empty predecessor can lie a
    chunk (of 4096 tiles) back in the changed-key scan."""
    a, b = W.config2(n_keys=4_300_000, seed=11)
    rng = np.random.default_rng(11)
    keys = np.unique(rng.choice(a["rows"][0], size=40, replace=False)).astype(np.uint64)
    sel = np.isin(b["rows"][0], keys)
    bs = {"rows": tuple(c[sel] for c in b["rows"]), "ctx": b["ctx"]}
    n = check(engine, a, bs, keys)
    assert 0 < n <= len(keys)
