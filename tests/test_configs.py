"""BASELINE configs 3, 4 and 5 on the CPU: each generator against the term oracle
replaying the same operations (AWLWWMap.add/4, remove/3 joined as CausalCrdt does),
and the C oracle's keyed delta fold / join / read against the term oracle.  The GPU
side of the same configs is tests/test_gpu_configs.py."""
import numpy as np
import pytest

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.interning import Universe, splitmix64
from oracle import awlww_term as T
from oracle import convert as CV
from oracle import ref as R
from test_c_oracle import ctx_equal, rows_equal, soa_to_term, term_to_soa_raw


def _base_term(n, node=0):
    """Replica `node` (a node term) adds k => k with ts = k * 1000 for k = 1..n (config
    2/3 base)."""
    st = T.compress_dots(T.new())
    for k in range(1, n + 1):
        st = T.join(st, T.add(k, k, node, st, k * 1000), [k])
    return st


def _take(state, keys):
    return T.AW(state.dots, {k: v for k, v in state.value.items() if k in keys})


# ------------------------------------------------------------------ config 3

def test_config3_generator_matches_term_replay():
    n, R_ = 150, 3
    base, deltas = W.config3(n_keys=n, n_replicas=R_, touch=0.12, seed=11)
    N = base["nodes"]
    assert all(1 <= x <= 1_000_000_000 for x in N.raw.tolist())  # :rand.uniform(1e9) terms
    kterm = {splitmix64(k): k for k in range(1, n + 1)}
    st0 = _base_term(n, int(N.raw[0]))
    rows, ctx = CV.state_to_soa_ints(st0, N)
    assert rows_equal(rows, base["rows"]) and ctx_equal(ctx, base["ctx"])
    for r, d in enumerate(deltas, start=1):
        keys = [kterm[int(x)] for x in d["keys"]]
        k, v, t, nd, c = d["rows"]
        adds = {kterm[int(k[i])]: (int(v[i]) - (1 << 62), int(t[i]), int(c[i])) for i in range(len(k))}
        st = st0
        # adds in counter order (next_dot numbers them), removes anywhere
        for key, (val, ts, _c) in sorted(adds.items(), key=lambda kv: kv[1][2]):
            st = T.join(st, T.add(key, val, int(N.raw[r]), st, ts), [key])
        for key in keys:
            if key not in adds:
                st = T.join(st, T.remove(key, int(N.raw[r]), st), [key])
        delta = _take(st, set(keys))
        drows, dctx = CV.state_to_soa_ints(delta, N)
        assert rows_equal(drows, d["rows"]), r
        assert ctx_equal(dctx, d["ctx"]), r


@pytest.mark.parametrize("seed", range(3))
def test_config3_keyed_fold_two_oracles(seed):
    """C restatement's fold of join(state, delta_i, keys_i) == the term oracle's."""
    base, deltas = W.config3(n_keys=200, n_replicas=6, touch=0.1, seed=seed)
    rows, ctx = R.apply_deltas(base["rows"], base["ctx"], [d["rows"] for d in deltas],
                               [d["ctx"] for d in deltas], [d["keys"] for d in deltas])
    st = soa_to_term(base["rows"], base["ctx"])
    for d in deltas:
        st = T.join(st, soa_to_term(d["rows"], d["ctx"]), [int(x) for x in d["keys"]])
    wrows, wctx = term_to_soa_raw(st)
    assert rows_equal(rows, wrows) and ctx_equal(ctx, wctx)
    # every touched key: the base row is gone; added keys carry their new rows
    touched = np.unique(np.concatenate([d["keys"] for d in deltas]))
    assert not np.any(np.isin(rows[0][rows[3] == base["nodes"][0]], touched))


def test_config3_keys_outside_keyset_are_right_biased():
    """A delta row whose key is not in the delta's keys replaces the state's rows of
    that key (Map.merge(Map.drop(..)) at aw_lww_map.ex:185-188) -- both oracles."""
    base, deltas = W.config3(n_keys=100, n_replicas=2, touch=0.2, seed=9)
    d = deltas[0]
    keys = d["keys"][: len(d["keys"]) // 2]
    rows, ctx = R.apply_deltas(base["rows"], base["ctx"], [d["rows"]], [d["ctx"]], [keys])
    st = T.join(soa_to_term(base["rows"], base["ctx"]), soa_to_term(d["rows"], d["ctx"]),
                [int(x) for x in keys])
    wrows, wctx = term_to_soa_raw(st)
    assert rows_equal(rows, wrows) and ctx_equal(ctx, wctx)


# ------------------------------------------------------------------ config 5

def test_config5_generator_matches_term_replay():
    """The config-5 generator's rows are what the reference's own mutators produce: every
    base writer adds its entries in key order (aw_lww_map.ex:99-112), replicas A and B
    re-add (add/4) and remove (remove/3) keys.  A writer's counter before an add is set
    to the generator's counter - 1 in its context, as its adds to keys elsewhere (other
    shards; later removed) would have left it -- next_dot takes vv[node] + 1 (:30-37)."""
    n, nn, seed = 50, 8, 3
    a, b = W.config5(n_keys=n, n_nodes=nn, seed=seed)
    N = a["nodes"]
    me, Wn = 3, nn - 2
    k = np.arange(1, n + 1, dtype=np.uint64)
    ne = (W._draw(k, seed, 1) % np.uint64(me)).astype(np.int64) + 1
    h = W._draw(k, seed, 2) % np.uint64(Wn)
    writers = {}
    for x in range(n):
        for j in range(int(ne[x])):
            w = int((h[x] + np.uint64(j)) % np.uint64(Wn))
            ek = np.array([(x + 1) * me + j], np.uint64)
            val = int(W._draw(ek, seed, 3)[0] % np.uint64(4))
            ts = int(W._draw(ek, seed, 4)[0] % np.uint64(16))
            writers.setdefault(w, []).append((x + 1, (x + 1) * me + j + 1, val, ts))
    base = T.compress_dots(T.new())
    for w, adds in writers.items():
        st = T.compress_dots(T.new())
        term = int(N.raw[w])
        for key, cnt, val, ts in adds:
            st = T.AW({**st.dots, term: cnt - 1}, st.value)  # its adds elsewhere
            st = T.join(st, T.add(key, val, term, st, ts), [key])
        base = T.join(base, st, sorted(set(base.value) | set(st.value)))
    base = T.AW({**base.dots, **{int(N.raw[w]): n * me + me for w in range(Wn)}}, base.value)
    for r, (node_id, gen) in enumerate(((nn - 2, a), (nn - 1, b))):
        term = int(N.raw[node_id])
        u = W._draw(k, seed, 10 + r)
        removed = (u % np.uint64(1 << 20)).astype(np.float64) < 0.5 * (1 << 20)
        v = W._draw(k, seed, 20 + r)
        readd = (~removed) & ((v % np.uint64(1 << 20)).astype(np.float64) < 0.2 * (1 << 20))
        st = base
        for x in np.flatnonzero(readd):
            key = int(x) + 1
            kk = np.array([key], np.uint64)
            val = int(W._draw(kk, seed, 30 + r)[0] % np.uint64(4))
            ts = int(W._draw(kk, seed, 40 + r)[0] % np.uint64(16))
            st = T.AW({**st.dots, term: key - 1}, st.value)
            st = T.join(st, T.add(key, val, term, st, ts), [key])
        for x in np.flatnonzero(removed):
            key = int(x) + 1
            st = T.join(st, T.remove(key, term, st), [key])
        st = T.AW({**st.dots, term: n}, st.value)  # its VV entry: the whole key space's
        rows, ctx = CV.state_to_soa_ints(st, N)
        assert rows_equal(rows, gen["rows"]), node_id
        assert ctx_equal(ctx, gen["ctx"]), node_id


@pytest.mark.parametrize("seed", range(3))
def test_config5_join_and_read_two_oracles(seed):
    a, b = W.config5(n_keys=80, n_nodes=10, seed=seed)
    rows, ctx = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    ta, tb = soa_to_term(a["rows"], a["ctx"]), soa_to_term(b["rows"], b["ctx"])
    want = T.join(ta, tb, sorted(set(ta.value) | set(tb.value)))
    wrows, wctx = term_to_soa_raw(want)
    assert rows_equal(rows, wrows) and ctx_equal(ctx, wctx)
    ok, ov = R.read_lww(rows)
    assert dict(zip(map(int, ok), map(int, ov))) == T.read(want)


# ------------------------------------------------------------------ config 4

@pytest.mark.parametrize("rank", range(4))
def test_config4_shard_anti_entropy_round(rank):
    """Per key-hash shard: the Merkle diff is the exact set of differing keys, and
    joining B's sync delta for those keys into A (causal_crdt.ex:324-335,383-384)
    equals the full-state join of the shard."""
    a, b = W.config4_shard(rank, 4, keys_per_rank=600, diff_frac=0.05)
    diff = R.store_diff(a["rows"], b["rows"])
    ta, tb = R.merkle_build(a["rows"], 8), R.merkle_build(b["rows"], 8)
    assert np.array_equal(R.merkle_diff(ta, a["rows"], tb, b["rows"]), diff)
    d = W.sync_delta(b, diff)
    rows, ctx = R.apply_deltas(a["rows"], a["ctx"], [d["rows"]], [d["ctx"]], [d["keys"]])
    frows, fctx = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    assert rows_equal(rows, frows) and ctx_equal(ctx, fctx)


# ------------------------------------------------------------------ keyed fold, adversarial

@pytest.mark.parametrize("seed", range(3))
def test_random_keyed_fold_two_oracles(seed):
    """The adversarial generator the GPU one-pass fold is tested on (tests/kfold_cases.py):
    the C restatement's delta-by-delta fold == the term oracle's, including shared tuples,
    rows outside keysets, full-state deltas and empty keysets."""
    from kfold_cases import random_fold
    st, ds = random_fold(seed, n_keys=40, k=6, rows_per_key=4, p_keys=0.3, p_take=0.6,
                         p_outside=0.1, p_full=0.2)
    if seed == 1:
        ds[0] = dict(ds[0], keys=np.zeros(0, np.uint64))
    rows, ctx = R.apply_deltas(st["rows"], st["ctx"], [d["rows"] for d in ds],
                               [d["ctx"] for d in ds], [d["keys"] for d in ds])
    t = soa_to_term(st["rows"], st["ctx"])
    for d in ds:
        dt = soa_to_term(d["rows"], d["ctx"])
        ks = sorted(set(t.value) | set(dt.value)) if d["keys"] is None else [int(x) for x in d["keys"]]
        t = T.join(t, dt, ks)
    wrows, wctx = term_to_soa_raw(t)
    assert rows_equal(rows, wrows) and ctx_equal(ctx, wctx)


# ------------------------------------------------------------------ changed keys (§8(f).1)

@pytest.mark.parametrize("seed", range(4))
def test_changed_keys_two_oracles(seed):
    """The changed keys dg_join2_changes is checked against (ref.changed_keys: the
    exact per-key row-set diff, restricted to `keys`) == the keys of the term oracle's
    diff/3 (causal_crdt.ex:343-351) after join/3."""
    from kfold_cases import random_fold
    st, ds = random_fold(40 + seed, n_keys=60, k=1, rows_per_key=4, p_keys=0.4, p_take=0.6,
                         p_outside=0.1, p_full=0.3 if seed == 3 else 0.0)
    d = ds[0]
    rows, ctx = R.join2(st["rows"], st["ctx"], d["rows"], d["ctx"], d["keys"])
    got = R.changed_keys(st["rows"], rows, d["keys"])
    old, dt = soa_to_term(st["rows"], st["ctx"]), soa_to_term(d["rows"], d["ctx"])
    keys = sorted(set(old.value) | set(dt.value)) if d["keys"] is None else [int(x) for x in d["keys"]]
    new = T.join(old, dt, keys)
    want = sorted(x[1] for x in T.causal_diff(old, new, keys))
    assert [int(x) for x in got] == want
    assert len(want) > 0


# ------------------------------------------------------------------ batched mutations (§8(f).3)

@pytest.mark.parametrize("seed", range(4))
def test_mutate_batch_equals_op_by_op(seed):
    """The batch delta (ref.mutate_batch, which dg_mutate_batch is checked against)
    joined with keys = the touched keys equals applying the ops one by one as
    CausalCrdt does (causal_crdt.ex:337-342: join(state, add/remove delta, [key]))."""
    from kfold_cases import random_fold
    rng = np.random.default_rng(seed)
    st0, _ = random_fold(60 + seed, n_keys=30, k=0, n_nodes=4, rows_per_key=3, p_state=0.7)
    ctx = R.compress_dots((1, *[np.asarray(x) for x in st0["ctx"][1:]])) if st0["ctx"][0] == 1 \
        else st0["ctx"]
    keys = np.unique(st0["rows"][0])
    node = 7
    ops = []
    for i in range(40):
        k = int(keys[rng.integers(0, len(keys))]) if rng.random() < 0.8 else int(rng.integers(1, 1 << 60))
        if rng.random() < 0.7:
            ops.append(("add", k, int(rng.integers(0, 5)) + (1 << 62), int(rng.integers(0, 50))))
        else:
            ops.append(("remove", k, 0, 0))
    # op by op on the term oracle
    t = soa_to_term(st0["rows"], ctx)
    for kind, k, v, ts in ops:
        d = T.add(k, v, node, t, ts) if kind == "add" else T.remove(k, node, t)
        t = T.join(t, d, [k])
    want_rows, want_ctx = term_to_soa_raw(t)
    # the batch delta, joined once
    drows, dctx, dkeys = R.mutate_batch(st0["rows"], ctx, node, ops)
    got_rows, got_ctx = R.join2(st0["rows"], ctx, drows, dctx, dkeys)
    assert rows_equal(got_rows, want_rows)
    assert ctx_equal(got_ctx, want_ctx)
