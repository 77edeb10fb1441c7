"""The C oracle (oracle/deltaref.c, the SoA restatement and the timed CPU baseline)
against the term-level oracle (oracle/awlww_term.py, pinned by the reference's own
tests in test_oracle_reference_tests.py), and the synthetic generators against the
term oracle replaying the same operations."""
import numpy as np
import pytest

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.interning import Universe, splitmix64
from oracle import awlww_term as T
from oracle import convert as CV
from oracle import ref as R


def soa_to_term(rows, ctx):
    """Raw-id term state (keys/values/nodes are their integer ids)."""
    k, v, t, n, c = rows
    value = {}
    for i in range(len(k)):
        value.setdefault(int(k[i]), {}).setdefault((int(v[i]), int(t[i])), set()).add(
            (int(n[i]), int(c[i])))
    value = {key: {e: frozenset(d) for e, d in ents.items()} for key, ents in value.items()}
    kind, node, cnt = ctx
    if kind == R.DOTS:
        dots = frozenset((int(a), int(b)) for a, b in zip(node, cnt))
    else:
        dots = {int(a): int(b) for a, b in zip(node, cnt)}
    return T.AW(dots, value)


def term_to_soa_raw(state):
    ks, vs, ts, ns, cs = [], [], [], [], []
    for key, ents in state.value.items():
        for (val, t), dots in ents.items():
            for (nd, c) in dots:
                ks.append(key)
                vs.append(val)
                ts.append(t)
                ns.append(nd)
                cs.append(c)
    rows = CV.sort_rows(ks, vs, ts, ns, cs)
    d = state.dots
    if isinstance(d, frozenset):
        pairs = sorted(d)
        ctx = (R.DOTS, np.array([p[0] for p in pairs], np.uint32), np.array([p[1] for p in pairs], np.uint64))
    else:
        pairs = sorted(d.items())
        ctx = (R.VV, np.array([p[0] for p in pairs], np.uint32), np.array([p[1] for p in pairs], np.uint64))
    return rows, ctx


def rows_equal(a, b):
    return len(a[0]) == len(b[0]) and all(np.array_equal(x, y) for x, y in zip(a, b))


def ctx_equal(a, b):
    return a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])


CASES = [
    dict(n_keys=40, ts_range=1 << 40, dense_ctx=True, ctx_kind=W.VV),
    dict(n_keys=40, ts_range=2, dense_ctx=True, ctx_kind=W.VV),        # LWW ties
    dict(n_keys=40, ts_range=1 << 40, dense_ctx=False, ctx_kind=W.VV),  # store not covered by own VV (H5)
    dict(n_keys=30, ts_range=4, dense_ctx=False, ctx_kind=W.DOTS),
    dict(n_keys=30, ts_range=4, dense_ctx=True, ctx_kind=W.DOTS),
    dict(n_keys=0, ts_range=4, dense_ctx=True, ctx_kind=W.VV),          # empty
]


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("seed", range(12))
def test_join2_matches_term_oracle(case, seed):
    rng = np.random.default_rng(1000 * case + seed)
    a, b = W.random_pair(rng, **CASES[case])
    ta, tb = soa_to_term(a["rows"], a["ctx"]), soa_to_term(b["rows"], b["ctx"])
    all_keys = sorted(set(ta.value) | set(tb.value))
    keysets = [None, all_keys, all_keys[: len(all_keys) // 2],
               [x for x in all_keys if x % 3 == 0] + [12345]]
    for ks in keysets:
        rows, ctx = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"], keys=ks)
        want = T.join(ta, tb, all_keys if ks is None else ks)
        wrows, wctx = term_to_soa_raw(want)
        assert rows_equal(rows, wrows), f"keys={ks is None}"
        assert ctx_equal(ctx, wctx)
        assert R.store_check(rows)


@pytest.mark.parametrize("seed", range(10))
def test_read_and_contexts_match_term_oracle(seed):
    rng = np.random.default_rng(seed)
    a, b = W.random_pair(rng, n_keys=50, ts_range=3, ctx_kind=W.DOTS if seed % 2 else W.VV)
    ta = soa_to_term(a["rows"], a["ctx"])
    ok, ov = R.read_lww(a["rows"])
    want = T.read(ta)
    assert dict(zip(map(int, ok), map(int, ov))) == want
    assert list(map(int, ok)) == sorted(want)
    sub = sorted(want)[::3]
    ok2, ov2 = R.read_lww(a["rows"], keys=sub)
    assert dict(zip(map(int, ok2), map(int, ov2))) == T.read(ta, list(sub))
    # Dots.union / compress
    u = R.context_union(a["ctx"], b["ctx"])
    tu = T.dots_union(soa_to_term(a["rows"], a["ctx"]).dots, soa_to_term(b["rows"], b["ctx"]).dots)
    assert ctx_equal(u, term_to_soa_raw(T.AW(tu, {}))[1])
    if a["ctx"][0] == R.DOTS:
        cc = R.compress_dots(a["ctx"])
        tc = T.dots_compress(ta.dots)
        assert ctx_equal(cc, term_to_soa_raw(T.AW(tc, {}))[1])
    else:
        with pytest.raises(Exception):
            R.compress_dots(a["ctx"])


@pytest.mark.parametrize("seed", range(6))
def test_joink_is_left_fold(seed):
    rng = np.random.default_rng(77 + seed)
    reps = []
    for _ in range(3):
        a, b = W.random_pair(rng, n_keys=25, ts_range=8, dense_ctx=bool(seed % 2))
        reps += [a, b]
    rows, ctx = R.joink([r["rows"] for r in reps], [r["ctx"] for r in reps])
    acc_r, acc_c = reps[0]["rows"], reps[0]["ctx"]
    for r in reps[1:]:
        acc_r, acc_c = R.join2(acc_r, acc_c, r["rows"], r["ctx"])
    assert rows_equal(rows, acc_r) and ctx_equal(ctx, acc_c)
    terms = [soa_to_term(r["rows"], r["ctx"]) for r in reps]
    keys = sorted(set().union(*[set(t.value) for t in terms]))
    want = T.join_k(terms, keys)
    wr, wc = term_to_soa_raw(want)
    assert rows_equal(rows, wr) and ctx_equal(ctx, wc)


@pytest.mark.parametrize("seed", range(5))
def test_merkle_tree_differs_exactly_above_differing_keys(seed):
    rng = np.random.default_rng(seed)
    a, b = W.random_pair(rng, n_keys=300, ts_range=1 << 30)
    d = R.store_diff(a["rows"], b["rows"])
    for depth in (1, 3, 8, 12):
        ta, tb = R.merkle_build(a["rows"], depth), R.merkle_build(b["rows"], depth)
        # the differing buckets are exactly the buckets of the differing keys
        diff_b = np.flatnonzero(ta.level(depth) != tb.level(depth))
        assert np.array_equal(diff_b, np.unique(ta.bucket_of(d)))
        assert np.array_equal(R.merkle_diff(ta, a["rows"], tb, b["rows"]), d)
        same = R.merkle_build(a["rows"], depth)
        assert np.array_equal(same.nodes, ta.nodes)
        assert (ta.nodes[0] != tb.nodes[0]) == (len(d) > 0)
        assert ta.n_keys == len(np.unique(a["rows"][0]))
        keys, total = R.merkle_diff(ta, a["rows"], tb, b["rows"], cap=7)
        assert total == len(d) and np.array_equal(keys, d[:7])


@pytest.mark.parametrize("bits", [1, 2, 3])
def test_merkle_shard_trees_fold_to_the_unsharded_root(bits):
    from delta_crdt_ex_amd.sharding import shard_of
    a, _ = W.merkle_pair(n_keys=4000, seed=bits)
    depth = 10
    whole = R.merkle_build(a["rows"], depth)
    roots = []
    for s in range(1 << bits):
        m = shard_of(a["rows"][0], 1 << bits) == s
        t = R.merkle_build(tuple(c[m] for c in a["rows"]), depth - bits, bits, s)
        assert np.array_equal(t.nodes[0:1], whole.level(bits)[s:s + 1])
        roots.append(int(t.nodes[0]))
    assert R.fold_roots(roots) == int(whole.nodes[0])
    with pytest.raises(RuntimeError):  # a row outside the shard
        R.merkle_build(a["rows"], depth - bits, bits, 0)


@pytest.mark.parametrize("levels", [1, 3, 8])
def test_merkle_partial_diff_protocol_ends_in_the_diff(levels):
    a, b = W.merkle_pair(n_keys=3000, diff_frac=0.02, seed=levels)
    d = R.store_diff(a["rows"], b["rows"])
    depth = 9
    ta, tb = R.merkle_build(a["rows"], depth), R.merkle_build(b["rows"], depth)
    # A prepares, B continues, A continues, ... (the ping-pong of causal_crdt.ex:91-110)
    cont = R.merkle_prepare(ta, levels)
    side = [(tb, b["rows"]), (ta, a["rows"])]
    hops = 0
    while True:
        t, rows = side[hops % 2]
        res = R.merkle_continue(t, rows, cont, levels)
        hops += 1
        if res[0] == "ok":
            break
        cont = res[1]
    assert np.array_equal(res[1], d)
    assert hops == -(-depth // levels) + 1  # node hops down to the buckets, then the leaf hop


# ------------------------------------------------------------- generators vs term replay

def test_config1_generator_matches_term_replay():
    n = 200
    ga, gb = W.config1(n)
    N = ga["nodes"]
    n1, n2 = int(N.raw[1]), int(N.raw[2])  # the replicas' 30-bit node terms
    # replica 1 adds k => k with ts = k * 1000
    A = T.compress_dots(T.new())
    for k in range(1, n + 1):
        A = T.join(A, T.add(k, k, n1, A, k * 1000), [k])
    B = A
    for k in range(1, n + 1):
        if k % 10 == 0:
            A = T.join(A, T.remove(k, n1, A), [k])
    for k in range(1, n + 1):
        if k % 10 == 5:
            B = T.join(B, T.add(k, k + 1, n2, B, n * 1000 + k), [k])
    for term_state, gen in ((A, ga), (B, gb)):
        rows, ctx = CV.state_to_soa_ints(term_state, N)
        assert rows_equal(rows, gen["rows"])
        assert ctx_equal(ctx, gen["ctx"])
    # and the config-1 join (CPU path) agrees across the two oracles
    rows, ctx = R.join2(ga["rows"], ga["ctx"], gb["rows"], gb["ctx"])
    want = T.join(A, B, sorted(set(A.value) | set(B.value)))
    wrows, wctx = CV.state_to_soa_ints(want, N)
    assert rows_equal(rows, wrows) and ctx_equal(ctx, wctx)
    ok, ov = R.read_lww(rows)
    kterm = {splitmix64(k): k for k in range(1, n + 1)}
    got = {kterm[int(k)]: int(v) - (1 << 62) for k, v in zip(ok, ov)}
    assert got == T.read(want)


def test_config2_generator_matches_term_replay():
    n = 300
    ga, gb = W.config2(n_keys=n, seed=5)
    N = ga["nodes"]
    base = T.compress_dots(T.new())
    for k in range(1, n + 1):
        base = T.join(base, T.add(k, k, int(N.raw[0]), base, k * 1000), [k])
    kterm = {splitmix64(k): k for k in range(1, n + 1)}
    # recover the generator's choices (which keys, which values/ts) from its rows
    for logical, gen in ((1, ga), (2, gb)):
        k, v, t, nd, c = gen["rows"]
        mine = nd == N[logical]
        order = np.argsort(c[mine])
        st = base
        for kid, vid, ts in zip(k[mine][order], v[mine][order], t[mine][order]):
            key = kterm[int(kid)]
            val = int(vid) - (1 << 62)
            st = T.join(st, T.add(key, val, int(N.raw[logical]), st, int(ts)), [key])
        rows, ctx = CV.state_to_soa_ints(st, N)
        assert rows_equal(rows, gen["rows"])
        assert ctx_equal(ctx, gen["ctx"])


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_join2_mt_equals_single_thread(threads):
    """deltaref_mt.c (bench.py's all-core CPU baseline) == ref_join2, including more
    shards than keys and a skewed split."""
    from delta_crdt_ex_amd import workloads as W
    a, b = W.config2(n_keys=20_000, seed=5)
    want_rows, want_ctx = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    got_rows, got_ctx = R.JoinMT(a["rows"], a["ctx"], b["rows"], b["ctx"], threads)()
    assert rows_equal(got_rows, want_rows) and ctx_equal(got_ctx, want_ctx)
    small = tuple(c[:5] for c in a["rows"])
    want_rows, _ = R.join2(small, a["ctx"], b["rows"], b["ctx"])
    got_rows, _ = R.JoinMT(small, a["ctx"], b["rows"], b["ctx"], threads)()
    assert rows_equal(got_rows, want_rows)
