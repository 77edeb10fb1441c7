"""ctypes wrapper around oracle/_build/libdeltaref.so (the C restatement) over
numpy arrays.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Rows are a tuple of five numpy arrays ``(key u64, val u64, ts i64, node u32, cnt u64)``
sorted by the full tuple; a context is ``(kind, node u32, cnt u64)``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from delta_crdt_ex_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libdeltaref.so")

VV, DOTS = _abi.DG_CTX_VV, _abi.DG_CTX_DOTS

_lib = None


def build():
    r = subprocess.run(["make", "-s", "-C", HERE], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + r.stdout + r.stderr)
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()  # make: a no-op when libdeltaref.so is newer than its sources
        L = C.CDLL(LIB)
        S, X = C.POINTER(_abi.dg_store), C.POINTER(_abi.dg_context)
        L.ref_join2.argtypes = [S, X, S, X, _abi.P64, C.c_uint64, S, X]
        L.ref_joink.argtypes = [C.c_int, S, X, S, X]
        L.ref_join2_mt.argtypes = [S, X, S, X, _abi.P64, C.c_uint64, S, X, S, C.c_int]
        L.ref_context_union.argtypes = [X, X, X]
        L.ref_compress_dots.argtypes = [X, X]
        L.ref_read_lww.argtypes = [S, _abi.P64, C.c_uint64, _abi.P64, _abi.P64, C.c_uint64,
                                   _abi.P64]
        TH = C.POINTER(_abi.dg_term_hashes)
        L.ref_merkle_build.argtypes = [S, C.c_uint32, C.c_uint32, C.c_uint64, TH, _abi.P64,
                                       C.c_void_p, _abi.P64]
        L.ref_term_val.argtypes = [TH, C.c_uint64]
        L.ref_term_val.restype = C.c_uint64
        L.ref_term_node.argtypes = [TH, C.c_uint32]
        L.ref_term_node.restype = C.c_uint64
        L.ref_store_diff.argtypes = [S, S, _abi.P64, C.c_uint64, _abi.P64]
        L.ref_store_check.argtypes = [S]
        L.ref_row_hash.argtypes = [C.c_uint64, C.c_uint64, C.c_int64, C.c_uint64, C.c_uint64]
        L.ref_row_hash.restype = C.c_uint64
        L.ref_node_hash.argtypes = [C.c_uint64, C.c_uint64]
        L.ref_node_hash.restype = C.c_uint64
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def empty_rows(n=0):
    return (np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(n, np.int64),
            np.zeros(n, np.uint32), np.zeros(n, np.uint64))


def as_rows(rows):
    k, v, t, nd, c = rows
    return (np.ascontiguousarray(k, np.uint64), np.ascontiguousarray(v, np.uint64),
            np.ascontiguousarray(t, np.int64), np.ascontiguousarray(nd, np.uint32),
            np.ascontiguousarray(c, np.uint64))


def _store(rows, cap=None):
    rows = as_rows(rows)
    s = _abi.dg_store()
    s.key = rows[0].ctypes.data
    s.val = rows[1].ctypes.data
    s.ts = rows[2].ctypes.data
    s.node = rows[3].ctypes.data
    s.cnt = rows[4].ctypes.data
    s.n = len(rows[0])
    s.cap = len(rows[0]) if cap is None else cap
    return s, rows


def _ctx(ctx):
    kind, node, cnt = ctx
    node = np.ascontiguousarray(node, np.uint32)
    cnt = np.ascontiguousarray(cnt, np.uint64)
    c = _abi.dg_context()
    c.kind = kind
    c.node = node.ctypes.data
    c.cnt = cnt.ctypes.data
    c.n = len(node)
    c.cap = len(node)
    return c, (kind, node, cnt)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with {rc}")


def join2(a, ca, b, cb, keys=None):
    """AWLWWMap.join/3 over SoA rows (aw_lww_map.ex:153-209)."""
    sa, a = _store(a)
    sb, b = _store(b)
    xa, ca = _ctx(ca)
    xb, cb = _ctx(cb)
    n = len(a[0]) + len(b[0])
    out = empty_rows(n + 1)
    so, _ = _store(out, cap=n)
    so.n = 0
    nc = len(ca[1]) + len(cb[1])
    onode, ocnt = np.zeros(nc + 1, np.uint32), np.zeros(nc + 1, np.uint64)
    xo, _ = _ctx((VV, onode, ocnt))
    xo.cap = nc
    if keys is not None:
        keys = np.ascontiguousarray(np.unique(np.asarray(keys, np.uint64)))
        kp, nk = _p(keys, _abi.P64), len(keys)
    else:
        kp, nk = None, 0
    _check(lib().ref_join2(C.byref(sa), C.byref(xa), C.byref(sb), C.byref(xb), kp, nk,
                           C.byref(so), C.byref(xo)), "ref_join2")
    m = so.n
    return tuple(col[:m] for col in out), (xo.kind, onode[: xo.n], ocnt[: xo.n])


class JoinMT:
    """join/3 of the C restatement on `threads` host cores (deltaref_mt.c: key-range
    shards under OpenMP), with its output and scratch buffers allocated once for
    repeated calls on inputs of the same sizes (bench.py's cpu_baseline)."""

    def __init__(self, a, ca, b, cb, threads):
        self.sa, self.a = _store(a)
        self.sb, self.b = _store(b)
        self.xa, self.ca = _ctx(ca)
        self.xb, self.cb = _ctx(cb)
        n = len(self.a[0]) + len(self.b[0])
        self.out, self.tmp = empty_rows(n + 1), empty_rows(n + 1)
        self.so, _ = _store(self.out, cap=n)
        self.st, _ = _store(self.tmp, cap=n)
        nc = len(self.ca[1]) + len(self.cb[1])
        self.onode, self.ocnt = np.zeros(nc + 1, np.uint32), np.zeros(nc + 1, np.uint64)
        self.xo, _ = _ctx((VV, self.onode, self.ocnt))
        self.xo.cap = nc
        self.threads = threads

    def __call__(self):
        self.so.n = 0
        _check(lib().ref_join2_mt(C.byref(self.sa), C.byref(self.xa), C.byref(self.sb),
                                  C.byref(self.xb), None, 0, C.byref(self.so), C.byref(self.xo),
                                  C.byref(self.st), self.threads), "ref_join2_mt")
        m = self.so.n
        return (tuple(col[:m] for col in self.out),
                (self.xo.kind, self.onode[: self.xo.n], self.ocnt[: self.xo.n]))


def joink(stores, ctxs):
    k = len(stores)
    keep = []
    S = (_abi.dg_store * k)()
    X = (_abi.dg_context * k)()
    for i in range(k):
        S[i], r = _store(stores[i])
        X[i], c = _ctx(ctxs[i])
        keep.append((r, c))
    n = sum(len(s[0]) for s in stores)
    nc = sum(len(c[1]) for c in ctxs)
    out = empty_rows(n + 1)
    so, _ = _store(out, cap=n)
    so.n = 0
    onode, ocnt = np.zeros(nc + 1, np.uint32), np.zeros(nc + 1, np.uint64)
    xo, _ = _ctx((VV, onode, ocnt))
    xo.cap = nc
    _check(lib().ref_joink(k, S, X, C.byref(so), C.byref(xo)), "ref_joink")
    return tuple(col[: so.n] for col in out), (xo.kind, onode[: xo.n], ocnt[: xo.n])


def apply_deltas(state, ctx, deltas, dctxs, keys=None):
    """Left fold of join(state, delta_i, keys_i) (causal_crdt.ex:383-384): the C
    restatement's join/3 applied once per delta.  keys[i] None = all keys."""
    for i, (d, c) in enumerate(zip(deltas, dctxs)):
        state, ctx = join2(state, ctx, d, c, None if keys is None else keys[i])
    return state, ctx


def context_union(ca, cb):
    xa, ca = _ctx(ca)
    xb, cb = _ctx(cb)
    nc = len(ca[1]) + len(cb[1])
    onode, ocnt = np.zeros(nc + 1, np.uint32), np.zeros(nc + 1, np.uint64)
    xo, _ = _ctx((VV, onode, ocnt))
    xo.cap = nc
    _check(lib().ref_context_union(C.byref(xa), C.byref(xb), C.byref(xo)), "ref_context_union")
    return (xo.kind, onode[: xo.n], ocnt[: xo.n])


def compress_dots(c):
    xa, c = _ctx(c)
    onode, ocnt = np.zeros(len(c[1]) + 1, np.uint32), np.zeros(len(c[1]) + 1, np.uint64)
    xo, _ = _ctx((VV, onode, ocnt))
    xo.cap = len(c[1])
    rc = lib().ref_compress_dots(C.byref(xa), C.byref(xo))
    if rc == _abi.DG_E_CLAUSE:
        raise _abi.FunctionClauseError(rc, "compress/1 on a VV")
    _check(rc, "ref_compress_dots")
    return (xo.kind, onode[: xo.n], ocnt[: xo.n])


def read_lww(rows, keys=None):
    s, rows = _store(rows)
    n = len(rows[0])
    ok, ov = np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64)
    cnt = np.zeros(1, np.uint64)
    if keys is not None:
        keys = np.ascontiguousarray(np.unique(np.asarray(keys, np.uint64)))
        kp, nk = _p(keys, _abi.P64), len(keys)
    else:
        kp, nk = None, 0
    _check(lib().ref_read_lww(C.byref(s), kp, nk, _p(ok, _abi.P64), _p(ov, _abi.P64), n,
                              _p(cnt, _abi.P64)), "ref_read_lww")
    m = int(cnt[0])
    return ok[:m], ov[:m]


class Terms:
    """Term-hash tables (dg_term_hashes) as host arrays: node_hash[node id], and the
    ascending non-canonical value ids with their hashes (interning.Universe.term_tables)."""

    def __init__(self, node_hash, val_id, val_hash):
        self.arrays = (np.ascontiguousarray(node_hash, np.uint64),
                       np.ascontiguousarray(val_id, np.uint64),
                       np.ascontiguousarray(val_hash, np.uint64))
        nh, vi, vh = self.arrays
        self.c = _abi.dg_term_hashes(nh.ctypes.data, len(nh), vi.ctypes.data, vh.ctypes.data, len(vi))

    def ptr(self):
        return C.pointer(self.c)


class Tree:
    """The oracle's Merkle tree (deltaref.c ref_merkle_build): `nodes` in level order,
    `counts` rows per bucket, `terms` the term hashes it was built with (or None)."""

    def __init__(self, depth, shard_bits=0, shard=0, terms=None):
        self.depth, self.shard_bits, self.shard = depth, shard_bits, shard
        self.nodes = np.zeros(2 * (1 << depth) - 1, np.uint64)
        self.counts = np.zeros(1 << depth, np.uint16)
        self.n_keys = 0
        self.terms = terms

    def level(self, lv):
        return self.nodes[(1 << lv) - 1: (1 << (lv + 1)) - 1]

    def bucket_of(self, keys):
        k = np.asarray(keys, np.uint64)
        with np.errstate(over="ignore"):
            return ((k << np.uint64(self.shard_bits)) >> np.uint64(64 - self.depth)).astype(np.int64)


def merkle_build(rows, depth, shard_bits=0, shard=0, terms: Terms | None = None):
    s, rows = _store(rows)
    t = Tree(depth, shard_bits, shard, terms)
    nk = np.zeros(1, np.uint64)
    _check(lib().ref_merkle_build(C.byref(s), depth, shard_bits, shard,
                                  terms.ptr() if terms is not None else None,
                                  _p(t.nodes, _abi.P64), t.counts.ctypes.data, _p(nk, _abi.P64)),
           "ref_merkle_build")
    t.n_keys = int(nk[0])
    return t


def row_hashes(rows, terms: Terms | None = None) -> np.ndarray:
    """The Merkle row hash of every row (with the tree's term hashes, if any)."""
    L = lib()
    th = terms.ptr() if terms is not None else None
    k, v, t, nd, c = as_rows(rows)
    return np.array([L.ref_row_hash(int(k[i]), L.ref_term_val(th, int(v[i])), int(t[i]),
                                    L.ref_term_node(th, int(nd[i])), int(c[i]))
                     for i in range(len(k))], np.uint64)


def merkle_diff(ta: Tree, ra, tb: Tree, rb, cap=None):
    """The keys whose raw value maps differ (hash trees agree with the exact row-set diff
    barring a 64-bit collision), ascending; with `cap`: (first cap keys, total) -- the
    reference's Enum.take(keys, max_sync_size), causal_crdt.ex:105,206-210."""
    assert (ta.depth, ta.shard_bits, ta.shard) == (tb.depth, tb.shard_bits, tb.shard)
    d = store_diff(ra, rb)
    return d if cap is None else (d[:cap], len(d))


def fold_roots(roots):
    """The unsharded root from 2^b shard roots (shard order)."""
    lv = [int(x) for x in roots]
    while len(lv) > 1:
        lv = [int(lib().ref_node_hash(lv[2 * i], lv[2 * i + 1])) for i in range(len(lv) // 2)]
    return lv[0]


def leaf_pairs(rows, tree: Tree, buckets):
    """(key, Σ row hash) of every key of `rows` in the given buckets, ascending."""
    L = lib()
    th = tree.terms.ptr() if tree.terms is not None else None
    k = rows[0]
    b = tree.bucket_of(k)
    m = np.isin(b, np.asarray(buckets, np.int64))
    keys, hs = [], []
    for i in np.flatnonzero(m):
        h = int(L.ref_row_hash(int(k[i]), L.ref_term_val(th, int(rows[1][i])), int(rows[2][i]),
                               L.ref_term_node(th, int(rows[3][i])), int(rows[4][i])))
        if keys and keys[-1] == int(k[i]):
            hs[-1] = (hs[-1] + h) & ((1 << 64) - 1)
        else:
            keys.append(int(k[i]))
            hs.append(h)
    return np.array(keys, np.uint64), np.array(hs, np.uint64)


def merkle_prepare(t: Tree, levels):
    """prepare_partial_diff: ("node", level, positions, hashes) of level min(levels, depth)."""
    L = min(levels, t.depth)
    return ("node", L, np.arange(1 << L, dtype=np.uint64), t.level(L).copy())


def merkle_continue(t: Tree, rows, cont, levels):
    """continue_partial_diff on the receiver (tree t over rows) -- the protocol
    include/deltagpu.h documents: ("ok", keys) or ("continue", cont')."""
    if cont[0] == "leaf":
        _, buckets, pk, ph = cont
        own_k, own_h = leaf_pairs(rows, t, buckets)
        mine = dict(zip(own_k.tolist(), own_h.tolist()))
        theirs = dict(zip(np.asarray(pk).tolist(), np.asarray(ph).tolist()))
        keys = sorted(k for k in set(mine) | set(theirs) if mine.get(k) != theirs.get(k))
        return ("ok", np.array(keys, np.uint64))
    _, L, pos, hs = cont
    own = t.level(L)[np.asarray(pos, np.int64)]
    dpos = np.asarray(pos, np.uint64)[own != np.asarray(hs, np.uint64)]
    if len(dpos) == 0:
        return ("ok", np.zeros(0, np.uint64))
    if L < t.depth:
        k = min(levels, t.depth - L)
        child = ((dpos[:, None] << np.uint64(k)) | np.arange(1 << k, dtype=np.uint64)[None, :]).ravel()
        return ("continue", ("node", L + k, child, t.level(L + k)[child.astype(np.int64)].copy()))
    pk, ph = leaf_pairs(rows, t, dpos)
    return ("continue", ("leaf", dpos, pk, ph))


def merkle_truncate(t: Tree, cont, max_entries):
    """truncate_diff(cont, max_sync_size) (causal_crdt.ex:98,212-214) on the oracle's
    continuations: a node form keeps its first `max_entries` entries, a leaf form its first
    `max_entries` buckets and the (key, leaf) pairs of those buckets (include/deltagpu.h
    dg_merkle_truncate)."""
    if cont[0] == "node":
        _, L, pos, hs = cont
        return ("node", L, pos[:max_entries], hs[:max_entries])
    _, buckets, pk, ph = cont
    keep = np.asarray(buckets)[:max_entries]
    m = np.isin(t.bucket_of(pk), keep.astype(np.int64))
    return ("leaf", keep, np.asarray(pk)[m], np.asarray(ph)[m])


def store_diff(ra, rb):
    sa, ra = _store(ra)
    sb, rb = _store(rb)
    cap = len(ra[0]) + len(rb[0]) + 1
    out = np.zeros(cap, np.uint64)
    n = np.zeros(1, np.uint64)
    _check(lib().ref_store_diff(C.byref(sa), C.byref(sb), _p(out, _abi.P64), cap, _p(n, _abi.P64)),
           "ref_store_diff")
    return out[: int(n[0])]


def changed_keys(old_rows, new_rows, keys=None):
    """CausalCrdt's diff/3 (causal_crdt.ex:343-351) on SoA rows: the keys (of `keys`, or
    all) whose row sets differ between the state before and after a join -- equal
    per-key value maps are equal row sets -- ascending."""
    d = store_diff(old_rows, new_rows)
    if keys is None:
        return d
    return d[np.isin(d, np.asarray(keys, np.uint64))]


def mutate_batch(rows, ctx, node, ops):
    """A batch of add/4 and remove/3 ops by `node` as one delta (aw_lww_map.ex:99-146
    per op, folded in batch order): ops = [(kind, key, val, ts)] with kind "add" /
    "remove", key/val ids.  ctx is the state's VV.  Returns (delta rows, delta context
    as a sorted dot list, touched keys ascending) -- see csrc/mutate.hip's header for
    the derivation, which tests/test_configs.py checks against the term oracle."""
    kind, node_ids, cnts = ctx
    assert kind == VV
    vv = {int(n): int(c) for n, c in zip(node_ids, cnts)}
    c0 = vv.get(int(node), 0) + 1
    last, gen, r = {}, [], 0
    for k, key, val, ts in ops:
        if k == "add":
            last[int(key)] = (int(val), int(ts), c0 + r)
            gen.append((int(node), c0 + r))
            r += 1
        else:
            last[int(key)] = None
    keys = np.array(sorted(last), np.uint64)
    drows = [(k, v, t, int(node), c) for k, x in sorted(last.items()) if x is not None
             for (v, t, c) in [x]]
    sel = np.isin(rows[0], keys)
    dots = sorted(set(zip(rows[3][sel].tolist(), rows[4][sel].tolist())) | set(gen))
    delta = (np.array([x[0] for x in drows], np.uint64), np.array([x[1] for x in drows], np.uint64),
             np.array([x[2] for x in drows], np.int64), np.array([x[3] for x in drows], np.uint32),
             np.array([x[4] for x in drows], np.uint64))
    dctx = (DOTS, np.array([d[0] for d in dots], np.uint32), np.array([d[1] for d in dots], np.uint64))
    return delta, dctx, keys


def store_check(rows) -> bool:
    s, _ = _store(rows)
    return lib().ref_store_check(C.byref(s)) == 0
