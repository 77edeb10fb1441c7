"""Host mirror of `DeltaCrdt.AWLWWMap` (reference lib/delta_crdt/aw_lww_map.ex) on top
of libdeltagpu: the same functions, argument meaning and error behaviour, with the
state kept device-resident as SoA dot rows.

    from delta_crdt_ex_amd import aw_lww_map as AWLWWMap
    s = AWLWWMap.compress_dots(AWLWWMap.new())
    s = AWLWWMap.join(s, AWLWWMap.add("k", "v", node_id, s), ["k"])
    AWLWWMap.read(s)                       # => {"k": "v"}

Terms (keys, values, node ids) are interned exactly through a `Universe`
(interning.py); a state remembers its universe.  `join/3` and `read/1,2` run on the
GPU (dg_join2 / dg_read_lww); `compress_dots/1` too (dg_compress_dots).  The mutators
`add/4` and `remove/3` build per-op deltas on the host from the state's rows for one
key, exactly as the reference does (:99-146) — a handful of rows, not the hot path.
There is no CPU fallback: without a GPU the Engine raises.
"""
from __future__ import annotations

import time
import weakref

import numpy as np
import torch

from . import interning
from ._abi import DG_CTX_DOTS, DG_CTX_VV, FunctionClauseError
from .store import Context, Engine, MerkleTree, Store, TermHashes, u64

_ENGINE: Engine | None = None
_LIVE: "weakref.WeakSet[AWLWWMap]" = weakref.WeakSet()  # host row caches to drop on a relabel


def engine() -> Engine:
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = Engine(0)
    return _ENGINE


def _dev():
    return engine().device


def _remap_hook(universe: interning.Universe):
    """The Universe's relabel hook: rewrite the val column of every device store that
    still holds its ids (dg_remap_values; the map is monotone, stores stay sorted)."""
    def hook(old_ids, new_ids):
        eng = engine()
        for st in universe.tracked():
            if st.n:
                eng.remap_values(st, old_ids, new_ids)
        for m in list(_LIVE):
            if m.universe is universe:
                m._host = None
    return hook


class AWLWWMap:
    """`%DeltaCrdt.AWLWWMap{dots, value}` (aw_lww_map.ex:2-3), device-resident."""

    __slots__ = ("rows", "ctx", "universe", "_host", "__weakref__")

    def __init__(self, rows: Store, ctx: Context, universe: interning.Universe):
        self.rows = rows
        self.ctx = ctx
        self.universe = universe
        self._host = None
        if universe.remap_hook is None:
            universe.remap_hook = _remap_hook(universe)
        universe.track(rows)
        _LIVE.add(self)

    # -- host views (small states / single keys only)
    def _host_rows(self):
        if self._host is None:
            self._host = self.rows.to_numpy()
        return self._host

    def _rows_of_key(self, kid: int):
        k, v, t, n, c = self._host_rows()
        lo = int(np.searchsorted(k, np.uint64(kid), side="left"))
        hi = int(np.searchsorted(k, np.uint64(kid), side="right"))
        return v[lo:hi], t[lo:hi], n[lo:hi], c[lo:hi]

    @property
    def dots(self):
        """The causal context as terms: a frozenset of dots or a {node: max} dict."""
        node, cnt = self.ctx.to_numpy()
        U = self.universe
        if self.ctx.kind == DG_CTX_DOTS:
            return frozenset((U.node_term(int(a)), int(b)) for a, b in zip(node, cnt))
        return {U.node_term(int(a)): int(b) for a, b in zip(node, cnt)}

    @property
    def value(self):
        """The value map as terms: {key: {(value, ts): frozenset(dots)}}."""
        U = self.universe
        k, v, t, n, c = self._host_rows()
        out: dict = {}
        for i in range(len(k)):
            ent = out.setdefault(U.key_term(int(k[i])), {})
            ent.setdefault((U.value_term(int(v[i])), int(t[i])), set()).add(
                (U.node_term(int(n[i])), int(c[i])))
        return {key: {e: frozenset(d) for e, d in ents.items()} for key, ents in out.items()}


def _ctx_from_pairs(kind, pairs) -> Context:
    pairs = sorted(set(pairs))
    return Context.from_numpy(kind, np.array([p[0] for p in pairs], np.uint32),
                              np.array([p[1] for p in pairs], np.uint64), _dev())


def _empty_rows() -> Store:
    return Store.empty(1, _dev())


def new(universe: interning.Universe | None = None) -> AWLWWMap:
    """aw_lww_map.ex:8 — empty value, empty MapSet context."""
    return AWLWWMap(_empty_rows(), Context.empty(DG_CTX_DOTS, 1, _dev()),
                    universe or interning.DEFAULT)


def compress_dots(state: AWLWWMap) -> AWLWWMap:
    """aw_lww_map.ex:115-117 (FunctionClauseError on an already compressed state)."""
    if state.ctx.kind != DG_CTX_DOTS:
        raise FunctionClauseError(-6, "no function clause matching in Dots.compress/1")
    return AWLWWMap(state.rows, engine().compress_dots(state.ctx), state.universe)


def _next_dot(nid: int, ctx: Context):
    """Dots.next_dot/2 (aw_lww_map.ex:30-37)."""
    node, cnt = ctx.to_numpy()
    if ctx.kind == DG_CTX_DOTS:  # compress (the reference logs "inefficient next_dot")
        m = cnt[node == nid]
        top = int(m.max()) if len(m) else 0
    else:
        m = cnt[node == nid]
        top = int(m[0]) if len(m) else 0
    return nid, top + 1


def remove(key, node_id, state: AWLWWMap) -> AWLWWMap:
    """aw_lww_map.ex:133-146: a delta whose context holds the key's current dots."""
    U = state.universe
    kid = U.key(key)
    _v, _t, n, c = state._rows_of_key(kid)
    return AWLWWMap(_empty_rows(), _ctx_from_pairs(DG_CTX_DOTS, zip(n.tolist(), c.tolist())), U)


def add(key, value, node_id, state: AWLWWMap, ts: int | None = None) -> AWLWWMap:
    """aw_lww_map.ex:99-112.  `ts` defaults to time.monotonic_ns() (the reference's
    System.monotonic_time(:nanosecond))."""
    U = state.universe
    if ts is None:
        ts = time.monotonic_ns()
    kid, vid, nid = U.key(key), U.value(value), U.node(node_id)
    rem = remove(key, node_id, state)
    d_node, d_cnt = _next_dot(nid, state.ctx)
    # aw_set_add (:119-122): the new dot plus any dots of an identical {value, ts} entry
    v, t, n, c = state._rows_of_key(kid)
    same = (v == np.uint64(vid)) & (t == np.int64(ts))
    ctx_pairs = [(d_node, d_cnt)] + list(zip(n[same].tolist(), c[same].tolist()))
    rows = Store.from_numpy(np.array([kid], np.uint64), np.array([vid], np.uint64),
                            np.array([ts], np.int64), np.array([d_node], np.uint32),
                            np.array([d_cnt], np.uint64), _dev())
    addd = AWLWWMap(rows, _ctx_from_pairs(DG_CTX_DOTS, ctx_pairs), U)
    if rem.ctx.n == 0:
        return addd
    return join(rem, addd, [key])


def clear(_node_id, state: AWLWWMap) -> AWLWWMap:
    """aw_lww_map.ex:148-150."""
    return AWLWWMap(_empty_rows(), state.ctx, state.universe)


def join(delta1: AWLWWMap, delta2: AWLWWMap, keys) -> AWLWWMap:
    """aw_lww_map.ex:153-158 on the GPU (dg_join2)."""
    U = delta1.universe
    kids = np.unique(np.array([U.key(k) for k in keys], dtype=np.uint64))
    kt = torch.from_numpy(np.ascontiguousarray(kids).view(np.int64)).to(_dev())
    out, octx = engine().join2(delta1.rows, delta1.ctx, delta2.rows, delta2.ctx, keys=kt)
    return AWLWWMap(out, octx, U)


def join_all(delta1: AWLWWMap, delta2: AWLWWMap) -> AWLWWMap:
    """join/3 over every key of both states (the full-state anti-entropy join)."""
    out, octx = engine().join2(delta1.rows, delta1.ctx, delta2.rows, delta2.ctx)
    return AWLWWMap(out, octx, delta1.universe)


def from_terms(value: dict, dots, universe: interning.Universe | None = None) -> AWLWWMap:
    """Marshal a term-level `%AWLWWMap{dots, value}` (aw_lww_map.ex:2-3) onto the device,
    as the NIF's marshal_state does (c_src/marshal.c): walk value = %{key => %{{v, ts} =>
    MapSet[{node, counter}]}} in map iteration order, intern every term, upload the rows
    and the context unsorted and order them on the device (dg_sort_store /
    dg_sort_context).  `dots` is a set of (node, counter) dots or a {node: max} VV."""
    U = universe or interning.DEFAULT
    for entries in value.values():  # values first: a relabel re-spaces value ids
        for (v, _t) in entries:
            U.value(v)
    ks, vs, ts, ns, cs = [], [], [], [], []
    for key, entries in value.items():
        kid = U.key(key)
        for (v, t), ds in entries.items():
            vid = U.value(v)
            for (nd, c) in ds:
                ks.append(kid)
                vs.append(vid)
                ts.append(t)
                ns.append(U.node(nd))
                cs.append(c)
    dev = _dev()
    raw = Store.from_numpy(np.array(ks, np.uint64), np.array(vs, np.uint64), np.array(ts, np.int64),
                           np.array(ns, np.uint32), np.array(cs, np.uint64), dev)
    if isinstance(dots, dict):
        kind, pairs = DG_CTX_VV, [(U.node(nd), c) for nd, c in dots.items()]
    else:
        kind, pairs = DG_CTX_DOTS, [(U.node(nd), c) for nd, c in dots]
    ctx = Context.from_numpy(kind, np.array([p[0] for p in pairs], np.uint32),
                             np.array([p[1] for p in pairs], np.uint64), dev)
    eng = engine()
    rows = eng.sort_store(raw) if raw.n else _empty_rows()
    return AWLWWMap(rows, eng.sort_context(ctx) if ctx.n else ctx, U)


def read(state: AWLWWMap, keys=None) -> dict:
    """aw_lww_map.ex:211-224 (read/1, read/2 with a list, read/3 with one key)."""
    U = state.universe
    kt = None
    if keys is not None:
        if not isinstance(keys, list):
            keys = [keys]
        kids = np.unique(np.array([U.key(k) for k in keys], dtype=np.uint64))
        kt = torch.from_numpy(np.ascontiguousarray(kids).view(np.int64)).to(_dev())
    if state.rows.n == 0:
        return {}
    ok, ov = engine().read_lww(state.rows, keys=kt)
    return {U.key_term(int(k)): U.value_term(int(v)) for k, v in zip(u64(ok), u64(ov))}


def merkle_map(state: AWLWWMap, depth: int | None = None, shard_bits: int = 0,
               shard: int = 0) -> MerkleTree:
    """The state's MerkleMap (MerkleMap.new + put of every key's raw value map,
    causal_crdt.ex:21,390-394) on the device.  Rows are hashed through their TERMS
    (the Universe's term hashes, interning.py), so the tree compares bit for bit with a
    replica's built through another Universe -- a neighbour on another BEAM node
    (causal_crdt_test.exs:68-78).  depth: ~3 keys per bucket by default."""
    if depth is None:
        n = max(int(np.unique(u64(state.rows.key[: state.rows.n])).size) if state.rows.n else 1, 2)
        depth = max(1, min(28, int(np.ceil(np.log2(n / 3))) if n > 3 else 1))
    return engine().merkle_build(state.rows, depth, shard_bits=shard_bits, shard=shard,
                                 terms=TermHashes.of(state.universe, _dev()))


def merkle_diff(a: AWLWWMap, ta: MerkleTree, b: AWLWWMap, tb: MerkleTree, cap: int | None = None):
    """The keys (terms, ascending by key id) whose raw value maps differ between two
    replicas, from their trees (continue_partial_diff run to the keys, causal_crdt.ex:96,
    104-105; Enum.take(keys, max_sync_size) with `cap`).  Key ids are term hashes, so the
    replicas' Universes may differ."""
    keys = engine().merkle_diff(ta, tb, cap=cap)
    out = []
    for k in u64(keys):
        k = int(k)
        try:
            out.append(a.universe.key_term(k))
        except KeyError:
            out.append(b.universe.key_term(k))
    return out


def mutate_batch(ops, node_id, state: AWLWWMap):
    """Many add/4 and remove/3 calls by one node as ONE delta on the GPU
    (dg_mutate_batch): ops = [("add", key, value[, ts]) or ("remove",
    key)] in order.  Returns (delta, keys): join(state, delta, keys) equals applying the
    ops one by one as CausalCrdt does.  The state's context must be a version vector
    (compress_dots/1, as CausalCrdt keeps it)."""
    U = state.universe
    nid = U.node(node_id)
    m = len(ops)
    kind = np.zeros(m, np.uint8)
    key = np.zeros(m, np.uint64)
    val = np.zeros(m, np.uint64)
    ts = np.zeros(m, np.int64)
    for op in ops:  # intern every value first: a relabel would stale earlier ids
        if op[0] == "add":
            U.value(op[2])
        elif op[0] != "remove":
            raise ValueError(f"unknown op {op[0]!r}")
    for i, op in enumerate(ops):
        key[i] = U.key(op[1])
        if op[0] == "add":
            kind[i] = 1
            val[i] = U.value(op[2])
            ts[i] = op[3] if len(op) > 3 else time.monotonic_ns()
    rank = np.cumsum(kind, dtype=np.uint64) - kind  # adds before each op, batch order
    order = np.argsort(key, kind="stable")           # by key, batch order within a key
    dev = _dev()

    def d(a, view):
        return torch.from_numpy(np.ascontiguousarray(a[order]).view(view)).to(dev)

    delta, dots, keys = engine().mutate_batch(
        state.rows, state.ctx, nid, torch.from_numpy(kind[order]).to(dev), d(key, np.int64),
        d(val, np.int64), d(ts, np.int64), d(rank, np.int64), int(kind.sum()))
    return AWLWWMap(delta, dots, U), [U.key_term(int(k)) for k in u64(keys)]


__all__ = ["AWLWWMap", "new", "compress_dots", "add", "remove", "clear", "join", "join_all", "read",
           "mutate_batch", "from_terms", "merkle_map", "merkle_diff", "DG_CTX_VV", "DG_CTX_DOTS"]
