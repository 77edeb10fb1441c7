"""Conversions between term-level oracle states (oracle/awlww_term.py) and the SoA
dot rows of include/deltagpu.h.  TEST INFRASTRUCTURE ONLY.

Interning goes through the product's `delta_crdt_ex_amd.interning.Universe`, so a
term state converted here is exactly what the host mirror would upload.
"""
from __future__ import annotations

import numpy as np

from delta_crdt_ex_amd.interning import Universe

from . import awlww_term as T
from .ref import DOTS, VV


def sort_rows(k, v, t, n, c):
    k = np.asarray(k, np.uint64)
    v = np.asarray(v, np.uint64)
    t = np.asarray(t, np.int64)
    n = np.asarray(n, np.uint32)
    c = np.asarray(c, np.uint64)
    order = np.lexsort((c, n, t, v, k))
    return k[order], v[order], t[order], n[order], c[order]


def ctx_arrays(dots, U: Universe):
    """A term context (frozenset of dots, or dict VV) -> (kind, node u32, cnt u64) sorted."""
    if isinstance(dots, (frozenset, set)):
        pairs = sorted((U.node(nd), c) for (nd, c) in dots)
        kind = DOTS
    else:
        pairs = sorted((U.node(nd), c) for nd, c in dots.items())
        kind = VV
    node = np.array([p[0] for p in pairs], np.uint32)
    cnt = np.array([p[1] for p in pairs], np.uint64)
    return kind, node, cnt


def state_to_soa(state: T.AW, U: Universe):
    for entries in state.value.values():  # intern every value first (a relabel re-spaces ids)
        for (val, _t) in entries:
            U.value(val)
    ks, vs, ts, ns, cs = [], [], [], [], []
    for key, entries in state.value.items():
        kid = U.key(key)
        for (val, t), dots in entries.items():
            vid = U.value(val)
            for (nd, c) in dots:
                ks.append(kid)
                vs.append(vid)
                ts.append(t)
                ns.append(U.node(nd))
                cs.append(c)
    rows = sort_rows(ks, vs, ts, ns, cs)
    return rows, ctx_arrays(state.dots, U)


def state_to_soa_ints(state: T.AW, nodes):
    """A term state whose keys and values are integers -> SoA rows in the synthetic
    workloads' id space (key = splitmix64(k), val = encode_int_value(v)) with node
    terms interned through `nodes` (a workloads.NodeTable: 30-bit term -> dense id)."""
    from delta_crdt_ex_amd.interning import encode_int_value, splitmix64
    dense = nodes.dense_of_term()
    ks, vs, ts, ns, cs = [], [], [], [], []
    for key, entries in state.value.items():
        for (val, t), dots in entries.items():
            for (nd, c) in dots:
                ks.append(splitmix64(key))
                vs.append(int(encode_int_value(val)))
                ts.append(t)
                ns.append(dense[nd])
                cs.append(c)
    rows = sort_rows(ks, vs, ts, ns, cs)
    d = state.dots
    if isinstance(d, (frozenset, set)):
        pairs, kind = sorted((dense[nd], c) for (nd, c) in d), DOTS
    else:
        pairs, kind = sorted((dense[nd], c) for nd, c in d.items()), VV
    return rows, (kind, np.array([p[0] for p in pairs], np.uint32),
                  np.array([p[1] for p in pairs], np.uint64))


def soa_canon(rows, ctx, U: Universe):
    """Canonical comparable form of SoA rows + context, in term space."""
    out = _canon_rows(rows, U)
    kind, node, cnt = ctx
    if kind == DOTS:
        cx = ("set", frozenset((U.node_term(int(a)), int(b)) for a, b in zip(node, cnt)))
    else:
        cx = ("vv", frozenset((U.node_term(int(a)), int(b)) for a, b in zip(node, cnt)))
    return cx, out


def _canon_rows(rows, U):
    k, v, t, n, c = rows
    return frozenset(
        (_hk(U.key_term(int(k[i]))), _hk(U.value_term(int(v[i]))), int(t[i]),
         _hk(U.node_term(int(n[i]))), int(c[i]))
        for i in range(len(k)))


def _hk(x):
    return (type(x).__name__, x)


def term_canon(state: T.AW):
    d = state.dots
    if isinstance(d, (frozenset, set)):
        cx = ("set", frozenset(d))
    else:
        cx = ("vv", frozenset(d.items()))
    rows = frozenset((_hk(key), _hk(val), ts, _hk(nd), c)
                     for key, entries in state.value.items()
                     for (val, ts), dots in entries.items()
                     for (nd, c) in dots)
    return cx, rows
