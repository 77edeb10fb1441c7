"""Python mirror of the Erlang NIF `DeltaCrdt.GPU` (c_src/deltagpu_nif.c).

The NIF is a term layer over c_src/replica.c (the device-resident replica state with
versions, replica.h); this module is the same term layer over the SAME compiled code
(c_src/_build/libdgreplica.so, ctypes), function for function and with the NIF's return
shapes, so the Elixir dispatch of INTEGRATION.md §3 can be exercised without a BEAM
(tests/binding_mirror.py, tests/test_gpu_binding.py):

    engine_open(device)                             -> ("ok", engine)
    state_load(engine, dots, value)                 -> ("ok", state, version)
    join_delta(state, version, dots, value, keys)   -> ("ok", version', new_dots, changed)
    mutate_batch(state, version, node, ops)         -> ("ok", version', new_dots, changed)
    read(state, version, keys | "all")              -> ("ok", {key: value})
    take(state, version, keys)                      -> ("ok", value_map)
    merkle_build(state, version, depth)             -> "ok"
    merkle_prepare(state, version, levels)          -> ("continue", bytes)
    merkle_continue(state, version, cont, levels, max_sync_size | "infinite")
                                                    -> ("continue", bytes) | ("ok", keys)
    resolve_keys(engine, keys)                      -> keys
    errors: ("error", "stale") for a version that is not the state's (an older struct),
            ("error", (code, message)) otherwise.

Terms are the package's stand-ins (delta_crdt_ex_amd/terms.py): a MapSet of dots is a
frozenset of (node, counter), a compressed context a {node: max} dict, a value map
{key: {(value, ts): frozenset(dots)}}, nil None.  An engine may be opened with `wrap` /
`unwrap` functions applied to every term crossing it (the tests keep their terms in an
exact-equality form, as BEAM maps compare keys, and pass the conversions).

Interning is the NIF's (c_src/marshal.c), mirrored by interning.Universe with the same
ids: key ids are hashes, value ids order-preserving, node ids dense; a relabel rewrites
every live state of the engine (dgr_remap).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi, interning
from ._abi import DG_CTX_DOTS, DG_CTX_VV, dg_context, dg_store
from .terms import Atom

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "c_src", "_build", "libdgreplica.so")

DGR_E_STALE = -16
U64_MAX = (1 << 64) - 1


class dgr_changed(C.Structure):
    _fields_ = [("version", C.c_uint64), ("n_changed", C.c_uint64), ("keys", C.c_void_p),
                ("rows", dg_store), ("ctx", dg_context)]


VP, U64, I32 = C.c_void_p, C.c_uint64, C.c_int
PU64 = C.POINTER(C.c_uint64)
_SIGS = {
    "dgr_engine_open": (I32, [I32, C.POINTER(VP)]),
    "dgr_engine_close": (I32, [VP]),
    "dgr_live_states": (U64, [VP]),
    "dgr_dg": (VP, [VP]),
    "dgr_refresh_terms": (I32, [VP, VP, U64, VP, VP, U64]),
    "dgr_remap": (I32, [VP, VP, VP, U64]),
    "dgr_state_load": (I32, [VP, C.POINTER(dg_store), C.POINTER(dg_context), C.POINTER(VP)]),
    "dgr_state_free": (I32, [VP]),
    "dgr_state_version": (U64, [VP]),
    "dgr_state_rows": (U64, [VP]),
    "dgr_state_has_tree": (I32, [VP]),
    "dgr_join_delta": (I32, [VP, U64, C.POINTER(dg_store), C.POINTER(dg_context), VP, U64,
                             C.POINTER(dgr_changed)]),
    "dgr_mutate_batch": (I32, [VP, U64, C.c_uint32, U64, VP, VP, VP, VP, C.POINTER(dgr_changed)]),
    "dgr_read": (I32, [VP, U64, I32, VP, U64, C.POINTER(VP), C.POINTER(VP), PU64]),
    "dgr_take": (I32, [VP, U64, VP, U64, C.POINTER(dg_store)]),
    "dgr_merkle_build": (I32, [VP, U64, C.c_uint32]),
    "dgr_merkle_prepare": (I32, [VP, U64, C.c_uint32, C.POINTER(VP), PU64]),
    "dgr_merkle_continue": (I32, [VP, U64, C.c_char_p, U64, C.c_uint32, U64, C.POINTER(I32),
                                  C.POINTER(VP), PU64, C.POINTER(VP), PU64]),
}

_lib = None


def load():
    """libdgreplica.so over the in-tree libdeltagpu.so (raises if either is missing or
    stale: there is no fallback)."""
    global _lib
    if _lib is None:
        _abi.load()  # the digest check of the library libdgreplica links
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C c_src`")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
    return _lib


def _err(rc):
    if rc == DGR_E_STALE:
        return ("error", "stale")
    msg = (_abi.load().dg_last_error() or b"").decode(errors="replace")
    return ("error", (rc, msg))


def _ident(t):
    return t


class Engine:
    """`engine` resource: a dgr_engine (one dg_engine, one HIP stream) and the interning
    universe of this "BEAM node"."""

    def __init__(self, device: int = 0, wrap=None, unwrap=None):
        self.lib = load()
        self.ptr = VP()
        rc = self.lib.dgr_engine_open(device, C.byref(self.ptr))
        if rc:
            raise _abi.DeltaGpuError(rc, "dgr_engine_open failed")
        self.universe = interning.Universe()
        self.universe.remap_hook = self._remap
        self.wrap = wrap or _ident
        self.unwrap = unwrap or _ident
        self.states = []

    def _remap(self, old_ids, new_ids):  # remap_live
        old = np.ascontiguousarray(old_ids, np.uint64)
        new = np.ascontiguousarray(new_ids, np.uint64)
        rc = self.lib.dgr_remap(self.ptr, old.ctypes.data, new.ctypes.data, len(old))
        if rc:
            raise _abi.DeltaGpuError(rc, "dgr_remap failed")

    def refresh_terms(self):
        nh, vid, vh = self.universe.term_tables()
        return self.lib.dgr_refresh_terms(self.ptr, nh.ctypes.data, len(nh), vid.ctypes.data,
                                          vh.ctypes.data, len(vid))

    def close(self):
        for s in self.states:
            s.free()
        self.states = []
        if self.ptr:
            self.lib.dgr_engine_close(self.ptr)
            self.ptr = VP()


class State:
    """`state` resource: one device-resident replica state (dgr_state)."""

    def __init__(self, engine: Engine, ptr):
        self.engine = engine
        self.ptr = ptr

    def free(self):
        if self.ptr:
            self.engine.lib.dgr_state_free(self.ptr)
            self.ptr = None

    @property
    def version(self):
        return int(self.engine.lib.dgr_state_version(self.ptr))

    @property
    def n_rows(self):
        return int(self.engine.lib.dgr_state_rows(self.ptr))


# ------------------------------------------------------------------ marshal
class _Rows:
    """Host rows and a context, as dgm_rows (the columns of a dg_store / dg_context)."""

    def __init__(self):
        self.k, self.v, self.t, self.n, self.c = [], [], [], [], []
        self.kind, self.cn, self.cc = DG_CTX_DOTS, [], []

    def store(self):
        self._a = (np.array(self.k, np.uint64), np.array(self.v, np.uint64),
                   np.array(self.t, np.int64), np.array(self.n, np.uint32),
                   np.array(self.c, np.uint64))
        k, v, t, n, c = self._a
        return dg_store(k.ctypes.data, v.ctypes.data, t.ctypes.data, n.ctypes.data, c.ctypes.data,
                        len(k), len(k))

    def context(self):
        self._c = (np.array(self.cn, np.uint32), np.array(self.cc, np.uint64))
        n, c = self._c
        return dg_context(self.kind, 0, n.ctypes.data, c.ctypes.data, len(n), len(n))


def _marshal_dots(eng: Engine, dots, out: _Rows):
    """a context: a MapSet of dots (DG_CTX_DOTS) or a %{node => max} VV (DG_CTX_VV)"""
    U, un = eng.universe, eng.unwrap
    if isinstance(dots, dict):
        out.kind = DG_CTX_VV
        items = dots.items()
    else:
        out.kind = DG_CTX_DOTS
        items = dots
    for node, cnt in items:
        out.cn.append(U.node(un(node)))
        out.cc.append(int(cnt))


def _marshal_value(eng: Engine, value, out: _Rows):
    """walk %{key => %{{v, ts} => MapSet[{node, counter}]}} in map order into host rows"""
    U, un = eng.universe, eng.unwrap
    for entries in value.values():  # pass 1: values first (a relabel re-spaces ids)
        for (v, _ts) in entries:
            U.value(un(v))
    for key, entries in value.items():
        kid = U.key(un(key))
        for (v, ts), dots in entries.items():
            vid = U.value(un(v))
            for node, cnt in dots:
                out.k.append(kid)
                out.v.append(vid)
                out.t.append(int(ts))
                out.n.append(U.node(un(node)))
                out.c.append(int(cnt))


KEY_TAG = Atom("$dg_key")


def key_placeholder(kid: int):
    """`{:"$dg_key", id}`: a differing key this node never interned (only the peer holds
    it), named by its id.  Every NIF that takes keys accepts it as that id; resolve_keys
    turns it back into the key's term on a node that knows the key."""
    return (KEY_TAG, int(kid))


def _key_id(eng: Engine, k):
    t = eng.unwrap(k)
    if isinstance(t, tuple) and len(t) == 2 and isinstance(t[0], Atom) and t[0] == KEY_TAG:
        return int(t[1])
    return eng.universe.key(t)


def _marshal_keys(eng: Engine, keys):
    return np.array([_key_id(eng, k) for k in keys], np.uint64)


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype)
    ct = {np.uint64: C.c_uint64, np.int64: C.c_int64, np.uint32: C.c_uint32}[dtype]
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(n,)).copy()


def _value_term(eng: Engine, vid: int):
    return eng.wrap(eng.universe.value_term(int(vid)))


def _unmarshal_rows(eng: Engine, s: dg_store):
    """host rows (store order) -> {key: {(v, ts): frozenset(dots)}}"""
    n = int(s.n)
    k, v = _arr(s.key, n, np.uint64), _arr(s.val, n, np.uint64)
    t, nd, c = _arr(s.ts, n, np.int64), _arr(s.node, n, np.uint32), _arr(s.cnt, n, np.uint64)
    U, w = eng.universe, eng.wrap
    out: dict = {}
    for i in range(n):
        ent = out.setdefault(w(U.key_term(int(k[i]))), {})
        ent.setdefault((_value_term(eng, v[i]), int(t[i])), set()).add(
            (w(U.node_term(int(nd[i]))), int(c[i])))
    return {key: {e: frozenset(d) for e, d in ents.items()} for key, ents in out.items()}


def _unmarshal_dots(eng: Engine, c: dg_context):
    n = int(c.n)
    node, cnt = _arr(c.node, n, np.uint32), _arr(c.cnt, n, np.uint64)
    U, w = eng.universe, eng.wrap
    if c.kind == DG_CTX_VV:
        return {w(U.node_term(int(a))): int(b) for a, b in zip(node, cnt)}
    return frozenset((w(U.node_term(int(a))), int(b)) for a, b in zip(node, cnt))


def _changed_result(eng: Engine, ch: dgr_changed):
    values = _unmarshal_rows(eng, ch.rows)
    dots = _unmarshal_dots(eng, ch.ctx)
    keys = _arr(ch.keys, int(ch.n_changed), np.uint64)
    changed = []
    for kid in keys:
        k = eng.wrap(eng.universe.key_term(int(kid)))
        changed.append((k, values.get(k)))  # None: the key's entries all went
    return ("ok", int(ch.version), dots, changed)


# ------------------------------------------------------------------ the NIFs
def engine_open(device: int = 0, wrap=None, unwrap=None):
    return ("ok", Engine(device, wrap, unwrap))


def state_load(engine: Engine, dots, value):
    h = _Rows()
    _marshal_dots(engine, dots, h)
    _marshal_value(engine, value, h)
    st, cx = h.store(), h.context()
    ptr = VP()
    rc = engine.lib.dgr_state_load(engine.ptr, C.byref(st), C.byref(cx), C.byref(ptr))
    if rc:
        return _err(rc)
    s = State(engine, ptr)
    engine.states.append(s)
    return ("ok", s, s.version)


def join_delta(state: State, version: int, dots, value, keys):
    eng = state.engine
    h = _Rows()
    _marshal_dots(eng, dots, h)
    _marshal_value(eng, value, h)
    kid = _marshal_keys(eng, keys)
    if eng.lib.dgr_state_has_tree(state.ptr):
        rc = eng.refresh_terms()
        if rc:
            return _err(rc)
    st, cx = h.store(), h.context()
    ch = dgr_changed()
    rc = eng.lib.dgr_join_delta(state.ptr, version, C.byref(st), C.byref(cx), kid.ctypes.data,
                                len(kid), C.byref(ch))
    if rc:
        return _err(rc)
    return _changed_result(eng, ch)


def mutate_batch(state: State, version: int, node, ops):
    """ops = [("add", key, value, ts) | ("remove", key)] in the order they were made"""
    eng = state.engine
    U, un = eng.universe, eng.unwrap
    nid = U.node(un(node))
    m = len(ops)
    kind = np.zeros(max(m, 1), np.uint8)
    key = np.zeros(max(m, 1), np.uint64)
    val = np.zeros(max(m, 1), np.uint64)
    ts = np.zeros(max(m, 1), np.int64)
    for op in ops:  # pass 1: values (a relabel re-spaces ids already handed out)
        if op[0] == "add":
            U.value(un(op[2]))
        elif op[0] != "remove":
            return ("error", (_abi.DG_E_INVAL, f"unknown op {op[0]!r}"))
    for i, op in enumerate(ops):
        key[i] = U.key(un(op[1]))
        if op[0] == "add":
            kind[i] = 1
            val[i] = U.value(un(op[2]))
            ts[i] = op[3]
    if eng.lib.dgr_state_has_tree(state.ptr):
        rc = eng.refresh_terms()
        if rc:
            return _err(rc)
    ch = dgr_changed()
    rc = eng.lib.dgr_mutate_batch(state.ptr, version, nid, m, kind.ctypes.data, key.ctypes.data,
                                  val.ctypes.data, ts.ctypes.data, C.byref(ch))
    if rc:
        return _err(rc)
    return _changed_result(eng, ch)


def read(state: State, version: int, keys):
    eng = state.engine
    all_ = isinstance(keys, str) and keys == "all"
    kid = np.zeros(1, np.uint64) if all_ else _marshal_keys(eng, keys)
    pk, pv, n = VP(), VP(), C.c_uint64()
    rc = eng.lib.dgr_read(state.ptr, version, 1 if all_ else 0, kid.ctypes.data,
                          0 if all_ else len(kid), C.byref(pk), C.byref(pv), C.byref(n))
    if rc:
        return _err(rc)
    k, v = _arr(pk, n.value, np.uint64), _arr(pv, n.value, np.uint64)
    U, w = eng.universe, eng.wrap
    return ("ok", {w(U.key_term(int(a))): _value_term(eng, b) for a, b in zip(k, v)})


def take(state: State, version: int, keys):
    eng = state.engine
    kid = _marshal_keys(eng, keys)
    out = dg_store()
    rc = eng.lib.dgr_take(state.ptr, version, kid.ctypes.data, len(kid), C.byref(out))
    if rc:
        return _err(rc)
    return ("ok", _unmarshal_rows(eng, out))


def merkle_build(state: State, version: int, depth: int):
    eng = state.engine
    rc = eng.refresh_terms() or eng.lib.dgr_merkle_build(state.ptr, version, depth)
    return "ok" if rc == 0 else _err(rc)


def merkle_prepare(state: State, version: int, levels: int):
    eng = state.engine
    p, n = VP(), C.c_uint64()
    rc = eng.lib.dgr_merkle_prepare(state.ptr, version, levels, C.byref(p), C.byref(n))
    if rc:
        return _err(rc)
    return ("continue", C.string_at(p, n.value))


def merkle_continue(state: State, version: int, cont: bytes, levels: int, max_sync):
    eng = state.engine
    rc = eng.refresh_terms()
    if rc:
        return _err(rc)
    mx = U64_MAX if max_sync == "infinite" else int(max_sync)
    status, p, n, pk, nk = C.c_int(), VP(), C.c_uint64(), VP(), C.c_uint64()
    rc = eng.lib.dgr_merkle_continue(state.ptr, version, cont, len(cont), levels, mx,
                                     C.byref(status), C.byref(p), C.byref(n), C.byref(pk),
                                     C.byref(nk))
    if rc:
        return _err(rc)
    if status.value == 1:
        return ("continue", C.string_at(p, n.value))
    return ("ok", [_key_term(eng, kid) for kid in _arr(pk, nk.value, np.uint64)])


def _key_term(eng: Engine, kid):
    """the key's term, or its placeholder when this node never interned it"""
    try:
        return eng.wrap(eng.universe.key_term(int(kid)))
    except KeyError:
        return eng.wrap(key_placeholder(kid))


def resolve_keys(engine: Engine, keys):
    """Placeholders of keys this node knows -> their terms (others stay placeholders):
    the originator's get_diff (causal_crdt.ex:112-123) takes its values of the keys a
    peer's continue_partial_diff named by id."""
    out = []
    for k in keys:
        t = engine.unwrap(k)
        if isinstance(t, tuple) and len(t) == 2 and isinstance(t[0], Atom) and t[0] == KEY_TAG:
            out.append(_key_term(engine, t[1]))
        else:
            out.append(k)
    return out


__all__ = ["engine_open", "state_load", "join_delta", "mutate_batch", "read", "take",
           "merkle_build", "merkle_prepare", "merkle_continue", "resolve_keys", "key_placeholder",
           "Engine", "State", "DGR_E_STALE"]
