"""One definition of the term hashes on both host sides: the canonical encoding, the key
ids and the node / value term hashes of delta_crdt_ex_amd/interning.py (the Python
mirror) and of c_src/marshal.c (the NIF's term-independent half, driven here through
ctypes exactly as the NIF's term walk drives it) agree with each other and with the
committed vectors (tests/golden/term_hash_vectors.json, made by make_golden.py).

Also: the C universe hands out the same key ids, value ids (closed-form integers, the two
gapped regions, relabels) and dense node ids as the Python Universe for the same insert
sequence, with the same term-hash tables -- so a tree built from either side's ids and
tables is the same tree (Merkle trees compare across universes and BEAM
nodes; reference causal_crdt.ex:390-394, causal_crdt_test.exs:68-78)."""
import ctypes as C
import json
import os
import random
import subprocess

import numpy as np
import pytest

from delta_crdt_ex_amd import interning as I
from delta_crdt_ex_amd.storage import _unpack
from delta_crdt_ex_amd.terms import Atom, EList, EMap
from oracle import erlterm as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "c_src", "_build", "libdgmarshal.so")
VECTORS = os.path.join(ROOT, "tests", "golden", "term_hash_vectors.json")


def _junpack(x):
    if isinstance(x, list):
        if x and x[0] == "yh":
            return ["y", bytes.fromhex(x[1])]
        return [_junpack(y) for y in x]
    return x


def _vectors():
    with open(VECTORS) as f:
        return [(_unpack(_junpack(v["term"])), v) for v in json.load(f)]


class dgm_buf(C.Structure):
    _fields_ = [("p", C.POINTER(C.c_ubyte)), ("n", C.c_size_t), ("cap", C.c_size_t)]


CMP = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p)
ENC = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(dgm_buf), C.c_void_p)
HASH = C.CFUNCTYPE(C.c_uint64, C.c_void_p, C.c_void_p)
KEEP = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_void_p)
DROP = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p)


class dgm_term_ops(C.Structure):
    _fields_ = [("cmp", CMP), ("encode", ENC), ("hash", C.c_void_p), ("keep", KEEP),
                ("drop", DROP), ("ud", C.c_void_p)]


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "c_src"), "_build/libdgmarshal.so"],
                       check=True)
    L = C.CDLL(LIB)
    B = C.POINTER(dgm_buf)
    for name, args in {"dgm_enc_atom": [B, C.c_char_p, C.c_size_t],
                       "dgm_enc_int": [B, C.c_int, C.c_char_p, C.c_size_t],
                       "dgm_enc_float": [B, C.c_double],
                       "dgm_enc_binary": [B, C.c_char_p, C.c_size_t],
                       "dgm_enc_tuple": [B, C.c_uint32], "dgm_enc_list": [B, C.c_uint32],
                       "dgm_enc_map": [B, C.c_uint32], "dgm_enc_i64": [B, C.c_int64],
                       "dgm_enc_u64": [B, C.c_uint64]}.items():
        getattr(L, name).argtypes = args
        getattr(L, name).restype = C.c_int
    L.dgm_buf_free.argtypes = [B]
    L.dgm_key_id.argtypes = [C.POINTER(C.c_ubyte), C.c_size_t]
    L.dgm_key_id.restype = C.c_uint64
    L.dgm_hash_bytes.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
    L.dgm_hash_bytes.restype = C.c_uint64
    L.dgm_value_is_canonical.argtypes = [C.c_uint64, C.POINTER(C.c_int64)]
    L.dgm_universe_new.argtypes = [C.POINTER(dgm_term_ops)]
    L.dgm_universe_new.restype = C.c_void_p
    L.dgm_universe_free.argtypes = [C.c_void_p]
    L.dgm_key.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
    L.dgm_value.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_int)]
    L.dgm_node.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint32)]
    L.dgm_node_hashes.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.c_uint32)]
    L.dgm_value_hashes.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint64)),
                                   C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.c_uint64)]
    L.dgm_last_relabel.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint64)),
                                   C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.c_uint64)]
    return L


def c_encode(L, t, b) -> int:
    """The NIF's term walk, restated over the Python stand-ins: the same dgm_enc_* calls
    c_src/deltagpu_nif.c makes for each term class."""
    if isinstance(t, bool) or t is None or isinstance(t, Atom):
        s = ("nil" if t is None else "true" if t is True else "false" if t is False
             else str.__str__(t)).encode()
        return L.dgm_enc_atom(b, s, len(s))
    if isinstance(t, int):
        m = abs(t).to_bytes((abs(t).bit_length() + 7) // 8 or 1, "little")
        return L.dgm_enc_int(b, 1 if t < 0 else 0, m, len(m))
    if isinstance(t, float):
        return L.dgm_enc_float(b, t)
    if isinstance(t, EList):
        rc = L.dgm_enc_list(b, len(t))
        for x in t:
            rc = rc or c_encode(L, x, b)
        return rc
    if isinstance(t, EMap):
        rc = L.dgm_enc_map(b, len(t))
        for k, v in sorted(t, key=lambda kv: E.sort_key(kv[0])):  # the NIF sorts the keys
            rc = rc or c_encode(L, k, b) or c_encode(L, v, b)
        return rc
    if isinstance(t, tuple):
        rc = L.dgm_enc_tuple(b, len(t))
        for x in t:
            rc = rc or c_encode(L, x, b)
        return rc
    s = t.encode() if isinstance(t, str) else t
    return L.dgm_enc_binary(b, s, len(s))


def c_canon(L, t) -> bytes:
    b = dgm_buf()
    assert c_encode(L, t, C.byref(b)) == 0
    out = bytes(C.string_at(b.p, b.n)) if b.n else b""
    L.dgm_buf_free(C.byref(b))
    return out


def test_python_side_matches_the_vectors():
    for t, v in _vectors():
        assert bytes(I.canon(t)).hex() == v["canon"], t
        assert str(I.key_id(t)) == v["key_id"]
        assert str(I.node_hash(t)) == v["node_hash"]
        assert str(I.value_hash(t)) == v["value_hash"]
        assert I.is_canonical_int(t) == v["canonical_value"]


def test_c_side_matches_the_vectors(lib):
    L = lib
    for t, v in _vectors():
        enc = c_canon(L, t)
        assert enc.hex() == v["canon"], t
        arr = (C.c_ubyte * len(enc)).from_buffer_copy(enc)
        assert L.dgm_key_id(arr, len(enc)) == int(v["key_id"])
        assert L.dgm_hash_bytes(arr, len(enc), I.NODE_SEED) == int(v["node_hash"])
        if not v["canonical_value"]:
            assert L.dgm_hash_bytes(arr, len(enc), I.VAL_SEED) == int(v["value_hash"])
        else:  # a canonical integer's value hash is its closed-form id
            back = C.c_int64()
            assert L.dgm_value_is_canonical(int(v["value_hash"]), C.byref(back)) == 1
            assert back.value == t


def test_c_integer_shortcuts_encode_alike(lib):
    L = lib
    for x in (0, 1, -1, 255, -256, (1 << 63) - 1, -(1 << 63)):
        b = dgm_buf()
        L.dgm_enc_i64(C.byref(b), x)
        assert bytes(C.string_at(b.p, b.n)) == bytes(I.canon(x))
        L.dgm_buf_free(C.byref(b))
    for x in (0, 7, (1 << 64) - 1):
        b = dgm_buf()
        L.dgm_enc_u64(C.byref(b), x)
        assert bytes(C.string_at(b.p, b.n)) == bytes(I.canon(x))
        L.dgm_buf_free(C.byref(b))


class _CUniverse:
    """A marshal.c universe whose term operations are the Python stand-ins'."""

    def __init__(self, L):
        self.L = L
        self.terms = [None]
        self.ops = dgm_term_ops(
            CMP(lambda a, b, ud: E.compare(self.terms[a], self.terms[b])),
            ENC(lambda t, b, ud: c_encode(L, self.terms[t], b)),
            None,
            KEEP(lambda t, ud: t),
            DROP(lambda t, ud: None), None)
        self.u = L.dgm_universe_new(C.byref(self.ops))
        assert self.u

    def _h(self, t):
        self.terms.append(t)
        return len(self.terms) - 1

    def key(self, t):
        x = C.c_uint64()
        assert self.L.dgm_key(self.u, self._h(t), C.byref(x)) == 0
        return x.value

    def value(self, t):
        x, rl = C.c_uint64(), C.c_int()
        assert self.L.dgm_value(self.u, self._h(t), C.byref(x), C.byref(rl)) == 0
        return x.value, rl.value

    def node(self, t):
        x = C.c_uint32()
        assert self.L.dgm_node(self.u, self._h(t), C.byref(x)) == 0
        return x.value

    def tables(self):
        nh, nn = C.POINTER(C.c_uint64)(), C.c_uint32()
        self.L.dgm_node_hashes(self.u, C.byref(nh), C.byref(nn))
        vi, vh, nv = C.POINTER(C.c_uint64)(), C.POINTER(C.c_uint64)(), C.c_uint64()
        self.L.dgm_value_hashes(self.u, C.byref(vi), C.byref(vh), C.byref(nv))
        return (np.array(nh[: nn.value], np.uint64), np.array(vi[: nv.value], np.uint64),
                np.array(vh[: nv.value], np.uint64))

    def close(self):
        self.L.dgm_universe_free(self.u)


def _random_terms(rng, n):
    pool = [lambda: rng.randint(-20, 20), lambda: rng.randint(-(1 << 70), 1 << 70),
            lambda: rng.choice([1 << 62, -(1 << 62), (1 << 64) + 3]),
            lambda: rng.random() * 10 - 5, lambda: Atom(rng.choice("abcxyz")),
            lambda: rng.choice(["", "a", "ab", "b"]), lambda: (rng.randint(0, 3), "t"),
            lambda: EList([rng.randint(0, 2)] * rng.randint(0, 2))]
    return [rng.choice(pool)() for _ in range(n)]


def test_c_universe_matches_the_python_universe(lib):
    rng = random.Random(9)
    U, V = I.Universe(), _CUniverse(lib)
    try:
        terms = _random_terms(rng, 1500)
        # squeeze floats into one gap so that both relabel (the same call must do it)
        lo, hi = 1.0, 1.5
        for _ in range(75):
            hi = (lo + hi) / 2
            terms.append(hi)
        relabels = 0
        for t in terms:
            e0 = U.val_epoch
            vid = U.value(t)
            cid, rl = V.value(t)
            assert cid == vid, t
            assert rl == (U.val_epoch != e0)
            relabels += rl
            assert V.key(t) == U.key(t)
            assert V.node(t) == U.node(t)
        assert relabels >= 1
        for t in terms:  # ids after the relabels
            assert V.value(t)[0] == U.value(t)
        got, want = V.tables(), U.term_tables()
        for g, w in zip(got, want):
            assert np.array_equal(g, w)
    finally:
        V.close()
