"""Exact interning of BEAM-style terms to the fixed-width ids of a dot row.

* key  -> u64 key id.  Integer keys 0 <= k < 2^64 map through splitmix64 (a
  bijection on u64, so distinct keys never collide); other terms through a 64-bit
  BLAKE2b of a canonical encoding, with an exact collision check.  Because key ids
  are hashes, sorting a store by key id also groups it into Merkle buckets and
  key-hash shards (bucket / shard = the id's high bits).
* value -> u64 value id, ORDER-PRESERVING for integers (the
  read tie-break is "smallest value in Erlang term order").  Integers in
  [-2^62, 2^62) get id = v + 2^62.  Other terms get ids above 2^63 grouped by
  Erlang term class (number < atom < tuple < map < nil < list < bitstring), in
  insertion order inside a class: a tie between two non-integer values of the same
  class with the same ts is "parity unpinned" (the synthetic workloads use ints,
  as the reference's bench does, bench/basic_operations.exs:4).
* node -> u32 node id (integers 0 <= n < 2^31 are kept as is; the reference draws
  node ids from :rand.uniform(1_000_000_000), causal_crdt.ex:65).
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np

MASK64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & MASK64
    return x ^ (x >> 31)


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 over a uint64 array (wrap-around arithmetic)."""
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x += np.uint64(0x9E3779B97F4A7C15)
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return x


def encode_int_value(v) -> np.ndarray:
    """Order-preserving value ids for integers in [-2^62, 2^62) (vectorised)."""
    v = np.asarray(v, dtype=np.int64)
    return (v.astype(np.uint64) + np.uint64(1 << 62))


class _Enc:
    @staticmethod
    def enc(t, out: bytearray):
        # local import keeps the product free of the oracle package
        from .terms import Atom, EList, EMap
        if isinstance(t, bool) or t is None or isinstance(t, Atom):
            s = ("nil" if t is None else "true" if t is True else "false" if t is False
                 else str.__str__(t)).encode()
            out += b"a" + struct.pack("<I", len(s)) + s
        elif isinstance(t, int):
            s = str(t).encode()
            out += b"i" + struct.pack("<I", len(s)) + s
        elif isinstance(t, float):
            out += b"f" + struct.pack("<d", t)
        elif isinstance(t, EList):
            out += b"l" + struct.pack("<I", len(t))
            for x in t:
                _Enc.enc(x, out)
        elif isinstance(t, EMap):
            out += b"m" + struct.pack("<I", len(t))
            for k, v in t:
                _Enc.enc(k, out)
                _Enc.enc(v, out)
        elif isinstance(t, tuple):
            out += b"t" + struct.pack("<I", len(t))
            for x in t:
                _Enc.enc(x, out)
        elif isinstance(t, (str, bytes)):
            b = t.encode() if isinstance(t, str) else t
            out += b"b" + struct.pack("<I", len(b)) + b
        else:
            raise TypeError(f"cannot intern a {type(t).__name__}")


def term_hash64(t) -> int:
    buf = bytearray()
    _Enc.enc(t, buf)
    return int.from_bytes(hashlib.blake2b(bytes(buf), digest_size=8).digest(), "little")


def _term_class(t) -> int:
    from .terms import Atom, EList, EMap
    if isinstance(t, bool) or t is None or isinstance(t, Atom):
        return 1
    if isinstance(t, (int, float)):
        return 0
    if isinstance(t, EList):
        return 8 if len(t) == 0 else 9
    if isinstance(t, EMap):
        return 7
    if isinstance(t, tuple):
        return 6
    if isinstance(t, (str, bytes)):
        return 10
    raise TypeError(f"cannot intern a {type(t).__name__}")


def _hkey(t):
    """Dict key that keeps `1`, `1.0`, `True` and `b"a"`/`"a"` distinct where the BEAM does."""
    if isinstance(t, str):
        return ("b", t.encode())
    if isinstance(t, bytes):
        return ("b", t)
    return (type(t).__name__, t)


class Universe:
    """The interning tables shared by every state of one process (one replica set)."""

    def __init__(self):
        self._key_id = {}
        self._key_term = {}
        self._val_id = {}
        self._val_term = {}
        self._class_next = {}
        self._node_id = {}
        self._node_term = {}
        self._node_next = 1 << 31

    # -- keys
    def key(self, t) -> int:
        hk = _hkey(t)
        kid = self._key_id.get(hk)
        if kid is not None:
            return kid
        if isinstance(t, int) and not isinstance(t, bool) and 0 <= t <= MASK64:
            kid = splitmix64(t)
        else:
            kid = term_hash64(t)
        other = self._key_term.get(kid)
        if other is not None and _hkey(other) != hk:
            raise RuntimeError(f"64-bit key id collision between {other!r} and {t!r}")
        self._key_id[hk] = kid
        self._key_term[kid] = t
        return kid

    def key_term(self, kid: int):
        return self._key_term[kid]

    # -- values
    def value(self, t) -> int:
        hk = _hkey(t)
        vid = self._val_id.get(hk)
        if vid is not None:
            return vid
        if isinstance(t, int) and not isinstance(t, bool) and -(1 << 62) <= t < (1 << 62):
            vid = t + (1 << 62)
        else:
            c = _term_class(t)
            seq = self._class_next.get(c, 0)
            if seq >= (1 << 56):
                raise RuntimeError("value id space exhausted")
            self._class_next[c] = seq + 1
            vid = (1 << 63) | (c << 56) | seq
        self._val_id[hk] = vid
        self._val_term[vid] = t
        return vid

    def value_term(self, vid: int):
        if vid in self._val_term:
            return self._val_term[vid]
        if vid < (1 << 63):
            return vid - (1 << 62)
        raise KeyError(vid)

    # -- nodes
    def node(self, t) -> int:
        hk = _hkey(t)
        nid = self._node_id.get(hk)
        if nid is not None:
            return nid
        if isinstance(t, int) and not isinstance(t, bool) and 0 <= t < (1 << 31):
            nid = t
        else:
            nid = self._node_next
            self._node_next += 1
            if nid > 0xFFFFFFFF:
                raise RuntimeError("node id space exhausted")
        self._node_id[hk] = nid
        self._node_term[nid] = t
        return nid

    def node_term(self, nid: int):
        return self._node_term.get(nid, nid)


DEFAULT = Universe()
