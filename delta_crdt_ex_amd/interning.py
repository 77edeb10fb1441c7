"""Exact interning of BEAM-style terms to the fixed-width ids of a dot row.

* key  -> u64 key id.  Integer keys 0 <= k < 2^64 map through splitmix64 (a
  bijection on u64, so distinct keys never collide); other terms through a 64-bit
  BLAKE2b of a canonical encoding, with an exact collision check.  Because key ids
  are hashes, sorting a store by key id also groups it into Merkle buckets and
  key-hash shards (bucket / shard = the id's high bits).
* value -> u64 value id, ORDER-PRESERVING over every term (the
  read tie-break is "smallest {value, ts} in Erlang term order",
  aw_lww_map.ex:211-216).  A Universe keeps its values sorted by `terms.order_key`
  and gives each a rank-like id with gaps: a new value takes an id between its two
  neighbours' (the midpoint; a fixed stride when it lands past either end).  When a
  gap is used up, every value is RELABELLED with evenly spaced ids -- a monotone map
  old id -> new id, so stores stay sorted -- and `remap_hook` rewrites the `val`
  column of every device store the Universe tracks (dg_remap_values).  Ids are
  therefore per-Universe; the synthetic workloads use the closed-form integer
  encoding `encode_int_value` (ints only, as bench/basic_operations.exs:4).
* node -> u32 node id, DENSE: the Universe's n-th distinct node term gets id n.
  The reference draws node ids from :rand.uniform(1_000_000_000)
  (causal_crdt.ex:65); dense ids keep every context inside the kernels' table
  lookups (the join's LDS VV table, the one-pass fold's KNT-entry tables).  Node
  order carries no meaning in the reference (dots are set members), so any
  bijection is exact.
"""
from __future__ import annotations

import bisect
import hashlib
import struct
import weakref

import numpy as np

from .terms import order_key

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


def _hkey(t):
    """Exact dict key of a term: equal exactly when the terms are `=:=` in Erlang
    (keeps `1`, `1.0` and `True` apart, also inside tuples and lists)."""
    return order_key(t)


ID_SPAN = 1 << 64
VAL_STRIDE = 1 << 32     # id step of a value that lands past either end of the order


class Universe:
    """The interning tables shared by every state of one process (one replica set).

    `remap_hook(old_ids, new_ids)` (uint64 arrays, both ascending) is called after a
    value relabel; the host mirror sets it to rewrite the tracked device stores.
    `val_epoch` counts relabels (a Merkle tree built before one is stale)."""

    def __init__(self):
        self._key_id = {}
        self._key_term = {}
        self._val_id = {}
        self._val_term = {}
        self._val_keys = []      # order keys of the values, ascending
        self._val_ids = []       # their ids, ascending (same order)
        self._node_id = {}
        self._node_term = []     # dense: node id -> term
        self.val_epoch = 0
        self.remap_hook = None
        self._tracked = weakref.WeakSet()

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
        p = bisect.bisect_left(self._val_keys, hk)
        vid = self._gap_id(p)
        if vid is None:
            self.relabel(extra=1)
            vid = self._gap_id(p)
        self._val_keys.insert(p, hk)
        self._val_ids.insert(p, vid)
        self._val_id[hk] = vid
        self._val_term[vid] = t
        return vid

    def _gap_id(self, p: int):
        """An id strictly between the neighbours of insertion point p, or None."""
        n = len(self._val_ids)
        if n == 0:
            return 1 << 63
        lo = self._val_ids[p - 1] if p > 0 else 0          # ids are >= 1
        hi = self._val_ids[p] if p < n else ID_SPAN
        if hi - lo < 2:
            return None
        if p == n:
            return lo + min(VAL_STRIDE, (hi - lo) // 2)
        if p == 0:
            return hi - min(VAL_STRIDE, (hi - lo) // 2)
        return lo + (hi - lo) // 2

    def relabel(self, extra: int = 0):
        """Re-space every value id evenly over the id range (order kept), then let
        `remap_hook` rewrite the device stores.  Returns (old_ids, new_ids)."""
        n = len(self._val_ids)
        step = ID_SPAN // (n + extra + 1)
        old = np.array(self._val_ids, dtype=np.uint64)
        new_ids = [(i + 1) * step for i in range(n)]
        new = np.array(new_ids, dtype=np.uint64)
        terms = [self._val_term[v] for v in self._val_ids]
        self._val_ids = new_ids
        self._val_term = {v: t for v, t in zip(new_ids, terms)}
        self._val_id = {k: v for k, v in zip(self._val_keys, new_ids)}
        self.val_epoch += 1
        if self.remap_hook is not None and n:
            self.remap_hook(old, new)
        return old, new

    def value_term(self, vid: int):
        return self._val_term[vid]

    def value_ids(self):
        """(ids, terms) of every value, ascending (= Erlang term order)."""
        return list(self._val_ids), [self._val_term[v] for v in self._val_ids]

    def track(self, store):
        """Remember a device store whose `val` column holds this Universe's ids (the
        remap hook rewrites it on a relabel)."""
        self._tracked.add(store)
        return store

    def tracked(self):
        return list(self._tracked)

    # -- nodes
    def node(self, t) -> int:
        hk = _hkey(t)
        nid = self._node_id.get(hk)
        if nid is not None:
            return nid
        nid = len(self._node_term)
        if nid > 0xFFFFFFFF:
            raise RuntimeError("node id space exhausted")
        self._node_id[hk] = nid
        self._node_term.append(t)
        return nid

    def node_term(self, nid: int):
        return self._node_term[nid]

    def node_ids(self, raw) -> np.ndarray:
        """Dense ids of an array of integer node terms (vectorised marshalling of a
        replica's `node` column or context, e.g. 30-bit :rand.uniform ids)."""
        raw = np.asarray(raw)
        if raw.size == 0:
            return np.zeros(0, np.uint32)
        uniq, inv = np.unique(raw, return_inverse=True)
        ids = np.array([self.node(int(u)) for u in uniq], np.uint32)
        return ids[inv].reshape(raw.shape)


DEFAULT = Universe()
