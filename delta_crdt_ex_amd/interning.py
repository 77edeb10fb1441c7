"""Exact interning of BEAM-style terms to the fixed-width ids of a dot row, and the
term hashes that make Merkle trees independent of the interning tables.

* key  -> u64 key id.  Integer keys 0 <= k < 2^64 map through splitmix64 (a
  bijection on u64, so distinct keys never collide); other terms to `term_hash(t, 0)`,
  the xxh64 of the term's canonical encoding (below), with an exact collision check.
  The NIF computes the same ids (c_src/marshal.c, dgm_key), so key ids agree between
  BEAM nodes.  Because key ids are hashes, sorting a store by key id also groups it
  into Merkle buckets and key-hash shards (bucket / shard = the id's high bits).
* value -> u64 value id, ORDER-PRESERVING over every term (the
  read tie-break is "smallest {value, ts} in map-key order", aw_lww_map.ex:211-216):
    - integers v in [CANON_LO, 2^62) have the CLOSED-FORM id v + 2^62, in
      [2^58, 2^63): the same on every node, no table entry (`encode_int_value`);
    - the other terms get gapped ids from the Universe's sorted table: integers below
      CANON_LO in (0, 2^58), everything above the canonical integers (larger integers,
      floats, atoms, tuples, ...) in [2^63, 2^64).  In map-key order every integer
      precedes every float and numbers precede every other class, so both regions keep
      term order.  A new value takes the midpoint of its neighbours' ids in its region
      (a 2^32 stride past either end); when a gap is used up, the region's values are
      RELABELLED with evenly spaced ids -- a monotone map old id -> new id, so stores
      stay sorted -- and `remap_hook` rewrites the `val` column of every device store
      the Universe tracks (dg_remap_values).
* node -> u32 node id, DENSE: the Universe's n-th distinct node term gets id n.
  The reference draws node ids from :rand.uniform(1_000_000_000)
  (causal_crdt.ex:65); dense ids keep every context inside the kernels' table
  lookups (the join's LDS VV table, the one-pass fold's KNT-entry tables).  Node
  order carries no meaning in the reference (dots are set members), so any
  bijection is exact.

Canonical encoding (`canon`, the input of every term hash; c_src/marshal.c builds the
same bytes from a NIF term walk): a tag byte and a little-endian u32 length, then

    a <utf8 text>             atom           f <f64 LE>           float (no length)
    i <sign byte><magnitude>  integer: sign 0/1, magnitude little-endian, minimal bytes
    t <n> <elements>          tuple          l <n> <elements>     proper list
    m <n> <key, value>...     map, pairs in map-key order         b <bytes>  binary

Term hashes of the Merkle rows (dg_term_hashes, include/deltagpu.h): a node's is
`term_hash(node, NODE_SEED)`, a non-canonical value's `term_hash(value, VAL_SEED)`;
a canonical integer value hashes as its closed-form id.  Trees built with them are
bit-identical for equal states whatever order two Universes interned the terms in, so
two replicas on different BEAM nodes compare their trees directly (causal_crdt.ex:
390-394, causal_crdt_test.exs:68-78).
"""
from __future__ import annotations

import bisect
import struct
import weakref

import numpy as np
import xxhash

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


CANON_LO = -(1 << 62) + (1 << 58)   # the canonical integer values: [CANON_LO, CANON_HI)
CANON_HI = 1 << 62
CANON_ID_LO = 1 << 58               # their ids: [CANON_ID_LO, CANON_ID_HI)
CANON_ID_HI = 1 << 63
NODE_SEED = 0x6E6F6465              # term_hash seeds of node and value terms
VAL_SEED = 0x76616C75


def encode_int_value(v) -> np.ndarray:
    """Closed-form (canonical) value ids of integers in [CANON_LO, 2^62) (vectorised):
    v + 2^62.  The Universe hands out exactly these ids for such integers."""
    v = np.asarray(v, dtype=np.int64)
    if v.size and (int(v.min()) < CANON_LO or int(v.max()) >= CANON_HI):
        raise ValueError("encode_int_value: integer outside the canonical range")
    return (v.astype(np.uint64) + np.uint64(1 << 62))


def is_canonical_int(t) -> bool:
    return isinstance(t, int) and not isinstance(t, bool) and CANON_LO <= t < CANON_HI


def canon(t, out: bytearray | None = None) -> bytearray:
    """The canonical encoding of a term (module docstring)."""
    from .terms import Atom, EList, EMap
    if out is None:
        out = bytearray()
    if isinstance(t, bool) or t is None or isinstance(t, Atom):
        b = ("nil" if t is None else "true" if t is True else "false" if t is False
             else str.__str__(t)).encode()
        out += b"a" + struct.pack("<I", len(b)) + b
    elif isinstance(t, int):
        m = abs(t)
        mag = m.to_bytes((m.bit_length() + 7) // 8, "little")
        out += b"i" + struct.pack("<I", len(mag) + 1) + (b"\x01" if t < 0 else b"\x00") + mag
    elif isinstance(t, float):
        out += b"f" + struct.pack("<d", t)
    elif isinstance(t, EList):
        out += b"l" + struct.pack("<I", len(t))
        for x in t:
            canon(x, out)
    elif isinstance(t, EMap):  # EMap pairs are in map-key order (oracle.erlterm.emap)
        out += b"m" + struct.pack("<I", len(t))
        for k, v in t:
            canon(k, out)
            canon(v, out)
    elif isinstance(t, tuple):
        out += b"t" + struct.pack("<I", len(t))
        for x in t:
            canon(x, out)
    elif isinstance(t, (str, bytes)):
        b = t.encode() if isinstance(t, str) else t
        out += b"b" + struct.pack("<I", len(b)) + b
    else:
        raise TypeError(f"cannot intern a {type(t).__name__}")
    return out


def term_hash(t, seed: int = 0) -> int:
    """xxh64 of the canonical encoding (c_src/marshal.c dgm_hash_bytes)."""
    return xxhash.xxh64_intdigest(bytes(canon(t)), seed)


def key_id(t) -> int:
    """The key id of a key term (dgm_key in c_src/marshal.c computes the same)."""
    if isinstance(t, int) and not isinstance(t, bool) and 0 <= t <= MASK64:
        return splitmix64(t)
    return term_hash(t, 0)


def node_hash(t) -> int:
    return term_hash(t, NODE_SEED)


def value_hash(t) -> int:
    """A value's term in the Merkle row hash: its closed-form id when canonical."""
    if is_canonical_int(t):
        return int(t) + (1 << 62)
    return term_hash(t, VAL_SEED)


def _hkey(t):
    """Exact dict key of a term: equal exactly when the terms are `=:=` in Erlang
    (keeps `1`, `1.0` and `True` apart, also inside tuples and lists)."""
    return order_key(t)


VAL_STRIDE = 1 << 32     # id step of a value that lands past either end of its region
# the two table regions (exclusive bounds): below and above the canonical integers
LOW = (0, CANON_ID_LO)
HIGH = (CANON_ID_HI - 1, 1 << 64)


class Universe:
    """The interning tables shared by every state of one process (one replica set).

    `remap_hook(old_ids, new_ids)` (uint64 arrays, both ascending) is called after a
    value relabel; the host mirror sets it to rewrite the tracked device stores.
    `val_epoch` counts relabels; `terms_version` changes whenever the term-hash tables
    (`term_tables`) do: a new node, a new table value or a relabel."""

    def __init__(self):
        self._key_id = {}
        self._key_term = {}
        self._val_id = {}        # table values only (canonical integers are closed-form)
        self._val_term = {}
        self._val_keys = []      # order keys of the table values, ascending
        self._val_ids = []       # their ids, ascending (same order)
        self._val_hash = []      # their term hashes (same order)
        self._node_id = {}
        self._node_term = []     # dense: node id -> term
        self._node_hash = []
        self.val_epoch = 0
        self.terms_version = 0
        self.remap_hook = None
        self._tracked = weakref.WeakSet()

    # -- keys
    def key(self, t) -> int:
        hk = _hkey(t)
        kid = self._key_id.get(hk)
        if kid is not None:
            return kid
        kid = key_id(t)
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
        if is_canonical_int(t):
            return int(t) + (1 << 62)
        hk = _hkey(t)
        vid = self._val_id.get(hk)
        if vid is not None:
            return vid
        low = isinstance(t, int) and not isinstance(t, bool) and t < CANON_LO
        p = bisect.bisect_left(self._val_keys, hk)
        vid = self._gap_id(p, low)
        if vid is None:
            self.relabel(extra=1, low=low)
            vid = self._gap_id(p, low)
        self._val_keys.insert(p, hk)
        self._val_ids.insert(p, vid)
        self._val_hash.insert(p, term_hash(t, VAL_SEED))
        self._val_id[hk] = vid
        self._val_term[vid] = t
        self.terms_version += 1
        return vid

    def _gap_id(self, p: int, low: bool):
        """An id strictly between the neighbours of insertion point p inside the value's
        region (LOW or HIGH, exclusive bounds), or None when the gap is used up."""
        rlo, rhi = LOW if low else HIGH
        ids = self._val_ids
        lo = ids[p - 1] if p > 0 and rlo < ids[p - 1] < rhi else None
        hi = ids[p] if p < len(ids) and rlo < ids[p] < rhi else None
        a, b = (lo if lo is not None else rlo), (hi if hi is not None else rhi)
        if b - a < 2:
            return None
        if lo is None and hi is None:
            return a + (b - a) // 2
        if hi is None:
            return a + min(VAL_STRIDE, (b - a) // 2)
        if lo is None:
            return b - min(VAL_STRIDE, (b - a) // 2)
        return a + (b - a) // 2

    def relabel(self, extra: int = 0, low: bool = False):
        """Re-space the value ids of one region evenly over it (order kept), then let
        `remap_hook` rewrite the device stores.  Returns (old_ids, new_ids)."""
        rlo, rhi = LOW if low else HIGH
        idx = [i for i, v in enumerate(self._val_ids) if rlo < v < rhi]
        n = len(idx)
        step = (rhi - rlo) // (n + extra + 1)
        old = np.array([self._val_ids[i] for i in idx], dtype=np.uint64)
        new_ids = [rlo + (j + 1) * step for j in range(n)]
        new = np.array(new_ids, dtype=np.uint64)
        # every old entry out before any new one goes in: a new id can equal an old id not
        # yet moved (evenly spaced ids meet earlier midpoints), and moving them one by one
        # then overwrote that value's term and lost the moved one
        terms = [self._val_term.pop(self._val_ids[i]) for i in idx]
        for j, i in enumerate(idx):
            self._val_ids[i] = new_ids[j]
            self._val_term[new_ids[j]] = terms[j]
            self._val_id[self._val_keys[i]] = new_ids[j]
        self.val_epoch += 1
        self.terms_version += 1
        if self.remap_hook is not None and n:
            self.remap_hook(old, new)
        return old, new

    def value_term(self, vid: int):
        if CANON_ID_LO <= vid < CANON_ID_HI:
            return vid - (1 << 62)
        return self._val_term[vid]

    def value_ids(self):
        """(ids, terms) of the table values (every value but the canonical integers),
        ascending (= term order)."""
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
        self._node_hash.append(node_hash(t))
        self.terms_version += 1
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

    # -- term hashes (dg_term_hashes)
    def term_tables(self):
        """(node_hash[n_nodes], val_ids[n], val_hash[n]) as uint64 arrays: the node hash
        of every dense node id, and the ascending table value ids with their hashes (the
        canonical integers need no entry)."""
        return (np.array(self._node_hash, dtype=np.uint64),
                np.array(self._val_ids, dtype=np.uint64),
                np.array(self._val_hash, dtype=np.uint64))


DEFAULT = Universe()
