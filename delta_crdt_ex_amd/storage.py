"""SoA snapshots of a replica's state: what `DeltaCrdt.Storage`
persists -- `{node_id, sequence_number, crdt_state, merkle_map}` (reference
lib/delta_crdt/storage.ex:12-16, written by causal_crdt.ex:238-250 after every delta
and read back at start-up by :216-234) -- stored as the device-resident dot store
itself instead of the term tree.

    storage.write(path, node_id, sequence_number, state, tree)   # AWLWWMap mirror state
    node_id, sequence_number, state, tree = storage.read(path)

File layout (little-endian), one self-describing file per replica:

    b"DGSNAP02" | u64 header length | header (msgpack) | column bytes ...

The header holds node_id, sequence_number, the row and context counts, the context
kind, the byte length and xxh64 of each column, and the exact interning tables of
the state's Universe (keys, values and nodes as tagged terms), so `read` restores the
same terms, ids and rows.  Columns are the raw SoA arrays (key, val, ts, node, cnt,
ctx node, ctx cnt, and the Merkle tree's nodes and per-bucket row counts when one is
persisted; the header records whether the tree hashed terms or ids): 36 B per dot + 12 B per context entry + 8 B per tree node + 2 B per bucket,
copied device -> host by one D2H copy each.  A persisted tree hashes terms (the
Universe's term hashes, interning.py), so it is valid for the restored ids.  The header names the tree's depth and key-hash shard.  A checksum mismatch
raises; the file is written to a temporary name, fsynced and renamed over the old one.
"""
from __future__ import annotations

import os
import struct

import msgpack
import numpy as np
import xxhash

from . import interning
from .terms import Atom, EList, EMap

MAGIC = b"DGSNAP02"
# DGSNAP01 (round 2): [id, term] node pairs and one value-id region; its ids do not carry
# over to the closed-form integer ids of DGSNAP02, so such a file is refused, not guessed.
_OLD_MAGICS = (b"DGSNAP01",)
_COLS = (("key", np.uint64), ("val", np.uint64), ("ts", np.int64), ("node", np.uint32),
         ("cnt", np.uint64))


def _pack(t):
    """A term as a tagged msgpack-able value (exact: no pickling)."""
    if t is None:
        return ["n"]
    if isinstance(t, bool):
        return ["b", t]
    if isinstance(t, Atom):
        return ["a", str(t)]
    if isinstance(t, int):
        return ["i", str(t)]
    if isinstance(t, float):
        return ["f", t]
    if isinstance(t, EList):
        return ["l", [_pack(x) for x in t]]
    if isinstance(t, EMap):
        return ["m", [[_pack(k), _pack(v)] for k, v in t]]
    if isinstance(t, tuple):
        return ["t", [_pack(x) for x in t]]
    if isinstance(t, str):
        return ["s", t]
    if isinstance(t, bytes):
        return ["y", t]
    raise TypeError(f"cannot snapshot term {t!r}")


def _unpack(x):
    tag = x[0]
    if tag == "n":
        return None
    if tag == "b":
        return bool(x[1])
    if tag == "a":
        return Atom(x[1])
    if tag == "i":
        return int(x[1])
    if tag == "f":
        return float(x[1])
    if tag == "l":
        return EList(_unpack(v) for v in x[1])
    if tag == "m":
        return EMap((_unpack(k), _unpack(v)) for k, v in x[1])
    if tag == "t":
        return tuple(_unpack(v) for v in x[1])
    if tag == "s":
        return x[1]
    if tag == "y":
        return bytes(x[1])
    raise ValueError(f"bad term tag {tag!r}")


def _universe_tables(U: interning.Universe):
    ids, terms = U.value_ids()
    return {
        "keys": [[str(k), _pack(t)] for k, t in U._key_term.items()],
        "vals": [[str(v), _pack(t)] for v, t in zip(ids, terms)],   # table values, ascending ids
        "nodes": [_pack(t) for t in U._node_term],                  # dense ids 0..n-1
        "val_epoch": U.val_epoch,
    }


def _universe_from(tables) -> interning.Universe:
    U = interning.Universe()
    for k, t in tables["keys"]:
        term = _unpack(t)
        U._key_term[int(k)] = term
        U._key_id[interning._hkey(term)] = int(k)
    for v, t in tables["vals"]:  # ascending ids = term order: appends keep the lists sorted
        term = _unpack(t)
        hk = interning._hkey(term)
        U._val_term[int(v)] = term
        U._val_id[hk] = int(v)
        U._val_keys.append(hk)
        U._val_ids.append(int(v))
        U._val_hash.append(interning.term_hash(term, interning.VAL_SEED))
    for t in tables["nodes"]:
        U.node(_unpack(t))
    U.val_epoch = int(tables.get("val_epoch", 0))
    return U


def write_arrays(path, node_id, sequence_number: int, rows, ctx, universe, merkle=None) -> None:
    """The snapshot file from host arrays: rows = (key, val, ts, node, cnt) numpy columns,
    ctx = (kind, node, cnt), merkle = None or (depth, shard_bits, shard, nodes uint64,
    counts uint16[, terms]) -- `terms` (default True): the tree hashed the rows' terms
    (the Universe's term hashes) rather than their ids; the reader restores it so."""
    cols = [np.ascontiguousarray(c, dt) for c, (_, dt) in zip(rows, _COLS)]
    cols += [np.ascontiguousarray(ctx[1], np.uint32), np.ascontiguousarray(ctx[2], np.uint64)]
    if merkle is not None:
        cols.append(np.ascontiguousarray(merkle[3], np.uint64))
        cols.append(np.ascontiguousarray(merkle[4], np.uint16))
    blobs = [c.tobytes() for c in cols]
    header = {
        "node_id": _pack(node_id),
        "sequence_number": int(sequence_number),
        "rows": int(len(cols[0])),
        "ctx_kind": int(ctx[0]),
        "ctx_n": int(len(cols[5])),
        "merkle": None if merkle is None else [int(merkle[0]), int(merkle[1]), str(int(merkle[2])),
                                               bool(merkle[5]) if len(merkle) > 5 else True],
        "columns": [[len(b), xxhash.xxh64_intdigest(b)] for b in blobs],
        "universe": _universe_tables(universe),
    }
    h = msgpack.packb(header, use_bin_type=True)
    # write-then-rename: a crash mid-write leaves the previous snapshot intact
    tmp = f"{path}.tmp"
    with open(tmp, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<Q", len(h)))
        f.write(h)
        for b in blobs:
            f.write(b)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def read_arrays(path):
    """(node_id, sequence_number, rows, ctx, universe, merkle) from a snapshot file as
    host arrays (merkle: None or (depth, shard_bits, shard, nodes, counts)); None if absent."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        magic = f.read(8)
        if magic in _OLD_MAGICS:
            raise ValueError(f"{path}: a {magic.decode()} snapshot (an older layout whose value "
                             f"ids {MAGIC.decode()} does not read); re-create it")
        if magic != MAGIC:
            raise ValueError(f"{path}: not a deltagpu snapshot")
        (hl,) = struct.unpack("<Q", f.read(8))
        header = msgpack.unpackb(f.read(hl), raw=False, strict_map_key=False)
        arrays = []
        dtypes = [d for _, d in _COLS] + [np.uint32, np.uint64, np.uint64, np.uint16]
        for (nbytes, digest), dt in zip(header["columns"], dtypes):
            b = f.read(nbytes)
            if len(b) != nbytes or xxhash.xxh64_intdigest(b) != digest:
                raise ValueError(f"{path}: column checksum mismatch")
            arrays.append(np.frombuffer(b, dtype=dt).copy())
    m = header.get("merkle")
    # the 4th entry: term-hashed tree (files without it hold term-hashed trees)
    merkle = None if m is None else (int(m[0]), int(m[1]), int(m[2]), arrays[7], arrays[8],
                                     bool(m[3]) if len(m) > 3 else True)
    return (_unpack(header["node_id"]), header["sequence_number"], tuple(arrays[:5]),
            (header["ctx_kind"], arrays[5], arrays[6]), _universe_from(header["universe"]), merkle)


def write(path, node_id, sequence_number: int, state, merkle_map=None) -> None:
    """Storage.write/2's payload {node_id, sequence_number, crdt_state, merkle_map}
    (causal_crdt.ex:242-250) for an AWLWWMap mirror state and its device MerkleTree
    (store.MerkleTree; None: not persisted, rebuilt on read)."""
    m = None
    if merkle_map is not None:
        m = (merkle_map.depth, merkle_map.shard_bits, merkle_map.shard,
             merkle_map.nodes.cpu().numpy().view(np.uint64), merkle_map.bucket_counts(),
             merkle_map.terms is not None)
    write_arrays(path, node_id, sequence_number, state.rows.to_numpy(),
                 (state.ctx.kind,) + tuple(state.ctx.to_numpy()), state.universe, m)


def read(path, device=None):
    """Storage.read/1 (causal_crdt.ex:220-230): {node_id, sequence_number, crdt_state,
    merkle_map} or None if `path` is absent.  The merkle_map is the persisted device tree
    (indexing the restored rows), or a fresh dg_merkle_build when none was persisted."""
    import torch

    from . import aw_lww_map as M
    from .store import Context, MerkleTree, Store, TermHashes
    got = read_arrays(path)
    if got is None:
        return None
    node_id, seq, rows, ctx, U, merkle = got
    dev = device or M._dev()
    st = Store.from_numpy(*rows, device=dev)
    state = M.AWLWWMap(st, Context.from_numpy(ctx[0], ctx[1], ctx[2], dev), U)
    if merkle is None:
        tree = None
    else:
        depth, sb, shard, nodes, counts, terms = merkle
        # a tree over ids stays one: mixing term-hashed buckets into it after
        # the next update would leave its nodes matching neither kind of rebuild
        tree = MerkleTree.empty(depth, dev, sb, shard, TermHashes.of(U, dev) if terms else None)
        tree.nodes.copy_(torch.from_numpy(nodes.view(np.int64).copy()))
        tree.counts[: 1 << depth].copy_(torch.from_numpy(counts.view(np.int16).copy()))
        tree.store = st
        tree.starts = None  # the chunk index is not persisted: the diff searches until a build
        tree.n_keys = int(len(np.unique(rows[0])))
    return node_id, seq, state, tree


__all__ = ["write", "read", "write_arrays", "read_arrays", "MAGIC"]
