"""Device-resident dot stores and causal contexts, and the Engine that drives
libdeltagpu on them.

PyTorch is plumbing here: it owns HBM allocations and the stream.  Columns are
int64/int32 tensors holding the bits of the u64/i64/u32 columns of
include/deltagpu.h (u64 ids are reinterpreted, never compared in torch).
"""
from __future__ import annotations

import ctypes as C
import weakref
from dataclasses import dataclass

import numpy as np
import torch

from . import _abi
from ._abi import DG_CTX_DOTS, DG_CTX_VV, check

_I64 = torch.int64
_I32 = torch.int32


def _ptr(t: torch.Tensor | None, ctype):
    if t is None or t.numel() == 0:
        return C.cast(C.c_void_p(t.data_ptr() if t is not None and t.numel() else 0), ctype)
    return C.cast(C.c_void_p(t.data_ptr()), ctype)


def _np_to_dev(a: np.ndarray, dtype_view, device) -> torch.Tensor:
    a = np.ascontiguousarray(a).view(dtype_view)
    return torch.from_numpy(a.copy()).to(device, non_blocking=False)


@dataclass(eq=False)  # identity semantics: a Universe tracks stores in a WeakSet
class Store:
    """SoA dot rows on the device: key u64, val u64, ts i64, node u32, cnt u64."""

    key: torch.Tensor
    val: torch.Tensor
    ts: torch.Tensor
    node: torch.Tensor
    cnt: torch.Tensor
    n: int

    @property
    def cap(self) -> int:
        return int(self.key.numel())

    @property
    def device(self):
        return self.key.device

    @staticmethod
    def empty(cap: int, device) -> "Store":
        cap = max(int(cap), 1)
        return Store(
            torch.empty(cap, dtype=_I64, device=device),
            torch.empty(cap, dtype=_I64, device=device),
            torch.empty(cap, dtype=_I64, device=device),
            torch.empty(cap, dtype=_I32, device=device),
            torch.empty(cap, dtype=_I64, device=device),
            0,
        )

    @staticmethod
    def from_numpy(key, val, ts, node, cnt, device) -> "Store":
        n = len(key)
        if n == 0:
            return Store.empty(1, device)
        return Store(
            _np_to_dev(np.asarray(key, dtype=np.uint64), np.int64, device),
            _np_to_dev(np.asarray(val, dtype=np.uint64), np.int64, device),
            _np_to_dev(np.asarray(ts, dtype=np.int64), np.int64, device),
            _np_to_dev(np.asarray(node, dtype=np.uint32), np.int32, device),
            _np_to_dev(np.asarray(cnt, dtype=np.uint64), np.int64, device),
            n,
        )

    def to_numpy(self):
        n = self.n
        return (
            self.key[:n].cpu().numpy().view(np.uint64),
            self.val[:n].cpu().numpy().view(np.uint64),
            self.ts[:n].cpu().numpy().view(np.int64),
            self.node[:n].cpu().numpy().view(np.uint32),
            self.cnt[:n].cpu().numpy().view(np.uint64),
        )

    def abi(self) -> _abi.dg_store:
        return _abi.dg_store(self.key.data_ptr(), self.val.data_ptr(), self.ts.data_ptr(),
                             self.node.data_ptr(), self.cnt.data_ptr(), self.n, self.cap)


@dataclass
class Context:
    """A causal context: DG_CTX_VV (version vector) or DG_CTX_DOTS (dot set)."""

    kind: int
    node: torch.Tensor
    cnt: torch.Tensor
    n: int

    @property
    def cap(self) -> int:
        return int(self.node.numel())

    @staticmethod
    def empty(kind: int, cap: int, device) -> "Context":
        cap = max(int(cap), 1)
        return Context(kind, torch.empty(cap, dtype=_I32, device=device),
                       torch.empty(cap, dtype=_I64, device=device), 0)

    @staticmethod
    def from_numpy(kind, node, cnt, device) -> "Context":
        n = len(node)
        if n == 0:
            return Context.empty(kind, 1, device)
        return Context(kind, _np_to_dev(np.asarray(node, dtype=np.uint32), np.int32, device),
                       _np_to_dev(np.asarray(cnt, dtype=np.uint64), np.int64, device), n)

    def to_numpy(self):
        return (self.node[: self.n].cpu().numpy().view(np.uint32),
                self.cnt[: self.n].cpu().numpy().view(np.uint64))

    def abi(self) -> _abi.dg_context:
        return _abi.dg_context(self.kind, 0, self.node.data_ptr(), self.cnt.data_ptr(), self.n,
                               self.cap)


class TermHashes:
    """Device term-hash tables of a tree's rows (include/deltagpu.h dg_term_hashes):
    node_hash[node id], and the ascending non-canonical value ids with their hashes --
    `interning.Universe.term_tables()`.  Trees built with them compare across interning
    tables (replicas on other BEAM nodes)."""

    def __init__(self, node_hash, val_id, val_hash, device):
        def dev(a):
            a = np.ascontiguousarray(np.asarray(a, np.uint64))
            return _np_to_dev(a, np.int64, device) if len(a) else torch.zeros(1, dtype=_I64,
                                                                                 device=device)
        self.nh, self.vid, self.vh = dev(node_hash), dev(val_id), dev(val_hash)
        self.c = _abi.dg_term_hashes(self.nh.data_ptr(), len(node_hash), self.vid.data_ptr(),
                                     self.vh.data_ptr(), len(val_id))
        self.device = device
        self._universe = None  # set by `of`: tables that follow a Universe
        self.version = None

    @staticmethod
    def of(universe, device) -> "TermHashes":
        """The universe's current tables, uploaded once per version (cached on it)."""
        cached = getattr(universe, "_dev_terms", None)
        if cached is not None and cached[0] == universe.terms_version and cached[1] == str(device):
            return cached[2]
        th = TermHashes(*universe.term_tables(), device)
        th._universe = weakref.ref(universe)
        th.version = universe.terms_version
        universe._dev_terms = (universe.terms_version, str(device), th)
        return th

    def current(self) -> "TermHashes":
        """These tables, or their Universe's newer ones once it has interned new values or
        nodes or relabelled: ids missing from stale tables would hash as
        themselves, and the tree would stop matching a rebuild and a peer's tree.  Tables
        made from explicit arrays follow nothing and are returned as they are."""
        u = self._universe() if self._universe is not None else None
        if u is None or u.terms_version == self.version:
            return self
        return TermHashes.of(u, self.device)


@dataclass(eq=False)
class MerkleTree:
    """A device Merkle tree (include/deltagpu.h dg_merkle): its node heap, the rows per
    bucket, the term hashes its rows were hashed with (None: the ids), and the store it
    indexes (the diff recomputes key leaves from the store's rows)."""

    depth: int
    nodes: torch.Tensor
    n_keys: int = 0
    shard_bits: int = 0
    shard: int = 0
    store: Store | None = None
    counts: torch.Tensor | None = None
    terms: TermHashes | None = None
    starts: torch.Tensor | None = None  # the chunk index (dg_merkle.starts); None: not kept

    @staticmethod
    def empty(depth: int, device, shard_bits: int = 0, shard: int = 0,
              terms: TermHashes | None = None) -> "MerkleTree":
        chunks = 1 << max(depth - 11, 0)
        return MerkleTree(depth, torch.empty(2 * (1 << depth) - 1, dtype=_I64, device=device), 0,
                          shard_bits, shard, None,
                          torch.empty(max(1 << depth, 16), dtype=torch.int16, device=device), terms,
                          torch.empty(chunks + 1, dtype=_I64, device=device))

    def clone(self) -> "MerkleTree":
        return MerkleTree(self.depth, self.nodes.clone(), self.n_keys, self.shard_bits, self.shard,
                          self.store, self.counts.clone(), self.terms,
                          self.starts.clone() if self.starts is not None else None)

    def abi(self) -> _abi.dg_merkle:
        if self.terms is not None:  # follow the Universe's newest tables
            self.terms = self.terms.current()
        t = _abi.dg_merkle()
        t.depth = self.depth
        t.shard_bits = self.shard_bits
        t.shard = self.shard
        t.nodes = self.nodes.data_ptr()
        t.n_keys = self.n_keys
        t.counts = self.counts.data_ptr()
        t.terms = C.pointer(self.terms.c) if self.terms is not None else None
        t.starts = self.starts.data_ptr() if self.starts is not None else None
        return t

    def bucket_counts(self) -> np.ndarray:
        return self.counts[: 1 << self.depth].cpu().numpy().view(np.uint16)

    def root(self) -> int:
        return int(self.nodes[0].item()) & ((1 << 64) - 1)

    def level(self, lv: int) -> np.ndarray:
        return self.nodes[(1 << lv) - 1: (1 << (lv + 1)) - 1].cpu().numpy().view(np.uint64)


@dataclass(eq=False)
class MerkleCont:
    """A partial-diff continuation (dg_merkle_cont): node form (level <= depth) or leaf
    form (level == depth + 1, with the buckets its (key, leaf) pairs cover)."""

    level: int
    pos: torch.Tensor
    hash: torch.Tensor
    n: int
    bucket: torch.Tensor | None = None
    n_buckets: int = 0

    @staticmethod
    def empty(cap: int, cap_buckets: int, device) -> "MerkleCont":
        cap, cap_buckets = max(int(cap), 1), max(int(cap_buckets), 1)
        return MerkleCont(0, torch.empty(cap, dtype=_I64, device=device),
                          torch.empty(cap, dtype=_I64, device=device), 0,
                          torch.empty(cap_buckets, dtype=_I64, device=device), 0)

    @property
    def leaf(self) -> bool:
        return self.n_buckets > 0

    def abi(self) -> _abi.dg_merkle_cont:
        c = _abi.dg_merkle_cont()
        c.level = self.level
        c.pos = self.pos.data_ptr()
        c.hash = self.hash.data_ptr()
        c.n = self.n
        c.cap = int(self.pos.numel())
        c.bucket = self.bucket.data_ptr() if self.bucket is not None else None
        c.n_buckets = self.n_buckets
        c.cap_buckets = int(self.bucket.numel()) if self.bucket is not None else 0
        return c

    def _set(self, c: _abi.dg_merkle_cont):
        self.level, self.n, self.n_buckets = int(c.level), int(c.n), int(c.n_buckets)


def fold_roots(roots) -> int:
    """dg_merkle_fold_roots: the unsharded root from the 2^b shard roots (shard order)."""
    lib = _abi.load()
    r = np.ascontiguousarray(np.asarray(roots, dtype=np.uint64))
    b = int(len(r)).bit_length() - 1
    if len(r) != 1 << b:
        raise ValueError("fold_roots needs a power-of-two number of shard roots")
    out = C.c_uint64()
    check(lib.dg_merkle_fold_roots(r.ctypes.data_as(_abi.P64), b, C.byref(out)))
    return int(out.value)


class Engine:
    """One libdeltagpu engine (one HIP stream) on one device."""

    def __init__(self, device=None, stream=None):
        if not torch.cuda.is_available():
            raise RuntimeError("libdeltagpu needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _abi.load()
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else
                           torch.device(device).index or 0)
        self.device = dev
        if stream is None:
            # a dedicated stream: the legacy null stream (handle 0) would be ambiguous
            # at the C-ABI, where NULL means "create one"
            stream = torch.cuda.Stream(device=dev)
        self.stream = stream
        h = C.c_void_p()
        check(self.lib.dg_engine_create(dev.index, C.c_void_p(stream.cuda_stream), C.byref(h)))
        self.h = h
        self._d_counts = torch.zeros(8, dtype=_I64, device=dev)

    def _order(self):
        """Make the engine stream wait for work already queued on torch's current stream
        (uploads of the inputs), so a call never reads half-written tensors."""
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream != self.stream.cuda_stream:
            # one reused event (Stream.wait_stream creates a new one per call)
            if getattr(self, "_order_ev", None) is None:
                self._order_ev = torch.cuda.Event()
            self._order_ev.record(cur)
            self.stream.wait_event(self._order_ev)

    def close(self):
        if getattr(self, "h", None):
            if getattr(self, "_home", None) is not None:
                self.lib.dg_host_free(self.h, self._home)
                self._home = None
            self.lib.dg_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(self.lib.dg_engine_sync(self.h))

    # ---------------------------------------------------------------- join
    def _keys(self, keys: torch.Tensor | None):
        """(pointer, n) of a `keys` argument: None -> NULL (every key); an empty tensor
        -> a valid pointer with n = 0 (no key -- an empty tensor's data_ptr() is 0,
        which the C-ABI would read as NULL)."""
        if keys is None:
            return None, 0
        if keys.numel() == 0:
            if getattr(self, "_no_keys", None) is None:
                self._no_keys = torch.zeros(1, dtype=_I64, device=self.device)
            return _ptr(self._no_keys, _abi.P64), 0
        return _ptr(keys, _abi.P64), int(keys.numel())

    def join2(self, a: Store, ca: Context, b: Store, cb: Context, keys: torch.Tensor | None = None,
              out: Store | None = None, out_ctx: Context | None = None):
        self._order()
        if out is None:
            out = Store.empty(a.n + b.n, self.device)
        if out_ctx is None:
            out_ctx = Context.empty(DG_CTX_VV, ca.n + cb.n, self.device)
        so, co = out.abi(), out_ctx.abi()
        sa, sb, xa, xb = a.abi(), b.abi(), ca.abi(), cb.abi()
        kp, nk = self._keys(keys)
        check(self.lib.dg_join2(self.h, C.byref(sa), C.byref(xa), C.byref(sb), C.byref(xb),
                                kp, nk, C.byref(so), C.byref(co)))
        out.n = int(so.n)
        out_ctx.n = int(co.n)
        out_ctx.kind = int(co.kind)
        return out, out_ctx

    def join2_changes(self, a: Store, ca: Context, b: Store, cb: Context,
                      keys: torch.Tensor | None = None, out: Store | None = None,
                      out_ctx: Context | None = None):
        """join/3 plus CausalCrdt's changed-key diff (diff/3, causal_crdt.ex:343-351):
        returns (out, out_ctx, changed) with `changed` the ascending device int64 tensor
        of the keys (of `keys`, or all) whose rows in `out` differ from those in `a`."""
        self._order()
        if out is None:
            out = Store.empty(a.n + b.n, self.device)
        if out_ctx is None:
            out_ctx = Context.empty(DG_CTX_VV, ca.n + cb.n, self.device)
        cap = max(a.n + b.n, 1)
        changed = torch.empty(cap, dtype=_I64, device=self.device)
        so, co = out.abi(), out_ctx.abi()
        sa, sb, xa, xb = a.abi(), b.abi(), ca.abi(), cb.abi()
        kp, nk = self._keys(keys)
        n = C.c_uint64(0)
        check(self.lib.dg_join2_changes(self.h, C.byref(sa), C.byref(xa), C.byref(sb), C.byref(xb),
                                        kp, nk, C.byref(so), C.byref(co), _ptr(changed, _abi.P64),
                                        cap, C.byref(n)))
        out.n = int(so.n)
        out_ctx.n = int(co.n)
        out_ctx.kind = int(co.kind)
        return out, out_ctx, changed[: n.value]

    def join2_async(self, a: Store, ca: Context, b: Store, cb: Context, out: Store,
                    out_ctx: Context, keys: torch.Tensor | None = None, d_counts=None):
        """Enqueue the join; counts land in d_counts[0:2] (device)."""
        self._order()
        if d_counts is None:
            d_counts = self._d_counts
        so, co = out.abi(), out_ctx.abi()
        sa, sb, xa, xb = a.abi(), b.abi(), ca.abi(), cb.abi()
        kp, nk = self._keys(keys)
        check(self.lib.dg_join2_async(self.h, C.byref(sa), C.byref(xa), C.byref(sb), C.byref(xb),
                                      kp, nk, C.byref(so), C.byref(co), _ptr(d_counts, _abi.P64)))
        out_ctx.kind = int(co.kind)
        return d_counts

    def prepare_join2(self, a: Store, ca: Context, b: Store, cb: Context, out: Store,
                      out_ctx: Context, d_counts: torch.Tensor, keys: torch.Tensor | None = None):
        """Pre-marshal one join for repeated asynchronous launches (benchmark loops):
        returns a zero-argument callable that enqueues dg_join2_async."""
        args = [a.abi(), ca.abi(), b.abi(), cb.abi(), out.abi(), out_ctx.abi()]
        refs = [C.byref(x) for x in args]
        kp, nk = self._keys(keys)
        dp = _ptr(d_counts, _abi.P64)
        f, h = self.lib.dg_join2_async, self.h

        def launch():
            check(f(h, refs[0], refs[1], refs[2], refs[3], kp, nk, refs[4], refs[5], dp))

        # the device memory the raw pointers name stays alive as long as the callable
        launch._keep = (a, ca, b, cb, out, out_ctx, args, keys, d_counts)
        return launch

    def joink(self, stores, ctxs, out: Store | None = None, out_ctx: Context | None = None):
        self._order()
        k = len(stores)
        arr_s = (_abi.dg_store * k)(*[s.abi() for s in stores])
        arr_c = (_abi.dg_context * k)(*[c.abi() for c in ctxs])
        if out is None:
            out = Store.empty(sum(s.n for s in stores), self.device)
        if out_ctx is None:
            out_ctx = Context.empty(DG_CTX_VV, sum(c.n for c in ctxs), self.device)
        so, co = out.abi(), out_ctx.abi()
        check(self.lib.dg_joink(self.h, k, arr_s, arr_c, C.byref(so), C.byref(co)))
        out.n = int(so.n)
        out_ctx.n = int(co.n)
        out_ctx.kind = int(co.kind)
        return out, out_ctx

    def prepare_apply_deltas(self, state: Store, ctx: Context, deltas, dctxs, keys, out: Store,
                             out_ctx: Context):
        """Pre-marshal one dg_apply_deltas call for repeated use (benchmark loops, a
        replica re-applying the same batch shape): returns a zero-argument callable that
        runs it and returns (out, out_ctx)."""
        k = len(deltas)
        arr_s = (_abi.dg_store * max(k, 1))(*[d.abi() for d in deltas])
        arr_c = (_abi.dg_context * max(k, 1))(*[c.abi() for c in dctxs])
        kp = kn = None
        if keys is not None:
            ptrs = [self._keys(t)[0] if t is not None else None for t in keys]
            kp = (C.c_void_p * max(k, 1))(*[C.cast(x, C.c_void_p) if x is not None else None
                                           for x in ptrs])
            kn_np = np.array([int(t.numel()) if t is not None else 0 for t in keys] or [0], np.uint64)
            kn = kn_np.ctypes.data_as(_abi.P64)
        ss, xs, so, co = state.abi(), ctx.abi(), out.abi(), out_ctx.abi()
        refs = (C.byref(ss), C.byref(xs), C.byref(so), C.byref(co))
        f, h = self.lib.dg_apply_deltas, self.h

        def run():
            self._order()
            check(f(h, refs[0], refs[1], k, arr_s, arr_c, kp, kn, refs[2], refs[3]))
            out.n = int(so.n)
            out_ctx.n = int(co.n)
            out_ctx.kind = int(co.kind)
            return out, out_ctx

        run._keep = (arr_s, arr_c, kp, kn, keys, ss, xs, so, co, state, ctx, deltas, dctxs)
        if keys is not None:
            run._keep += (kn_np,)
        return run

    def apply_deltas(self, state: Store, ctx: Context, deltas, dctxs, keys=None,
                     out: Store | None = None, out_ctx: Context | None = None):
        """CausalCrdt's delta application (causal_crdt.ex:383-384): fold of
        join(state, deltas[i], keys[i]); keys[i] a sorted unique device int64 tensor of
        key ids, or None for a full-state join of that delta."""
        self._order()
        k = len(deltas)
        arr_s = (_abi.dg_store * max(k, 1))(*[d.abi() for d in deltas])
        arr_c = (_abi.dg_context * max(k, 1))(*[c.abi() for c in dctxs])
        kp = kn = None
        if keys is not None:
            kp = (C.c_void_p * max(k, 1))(*[C.c_void_p(t.data_ptr() if t is not None and t.numel()
                                                         else 0) for t in keys])
            kn_np = np.array([int(t.numel()) if t is not None else 0 for t in keys] or [0],
                             np.uint64)
            kn = kn_np.ctypes.data_as(_abi.P64)
            # an empty keyset is a join over no keys, not a full-state join: point it at
            # a one-element dummy with n_keys = 0
            dummy = torch.zeros(1, dtype=_I64, device=self.device)
            for i, t in enumerate(keys):
                if t is not None and t.numel() == 0:
                    kp[i] = C.c_void_p(dummy.data_ptr())
        if out is None:
            out = Store.empty(state.n + sum(d.n for d in deltas), self.device)
        if out_ctx is None:
            out_ctx = Context.empty(DG_CTX_VV, ctx.n + sum(c.n for c in dctxs), self.device)
        ss, xs, so, co = state.abi(), ctx.abi(), out.abi(), out_ctx.abi()
        check(self.lib.dg_apply_deltas(self.h, C.byref(ss), C.byref(xs), k, arr_s, arr_c, kp, kn,
                                       C.byref(so), C.byref(co)))
        out.n = int(so.n)
        out_ctx.n = int(co.n)
        out_ctx.kind = int(co.kind)
        return out, out_ctx

    def take_keys(self, s: Store, keys: torch.Tensor, out: Store | None = None) -> Store:
        """Map.take(value, keys) of a sync delta (causal_crdt.ex:324-335): the rows of `s`
        whose key is in `keys` (ascending unique device int64), in store order."""
        self._order()
        kp, nk = self._keys(keys)
        ss = s.abi()
        if out is None:
            # a sync delta holds a few rows per key: room for four (an output of the whole
            # store's size -- 450 MB at config 4 -- cost more than the call); more rows than
            # that: the call reports DG_E_CAPACITY and runs again into a store-sized output
            out = Store.empty(min(max(s.n, 1), max(4 * int(nk), 256)), self.device)
            so = out.abi()
            rc = self.lib.dg_take_keys(self.h, C.byref(ss), kp, nk, C.byref(so))
            if rc == _abi.DG_E_CAPACITY and out.cap < s.n:
                out = Store.empty(max(s.n, 1), self.device)
                so = out.abi()
                rc = self.lib.dg_take_keys(self.h, C.byref(ss), kp, nk, C.byref(so))
            check(rc)
        else:
            so = out.abi()
            check(self.lib.dg_take_keys(self.h, C.byref(ss), kp, nk, C.byref(so)))
        out.n = int(so.n)
        return out

    def mutate_batch(self, state: Store, ctx: Context, node: int, kind: torch.Tensor,
                     key: torch.Tensor, val: torch.Tensor, ts: torch.Tensor,
                     add_rank: torch.Tensor, n_adds: int):
        """A batch of add/remove ops by `node` as one delta (aw_lww_map.ex:99-146):
        device arrays sorted by key (batch order within a key); kind uint8 (1 add),
        add_rank = adds before the op in batch order.  Returns (delta Store, its dot-list
        Context, touched keys) -- join the delta with those keys."""
        self._order()
        m = int(key.numel())
        out = Store.empty(max(m, 1), self.device)
        keys = torch.empty(max(m, 1), dtype=_I64, device=self.device)
        nk = C.c_uint64(0)
        ss, xs, so = state.abi(), ctx.abi(), out.abi()
        args = [_ptr(kind, C.c_void_p) if m else None, _ptr(key, _abi.P64), _ptr(val, _abi.P64),
                _ptr(ts, _abi.PI64), _ptr(add_rank, _abi.P64)]
        for cap in (8 * m + n_adds + 1, state.n + n_adds + 1):
            dots = Context.empty(DG_CTX_DOTS, cap, self.device)
            xd = dots.abi()
            rc = self.lib.dg_mutate_batch(self.h, C.byref(ss), C.byref(xs), node, m, *args, n_adds,
                                          C.byref(so), C.byref(xd), _ptr(keys, _abi.P64),
                                          max(m, 1), C.byref(nk))
            if rc != _abi.DG_E_CAPACITY:
                break
        check(rc)
        out.n = int(so.n)
        dots.n = int(xd.n)
        dots.kind = int(xd.kind)
        return out, dots, keys[: nk.value]

    # ---------------------------------------------------------------- contexts
    def context_union(self, a: Context, b: Context, out: Context | None = None) -> Context:
        self._order()
        if out is None:
            out = Context.empty(DG_CTX_VV, a.n + b.n, self.device)
        xa, xb, xo = a.abi(), b.abi(), out.abi()
        check(self.lib.dg_context_union(self.h, C.byref(xa), C.byref(xb), C.byref(xo)))
        out.n = int(xo.n)
        out.kind = int(xo.kind)
        return out

    def compress_dots(self, dots: Context, out: Context | None = None) -> Context:
        self._order()
        if out is None:
            out = Context.empty(DG_CTX_VV, dots.n, self.device)
        xa, xo = dots.abi(), out.abi()
        check(self.lib.dg_compress_dots(self.h, C.byref(xa), C.byref(xo)))
        out.n = int(xo.n)
        out.kind = int(xo.kind)
        return out

    # ---------------------------------------------------------------- read
    def read_lww(self, s: Store, keys: torch.Tensor | None = None):
        self._order()
        cap = max(s.n, 1)
        ok = torch.empty(cap, dtype=_I64, device=self.device)
        ov = torch.empty(cap, dtype=_I64, device=self.device)
        n = C.c_uint64()
        ss = s.abi()
        kp, nk = self._keys(keys)
        check(self.lib.dg_read_lww(self.h, C.byref(ss), kp, nk, _ptr(ok, _abi.P64),
                                   _ptr(ov, _abi.P64), cap, C.byref(n)))
        return ok[: n.value], ov[: n.value]

    # ---------------------------------------------------------------- merkle
    def merkle_build(self, s: Store, depth: int, tree: MerkleTree | None = None,
                     shard_bits: int = 0, shard: int = 0,
                     terms: TermHashes | None = None) -> MerkleTree:
        """MerkleMap over every key of `s` (or of its key-hash shard); `terms`: hash the
        rows' terms instead of their ids (a given `tree` keeps its own)."""
        self._order()
        if tree is None or tree.depth != depth:
            tree = MerkleTree.empty(depth, self.device, shard_bits, shard,
                                    terms if terms is not None else (tree.terms if tree else None))
        elif terms is not None:
            tree.terms = terms
        tree.shard_bits, tree.shard = shard_bits, shard
        t = tree.abi()
        ss = s.abi()
        check(self.lib.dg_merkle_build(self.h, C.byref(ss), C.byref(t)))
        tree.n_keys = int(t.n_keys)
        tree.store = s
        return tree

    def prepare_merkle_build(self, s: Store, tree: MerkleTree, d_counts: torch.Tensor):
        """Pre-marshal one dg_merkle_build_async (benchmark loops): a zero-argument
        callable that enqueues the build on the engine stream."""
        args = [s.abi(), tree.abi()]
        refs = [C.byref(x) for x in args]
        dp = _ptr(d_counts, _abi.P64)
        f, h = self.lib.dg_merkle_build_async, self.h

        def launch():
            check(f(h, refs[0], refs[1], dp))

        launch._keep = (args, d_counts, s, tree)
        tree.store = s
        return launch

    def join_delta(self, state: Store, state_ctx: Context, delta: Store, delta_ctx: Context,
                   keys: torch.Tensor, spare: Store, tree: MerkleTree | None = None,
                   changed: torch.Tensor | None = None, rows: Store | None = None):
        """CausalCrdt.update_state_with_delta on a device-resident state
        (causal_crdt.ex:383-404, dg_join_delta): `state` and `state_ctx` become the keyed
        join with the sync delta, `tree` (indexing `state`) is updated for the changed keys.
        In place when every joined key keeps its row count; otherwise the result lands in
        `spare` and the two Store objects exchange their columns (so `state` always holds
        the joined rows).  `rows` (optional): receives the changed keys' joined rows
        (dg_join_delta_rows, what on_diffs reads).  Returns (changed keys, swapped)."""
        self._order()
        if changed is None:
            changed = torch.empty(max(int(keys.numel()), 1), dtype=_I64, device=self.device)
        ss, sc, sd, cd, sp = state.abi(), state_ctx.abi(), delta.abi(), delta_ctx.abi(), spare.abi()
        t = tree.abi() if tree is not None else None
        kp, nk = self._keys(keys)
        n = C.c_uint64(0)
        sw = C.c_int(0)
        args = (self.h, C.byref(ss), C.byref(sc), C.byref(sd), C.byref(cd), kp, nk, C.byref(sp),
                C.byref(t) if t is not None else None, _ptr(changed, _abi.P64), int(changed.numel()),
                C.byref(n), C.byref(sw))
        if rows is None:
            check(self.lib.dg_join_delta(*args))
        else:
            ro = rows.abi()
            check(self.lib.dg_join_delta_rows(*args, C.byref(ro)))
            rows.n = int(ro.n)
        if sw.value:
            for f in ("key", "val", "ts", "node", "cnt"):
                a, b = getattr(state, f), getattr(spare, f)
                setattr(state, f, b)
                setattr(spare, f, a)
            spare.n = 0
        state.n = int(ss.n)
        state_ctx.n = int(sc.n)
        state_ctx.kind = int(sc.kind)
        if tree is not None:
            tree.n_keys = int(t.n_keys) & ((1 << 64) - 1)
            tree.store = state
        return changed[: n.value], bool(sw.value)

    def join_delta_home(self, state: Store, state_ctx: Context, delta: Store, delta_ctx: Context,
                        keys: torch.Tensor, spare: Store, tree: MerkleTree | None = None):
        """dg_join_delta_home: join_delta for a small delta in one launch chain with one
        host wait, the result (changed keys, their rows, the new context) written into
        page-locked host memory.  Returns None when the library declined (DG_HOME_FALLBACK:
        nothing happened), else (changed keys, rows (key, val, ts, node, cnt), context
        (node, cnt), swapped) as numpy arrays."""
        self._order()
        if getattr(self, "_home", None) is None:
            p = C.c_void_p()
            check(self.lib.dg_host_alloc(self.h, _abi.DG_HOME_WORDS * 8, C.byref(p)))
            self._home = p
        ss, sc, sd, cd, sp = state.abi(), state_ctx.abi(), delta.abi(), delta_ctx.abi(), spare.abi()
        t = tree.abi() if tree is not None else None
        kp, nk = self._keys(keys)
        sw = C.c_int(0)
        check(self.lib.dg_join_delta_home(self.h, C.byref(ss), C.byref(sc), C.byref(sd), C.byref(cd), kp,
                                          nk, C.byref(sp), C.byref(t) if t is not None else None,
                                          self._home, C.byref(sw)))
        h = np.ctypeslib.as_array(C.cast(self._home, C.POINTER(C.c_uint64)), shape=(_abi.DG_HOME_WORDS,))
        if int(h[0]) & _abi.DG_HOME_FALLBACK:
            return None
        nch, nr, nc = int(h[1]), int(h[2]), int(h[3])
        S, R0 = _abi.DG_HOME_STRIDE, _abi.DG_HOME_ROWS
        keys_out = h[_abi.DG_HOME_KEYS:_abi.DG_HOME_KEYS + nch].copy()
        rows = (h[R0:R0 + nr].copy(), h[R0 + S:R0 + S + nr].copy(),
                h[R0 + 2 * S:R0 + 2 * S + nr].copy().view(np.int64),
                h[R0 + 4 * S:R0 + 5 * S].view(np.uint32)[:nr].copy(), h[R0 + 3 * S:R0 + 3 * S + nr].copy())
        C0 = _abi.DG_HOME_CTX
        ctx = (h[C0 + _abi.DG_HOME_NODES:C0 + 2 * _abi.DG_HOME_NODES].view(np.uint32)[:nc].copy(),
               h[C0:C0 + nc].copy())
        if sw.value:
            for f in ("key", "val", "ts", "node", "cnt"):
                a, b = getattr(state, f), getattr(spare, f)
                setattr(state, f, b)
                setattr(spare, f, a)
            spare.n = 0
        state.n = int(ss.n)
        state_ctx.n = int(sc.n)
        state_ctx.kind = int(sc.kind)
        if tree is not None:
            tree.n_keys = int(t.n_keys) & ((1 << 64) - 1)
            tree.store = state
        return keys_out, rows, ctx, bool(sw.value)

    def merkle_update(self, tree: MerkleTree, new: Store, keys: torch.Tensor) -> MerkleTree:
        """MerkleMap.put/delete of the changed `keys` + update_hashes: `tree` indexed
        tree.store; afterwards it indexes `new` (causal_crdt.ex:383-394)."""
        self._order()
        t = tree.abi()
        so, sn = tree.store.abi(), new.abi()
        kp, nk = self._keys(keys)
        check(self.lib.dg_merkle_update(self.h, C.byref(t), C.byref(so), C.byref(sn), kp, nk))
        tree.n_keys = int(t.n_keys) & ((1 << 64) - 1)
        tree.store = new
        return tree

    def merkle_diff(self, a: MerkleTree, b: MerkleTree, cap: int | None = None,
                    with_total: bool = False):
        """The differing keys of the two indexed stores, ascending; with `cap` only the
        first cap (Enum.take(keys, max_sync_size)).  with_total: (keys, total)."""
        self._order()
        if cap is None:
            cap = a.n_keys + b.n_keys
        cap = int(cap)
        # the kernels write into an engine-held buffer of `cap` keys (a fresh cap-sized
        # tensor per call -- 200 MB at config 4 -- cost ~100 us of allocation); the caller
        # gets its own copy of the n keys.  (The next engine call orders itself after the
        # copy: _order.)
        out = getattr(self, "_diff_out", None)
        if out is None or out.numel() < max(cap, 1):
            out = self._diff_out = torch.empty(max(cap, 1), dtype=_I64, device=self.device)
        n, tot = C.c_uint64(), C.c_uint64()
        ta, tb, sa, sb = a.abi(), b.abi(), a.store.abi(), b.store.abi()
        check(self.lib.dg_merkle_diff(self.h, C.byref(ta), C.byref(sa), C.byref(tb), C.byref(sb),
                                      _ptr(out, _abi.P64), cap, C.byref(n), C.byref(tot)))
        keys = out[: n.value].clone()
        return (keys, int(tot.value)) if with_total else keys

    def prepare_merkle_diff(self, a: MerkleTree, b: MerkleTree, out: torch.Tensor, cap: int,
                            d_total: torch.Tensor):
        """Pre-marshal dg_merkle_diff_async for repeated launches (benchmark loops, a
        replica's anti-entropy timer): returns a zero-argument callable that enqueues the
        diff; the first min(total, cap) keys land in `out`, the total in d_total[0]."""
        ta, tb, sa, sb = a.abi(), b.abi(), a.store.abi(), b.store.abi()
        refs = [C.byref(x) for x in (ta, sa, tb, sb)]
        op, dp, f, h = _ptr(out, _abi.P64), _ptr(d_total, _abi.P64), self.lib.dg_merkle_diff_async, self.h

        def launch():
            check(f(h, refs[0], refs[1], refs[2], refs[3], op, int(cap), dp))

        launch._keep = (a, b, out, d_total, ta, tb, sa, sb)
        return launch

    def merkle_prepare(self, tree: MerkleTree, levels: int = 8) -> MerkleCont:
        """MerkleMap.prepare_partial_diff(mm, levels) (causal_crdt.ex:255)."""
        self._order()
        L = min(levels, tree.depth)
        cont = MerkleCont.empty(1 << L, 1, self.device)
        c = cont.abi()
        check(self.lib.dg_merkle_prepare(self.h, C.byref(tree.abi()), levels, C.byref(c)))
        cont._set(c)
        return cont

    def merkle_continue(self, tree: MerkleTree, cont: MerkleCont, levels: int = 8,
                        cap: int | None = None):
        """MerkleMap.continue_partial_diff(cont, mm, levels) (causal_crdt.ex:96) on this
        replica's tree: ("continue", MerkleCont) or ("ok", keys, total)."""
        self._order()
        s = tree.store
        if cap is None:
            cap = max(cont.n, 1) + s.n
        keys = torch.empty(max(int(cap), 1), dtype=_I64, device=self.device)
        cin = cont.abi()
        t, ss = tree.abi(), s.abi()
        out_cap, out_bcap = 4 * max(cont.n, 1), max(cont.n, 1)
        for _ in range(3):  # grow the output continuation to the sizes the call reports
            out = MerkleCont.empty(out_cap, out_bcap, self.device)
            co = out.abi()
            nk, tot, st = C.c_uint64(), C.c_uint64(), C.c_int()
            rc = self.lib.dg_merkle_continue(self.h, C.byref(t), C.byref(ss), C.byref(cin), levels,
                                             C.byref(co), _ptr(keys, _abi.P64), int(cap),
                                             C.byref(nk), C.byref(tot), C.byref(st))
            if rc != _abi.DG_E_CAPACITY:
                break
            out_cap, out_bcap = max(int(co.n), out_cap), max(int(co.n_buckets), out_bcap)
        check(rc)
        if st.value == 1:
            out._set(co)
            return ("continue", out)
        return ("ok", keys[: nk.value], int(tot.value))

    def merkle_continue_home(self, tree: MerkleTree, cont: MerkleCont, levels: int = 8,
                             max_entries: int | None = None, cap: int | None = None):
        """dg_merkle_continue_home: one hop (continue_partial_diff + truncate_diff to
        max_entries; None: :infinite) in one launch with one host wait.  ("continue",
        MerkleCont), ("ok", keys, total), or ("declined",) for a continuation over the
        one-workgroup limits (then merkle_continue)."""
        self._order()
        s = tree.store
        mx = (1 << 64) - 1 if max_entries is None else int(max_entries)
        if cap is None:
            cap = max(cont.n, 1) + s.n
        keys = torch.empty(max(int(cap), 1), dtype=_I64, device=self.device)
        cin = cont.abi()
        t, ss = tree.abi(), s.abi()
        out_cap, out_bcap = 4 * max(cont.n, 1), max(cont.n, 1)
        if max_entries is not None:
            out_cap = min(out_cap, max(int(max_entries), 1))
        for _ in range(3):
            out = MerkleCont.empty(out_cap, out_bcap, self.device)
            co = out.abi()
            nk, tot, st = C.c_uint64(), C.c_uint64(), C.c_int()
            rc = self.lib.dg_merkle_continue_home(self.h, C.byref(t), C.byref(ss), C.byref(cin), levels,
                                                  mx, C.byref(co), _ptr(keys, _abi.P64), int(cap),
                                                  C.byref(nk), C.byref(tot), C.byref(st))
            if rc != _abi.DG_E_CAPACITY:
                break
            out_cap, out_bcap = max(int(co.n), out_cap), max(int(co.n_buckets), out_bcap)
        check(rc)
        if st.value == _abi.DG_CONT_DECLINED:
            return ("declined",)
        if st.value == 1:
            out._set(co)
            return ("continue", out)
        return ("ok", keys[: nk.value], int(tot.value))

    def merkle_truncate(self, tree: MerkleTree, cont: MerkleCont, max_entries: int) -> MerkleCont:
        """MerkleMap.truncate_diff(cont, max_sync_size) (causal_crdt.ex:98,212-214)."""
        c = cont.abi()
        check(self.lib.dg_merkle_truncate(self.h, C.byref(tree.abi()), C.byref(c), int(max_entries)))
        cont._set(c)
        return cont

    # ---------------------------------------------------------------- marshalling
    def sort_store(self, s: Store, out: Store | None = None) -> Store:
        """dg_sort_store: rows in any order (e.g. a map walk) -> sorted by (key, val, ts,
        node, cnt), duplicates dropped."""
        self._order()
        if out is None:
            out = Store.empty(max(s.n, 1), self.device)
        si, so = s.abi(), out.abi()
        check(self.lib.dg_sort_store(self.h, C.byref(si), C.byref(so)))
        out.n = int(so.n)
        return out

    def sort_context(self, c: Context, out: Context | None = None) -> Context:
        """dg_sort_context: a VV by node, a dot set by (node, cnt)."""
        self._order()
        if out is None:
            out = Context.empty(c.kind, max(c.n, 1), self.device)
        ci, co = c.abi(), out.abi()
        check(self.lib.dg_sort_context(self.h, C.byref(ci), C.byref(co)))
        out.n, out.kind = int(co.n), int(co.kind)
        return out

    # ---------------------------------------------------------------- interning
    def remap_values(self, s: Store, old_ids: np.ndarray, new_ids: np.ndarray):
        """Rewrite s.val in place after a value relabel (dg_remap_values): old_ids /
        new_ids ascending uint64, the monotone map the Universe produced."""
        self._order()
        o = _np_to_dev(np.asarray(old_ids, np.uint64), np.int64, self.device)
        w = _np_to_dev(np.asarray(new_ids, np.uint64), np.int64, self.device)
        ss = s.abi()
        check(self.lib.dg_remap_values(self.h, C.byref(ss), _ptr(o, _abi.P64), _ptr(w, _abi.P64),
                                       int(len(old_ids))))

    def store_check(self, s: Store):
        self._order()
        ss = s.abi()
        check(self.lib.dg_store_check(self.h, C.byref(ss)))


def u64(t: torch.Tensor) -> np.ndarray:
    """Device int64 tensor holding u64 bits -> numpy uint64."""
    return t.cpu().numpy().view(np.uint64)


__all__ = ["Store", "Context", "MerkleTree", "MerkleCont", "TermHashes", "Engine", "fold_roots", "u64",
           "DG_CTX_VV", "DG_CTX_DOTS"]
