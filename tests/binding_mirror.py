"""The Elixir side of INTEGRATION.md §3, restated in Python over the NIF's mirror
(delta_crdt_ex_amd/nif.py -> c_src/replica.c -> libdeltagpu), so the dispatch that makes
a GPU-attached replica behave like the reference's immutable states can run without a
BEAM.  TEST INFRASTRUCTURE: each function below is the Elixir function of the same name
in INTEGRATION.md §3, clause for clause; `join_cpu` / `read_cpu` are the reference's own
bodies (aw_lww_map.ex:153-224), here the term oracle.

Terms are kept in the oracle's exact-equality form (oracle.erlterm.tg) -- keys, values
and node ids alike -- so Python dicts compare keys as BEAM maps do; the NIF module
converts at its boundary (wrap=tg, unwrap=untg), as the BEAM hands the NIF its terms.

    %AWLWWMap{dots, value, gpu: nil | {res, version, pending}}       AW(dots, value, gpu)

`gpu` pairs the device-resident state (a NIF resource) with the version this struct's
terms correspond to, and `pending`, the local mutations joined into the terms but not yet
into the device state (newest first, as {delta, keys}).
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass, field, replace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from delta_crdt_ex_amd import nif  # noqa: E402
from oracle import awlww_term as T  # noqa: E402
from oracle.erlterm import tg, untg  # noqa: E402

# compile-time config of the patch (Application.compile_env); the tests set 0
GPU_MIN_DOTS = 10_000
GPU_MIN_READ_KEYS = 1_000
MERKLE_DEPTH = 10
LEVELS = 8  # continue_partial_diff(cont, mm, 8) (causal_crdt.ex:96,255)


@dataclass(frozen=True)
class AW:
    """%DeltaCrdt.AWLWWMap{dots, value, gpu} (aw_lww_map.ex:2-3 + the `gpu` field)."""

    dots: object = field(default_factory=frozenset)
    value: dict = field(default_factory=dict)
    gpu: object = None


def is_mapset(d):
    return isinstance(d, (frozenset, set))


# ------------------------------------------------------------------ DeltaCrdt.GPU (the NIF module)
class GPU:
    _engine = None

    @classmethod
    def load_nif(cls, device=0):
        """@on_load: open ONE engine for this node (a failed load keeps the CPU path)."""
        ok, eng = nif.engine_open(device, wrap=tg, unwrap=untg)
        cls._engine = eng if ok == "ok" else None

    @classmethod
    def engine(cls):
        return cls._engine

    @classmethod
    def close(cls):
        if cls._engine is not None:
            cls._engine.close()
        cls._engine = None

    state_load = staticmethod(nif.state_load)
    join_delta = staticmethod(nif.join_delta)
    mutate_batch = staticmethod(nif.mutate_batch)
    read = staticmethod(nif.read)
    take = staticmethod(nif.take)
    merkle_build = staticmethod(nif.merkle_build)
    merkle_prepare = staticmethod(nif.merkle_prepare)
    merkle_continue = staticmethod(nif.merkle_continue)
    resolve_keys = staticmethod(nif.resolve_keys)


# ------------------------------------------------------------------ the reference's bodies
def new():
    return AW(frozenset(), {})


def compress_dots(state):
    """aw_lww_map.ex:115-117 (keeps the struct's other fields)."""
    return replace(state, dots=T.dots_compress(state.dots))


def join_cpu(delta1, delta2, keys):
    """The unchanged join/3 body (aw_lww_map.ex:153-158): a FRESH struct, gpu: nil."""
    r = T.join(T.AW(delta1.dots, delta1.value), T.AW(delta2.dots, delta2.value), keys)
    return AW(r.dots, r.value)


def read_cpu(state, keys=None):
    """The unchanged read/1,2 bodies (aw_lww_map.ex:211-224): keys None is read/1, a list
    read/2, any other term the one key (`read(crdt, key)`, :222-224)."""
    if keys is not None and not isinstance(keys, list):  # (is_list)
        keys = [keys]
    return T.read(T.AW(state.dots, state.value), None if keys is None else list(keys))


def add(key, value, i, state, ts):
    r = T.add(key, value, i, T.AW(state.dots, state.value), ts)
    return AW(r.dots, r.value)


def remove(key, i, state):
    r = T.remove(key, i, T.AW(state.dots, state.value))
    return AW(r.dots, r.value)


# ------------------------------------------------------------------ the patch
def join(state, delta, keys):
    g = state.gpu
    if g is not None and is_mapset(delta.dots):
        # a local mutation (a MapSet context, :124-146): joined on the BEAM, queued
        res, ver, pending = g
        return replace(join_cpu(state, delta, keys), gpu=(res, ver, ((delta, tuple(keys)),) + pending))
    if g is not None:
        # a sync delta: the queue flushed, then joined on the device
        ok, flushed = flush(state)
        if ok == "ok":
            res, ver, _ = flushed.gpu
            r = GPU.join_delta(res, ver, delta.dots, delta.value, list(keys))
            if r[0] == "ok":
                _, ver2, dots, changed = r
                return apply_changed(flushed, (res, ver2, ()), dots, changed)
        return join_cpu(state, delta, keys)  # detached: the struct's terms are authoritative
    return join_cpu(state, delta, keys)


def delta_ops(delta, keys):
    """A mutation delta back into its op: an add's delta holds the key's one new entry
    (aw_lww_map.ex:99-112), a remove's none (:133-146)."""
    (key,) = keys
    entries = delta.value.get(key)
    if entries:
        ((v, ts),) = entries.keys()
        return [("add", key, v, ts)]
    return [("remove", key)]


def op_node(delta):
    """the node of an add's fresh dot (every pending op is this replica's own)"""
    for entries in delta.value.values():
        for dots in entries.values():
            for (node, _c) in dots:
                return node
    return None


def flush(state):
    """The pending mutations down as ONE mutate_batch; the device then holds the terms."""
    res, ver, pending = state.gpu
    if not pending:
        return ("ok", state)
    ordered = list(reversed(pending))
    ops = [op for delta, keys in ordered for op in delta_ops(delta, keys)]
    node = next((n for n in (op_node(d) for d, _ in ordered) if n is not None), tg("none"))
    r = GPU.mutate_batch(res, ver, node, ops)
    if r[0] != "ok":
        return r
    return ("ok", replace(state, gpu=(res, r[1], ())))


def apply_changed(state, gpu, dots, changed):
    value = dict(state.value)
    for k, v in changed:
        if v is None:
            value.pop(k, None)  # the key's entries all went (:177-181)
        else:
            value[k] = v
    return replace(state, dots=dots, value=value, gpu=gpu)


def attach_gpu(state, min_dots=None, eng=None):
    """CausalCrdt.init (:72) / read_from_storage (:220-232): the device copy and its tree.
    A handed-in struct's handle is never trusted -- a struct restored from storage may carry
    one of a VM that has gone, or of another engine -- so the copy is rebuilt from the
    struct's terms (which hold every queued mutation too)."""
    state = detach(state)
    eng = eng or GPU.engine()
    if eng is None or len(state.value) < (GPU_MIN_DOTS if min_dots is None else min_dots):
        return state
    r = GPU.state_load(eng, state.dots, state.value)
    if r[0] != "ok":
        return state
    _, res, ver = r
    if GPU.merkle_build(res, ver, MERKLE_DEPTH) != "ok":
        return state
    return replace(state, gpu=(res, ver, ()))


def detach(state):
    """What send_diff / get_diff ship (causal_crdt.ex:118,331): no device handle, no queue."""
    return replace(state, gpu=None)


def read(state, keys=None):
    """read/1 (keys None: the whole map -- the only way to the NIF's :all), read/2 of a
    list, and read(crdt, key) of any other term (a Tg is a tuple: only lists are lists) as [key] (aw_lww_map.ex:218-224): a map
    keyed by the atom :all reads its key :all, as the reference does."""
    if keys is not None and not isinstance(keys, list):  # (is_list)
        return read(state, [keys])
    g = state.gpu
    if g is not None and not g[2] and (keys is None or len(keys) >= GPU_MIN_READ_KEYS):
        res, ver, _ = g
        r = GPU.read(res, ver, "all" if keys is None else list(keys))
        if r[0] == "ok":
            return r[1]
        # ("error", "stale"): an older struct -- its own terms answer
    return read_cpu(state, keys)


def merkle_prepare(state, levels):
    """sync_interval_or_state_to_all (:254-255) on the device tree: the queue flushed first
    (the returned struct is the replica's new state)."""
    ok, st = flush(state)
    if ok != "ok":
        raise RuntimeError(f"flush failed: {st}")
    res, ver, _ = st.gpu
    r = GPU.merkle_prepare(res, ver, levels)
    if r[0] != "continue":
        raise RuntimeError(f"merkle_prepare failed: {r}")
    return st, r[1]


def merkle_continue(state, cont, levels, max_sync):
    """handle_info({:diff, diff}) (:91-110): continue_partial_diff + truncate on the device."""
    ok, st = flush(state)
    if ok != "ok":
        raise RuntimeError(f"flush failed: {st}")
    res, ver, _ = st.gpu
    r = GPU.merkle_continue(res, ver, cont, levels, max_sync)
    if r[0] not in ("continue", "ok"):
        raise RuntimeError(f"merkle_continue failed: {r}")
    return st, r


# ------------------------------------------------------------------ CausalCrdt (the data path)
@dataclass
class Diff:
    """%Diff{continuation, dots, from, to, originator} (causal_crdt.ex:29)."""

    continuation: bytes
    dots: object
    frm: object
    to: object
    originator: object


class MemoryStorage:
    """test/support/memory_storage.ex: write(name, state) / read(name) over a map."""

    def __init__(self):
        self.map = {}

    def write(self, name, state):
        self.map[name] = state

    def read(self, name):
        return self.map.get(name)


class Replica:
    """CausalCrdt's state and the handlers on the data path (causal_crdt.ex:45-413):
    handle_operation, update_state_with_delta (diff/3, diffs_to_callback/3), read, and
    the sync round (prepare, continue, send_diff / get_diff) run synchronously.

    gpu_merkle: the device tree replaces MerkleMap; False: the device
    does joins and reads only and the sync round is the CPU MerkleMap's (_sync_cpu)."""

    def __init__(self, node, clock, on_diffs=None, max_sync_size=200, gpu=True, min_dots=0,
                 engine=None, storage_module=None, name=None, gpu_merkle=True):
        self.engine = engine or GPU.engine()  # this replica's BEAM node's engine
        self.gpu = gpu
        self.min_dots = min_dots
        self.gpu_merkle = gpu_merkle
        self.node_id = tg(node)
        self.clock = clock
        self.on_diffs = on_diffs
        self.max_sync_size = max_sync_size
        self.storage_module = storage_module
        self.name = name
        self.sequence_number = 0
        st = compress_dots(new())  # init (:72)
        self.crdt_state = self._attach(st)
        self.received = []
        self.read_from_storage()  # handle_continue(:read_storage) (:78-80)

    def _attach(self, st):
        return attach_gpu(st, self.min_dots, self.engine) if self.gpu else detach(st)

    def read_from_storage(self):  # :216-232, the restored struct re-attached (§3.3)
        if self.storage_module is None:
            return
        stored = self.storage_module.read(self.name)
        if stored is None:
            return
        node_id, seq, crdt_state, _merkle_map = stored
        self.node_id, self.sequence_number = node_id, seq
        self.crdt_state = self._attach(crdt_state)

    def write_to_storage(self):  # :234-246: the struct detached (its terms hold the queue)
        if self.storage_module is None:
            return
        self.storage_module.write(self.name, (self.node_id, self.sequence_number,
                                              detach(self.crdt_state), None))

    # handle_operation (:337-342)
    def mutate(self, f, *args):
        key = tg(args[0])
        if f == "add":
            delta = add(key, tg(args[1]), self.node_id, self.crdt_state, self.clock())
        else:
            delta = remove(key, self.node_id, self.crdt_state)
        self.update_state_with_delta(delta, [key])

    # update_state_with_delta (:383-404); the tree's put/delete is the device's (join_delta)
    def update_state_with_delta(self, delta, keys):
        old = self.crdt_state
        new_state = join(old, delta, keys)
        diffs = diff(old, new_state, keys)
        self.crdt_state = new_state
        self.diffs_to_callback(old, new_state, [d[1] for d in diffs])
        self.write_to_storage()

    def diffs_to_callback(self, old_state, new_state, keys):  # :359-381
        if not keys:
            return None
        old = read(old_state, keys)
        new = read(new_state, keys)
        out = []
        nil = tg(None)
        for key in keys:
            o, n = old.get(key, nil), new.get(key, nil)  # Map.get: absent -> nil
            if o == n:
                continue  # {old, old}
            out.append(("remove", key) if n == nil else ("add", key, n))
        self.received.append(out)
        if self.on_diffs:
            self.on_diffs(out)
        return out

    def read(self):  # handle_call(:read) (:188-190): the reply only, no new state
        return read(self.crdt_state)

    # the sync round: sync_interval_or_state_to_all (:252-289) with one neighbour
    def sync_to(self, peer, trace=None):
        if self.crdt_state.gpu is None or not self.gpu_merkle or not peer.gpu_merkle:
            return self._sync_cpu(peer)
        self.crdt_state, cont = merkle_prepare(self.crdt_state, LEVELS)
        d = Diff(cont, self.crdt_state.dots, self, peer, self)
        msgs = [(peer, ("diff", d))]
        while msgs:
            dest, msg = msgs.pop(0)
            if trace is not None:
                trace.append(msg[0])
            msgs.extend(dest.handle(msg))

    def handle(self, msg):
        kind = msg[0]
        if kind == "diff" and len(msg) == 2:  # handle_info({:diff, diff}) (:91-110)
            d = msg[1]
            d = Diff(d.continuation, d.dots, d.to, d.frm, d.originator)  # reverse_diff
            self.crdt_state, r = merkle_continue(self.crdt_state, d.continuation, LEVELS,
                                                 self.max_sync_size)
            if r[0] == "continue":
                return [(d.to, ("diff", Diff(r[1], d.dots, d.frm, d.to, d.originator)))]
            keys = r[1]
            if not keys:
                return []  # ack_diff
            return self.send_diff(d, truncate(keys, self.max_sync_size))
        if kind == "get_diff":  # handle_info({:get_diff, diff, keys}) (:112-123)
            d, keys = msg[1], msg[2]
            d = Diff(d.continuation, d.dots, d.to, d.frm, d.originator)
            keys = GPU.resolve_keys(self.engine, keys)  # ids a peer could not name
            delta = replace(detach(self.crdt_state), dots=d.dots,
                            value={k: self.crdt_state.value[k] for k in keys if k in self.crdt_state.value})
            return [(d.to, ("diff", delta, keys))]
        if kind == "diff":  # handle_info({:diff, delta, keys}) (:86-89)
            self.update_state_with_delta(msg[1], msg[2])
            return []
        raise ValueError(kind)

    def send_diff(self, d, keys):  # :324-335
        if d.originator is d.to:
            return [(d.to, ("get_diff", d, keys))]
        delta = replace(detach(self.crdt_state), dots=d.dots,
                        value={k: self.crdt_state.value[k] for k in keys if k in self.crdt_state.value})
        return [(d.to, ("diff", delta, keys))]

    def _sync_cpu(self, peer):
        """A CPU-only pair (no device): the keys whose raw maps differ, as MerkleMap finds
        them, shipped as send_diff does."""
        a, b = self.crdt_state.value, peer.crdt_state.value
        keys = [k for k in set(a) | set(b) if a.get(k) != b.get(k)]
        if keys:
            delta = replace(detach(self.crdt_state), value={k: a[k] for k in keys if k in a})
            peer.update_state_with_delta(delta, keys)


def truncate(keys, size):  # causal_crdt.ex:206-210
    return keys if size == "infinite" else keys[:size]


def diff(old_state, new_state, keys):  # causal_crdt.ex:344-352, over the raw value maps
    out = []
    for key in keys:
        o, n = old_state.value.get(key), new_state.value.get(key)
        if o == n:
            continue
        out.append(("remove", key) if n is None else ("add", key, n))
    return out
