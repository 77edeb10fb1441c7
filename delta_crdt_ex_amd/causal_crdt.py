"""Host mirror of the data path of `DeltaCrdt.CausalCrdt` around the join (reference
lib/delta_crdt/causal_crdt.ex): applying a delta to a replica's state and the diffs
its `on_diffs` subscriber receives.  The GenServer, neighbours, sync messages,
MerkleMap and storage are out of scope.

    from delta_crdt_ex_amd import aw_lww_map as M, causal_crdt as CC
    st = M.compress_dots(M.new())
    st, diffs = CC.update_state_with_delta(st, M.add("k", "v", 1, st), ["k"])
    diffs                                   # => [("add", "k", "v")]

update_state_with_delta/3 (:383-404) runs join/3 and diff/3 (:343-351) as ONE
libdeltagpu call (dg_join2_changes: the changed keys come out of the join's merge),
then diffs_to_callback/3 (:359-381) reads the changed keys from the old and the new
state (dg_read_lww with those keys) and keeps the keys whose read value changed.
"""
from __future__ import annotations

import numpy as np
import torch

from . import aw_lww_map as M
from .store import u64


def update_state_with_delta(state: M.AWLWWMap, delta: M.AWLWWMap, keys):
    """Returns (new_state, diffs): diffs is what on_diffs would receive -- None when no
    key's value map changed (diffs_to_callback/3 is not reached), else a list of
    ("add", key, value) / ("remove", key) in `keys` order (possibly empty)."""
    U = state.universe
    order = list(dict.fromkeys(keys))
    kids = np.unique(np.array([U.key(k) for k in order], dtype=np.uint64))
    kt = torch.from_numpy(np.ascontiguousarray(kids).view(np.int64)).to(M._dev())
    out, octx, changed = M.engine().join2_changes(state.rows, state.ctx, delta.rows, delta.ctx,
                                                  keys=kt)
    new = M.AWLWWMap(out, octx, U)
    if changed.numel() == 0:
        return new, None
    ch = set(int(x) for x in u64(changed))
    ckeys = [k for k in order if U.key(k) in ch]
    old_v, new_v = M.read(state, ckeys), M.read(new, ckeys)
    diffs = []
    for k in ckeys:
        o, n = old_v.get(k), new_v.get(k)
        if o == n:
            continue
        diffs.append(("remove", k) if n is None else ("add", k, n))
    return new, diffs


def apply_ops(state: M.AWLWWMap, ops, node_id):
    """A batch of mutate/3 calls (causal_crdt.ex:337-342 per op) applied as ONE delta:
    (new_state, diffs) as update_state_with_delta/3 would give for the batch's touched
    keys (on_diffs sees the batch's net changes, not each op's)."""
    delta, keys = M.mutate_batch(ops, node_id, state)
    return update_state_with_delta(state, delta, keys)


__all__ = ["update_state_with_delta", "apply_ops"]
