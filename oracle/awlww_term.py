"""Term-level CPU restatement of `DeltaCrdt.AWLWWMap` — the ORACLE.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path imports this module; only
`tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may use it,
and only as the checker.

This is a line-by-line restatement of `lib/delta_crdt/aw_lww_map.ex` (reference
package delta_crdt 0.5.10) over Python stand-ins for BEAM terms:

* ``MapSet``  -> ``frozenset``          (a causal context given as an explicit dot set)
* ``%{}`` map -> ``dict``               (a compressed context = version vector, node -> max)
* a dot ``{node_id, counter}`` -> ``(node_id, counter)``
* ``%AWLWWMap{dots, value}`` -> ``AW(dots, value)`` with
  ``value = {key: {(val, ts): frozenset(dots)}}``

Map iteration order matters in exactly one place, `read/1`'s `Enum.max_by` tie-break
(aw_lww_map.ex:213).  For <= 32 entries the BEAM iterates a flatmap in term order of
its keys, so `read` walks entries sorted by Erlang term order (oracle/erlterm.py).
Above 32 entries the BEAM uses HAMT order, which is not reproducible off the BEAM:
`read` raises `TieOrderUnpinned` if a tie must be broken among > 32 entries.

Parity pinning: tests/test_oracle_reference_tests.py replays the reference's own
tests (`test/aw_lww_map_test.exs:7-86`, `test/aw_lww_map_property_test.exs:18-76`)
against this module; there is no BEAM in this image to run the reference itself
(SURVEY.md §8(c)).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field

from .erlterm import term_sorted, sort_key, tg


class TieOrderUnpinned(Exception):
    """An LWW tie among > 32 entries: BEAM HAMT iteration order decides."""


@dataclass(frozen=True)
class AW:
    """`%DeltaCrdt.AWLWWMap{dots: MapSet.new(), value: %{}}` (aw_lww_map.ex:2-3)."""

    dots: object = field(default_factory=frozenset)
    value: dict = field(default_factory=dict)


def new():
    """aw_lww_map.ex:8"""
    return AW(frozenset(), {})


# ---------------------------------------------------------------- Dots (aw_lww_map.ex:10-97)

def _is_set(d):
    return isinstance(d, (frozenset, set))


def dots_compress(dots):
    """aw_lww_map.ex:13-20 — MapSet -> %{node => max counter}."""
    assert _is_set(dots), "FunctionClauseError: compress/1 takes a MapSet"
    out = {}
    for (c, i) in dots:
        x = out.get(c)
        out[c] = x if (x is not None and x > i) else i
    return out


def dots_next_dot(i, c):
    """aw_lww_map.ex:30-37"""
    if _is_set(c):
        c = dots_compress(c)
    return (i, c.get(i, 0) + 1)


def dots_union(d1, d2):
    """aw_lww_map.ex:39-52"""
    if _is_set(d1) and _is_set(d2):
        return frozenset(d1) | frozenset(d2)
    if _is_set(d1):
        return dots_union(d2, d1)
    out = dict(d1)
    items = d2 if _is_set(d2) else d2.items()
    for (c, i) in items:
        x = out.get(c)
        out[c] = x if (x is not None and x > i) else i
    return out


def dots_member(dots, dot):
    """aw_lww_map.ex:67-73"""
    if _is_set(dots):
        return dot in dots
    i, x = dot
    return dots.get(i, 0) >= x


def dots_difference(d1, d2):
    """aw_lww_map.ex:54-65"""
    if _is_set(d1) and _is_set(d2):
        return frozenset(d1) - frozenset(d2)
    if _is_set(d2):
        raise RuntimeError("this should not happen")
    items = d1 if _is_set(d1) else d1.items()
    return frozenset(d for d in items if not dots_member(d2, d))


# ---------------------------------------------------------------- mutators (aw_lww_map.ex:99-150)

def add(key, value, i, state, ts):
    """aw_lww_map.ex:99-112.  `ts` stands in for System.monotonic_time(:nanosecond)."""
    rem = remove(key, i, state)

    def op(aw_set, context):
        return _aw_set_add(i, (value, ts), aw_set, context)

    addd = _apply_op(op, key, state)
    if len(rem.dots) == 0:
        return addd
    return join(rem, addd, [key])


def compress_dots(state):
    """aw_lww_map.ex:115-117"""
    return AW(dots_compress(state.dots), state.value)


def _aw_set_add(i, el, aw_set, c):
    """aw_lww_map.ex:119-122"""
    d = dots_next_dot(i, c)
    return {el: frozenset([d])}, frozenset(aw_set.get(el, frozenset())) | {d}


def _apply_op(op, key, state):
    """aw_lww_map.ex:124-131"""
    val, c_p = op(state.value.get(key, {}), state.dots)
    return AW(frozenset(c_p), {key: val})


def remove(key, _i, state):
    """aw_lww_map.ex:133-146"""
    to_remove = []
    if key in state.value:
        for _val, dots in state.value[key].items():
            to_remove.extend(dots)
    return AW(frozenset(to_remove), {})


def clear(_i, state):
    """aw_lww_map.ex:148-150"""
    return AW(state.dots, {})


# ---------------------------------------------------------------- join (aw_lww_map.ex:153-209)

def join(delta1, delta2, keys):
    """aw_lww_map.ex:153-158"""
    new_dots = dots_union(delta1.dots, delta2.dots)
    value = _join_or_maps(delta1, delta2, ["join_or_maps", "join_dot_sets"], keys)
    return AW(new_dots, value)


def _uniq(xs):
    seen, out = set(), []
    for x in xs:
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out


def _join_or_maps(delta1, delta2, nested_joins, keys):
    """aw_lww_map.ex:161-193; returns the joined `value` map."""
    resolved = {}
    for key in keys:
        sub1 = AW(delta1.dots, delta1.value.get(key, {}))
        sub2 = AW(delta2.dots, delta2.value.get(key, {}))
        sub_keys = _uniq(list(_map_keys(sub1.value)) + list(_map_keys(sub2.value)))
        nxt, other = nested_joins[0], nested_joins[1:]
        if nxt == "join_or_maps":
            new_sub = _join_or_maps(sub1, sub2, other, sub_keys)
        else:
            new_sub = _join_dot_sets(sub1, sub2, other, sub_keys)
        if len(new_sub) != 0:
            resolved[key] = new_sub
    new_val = {k: v for k, v in delta1.value.items() if k not in set(keys)}
    new_val.update({k: v for k, v in delta2.value.items() if k not in set(keys)})
    new_val.update(resolved)
    return new_val


def _map_keys(m):
    # Map.keys of a value map; a MapSet reached here would be a malformed state.
    return m.keys() if isinstance(m, dict) else ()


def _join_dot_sets(d1, d2, nested, _keys):
    """aw_lww_map.ex:196-209; returns the joined MapSet."""
    assert nested == []
    s1 = frozenset(d1.value) if not isinstance(d1.value, dict) else frozenset(d1.value.keys())
    s2 = frozenset(d2.value) if not isinstance(d2.value, dict) else frozenset(d2.value.keys())
    # MapSet.new(%{}) is the empty set; a missing entry arrives as %{}.
    parts = [s1 & s2, dots_difference(s1, d2.dots), dots_difference(s2, d1.dots)]
    return parts[0] | parts[1] | parts[2]


# ---------------------------------------------------------------- read (aw_lww_map.ex:211-224)

def read(state, keys=None):
    """aw_lww_map.ex:211-224 (`read/1`, `read/2`, `read/3` via a single key)."""
    values = state.value
    if keys is not None:
        if not isinstance(keys, list):
            keys = [keys]
        values = {k: values[k] for k in keys if k in values}
    out = {}
    for key, entries in values.items():
        out[key] = _max_by_ts(entries)[0]
    return out


def _max_by_ts(entries):
    """`Enum.max_by(values, fn {{_v, ts}, _c} -> ts end)`: first maximum in map order."""
    order = term_sorted(entries.keys())
    best = None
    for vt in order:
        if best is None or vt[1] > best[1]:
            best = vt
    if len(order) > 32:
        n_max = sum(1 for vt in order if vt[1] == best[1])
        if n_max > 1:
            raise TieOrderUnpinned(f"{n_max}-way ts tie among {len(order)} entries")
    return best


# ---------------------------------------------------------------- helpers for tests

def rows(state):
    """Flatten a state's value into canonical rows (key, val, ts, node, counter)."""
    out = []
    for key, entries in state.value.items():
        for (val, ts), dots in entries.items():
            for (node, counter) in dots:
                out.append((key, val, ts, node, counter))
    return term_sorted(out)


def canon(state):
    """A hashable canonical form of a state (for equality checks)."""
    d = state.dots
    ctx = ("set", frozenset(d)) if _is_set(d) else ("vv", frozenset(d.items()))
    return ctx, tuple(rows(state))


def join_k(states, keys):
    """Left fold of join/3 — how CausalCrdt applies a stream of deltas."""
    return list(itertools.accumulate(states, lambda a, b: join(a, b, keys)))[-1]


def causal_diff(old, new, keys):
    """causal_crdt.ex:343-351 (diff/3): per key of `keys`, in order, {:add, key,
    new_value_map} when the raw per-key value maps differ and the key survives,
    {:remove, key} when it does not."""
    out = []
    for key in keys:
        o, n = old.value.get(key), new.value.get(key)
        if o == n:
            continue
        out.append(("remove", key) if n is None else ("add", key, n))
    return out


def diffs_to_callback(old, new, keys):
    """causal_crdt.ex:361-381: what the `on_diffs` subscriber receives for the keys diff/3
    reported -- None when that list is empty (:361, the callback is not called), else per
    key, in order, from read/2 of both states (:364-365):
        {old, old} -> []              (exact match, `=:=`; nil/absent on both sides too)
        {_old, nil} -> {:remove, key} (Map.get gives nil for an absent key AND a nil value)
        {_old, new} -> {:add, key, new}
    `None` stands for the atom nil."""
    if len(keys) == 0:
        return None
    ro, rn = read(old, list(keys)), read(new, list(keys))
    out = []
    for key in keys:
        o, n = ro.get(key), rn.get(key)
        if tg(o) == tg(n):  # an absent key reads as None, i.e. as tg(nil)
            continue
        out.append(("remove", key) if tg(n) == _NIL else ("add", key, n))
    return out


_NIL = tg(None)


def update_state_with_delta(state, delta, keys):
    """causal_crdt.ex:383-404, the CRDT half: (joined state, what on_diffs receives):
    join/3 (:384), diff/3 (:388), diffs_to_callback/3 over diffs_keys (:354-359,400)."""
    new = join(state, delta, keys)
    diffs = causal_diff(state, new, keys)
    return new, diffs_to_callback(state, new, [d[1] for d in diffs])

