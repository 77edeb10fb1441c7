"""Erlang term order for the Python values the oracle and the host mirror use.

TEST INFRASTRUCTURE / HOST HELPER — not a compute path.

Why this exists: `DeltaCrdt.AWLWWMap.read/1` (reference
`lib/delta_crdt/aw_lww_map.ex:211-216`) picks `Enum.max_by(values, ts)`, and ties
go to the FIRST entry in map iteration order.  For maps of <= 32 keys the BEAM
iterates a "flatmap" in Erlang term order of the keys, which here are `{value, ts}`
tuples.  So the tie-break is "smallest value in Erlang term order" and any id we
give a value on the device must preserve that order.

Erlang term order (number < atom < reference < fun < port < pid < tuple < map <
nil < list < bitstring) restricted to the Python stand-ins used here:

* ``int`` / ``float``           -> number, in MAP-KEY order: every integer before every
                                   float, then by value (OTP: "in maps key order integers
                                   types are considered less than floats types"; a flatmap
                                   sorts its {value, ts} keys so, recursively inside
                                   tuples, lists and maps).  -0.0 sorts before 0.0 (distinct
                                   keys since OTP 27; their relative order is unpinned).
                                   The reference's tests never mix ints and floats.
* ``Atom`` / ``None`` / ``bool``  -> atom (``None`` is ``:nil``; ``True``/``False`` are
                                   ``:true``/``:false``); atoms compare by their text
* ``tuple``                     -> tuple: by size, then element-wise
* ``EMap``                      -> map: by size, then sorted keys, then values
* ``EList``                     -> list (``EList()`` is ``[]`` = nil); element-wise
* ``str`` / ``bytes``           -> bitstring (``str`` is its UTF-8 binary, as Elixir strings are)
"""
from __future__ import annotations

import functools
import math


from delta_crdt_ex_amd.terms import Atom, EList, EMap  # noqa: E402,F401  (shared stand-ins)


def _class(t):
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
    raise TypeError(f"no Erlang term class for {type(t).__name__}")


def _atom_text(t):
    if t is None:
        return "nil"
    if t is True:
        return "true"
    if t is False:
        return "false"
    return str.__str__(t)


class Tg(tuple):
    """Exact-equality wrapper ``(tag, payload)`` for a term.

    Python's ``==`` conflates terms the BEAM keeps apart as map keys (``0 == 0.0``,
    ``True == 1``, ``Atom("a") == "a"``, ``EList((1,)) == (1,)``).  Wrapped terms
    compare equal exactly when they are ``=:=`` in Erlang, so oracle maps keyed by
    them behave like BEAM maps."""

    __slots__ = ()


def tg(t):
    """Wrap a stand-in term (recursively) into its exact-equality form."""
    if isinstance(t, Tg):
        return t
    if isinstance(t, bool) or t is None or isinstance(t, Atom):
        return Tg(("a", "nil" if t is None else "true" if t is True else "false" if t is False
                   else str.__str__(t)))
    if isinstance(t, int):
        return Tg(("i", t))
    if isinstance(t, float):  # the sign keeps -0.0 and 0.0 apart (`=:=` since OTP 27)
        return Tg(("f", t, math.copysign(1.0, t) < 0))
    if isinstance(t, EList):
        return Tg(("l", tuple(tg(x) for x in t)))
    if isinstance(t, EMap):
        return Tg(("m", tuple((tg(k), tg(v)) for k, v in t)))
    if isinstance(t, tuple):
        return Tg(("t", tuple(tg(x) for x in t)))
    if isinstance(t, (str, bytes)):
        return Tg(("b", t.encode() if isinstance(t, str) else t))
    raise TypeError(type(t).__name__)


def untg(t):
    """Inverse of `tg` (binaries come back as bytes, atoms as Atom)."""
    if not isinstance(t, Tg):
        return t
    tag, p = t[0], t[1]
    if tag == "a":
        return Atom(p)
    if tag in ("i", "f", "b"):
        return p
    if tag == "l":
        return EList(untg(x) for x in p)
    if tag == "m":
        return EMap((untg(k), untg(v)) for k, v in p)
    return tuple(untg(x) for x in p)


def compare(a, b) -> int:
    """Erlang term comparison: -1, 0, 1 (exact equality `=:=` returns 0)."""
    if isinstance(a, Tg) or isinstance(b, Tg):
        return compare(untg(a), untg(b))
    ca, cb = _class(a), _class(b)
    if ca != cb:
        return -1 if ca < cb else 1
    if ca == 0:
        ia, ib = isinstance(a, int), isinstance(b, int)
        if ia != ib:  # map-key order: integers before floats, whatever their values
            return -1 if ia else 1
        if a < b:
            return -1
        if a > b:
            return 1
        if not ia and a == 0.0:  # -0.0 before 0.0
            sa, sb = math.copysign(1.0, a), math.copysign(1.0, b)
            return (sa > sb) - (sa < sb)
        return 0
    if ca == 1:
        x, y = _atom_text(a), _atom_text(b)
        return (x > y) - (x < y)
    if ca == 6 or ca == 7:
        if len(a) != len(b):
            return -1 if len(a) < len(b) else 1
        if ca == 7:
            for (ka, _), (kb, _) in zip(a, b):
                c = compare(ka, kb)
                if c:
                    return c
            for (_, va), (_, vb) in zip(a, b):
                c = compare(va, vb)
                if c:
                    return c
            return 0
        for x, y in zip(a, b):
            c = compare(x, y)
            if c:
                return c
        return 0
    if ca in (8, 9):
        for x, y in zip(a, b):
            c = compare(x, y)
            if c:
                return c
        return (len(a) > len(b)) - (len(a) < len(b))
    # bitstring
    x = a.encode() if isinstance(a, str) else a
    y = b.encode() if isinstance(b, str) else b
    return (x > y) - (x < y)


sort_key = functools.cmp_to_key(compare)


def term_sorted(items):
    return sorted(items, key=sort_key)


def emap(d):
    """An `EMap` from a dict, pairs in key term order (canonical form)."""
    return EMap(sorted(d.items(), key=lambda kv: sort_key(kv[0])))
