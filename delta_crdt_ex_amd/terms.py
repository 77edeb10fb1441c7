"""Python stand-ins for BEAM terms that have no direct Python equivalent.

Used by the host mirror (interning) and shared with the test oracle.
``None``/``True``/``False`` stand for the atoms ``nil``/``true``/``false``;
``str`` and ``bytes`` are binaries; ``tuple`` is a tuple.
"""
from __future__ import annotations

import math


class Atom(str):
    """An Erlang atom (``:foo``)."""

    def __repr__(self):
        return ":" + str.__str__(self)


class EList(tuple):
    """An Erlang proper list (hashable so it can be a map key / set member)."""

    def __repr__(self):
        return "[" + ", ".join(repr(x) for x in self) + "]"


class EMap(tuple):
    """An Erlang map as a hashable tuple of (k, v) pairs in key term order
    (build one with `oracle.erlterm.emap`)."""


# Erlang term classes in term order: number < atom < (reference < fun < port < pid) <
# tuple < map < nil < list < bitstring.  Only the classes with a stand-in here appear.
C_NUMBER, C_ATOM, C_TUPLE, C_MAP, C_NIL, C_LIST, C_BITSTRING = 0, 1, 6, 7, 8, 9, 10


def term_class(t) -> int:
    if isinstance(t, bool) or t is None or isinstance(t, Atom):
        return C_ATOM
    if isinstance(t, (int, float)):
        return C_NUMBER
    if isinstance(t, EList):
        return C_NIL if len(t) == 0 else C_LIST
    if isinstance(t, EMap):
        return C_MAP
    if isinstance(t, tuple):
        return C_TUPLE
    if isinstance(t, (str, bytes)):
        return C_BITSTRING
    raise TypeError(f"no Erlang term class for {type(t).__name__}")


def atom_text(t) -> str:
    if t is None:
        return "nil"
    if t is True:
        return "true"
    if t is False:
        return "false"
    return str.__str__(t)


def order_key(t):
    """A Python sort key that orders terms as Erlang's term order does (the order a
    flatmap of <= 32 keys iterates in, which decides AWLWWMap.read/1's tie-break,
    reference lib/delta_crdt/aw_lww_map.ex:211-216):

    * numbers in MAP-KEY order (the order a flatmap's `{value, ts}` keys are sorted in):
      every integer before every float ("in maps key order integers types are considered
      less than floats types", OTP's term-order rules), then by value; -0.0 before 0.0
      (distinct keys since OTP 27; the relative order of the two zeros is unpinned);
    * atoms by their text; tuples by size, then element-wise; maps by size, then keys
      in key order, then values; lists element-wise with a proper prefix first;
      bitstrings byte-wise (a ``str`` is its UTF-8 binary).

    Two keys are equal exactly when the terms are `=:=`."""
    c = term_class(t)
    if c == C_NUMBER:
        if isinstance(t, int):
            return (c, 0, t)
        return (c, 1, t, 0 if math.copysign(1.0, t) < 0 else 1)
    if c == C_ATOM:
        return (c, atom_text(t))
    if c == C_TUPLE:
        return (c, len(t), tuple(order_key(x) for x in t))
    if c == C_MAP:
        return (c, len(t), tuple(order_key(k) for k, _ in t), tuple(order_key(v) for _, v in t))
    if c == C_NIL:
        return (c,)
    if c == C_LIST:
        return (c, tuple(order_key(x) for x in t))
    return (c, t.encode() if isinstance(t, str) else bytes(t))
