"""Python stand-ins for BEAM terms that have no direct Python equivalent.

Used by the host mirror (interning) and shared with the test oracle.
``None``/``True``/``False`` stand for the atoms ``nil``/``true``/``false``;
``str`` and ``bytes`` are binaries; ``tuple`` is a tuple.
"""
from __future__ import annotations


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
