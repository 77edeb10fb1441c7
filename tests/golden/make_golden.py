"""Generate the golden fixtures in tests/golden/ from the term-level oracle.

    python tests/golden/make_golden.py

Every fixture is DATA: input replicas (SoA rows + causal context, as the GPU consumes
them) and the expected outputs computed by oracle/awlww_term.py — the line-by-line
restatement of lib/delta_crdt/aw_lww_map.ex that tests/test_oracle_reference_tests.py
pins to the reference's own unit tests and properties.  The reference (Elixir) cannot
run in this image, so these vectors are the oracle's, generated from
histories built with the reference's own mutators (add/4, remove/3) and joins.

Fixtures (one .npz each):
  kat_*         the five reference KATs (aw_lww_map_test.exs:7-49) as SoA joins
  history_*     random multi-replica histories (ops + directional syncs) with ts ties,
                joined pairwise: join rows/context, read/1, and the Merkle diff
  config1_small config-1-shaped replicas (bench/basic_operations.exs style), 500 keys
  term_hash_vectors.json  the canonical encoding, key id and node / value term hashes of
                terms of every class (delta_crdt_ex_amd/interning.py; c_src/marshal.c
                builds the same bytes and hashes, tests/test_term_hash.py checks both)
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from delta_crdt_ex_amd.interning import Universe  # noqa: E402
from oracle import awlww_term as T  # noqa: E402
from oracle import convert as CV  # noqa: E402
from delta_crdt_ex_amd import storage  # noqa: E402
from oracle import ref as R  # noqa: E402
from oracle.erlterm import Atom, EList  # noqa: E402


def snapshot_case():
    """tests/golden/snapshot_terms.dgsnap: what Storage.write persists after a delta,
    {node_id, sequence_number, crdt_state, merkle_map} (causal_crdt.ex:242-250), for a
    term-valued replica of history("terms", seed 7): its SoA rows and context through a
    fresh Universe, and the depth-6 Merkle tree of the C oracle over the rows' terms."""
    U = Universe()
    A = history(7, U, values=TERM_VALUES)[0]
    rows, ctx = CV.state_to_soa(A, U)
    tree = R.merkle_build(rows, 6, terms=R.Terms(*U.term_tables()))  # a tree over terms
    storage.write_arrays(os.path.join(HERE, "snapshot_terms.dgsnap"), Atom("replica_a"), 3, rows,
                         ctx, U, (6, 0, 0, tree.nodes, tree.counts))
    return A


def soa(state, U):
    rows, ctx = CV.state_to_soa(state, U)
    return rows, ctx


def pack(prefix, rows, ctx):
    k, v, t, n, c = rows
    kind, cn, cc = ctx
    return {f"{prefix}_key": k, f"{prefix}_val": v, f"{prefix}_ts": t, f"{prefix}_node": n,
            f"{prefix}_cnt": c, f"{prefix}_ctx_kind": np.array([kind], np.int32),
            f"{prefix}_ctx_node": cn, f"{prefix}_ctx_cnt": cc}


def write_case(name, A, B, keys, U, note):
    ra, ca = soa(A, U)
    rb, cb = soa(B, U)
    J = T.join(A, B, keys)
    rj, cj = soa(J, U)
    read = T.read(J)
    rk = np.array(sorted(U.key(k) for k in read), np.uint64)
    rv = np.array([U.value(read[U.key_term(int(k))]) for k in rk], np.uint64)
    key_ids = np.array(sorted(set(U.key(k) for k in keys)), np.uint64)
    # Merkle diff semantics: keys whose raw value maps differ (causal_crdt.ex:392)
    diff = sorted(U.key(k) for k in set(A.value) | set(B.value)
                  if A.value.get(k) != B.value.get(k))
    d = {}
    d.update(pack("a", ra, ca))
    d.update(pack("b", rb, cb))
    d.update(pack("out", rj, cj))
    d["keys"] = key_ids
    d["full"] = np.array([1 if set(keys) >= (set(A.value) | set(B.value)) else 0], np.int32)
    d["read_key"] = rk
    d["read_val"] = rv
    d["diff_keys"] = np.array(diff, np.uint64)
    d["note"] = np.array(note)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)


class Clock:
    def __init__(self, t=1000):
        self.t = t

    def __call__(self):
        self.t += 1
        return self.t


def kats(U):
    c = Clock()
    foo = Atom("foo_node")
    add1 = T.add(1, 2, foo, T.new(), c())
    add2 = T.add(2, 2, foo, add1, c())
    write_case("kat_join_two_adds", add1, add2, [1, 2], U, "aw_lww_map_test.exs:13-20")
    rem1 = T.remove(1, foo, add1)
    write_case("kat_remove", add1, rem1, [1], U, "aw_lww_map_test.exs:22-29")
    chg = T.add(1, 3, foo, add1, c())
    write_case("kat_resolve_conflicts", add1, chg, [1], U, "aw_lww_map_test.exs:31-49")


TERM_VALUES = ["a", "b", "ab", Atom("x"), Atom("nil_not"), (1,), (1, "z"), 2.5, 7, -1.5,
               EList([2]), b"\x00"]


def history(seed, U, n_keys=40, n_rep=3, steps=200, ts_ties=True, values=None):
    rnd = random.Random(seed)
    c = Clock()
    reps = [T.compress_dots(T.new()) for _ in range(n_rep)]
    nodes = [1000 + 17 * i for i in range(n_rep)]

    def mutate(i, op, k, v):
        st = reps[i]
        if op == "add":
            # ts ties across replicas: several adds share a timestamp
            ts = (c() // 3) if ts_ties else c()
            d = T.add(k, v, nodes[i], st, ts)
        else:
            d = T.remove(k, nodes[i], st)
        reps[i] = T.join(st, d, [k])

    def sync(i, j):
        a, b = reps[i], reps[j]
        keys = [k for k in set(a.value) | set(b.value) if a.value.get(k) != b.value.get(k)]
        if keys:
            delta = T.AW(a.dots, {k: a.value[k] for k in keys if k in a.value})
            reps[j] = T.join(b, delta, keys)

    for _ in range(steps):
        i = rnd.randrange(n_rep)
        r = rnd.random()
        if r < 0.55:
            mutate(i, "add", rnd.randrange(n_keys),
                   rnd.randrange(6) if values is None else rnd.choice(values))
        elif r < 0.8:
            mutate(i, "remove", rnd.randrange(n_keys), None)
        else:
            sync(i, rnd.randrange(n_rep))
    return reps


# terms of every class the mirror has a stand-in for, with the boundaries of the closed-form
# integer ids, bignums, the two zeros and nested containers
VECTOR_TERMS = [
    0, 1, -1, 255, 256, -(1 << 62) + (1 << 58), -(1 << 62) + (1 << 58) - 1, (1 << 62) - 1, 1 << 62,
    (1 << 64) - 1, 1 << 64, -(1 << 64), 1 << 100, -(3 ** 50),
    0.0, -0.0, 1.0, -2.5, 1e300, 5e-324,
    Atom("a"), Atom("hello_world"), Atom("ünïcode"), None, True, False,
    "", "k1", "ünïcode", b"\x00\xff",
    (), (1,), (1, 2.0, "x"), ((), (Atom("n"), -1)),
    EList(), EList([1, 2, 3]), EList([EList(), (1,)]),
]


def term_vectors():
    """tests/golden/term_hash_vectors.json (see the module docstring)."""
    import json
    from delta_crdt_ex_amd import interning as I
    from delta_crdt_ex_amd.storage import _pack
    from oracle.erlterm import emap
    terms = VECTOR_TERMS + [emap({1: 2, Atom("a"): "b"}), emap({2.0: 1, 2: (3,)}),
                            (emap({}), EList([emap({0: 0})]))]
    def jpack(x):  # storage._pack with binaries as hex (JSON-safe)
        if isinstance(x, list):
            if x and x[0] == "y":
                return ["yh", x[1].hex()]
            return [jpack(y) for y in x]
        return x

    out = []
    for t in terms:
        out.append({"term": jpack(_pack(t)), "canon": bytes(I.canon(t)).hex(), "key_id": str(I.key_id(t)),
                    "node_hash": str(I.node_hash(t)), "value_hash": str(I.value_hash(t)),
                    "canonical_value": I.is_canonical_int(t)})
    with open(os.path.join(HERE, "term_hash_vectors.json"), "w") as f:
        json.dump(out, f, indent=1, ensure_ascii=True)


def main():
    term_vectors()
    U = Universe()
    kats(U)
    for seed in range(4):
        reps = history(seed, U)
        A, B = reps[0], reps[1]
        allk = sorted(set(A.value) | set(B.value))
        write_case(f"history_{seed}_full", A, B, allk, U, f"random history seed {seed}, full join")
        part = allk[::2] + [999_999]
        write_case(f"history_{seed}_keys", A, B, part, U,
                   f"random history seed {seed}, join over a key subset")
        # sync-shaped delta: sender's VV snapshot + its values for the differing keys
        keys = [k for k in allk if A.value.get(k) != B.value.get(k)]
        delta = T.AW(A.dots, {k: A.value[k] for k in keys if k in A.value})
        write_case(f"history_{seed}_sync", B, delta, keys or [0], U,
                   f"random history seed {seed}, sync delta (causal_crdt.ex:324-335)")
    # term-valued histories: LWW ties between strings, atoms, tuples, floats, lists
    for seed in range(2):
        V = Universe()
        reps = history(100 + seed, V, values=TERM_VALUES)
        A, B = reps[0], reps[1]
        allk = sorted(set(A.value) | set(B.value))
        write_case(f"history_terms_{seed}_full", A, B, allk, V,
                   f"term-valued random history seed {100 + seed}, full join")
    snapshot_case()
    # config-1 shape, small
    A = T.compress_dots(T.new())
    n = 500
    for k in range(1, n + 1):
        A = T.join(A, T.add(k, k, 1, A, k * 1000), [k])
    B = A
    for k in range(1, n + 1):
        if k % 10 == 0:
            A = T.join(A, T.remove(k, 1, A), [k])
        if k % 10 == 5:
            B = T.join(B, T.add(k, k + 1, 2, B, n * 1000 + k), [k])
    write_case("config1_small", A, B, sorted(set(A.value) | set(B.value)), U,
               "config 1 shape (bench/basic_operations.exs), 500 keys")
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith((".npz", ".dgsnap", ".json"))))


if __name__ == "__main__":
    main()
