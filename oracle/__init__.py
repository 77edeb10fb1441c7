"""CPU oracle for delta_crdt_ex_amd — TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import anything from here, and only as the checker (never as the thing measured or
shipped).  Contents:

* `erlterm.py`     — Erlang term order for Python stand-ins of BEAM terms.
* `awlww_term.py`  — line-by-line restatement of `lib/delta_crdt/aw_lww_map.ex` over terms.
* `deltaref.c`     — C restatement of the same algorithm over the SoA dot rows the GPU
                     uses (join2, context union, read/LWW, Merkle build/diff, k-way fold);
                     built into `oracle/_build/libdeltaref.so` by `oracle/Makefile`.
* `ref.py`         — ctypes wrapper around `libdeltaref.so` (numpy in/out).

The reference (Elixir) cannot run here or on the GPU box (no BEAM), so
the oracle is pinned by the reference's own unit tests and properties restated in
`tests/test_oracle_reference_tests.py`, and by the golden fixtures in `tests/golden/`.
"""
