"""The C-ABI boundary (include/deltagpu.h) without a GPU: the library builds and
loads, exports every function the header declares, the ctypes mirror matches the
header's struct layouts, and the product fails loudly (no CPU fallback) when no
device is present."""
import ctypes as C
import os
import subprocess
import tempfile

import pytest

from delta_crdt_ex_amd import _abi
from delta_crdt_ex_amd.build import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    build()
    return _abi.load()


def test_every_header_function_is_exported(lib):
    names = _abi.header_functions()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name
        assert name in _abi._SIGS, f"ctypes signature missing for {name}"


def test_abi_version(lib):
    assert lib.dg_abi_version() == 4


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "deltagpu.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("dg_store %zu\n", sizeof(dg_store));
  F(dg_store, key) F(dg_store, val) F(dg_store, ts) F(dg_store, node) F(dg_store, cnt)
  F(dg_store, n) F(dg_store, cap)
  printf("dg_context %zu\n", sizeof(dg_context));
  F(dg_context, kind) F(dg_context, node) F(dg_context, cnt) F(dg_context, n) F(dg_context, cap)
  printf("dg_merkle %zu\n", sizeof(dg_merkle));
  F(dg_merkle, depth) F(dg_merkle, shard_bits) F(dg_merkle, shard) F(dg_merkle, nodes)
  F(dg_merkle, n_keys) F(dg_merkle, counts) F(dg_merkle, terms) F(dg_merkle, starts)
  printf("dg_term_hashes %zu\n", sizeof(dg_term_hashes));
  F(dg_term_hashes, node_hash) F(dg_term_hashes, n_nodes) F(dg_term_hashes, val_id)
  F(dg_term_hashes, val_hash) F(dg_term_hashes, n_vals)
  printf("dg_merkle_cont %zu\n", sizeof(dg_merkle_cont));
  F(dg_merkle_cont, level) F(dg_merkle_cont, pos) F(dg_merkle_cont, hash) F(dg_merkle_cont, n)
  F(dg_merkle_cont, cap) F(dg_merkle_cont, bucket) F(dg_merkle_cont, n_buckets)
  F(dg_merkle_cont, cap_buckets)
  return 0;
}
"""


def test_struct_layout_matches_header():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "layout.c")
        exe = os.path.join(d, "layout")
        open(src, "w").write(LAYOUT_C)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    want = {}
    for line in out.strip().splitlines():
        name, v = line.split()
        want[name] = int(v)
    for cls in (_abi.dg_store, _abi.dg_context, _abi.dg_merkle, _abi.dg_merkle_cont,
                _abi.dg_term_hashes):
        assert C.sizeof(cls) == want[cls.__name__]
        for fname, _ in cls._fields_:
            key = f"{cls.__name__}.{fname}"
            if key in want:
                assert getattr(cls, fname).offset == want[key], key


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """The library embeds its sources' digest (dg_build_digest); a library built from other
    sources is refused at load (a stale build must never be what runs)."""
    lib = _abi.load()
    assert lib.dg_build_digest().decode() == _abi.source_digest()
    hdr = tmp_path / "deltagpu.h"
    hdr.write_text(open(_abi.HEADER).read() + "\n/* changed */\n")
    monkeypatch.setattr(_abi, "HEADER", str(hdr))
    monkeypatch.setattr(_abi, "_lib", None)
    with pytest.raises(RuntimeError, match="stale"):
        _abi.load()


def test_no_device_fails_loudly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = C.c_void_p()
    rc = lib.dg_engine_create(0, None, C.byref(h))
    assert rc == _abi.DG_E_DEVICE
    assert b"hipGetDeviceCount" in lib.dg_last_error()
    from delta_crdt_ex_amd.store import Engine
    with pytest.raises(RuntimeError):
        Engine(0)


def test_null_arguments_are_rejected(lib):
    # argument validation happens before any device call
    s = _abi.dg_store()
    x = _abi.dg_context()
    assert lib.dg_join2(None, C.byref(s), C.byref(x), C.byref(s), C.byref(x), None, 0,
                        C.byref(s), C.byref(x)) == _abi.DG_E_INVAL
    assert lib.dg_read_lww(None, C.byref(s), None, 0, None, None, 0, None) == _abi.DG_E_INVAL


def test_replica_layer_exports_every_declared_function(lib):
    """c_src/replica.h (the NIF's device half, bound by delta_crdt_ex_amd/nif.py): the
    shared library exports every function the header declares, each with a ctypes
    signature in the mirror, and dgr_changed matches gcc's layout."""
    import re
    from delta_crdt_ex_amd import nif
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "c_src")], check=True)
    r = nif.load()
    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "c_src", "replica.h")).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(dgr_[a-z0-9_]+)\s*\(", text)))
    assert len(names) >= 15
    for name in names:
        assert hasattr(r, name), name
        assert name in nif._SIGS, f"ctypes signature missing for {name}"
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "replica.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(dgr_changed), offsetof(dgr_changed, version),
         offsetof(dgr_changed, n_changed), offsetof(dgr_changed, keys), offsetof(dgr_changed, rows),
         offsetof(dgr_changed, ctx));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "l")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "c_src"), c, "-o", exe], check=True)
        got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    D = nif.dgr_changed
    assert got == [C.sizeof(D), D.version.offset, D.n_changed.offset, D.keys.offset, D.rows.offset,
                   D.ctx.offset]
    assert nif.DGR_E_STALE == int(re.search(r"DGR_E_STALE \((-?\d+)\)", text).group(1))
