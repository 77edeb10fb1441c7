"""ctypes view of the libdeltagpu C-ABI (include/deltagpu.h).

The structs here mirror the header byte for byte; `tests/test_abi.py` checks that
every function the header declares is exported and that the struct layouts match.
Loading fails loudly: there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes as C
import glob
import hashlib
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DG_LIB_PATH") or os.path.join(HERE, "libdeltagpu.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "deltagpu.h")
CSRC = os.path.join(HERE, "csrc")


def source_files() -> list[str]:
    """The sources libdeltagpu.so is built from (the digest's inputs)."""
    return (sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")))
            + [HEADER])


def source_digest() -> str:
    """sha256 prefix over the library's sources (name + content), as build.py embeds it
    in the library (dg_build_digest)."""
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]

DG_OK = 0
DG_E_INVAL = -1
DG_E_CAPACITY = -2
DG_E_DEVICE = -3
DG_E_NOMEM = -4
DG_E_ORDER = -5
DG_E_CLAUSE = -6

DG_HOME_FALLBACK = 1
DG_CONT_DECLINED = 2
DG_CONT_HOME_ENTRIES = 4096
DG_CONT_HOME_BUCKETS = 512
DG_HOME_KEYS = 8
DG_HOME_STRIDE = 1536
DG_HOME_ROWS = DG_HOME_KEYS + 512
DG_HOME_NODES = 2048
DG_HOME_CTX = DG_HOME_ROWS + 4 * DG_HOME_STRIDE + DG_HOME_STRIDE // 2
DG_HOME_WORDS = DG_HOME_CTX + DG_HOME_NODES + DG_HOME_NODES // 2

DG_CTX_VV = 0
DG_CTX_DOTS = 1

P64 = C.POINTER(C.c_uint64)
PI64 = C.POINTER(C.c_int64)
P32 = C.POINTER(C.c_uint32)
# struct pointer fields are untyped (same size and offsets as the header's typed pointers):
# the host mirror sets them from tensor addresses without a ctypes cast per field
VP = C.c_void_p


class dg_store(C.Structure):
    _fields_ = [
        ("key", VP),
        ("val", VP),
        ("ts", VP),
        ("node", VP),
        ("cnt", VP),
        ("n", C.c_uint64),
        ("cap", C.c_uint64),
    ]


class dg_context(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("reserved", C.c_int32),
        ("node", VP),
        ("cnt", VP),
        ("n", C.c_uint64),
        ("cap", C.c_uint64),
    ]


class dg_term_hashes(C.Structure):
    _fields_ = [
        ("node_hash", VP),
        ("n_nodes", C.c_uint64),
        ("val_id", VP),
        ("val_hash", VP),
        ("n_vals", C.c_uint64),
    ]


class dg_merkle(C.Structure):
    _fields_ = [
        ("depth", C.c_uint32),
        ("shard_bits", C.c_uint32),
        ("shard", C.c_uint64),
        ("nodes", VP),
        ("n_keys", C.c_uint64),
        ("counts", VP),
        ("terms", C.POINTER(dg_term_hashes)),
        ("starts", VP),
    ]


class dg_merkle_cont(C.Structure):
    _fields_ = [
        ("level", C.c_uint32),
        ("reserved", C.c_uint32),
        ("pos", VP),
        ("hash", VP),
        ("n", C.c_uint64),
        ("cap", C.c_uint64),
        ("bucket", VP),
        ("n_buckets", C.c_uint64),
        ("cap_buckets", C.c_uint64),
    ]


class DeltaGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libdeltagpu error {code}: {msg}")
        self.code = code


class CapacityError(DeltaGpuError):
    pass


class FunctionClauseError(DeltaGpuError):
    """The reference raises FunctionClauseError here (e.g. compress_dots on a VV)."""


_SIGS = {
    "dg_abi_version": (C.c_int, []),
    "dg_build_digest": (C.c_char_p, []),
    "dg_last_error": (C.c_char_p, []),
    "dg_engine_create": (C.c_int, [C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]),
    "dg_engine_destroy": (C.c_int, [C.c_void_p]),
    "dg_engine_stream": (C.c_void_p, [C.c_void_p]),
    "dg_engine_sync": (C.c_int, [C.c_void_p]),
    "dg_store_check": (C.c_int, [C.c_void_p, C.POINTER(dg_store)]),
    "dg_join2": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context),
                           C.POINTER(dg_store), C.POINTER(dg_context), P64, C.c_uint64,
                           C.POINTER(dg_store), C.POINTER(dg_context)]),
    "dg_join2_changes": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context),
                                   C.POINTER(dg_store), C.POINTER(dg_context), P64, C.c_uint64,
                                   C.POINTER(dg_store), C.POINTER(dg_context), P64, C.c_uint64,
                                   P64]),
    "dg_join_delta": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context),
                                C.POINTER(dg_store), C.POINTER(dg_context), P64, C.c_uint64,
                                C.POINTER(dg_store), C.c_void_p, P64, C.c_uint64, P64,
                                C.POINTER(C.c_int)]),
    "dg_join_delta_home": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context),
                                     C.POINTER(dg_store), C.POINTER(dg_context), P64, C.c_uint64,
                                     C.POINTER(dg_store), C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]),
    "dg_join_delta_rows": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context),
                                     C.POINTER(dg_store), C.POINTER(dg_context), P64, C.c_uint64,
                                     C.POINTER(dg_store), C.c_void_p, P64, C.c_uint64, P64,
                                     C.POINTER(C.c_int), C.POINTER(dg_store)]),
    "dg_join_delta_out": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context),
                                    C.POINTER(dg_store), C.POINTER(dg_context), P64, C.c_uint64,
                                    C.POINTER(dg_store), C.c_void_p, P64, C.c_uint64, P64,
                                    C.POINTER(C.c_int), C.POINTER(dg_store), C.POINTER(dg_context)]),
    "dg_take_keys": (C.c_int, [C.c_void_p, C.POINTER(dg_store), P64, C.c_uint64,
                               C.POINTER(dg_store)]),
    "dg_mutate_batch": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context),
                                  C.c_uint32, C.c_uint64, C.c_void_p, P64, P64, PI64, P64,
                                  C.c_uint64, C.POINTER(dg_store), C.POINTER(dg_context), P64,
                                  C.c_uint64, P64]),
    "dg_mutate_batch_async": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context),
                                        C.c_uint32, C.c_uint64, C.c_void_p, P64, P64, PI64, P64,
                                        C.c_uint64, C.POINTER(dg_store), C.POINTER(dg_context), P64,
                                        C.c_uint64, P64]),
    "dg_join2_async": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context),
                                 C.POINTER(dg_store), C.POINTER(dg_context), P64, C.c_uint64,
                                 C.POINTER(dg_store), C.POINTER(dg_context), P64]),
    "dg_joink": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(dg_store), C.POINTER(dg_context),
                           C.POINTER(dg_store), C.POINTER(dg_context)]),
    "dg_apply_deltas": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_context), C.c_int,
                                  C.POINTER(dg_store), C.POINTER(dg_context),
                                  C.POINTER(C.c_void_p), P64, C.POINTER(dg_store),
                                  C.POINTER(dg_context)]),
    "dg_context_union": (C.c_int, [C.c_void_p, C.POINTER(dg_context), C.POINTER(dg_context),
                                   C.POINTER(dg_context)]),
    "dg_compress_dots": (C.c_int, [C.c_void_p, C.POINTER(dg_context), C.POINTER(dg_context)]),
    "dg_read_lww": (C.c_int, [C.c_void_p, C.POINTER(dg_store), P64, C.c_uint64, P64, P64,
                              C.c_uint64, P64]),
    "dg_store_alloc": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(dg_store)]),
    "dg_store_free": (C.c_int, [C.c_void_p, C.POINTER(dg_store)]),
    "dg_store_upload": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_store)]),
    "dg_store_download": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_store)]),
    "dg_context_alloc": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(dg_context)]),
    "dg_context_free": (C.c_int, [C.c_void_p, C.POINTER(dg_context)]),
    "dg_context_upload": (C.c_int, [C.c_void_p, C.POINTER(dg_context), C.POINTER(dg_context)]),
    "dg_context_download": (C.c_int, [C.c_void_p, C.POINTER(dg_context), C.POINTER(dg_context)]),
    "dg_buffer_alloc": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "dg_buffer_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "dg_copy_to_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "dg_copy_to_host": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "dg_copy_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "dg_host_alloc": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "dg_host_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "dg_sort_store": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_store)]),
    "dg_sort_context": (C.c_int, [C.c_void_p, C.POINTER(dg_context), C.POINTER(dg_context)]),
    "dg_remap_values": (C.c_int, [C.c_void_p, C.POINTER(dg_store), P64, P64, C.c_uint64]),
    "dg_merkle_chunks": (C.c_uint64, [C.c_uint32]),
    "dg_merkle_build": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_merkle)]),
    "dg_merkle_build_async": (C.c_int, [C.c_void_p, C.POINTER(dg_store), C.POINTER(dg_merkle),
                                        P64]),
    "dg_merkle_update": (C.c_int, [C.c_void_p, C.POINTER(dg_merkle), C.POINTER(dg_store),
                                   C.POINTER(dg_store), P64, C.c_uint64]),
    "dg_merkle_diff": (C.c_int, [C.c_void_p, C.POINTER(dg_merkle), C.POINTER(dg_store),
                                 C.POINTER(dg_merkle), C.POINTER(dg_store), P64, C.c_uint64, P64,
                                 P64]),
    "dg_merkle_diff_async": (C.c_int, [C.c_void_p, C.POINTER(dg_merkle), C.POINTER(dg_store),
                                       C.POINTER(dg_merkle), C.POINTER(dg_store), P64, C.c_uint64,
                                       P64]),
    "dg_merkle_prepare": (C.c_int, [C.c_void_p, C.POINTER(dg_merkle), C.c_uint32,
                                    C.POINTER(dg_merkle_cont)]),
    "dg_merkle_continue": (C.c_int, [C.c_void_p, C.POINTER(dg_merkle), C.POINTER(dg_store),
                                     C.POINTER(dg_merkle_cont), C.c_uint32,
                                     C.POINTER(dg_merkle_cont), P64, C.c_uint64, P64, P64,
                                     C.POINTER(C.c_int)]),
    "dg_merkle_continue_home": (C.c_int, [C.c_void_p, C.POINTER(dg_merkle), C.POINTER(dg_store),
                                          C.POINTER(dg_merkle_cont), C.c_uint32, C.c_uint64,
                                          C.POINTER(dg_merkle_cont), P64, C.c_uint64, P64, P64,
                                          C.POINTER(C.c_int)]),
    "dg_merkle_truncate": (C.c_int, [C.c_void_p, C.POINTER(dg_merkle), C.POINTER(dg_merkle_cont),
                                     C.c_uint64]),
    "dg_merkle_fold_roots": (C.c_int, [P64, C.c_uint32, P64]),
}


def header_functions(path: str = HEADER) -> list[str]:
    """Names of every function the public header declares."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dg_[a-z0-9_]+)\s*\(", text)))


_lib = None


def load(path: str = LIB_PATH):
    """Load libdeltagpu.so (raises if it is missing — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: build it with `python -m delta_crdt_ex_amd.build` "
            "(libdeltagpu has no CPU fallback)")
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    built = lib.dg_build_digest().decode()
    # (DG_LIB_ANY_DIGEST=1: an A/B against a build of an earlier commit, tools/build_base.sh)
    if os.path.isdir(CSRC) and built != source_digest() and os.environ.get("DG_LIB_ANY_DIGEST") != "1":
        raise RuntimeError(
            f"{path} is stale: built from sources {built}, the tree's are {source_digest()}; "
            "rebuild with `python -m delta_crdt_ex_amd.build`")
    _lib = lib
    return lib


def check(rc: int):
    if rc == DG_OK:
        return
    msg = (_lib.dg_last_error() or b"").decode(errors="replace")
    if rc == DG_E_CAPACITY:
        raise CapacityError(rc, msg)
    if rc == DG_E_CLAUSE:
        raise FunctionClauseError(rc, msg)
    raise DeltaGpuError(rc, msg)
