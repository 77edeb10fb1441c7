"""Build libdeltagpu.so in-tree with hipcc for gfx950 (no torch extension: the
boundary is a plain C-ABI library, include/deltagpu.h).

    python -m delta_crdt_ex_amd.build          # incremental
    python -m delta_crdt_ex_amd.build --force

Experiment builds (DG_VARIANT="-DNAME=V", DG_STAMPS=1) go to ab/libdeltagpu_<NAME>.so, a
directory that exists only while an A/B runs (tools/build_base.sh puts a build of an
earlier commit there too); select one with DG_LIB_PATH.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
STAMPS = os.environ.get("DG_STAMPS") == "1"  # diagnostic build with in-kernel phase stamps
VARIANT = os.environ.get("DG_VARIANT", "")     # experiment builds: extra -D flags, own .so
_SUFFIX = ("_stamps" if STAMPS else "") + (("_" + VARIANT.replace("=", "").replace("-D", "").replace(" ", "_")) if VARIANT else "")
OBJ = os.path.join(HERE, "_build" + _SUFFIX)
LIB = os.path.join(HERE, "ab", "libdeltagpu" + _SUFFIX + ".so") if _SUFFIX else os.path.join(HERE, "libdeltagpu.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
SOURCES = ["join.hip", "kfold.hip", "take.hip", "splice.hip", "small.hip", "kdelta.hip", "mutate.hip", "segred.hip", "merkle.hip", "remap.hip", "sort.hip", "api.hip"]
ARCH = os.environ.get("DG_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: libdeltagpu needs the ROCm toolchain")


def _deps() -> list[str]:
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return hdrs + [os.path.join(INCLUDE, "deltagpu.h")]


def _stale(target: str, inputs: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(i) > t for i in inputs)


def _digest_object(hipcc: str, run) -> str:
    """OBJ/digest.o defining dg_build_digest() = the sources' digest (rewritten, and so
    relinked, only when the digest changes)."""
    sys.path.insert(0, HERE)
    try:
        from _abi import source_digest  # noqa: E402  (no package import: no torch needed)
    finally:
        sys.path.pop(0)
    d = source_digest()
    src = os.path.join(OBJ, "digest.c")
    obj = os.path.join(OBJ, "digest.o")
    text = f'const char* dg_build_digest(void) {{ return "{d}"; }}\n'
    if not os.path.exists(src) or open(src).read() != text:
        with open(src, "w") as f:
            f.write(text)
    if _stale(obj, [src]):
        run([hipcc, "-x", "c", "-O2", "-fPIC", "-c", src, "-o", obj])
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    hipcc = _hipcc()
    deps = _deps()
    flags = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-Wno-unused-result", "-I" + INCLUDE] + (["-DDG_STAMPS"] if STAMPS else []) + VARIANT.split()
    jobs = []
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src.replace(".hip", ".o"))
        objs.append(o)
        if force or _stale(o, [s] + deps):
            jobs.append([hipcc] + flags + ["-c", s, "-o", o])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
        if verbose and (r.stdout or r.stderr):
            sys.stderr.write(r.stdout + r.stderr)

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    objs.append(_digest_object(hipcc, run))
    if force or jobs or _stale(LIB, objs):
        tmp = LIB + ".tmp"
        run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs)
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose))
