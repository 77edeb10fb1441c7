"""The NIF's term-independent half (c_src/marshal.c) and the C-ABI path the NIF drives,
run from C (c_src/test_marshal.c): value ids in Erlang term order across relabels, dense
node ids and key-id collisions on the CPU; on the GPU, replicas marshalled in map-walk
order are uploaded, ordered by dg_sort_store / dg_sort_context, joined and read through
the C-ABI, bit-exact against the C oracle, and a relabel rewrites a device store
(dg_remap_values)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "c_src", "_build", "test_marshal")


def _build():
    # built by __graft_entry__.build(); rebuilt here only when absent (CPU runs)
    if not os.path.exists(EXE):
        from oracle import ref
        ref.build()
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "c_src")], check=True)


def test_marshal_c_cpu():
    _build()
    env = dict(os.environ, DG_REQUIRE_GPU="0")
    r = subprocess.run([EXE], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "universe ok" in r.stdout


@pytest.mark.gpu
def test_marshal_c_gpu():
    """Runs as an early process of the session (conftest.EARLY_CMDS), started before
    this process touches the GPU."""
    from conftest import early_result
    assert os.path.exists(EXE), "c_src/_build/test_marshal is built by __graft_entry__.build()"
    rc, out = early_result("c_marshal")
    assert rc == 0, out
    assert "gpu marshal/sort/join/read ok" in out and "gpu relabel remap ok" in out


def test_nif_source_type_checks():
    """c_src/deltagpu_nif.c compiles (-fsyntax-only, warnings as errors) against the erl_nif
    API declarations restated in c_src/syntax_check/erl_nif.h -- this image has no
    Erlang/OTP, so the NIF itself is built by the Elixir project."""
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "c_src", "syntax_check"),
                        os.path.join(ROOT, "c_src", "deltagpu_nif.c")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
