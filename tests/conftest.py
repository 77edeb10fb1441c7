import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdeltagpu on cuda:0)")


# GPU programs that run in their own processes (the C-ABI test binary, the multi-rank
# sharded round).  They are started when the session starts, BEFORE any test of this
# process initialises the GPU: a process that has initialised the GPU must not start
# other programs.  Tests collect their results with early_result().
EARLY_CMDS = {
    "c_marshal": ([os.path.join(ROOT, "c_src", "_build", "test_marshal")], {"DG_REQUIRE_GPU": "1"}),
    "sharded2": ([sys.executable, "-u", os.path.join(ROOT, "tests", "sharded_round.py"), "--world", "2"],
                 {}),
    "sharded4": ([sys.executable, "-u", os.path.join(ROOT, "tests", "sharded_round.py"), "--world", "4",
                  "--keys-per-rank", "20000"], {}),
}
_EARLY: dict = {}


def _gpu_selected(config) -> bool:
    m = (config.getoption("-m") or "").replace(" ", "")
    return "gpu" in m and "notgpu" not in m


def _launch(name):
    import subprocess
    import tempfile
    cmd, env = EARLY_CMDS[name]
    log = tempfile.TemporaryFile(mode="w+")
    try:
        p = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, cwd=ROOT,
                             env=dict(os.environ, **env))
    except OSError as e:  # e.g. the binary was not built
        log.write(f"could not start {cmd[0]}: {e}")
        p = None
    _EARLY[name] = (p, log)


def pytest_sessionstart(session):
    if _gpu_selected(session.config):
        for name in EARLY_CMDS:
            _launch(name)


def early_result(name, timeout=300):
    """(exit status, output) of an early GPU program (started now if the session did not)."""
    if name not in _EARLY:
        _launch(name)
    p, log = _EARLY[name]
    rc = -1 if p is None else p.wait(timeout=timeout)
    log.seek(0)
    return rc, log.read()


@pytest.fixture(scope="session")
def engine():
    import torch
    from delta_crdt_ex_amd.store import Engine
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need an MI355X: torch.cuda.is_available() is False")
    e = Engine(0)
    yield e
    e.close()
