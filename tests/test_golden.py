"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from the
term-level oracle) replayed through the C oracle (CPU) and libdeltagpu (GPU)."""
import glob
import os

import numpy as np
import pytest

from oracle import ref as R

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)

    def rows(p):
        return (z[f"{p}_key"], z[f"{p}_val"], z[f"{p}_ts"], z[f"{p}_node"], z[f"{p}_cnt"])

    def ctx(p):
        return (int(z[f"{p}_ctx_kind"][0]), z[f"{p}_ctx_node"], z[f"{p}_ctx_cnt"])

    return z, rows, ctx


def test_fixtures_exist():
    assert len(FIXTURES) >= 10


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_c_oracle_reproduces_fixture(path):
    z, rows, ctx = load(path)
    keys = None if int(z["full"][0]) else z["keys"]
    got_rows, got_ctx = R.join2(rows("a"), ctx("a"), rows("b"), ctx("b"), keys=keys)
    want_rows, want_ctx = rows("out"), ctx("out")
    for x, y in zip(got_rows, want_rows):
        assert np.array_equal(x, y)
    assert got_ctx[0] == want_ctx[0]
    assert np.array_equal(got_ctx[1], want_ctx[1]) and np.array_equal(got_ctx[2], want_ctx[2])
    k, v = R.read_lww(want_rows)
    assert np.array_equal(k, z["read_key"]) and np.array_equal(v, z["read_val"])
    assert np.array_equal(R.store_diff(rows("a"), rows("b")), z["diff_keys"])
    ta, tb = R.merkle_build(rows("a"), 6), R.merkle_build(rows("b"), 6)
    d = np.unique(ta.bucket_of(z["diff_keys"]))
    assert np.array_equal(np.flatnonzero(ta.level(6) != tb.level(6)), d)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_gpu_reproduces_fixture(engine, path):
    import torch

    from delta_crdt_ex_amd.store import Context, Store, u64
    dev = "cuda:0"
    z, rows, ctx = load(path)
    sa = Store.from_numpy(*rows("a"), device=dev)
    sb = Store.from_numpy(*rows("b"), device=dev)
    ca = Context.from_numpy(*ctx("a"), dev)
    cb = Context.from_numpy(*ctx("b"), dev)
    keys = None
    if not int(z["full"][0]):
        keys = torch.from_numpy(np.ascontiguousarray(z["keys"]).view(np.int64)).to(dev)
    out, octx = engine.join2(sa, ca, sb, cb, keys=keys)
    for x, y in zip(out.to_numpy(), rows("out")):
        assert np.array_equal(x, y)
    want = ctx("out")
    assert octx.kind == want[0]
    node, cnt = octx.to_numpy()
    assert np.array_equal(node, want[1]) and np.array_equal(cnt, want[2])
    ok, ov = engine.read_lww(out)
    assert np.array_equal(u64(ok), z["read_key"]) and np.array_equal(u64(ov), z["read_val"])
    ta, tb = engine.merkle_build(sa, 6), engine.merkle_build(sb, 6)
    assert np.array_equal(u64(engine.merkle_diff(ta, tb)), z["diff_keys"])
    assert np.array_equal(ta.nodes.cpu().numpy().view(np.uint64), R.merkle_build(rows("a"), 6).nodes)
