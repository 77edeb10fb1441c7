"""Joins of two engines (two HIP streams) running at the same time on one GPU.

The single-pass join kernel is persistent: its workgroups hand tile counts to each
other, so a launch must never depend on workgroups that cannot become resident while
its own wait.  Two engines launching joins concurrently on their own
streams is the case that would interleave two such grids on the CUs; both joins must
finish with the same rows as when they run alone."""
import numpy as np
import pytest

from delta_crdt_ex_amd import workloads as W

pytestmark = pytest.mark.gpu


def _inputs(n_keys, seed, dev):
    from delta_crdt_ex_amd.store import Context, Store
    a, b = W.config5(n_keys=n_keys, n_nodes=64, seed=seed)
    sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
    ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
    return sa, ca, sb, cb


@pytest.mark.parametrize("n_keys", [400_000, 3_000_000])  # fused splits / partition launch
def test_two_engines_concurrent_joins(n_keys):
    import torch

    from delta_crdt_ex_amd.store import Context, Engine, Store
    dev = "cuda:0"
    engines = [Engine(0), Engine(0)]
    jobs = []
    for i, eng in enumerate(engines):
        sa, ca, sb, cb = _inputs(n_keys, 50 + i, dev)
        out = Store.empty(sa.n + sb.n, dev)
        octx = Context.empty(0, ca.n + cb.n, dev)
        d = torch.zeros(8, dtype=torch.int64, device=dev)
        launch = eng.prepare_join2(sa, ca, sb, cb, out, octx, d)
        jobs.append((eng, launch, out, d))
    torch.cuda.synchronize()
    # alone: the reference result of each engine
    want = []
    for eng, launch, out, d in jobs:
        launch()
        eng.sync()
        out.n = int(d[0].item())
        want.append(tuple(c.copy() for c in out.to_numpy()))
    # together, several times: both grids in flight at once
    for _ in range(5):
        for eng, launch, out, d in jobs:
            launch()
        for eng, launch, out, d in jobs:
            eng.sync()
        for (eng, launch, out, d), w in zip(jobs, want):
            out.n = int(d[0].item())
            for x, y in zip(out.to_numpy(), w):
                assert np.array_equal(x, y)
    for eng, *_ in jobs:
        eng.close()


def test_join_beside_long_kernels_on_another_stream():
    """A join while ordinary kernels of another stream hold CUs: the join's
    grid becomes resident as those workgroups retire; the result is the same as alone."""
    import torch

    from delta_crdt_ex_amd.store import Context, Engine, Store
    dev = "cuda:0"
    eng = Engine(0)
    sa, ca, sb, cb = _inputs(3_000_000, 61, dev)
    out = Store.empty(sa.n + sb.n, dev)
    octx = Context.empty(0, ca.n + cb.n, dev)
    d = torch.zeros(8, dtype=torch.int64, device=dev)
    launch = eng.prepare_join2(sa, ca, sb, cb, out, octx, d)
    torch.cuda.synchronize()
    launch()
    eng.sync()
    out.n = int(d[0].item())
    want = tuple(c.copy() for c in out.to_numpy())
    side = torch.cuda.Stream(device=dev)
    x = torch.randn(64 << 20, device=dev)  # elementwise kernels: many short workgroups
    torch.cuda.synchronize()
    for _ in range(3):
        with torch.cuda.stream(side):
            for _ in range(16):
                x = torch.sin(x) * 1.0001
        launch()
        eng.sync()
        side.synchronize()
        out.n = int(d[0].item())
        for a, b in zip(out.to_numpy(), want):
            assert np.array_equal(a, b)
    eng.close()


def test_overscheduled_grid_aborts_and_replays(monkeypatch):
    """A single-pass join grid twice the resident size (DG_JOIN_WORKERS=1024; 512
    workgroups fit): the resident half waits on workgroups that cannot start, raises the
    abort flag and runs on; dg_join2 re-runs on the two-pass kernels, dg_engine_sync
    replays the asynchronous joins, dg_join2_changes re-runs on a small grid.  Every
    result equals the one of a co-resident grid."""
    import torch

    from delta_crdt_ex_amd.store import Context, Engine, Store
    dev = "cuda:0"
    sa, ca, sb, cb = _inputs(3_000_000, 71, dev)
    ref = Engine(0)
    want_out, want_ctx, want_chg = ref.join2_changes(sa, ca, sb, cb)
    want = tuple(c.copy() for c in want_out.to_numpy())
    want_c = tuple(c.copy() for c in want_ctx.to_numpy())
    want_k = want_chg.cpu().numpy()
    ref.close()
    monkeypatch.setenv("DG_JOIN_WORKERS", "1024")
    eng = Engine(0)
    out, octx = eng.join2(sa, ca, sb, cb)
    for x, y in zip(out.to_numpy(), want):
        assert np.array_equal(x, y)
    for x, y in zip(octx.to_numpy(), want_c):
        assert np.array_equal(x, y)
    out, octx, chg = eng.join2_changes(sa, ca, sb, cb)
    assert np.array_equal(chg.cpu().numpy(), want_k)
    for x, y in zip(out.to_numpy(), want):
        assert np.array_equal(x, y)
    outs = []
    for _ in range(2):
        o = Store.empty(sa.n + sb.n, dev)
        oc = Context.empty(0, ca.n + cb.n, dev)
        d = torch.zeros(8, dtype=torch.int64, device=dev)
        eng.prepare_join2(sa, ca, sb, cb, o, oc, d)()
        outs.append((o, d))
    eng.sync()
    for o, d in outs:
        o.n = int(d[0].item())
        for x, y in zip(o.to_numpy(), want):
            assert np.array_equal(x, y)
    eng.close()


def test_aborted_async_join_then_synchronous_call(monkeypatch):
    """an asynchronous join whose grid aborts, followed by a synchronous
    call of another kind (dg_read_lww) before dg_engine_sync.  The synchronous call settles
    the pending join first (replays it on the two-pass kernels), so the join's output is
    right and the read sees it; dg_engine_sync afterwards is clean."""
    import torch

    from delta_crdt_ex_amd.store import Context, Engine, Store
    dev = "cuda:0"
    sa, ca, sb, cb = _inputs(3_000_000, 73, dev)
    ref = Engine(0)
    want_out, _ = ref.join2(sa, ca, sb, cb)
    want = tuple(c.copy() for c in want_out.to_numpy())
    wk, wv = ref.read_lww(want_out)
    wk, wv = wk.cpu().numpy(), wv.cpu().numpy()
    ref.close()
    monkeypatch.setenv("DG_JOIN_WORKERS", "1024")  # over-sized grid: the async join aborts
    eng = Engine(0)
    o = Store.empty(sa.n + sb.n, dev)
    oc = Context.empty(0, ca.n + cb.n, dev)
    d = torch.zeros(8, dtype=torch.int64, device=dev)
    eng.prepare_join2(sa, ca, sb, cb, o, oc, d)()
    o.n = sa.n + sb.n  # unknown until settled: read the count after the read call
    k0, v0 = eng.read_lww(sb)  # a synchronous call of another kind: settles the join first
    o.n = int(d[0].item())
    for x, y in zip(o.to_numpy(), want):
        assert np.array_equal(x, y)
    k, v = eng.read_lww(o)
    assert np.array_equal(k.cpu().numpy(), wk) and np.array_equal(v.cpu().numpy(), wv)
    eng.sync()
    eng.close()
