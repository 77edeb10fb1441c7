"""bench.py — merged dots/s of the AWLWWMap delta join on MI355X (BASELINE.json metric).

A "step" is one AWLWWMap.join/3 (full-state, all keys) of two replicas resident in
HBM — BASELINE config 2 per GPU: 1M keys, ~10 % concurrent-write conflicts,
N_in = 2M rows, N_out ~= 1.1M rows.  At N GPUs (one process per GPU, launched by
torch.distributed.run) every rank joins its own key-hash range shard of an N x 1M-key
key space (weak scaling); there is no collective in the data path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]

Rank 0 prints ONE JSON line.  `value` = Σ input rows over all ranks x K / the max
over ranks of the timed region.  `roofline` prices the join kernel (one launch per
step: rows + context union) by its algorithmic bytes 36·(N_in + N_out) + 12·(|c_a| +
|c_b| + |c_out|) over its average duration from HIP events on the engine stream.
`cpu_baseline` times the C restatement (oracle/deltaref.c) on the same config-2
inputs on all host cores (OpenMP over key shards, oracle/deltaref_mt.c) and on one core,
~6 s each.  A secondary Merkle hash+diff rate (config-4
shape, 1M keys, 1 % differing) is reported under `merkle`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
KEYS_PER_GPU = 1_000_000


def kernel_source_digest():
    """The digest of libdeltagpu's sources (the one the library embeds, dg_build_digest):
    ties a PMC summary to the kernels it measured."""
    from delta_crdt_ex_amd._abi import source_digest
    return source_digest()


def _traffic_from_profiles(n_in, n_out):
    """HBM bytes per launch of the join from the committed PMC summary, if one exists
    for this exact workload and these exact kernel sources (profiles/join2_pmc.json,
    written by tools/pmc_traffic.py); else None."""
    p = os.path.join(ROOT, "profiles", "join2_pmc.json")
    try:
        d = json.load(open(p))
    except Exception:
        return None
    if d.get("rows_in") != n_in or d.get("rows_out") != n_out:
        return None
    if d.get("kernel_sources") != kernel_source_digest():
        return None
    return d.get("hbm_bytes_per_launch")


def _host_threads():
    """The host cores this process may use (the GPU box pins OMP_NUM_THREADS to its
    CPU share; os.cpu_count() there shows the whole machine)."""
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    return len(os.sched_getaffinity(0))


def cpu_baseline(a, b, budget_s=6.0):
    """The C restatement of join/3 on the same config-2 replicas: on all host cores
    (deltaref_mt.c, OpenMP over key shards; the reported value) and on one core."""
    from oracle import ref as R  # the checker / CPU baseline only
    R.lib()
    n_in = len(a["rows"][0]) + len(b["rows"][0])

    def rate(fn):
        reps, t0 = 0, time.perf_counter()
        while True:
            fn()
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget_s or reps >= 2000:
                return n_in * reps / el, reps, el

    threads = _host_threads()
    mt = R.JoinMT(a["rows"], a["ctx"], b["rows"], b["ctx"], threads)
    v_mt, r_mt, e_mt = rate(mt)
    v_1, r_1, e_1 = rate(R.JoinMT(a["rows"], a["ctx"], b["rows"], b["ctx"], 1))
    return {
        "value": v_mt,
        "unit": "merged dots/s",
        "cores": threads,
        "kind": "port",
        "sample": f"C restatement of aw_lww_map.ex join/3 (oracle/deltaref.c + deltaref_mt.c, gcc "
                  f"-O2 -fopenmp, {threads} threads over key-range shards) on the same config-2 "
                  f"replicas ({n_in} rows in), {r_mt} joins in {e_mt:.1f} s",
        "single_core": {"value": v_1, "cores": 1,
                        "sample": f"the same, 1 thread: {r_1} joins in {e_1:.1f} s"},
    }


def _diff_accounting(ta, tb):
    """Algorithmic bytes of a dg_merkle_diff (16 B per node pair visited +
    8 B per differing key, plus what the descent reads to reach the rows: the u16 row
    counts of both trees over every dirty subtree, and 36 B per row of a differing
    bucket).  Node pairs visited: every subtree root, then both children of each
    differing node, level by level (csrc/merkle.hip merkle_diff_count_kernel)."""
    depth = ta.depth
    sub = min(depth, 12)
    Ls = depth - sub
    na = ta.nodes.cpu().numpy().view(np.uint64)
    nb = tb.nodes.cpu().numpy().view(np.uint64)
    lvl = lambda a, l: a[(1 << l) - 1: (1 << (l + 1)) - 1]  # noqa: E731
    differ = lvl(na, Ls) != lvl(nb, Ls)
    dirty = int(differ.sum())
    visited = 1 << Ls
    for l in range(Ls + 1, depth + 1):
        parent = np.repeat(differ, 2)
        visited += 2 * int(differ.sum())
        differ = parent & (lvl(na, l) != lvl(nb, l))
    ca, cb = ta.bucket_counts(), tb.bucket_counts()
    rows = int(ca[differ].astype(np.int64).sum() + cb[differ].astype(np.int64).sum())
    return {"node_pairs_visited": visited, "dirty_subtrees": dirty, "subtrees": 1 << Ls,
            "differing_buckets": int(differ.sum()), "rows_read": rows,
            "bytes_no_keys": 16 * visited + 4 * dirty * (1 << sub) + 36 * rows}


def _join_delta_roofline(last, t_dev):
    """dg_join_delta's algorithmic bytes (§8(d)'s join bytes over the rows it touches: the
    keyset's state rows read, the delta's rows read, the joined rows written, the keyset
    read, and per changed key its bucket's leaf and row count read and written) over the
    call's device time.  Latency-bound: a few searches and hashes per key, one wait."""
    alg = 36 * (last["n_ak"] + last["rows"] + last["n_e"]) + 8 * last["keys"] + 20 * last["changed"]
    return {"bound": "hbm (latency: per-key search chains)", "alg_bytes": alg,
            "device_us": t_dev * 1e6, "achieved": alg / t_dev / 1e9, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": alg / t_dev / 1e9 / HBM_PEAK_GBS,
            "rows": {"state_rows_of_keyset": last["n_ak"], "delta_rows": last["rows"],
                     "joined_rows_of_keyset": last["n_e"], "keys": last["keys"],
                     "changed": last["changed"]}}


def config4_round(eng, torch, dev, rank=0, world=1, keys_per_rank=12_500_000, steps=10,
                  max_sync_size=None, cdev=None):
    """BASELINE config 4 on this rank's key-hash shard (12.5M keys per GPU: 100M over 8):
    two replicas differing on 1 % of the keys.  Measures
      * build: dg_merkle_build_async of both replicas' shard trees (MerkleMap over every
        key, rows hashed through their node TERMS: dg_term_hashes), HIP events on the
        engine stream around `steps` builds -> the roofline of the one-launch build
        (36 B/row read, the node heap written once: 16 B per bucket, the u16 row counts);
      * the anti-entropy round as CausalCrdt runs it (causal_crdt.ex:91-123,324-335,
        383-394), each a synchronous call: Merkle diff (keys, truncated to
        max_sync_size), the sync delta Map.take(B.value, keys) (dg_take_keys), the
        keyed join with its changed keys (dg_join2_changes), and the MerkleMap
        put/delete + update_hashes of those keys (dg_merkle_update, incremental);
        the diff's roofline from its algorithmic bytes (_diff_accounting);
      * at world > 1: the shard roots all-gathered and folded (== the unsharded root)
        and the VV all-reduce(max) on the device context, over RCCL.
    Returns the rank's dict and the (keys, seconds) its aggregate needs."""
    from delta_crdt_ex_amd import sharding as S
    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Context, MerkleTree, Store, TermHashes
    a, b = W.config4_shard(rank, max(world, 1), keys_per_rank=keys_per_rank, diff_frac=0.01)
    N = a["nodes"]
    terms = TermHashes(*N.universe.term_tables(), dev)  # node term hashes of the replicas
    sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
    ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
    sbits = S.shard_bits(world) if world > 1 else 0
    n_keys = len(a["rows"][0])
    depth = max(8, min(28, int(np.ceil(np.log2(max(n_keys, 2) / 3)))))  # ~3 keys per bucket
    ta = MerkleTree.empty(depth, dev, sbits, rank if sbits else 0, terms)
    tb = MerkleTree.empty(depth, dev, sbits, rank if sbits else 0, terms)
    dk = torch.zeros(8, dtype=torch.int64, device=dev)
    la, lb = eng.prepare_merkle_build(sa, ta, dk[0:1]), eng.prepare_merkle_build(sb, tb, dk[1:2])
    la(), lb()
    eng.sync()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(eng.stream)
    for _ in range(steps):
        la()
        lb()
    ev1.record(eng.stream)
    eng.sync()
    build_us = ev0.elapsed_time(ev1) * 1e3 / (2 * steps)
    rows = (sa.n + sb.n) / 2
    nb = 1 << depth
    build_alg = 36 * rows + 16 * nb + 2 * nb
    eng.merkle_build(sa, depth, ta, sbits, rank if sbits else 0)  # n_keys, shard check
    eng.merkle_build(sb, depth, tb, sbits, rank if sbits else 0)
    cap = max_sync_size or (ta.n_keys + tb.n_keys)
    # the diff's kernels alone: `steps` asynchronous diffs back to back, HIP events on the
    # engine stream (as the builds above); the synchronous call is timed in the rounds
    d_keys = torch.empty(max(int(cap), 1), dtype=torch.int64, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    ld = eng.prepare_merkle_diff(ta, tb, d_keys, cap, d_tot)
    ld()
    eng.sync()
    ev0.record(eng.stream)
    for _ in range(steps):
        ld()
    ev1.record(eng.stream)
    eng.sync()
    diff_us = ev0.elapsed_time(ev1) * 1e3 / steps

    # the round as CausalCrdt runs it on the receiving replica: update_state_with_delta
    # REPLACES A's state (causal_crdt.ex:383-404), so the keyed join is applied in place
    # (dg_join_delta, with its MerkleMap update); A's state and tree are restored from a
    # pristine copy before each round, outside the clock
    st = Store.empty(sa.n + sb.n, dev)
    spare = Store.empty(sa.n + sb.n, dev)
    sc = Context.empty(ca.kind, ca.n + cb.n, dev)

    def one_round():
        t = {}
        for f in ("key", "val", "ts", "node", "cnt"):
            getattr(st, f)[: sa.n].copy_(getattr(sa, f)[: sa.n])
        st.n = sa.n
        sc.node[: ca.n].copy_(ca.node[: ca.n])
        sc.cnt[: ca.n].copy_(ca.cnt[: ca.n])
        sc.n, sc.kind = ca.n, ca.kind
        tt = ta.clone()
        tt.store = st
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # the calls run on the engine's own stream (as a caller that issues its work there:
        # no cross-stream ordering per call); each is synchronous -- it returns once its
        # results are on the host -- so the wall clock stops at its return
        with torch.cuda.stream(eng.stream):
            t0 = time.perf_counter()
            e0.record(eng.stream)
            keys, total = eng.merkle_diff(ta, tb, cap=cap, with_total=True)
            e1.record(eng.stream)
            t1 = time.perf_counter()
            delta = eng.take_keys(sb, keys)
            t2 = time.perf_counter()
            e2.record(eng.stream)
            changed, swapped = eng.join_delta(st, sc, delta, cb, keys, spare, tt)
            t3 = time.perf_counter()
            e3.record(eng.stream)
        torch.cuda.synchronize()
        t.update(diff=t1 - t0, take=t2 - t1, join_delta=t3 - t2, total=t3 - t0,
                 join_delta_ev=e2.elapsed_time(e3) * 1e-3,
                 diff_ev=e0.elapsed_time(e1) * 1e-3, keys=int(keys.numel()), total_keys=total,
                 rows=delta.n, changed=int(changed.numel()), in_place=not swapped)
        t["ok"] = tt.root() == eng.merkle_build(st, depth, None, sbits, rank if sbits else 0,
                                                terms=terms).root()
        # (outside the clock) the keyset's rows before and after: the join's row bytes
        t["n_ak"] = int(torch.isin(sa.key[: sa.n], keys).sum())
        t["n_e"] = int(torch.isin(st.key[: st.n], keys).sum())
        return t

    one_round()
    rounds = [one_round() for _ in range(5)]

    def c_abi_join_delta(reps=5):
        """dg_join_delta as the NIF calls it: the C-ABI call alone (its arguments built
        beforehand), from the round's state, delta and keys, A restored outside the clock."""
        import ctypes as C
        from delta_crdt_ex_amd import _abi
        from delta_crdt_ex_amd.store import _ptr, check
        keys = eng.merkle_diff(ta, tb, cap=cap)
        delta = eng.take_keys(sb, keys)
        chg = torch.empty(max(int(keys.numel()), 1), dtype=torch.int64, device=dev)
        out = []
        for _ in range(reps + 1):
            for f in ("key", "val", "ts", "node", "cnt"):
                getattr(st, f)[: sa.n].copy_(getattr(sa, f)[: sa.n])
            st.n = sa.n
            sc.node[: ca.n].copy_(ca.node[: ca.n])
            sc.cnt[: ca.n].copy_(ca.cnt[: ca.n])
            sc.n, sc.kind = ca.n, ca.kind
            tt = ta.clone()
            tt.store = st
            ss, scc, sd, cd, sp, tr = st.abi(), sc.abi(), delta.abi(), cb.abi(), spare.abi(), tt.abi()
            kp, nk = eng._keys(keys)
            nn, sw = C.c_uint64(0), C.c_int(0)
            args = (eng.h, C.byref(ss), C.byref(scc), C.byref(sd), C.byref(cd), kp, nk, C.byref(sp),
                    C.byref(tr), _ptr(chg, _abi.P64), int(chg.numel()), C.byref(nn), C.byref(sw))
            fn = eng.lib.dg_join_delta
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc = fn(*args)
            out.append(time.perf_counter() - t0)
            check(rc)
            torch.cuda.synchronize()
        return float(np.median(out[1:])) * 1e6

    join_delta_c_us = c_abi_join_delta()

    def c_abi_diff(reps=7):
        """dg_merkle_diff as the NIF calls it: the synchronous C-ABI call alone (arguments and
        the output buffer built beforehand), median of reps."""
        import ctypes as C
        from delta_crdt_ex_amd import _abi
        from delta_crdt_ex_amd.store import _ptr, check
        out_k = torch.empty(max(int(cap), 1), dtype=torch.int64, device=dev)
        xa, xb, ya, yb = ta.abi(), tb.abi(), ta.store.abi(), tb.store.abi()
        n_o, n_t = C.c_uint64(), C.c_uint64()
        args = (eng.h, C.byref(xa), C.byref(ya), C.byref(xb), C.byref(yb), _ptr(out_k, _abi.P64), int(cap),
                C.byref(n_o), C.byref(n_t))
        fn = eng.lib.dg_merkle_diff
        out = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc = fn(*args)
            out.append(time.perf_counter() - t0)
            check(rc)
        return float(np.median(out[1:])) * 1e6

    diff_c_us = c_abi_diff()
    resident = resident_delta(eng, torch, sa, ca, cb, ta, tb, b)
    partial = {"max_sync_size_200": partial_round(eng, torch, ta, tb, max_sync_size=200),
               "infinite": partial_round(eng, torch, ta, tb, max_sync_size=None, reps=3),
               "note": "prepare on A, continue on B, A, B, A ...: the message exchange of "
                       "causal_crdt.ex:91-110,252-270 with both replicas on this GPU (between "
                       "BEAM nodes each hop is one message); synchronous calls, wall time"}
    med = {k: float(np.median([r[k] for r in rounds]))
           for k in ("diff", "take", "join_delta", "total", "diff_ev", "join_delta_ev")}
    last = rounds[-1]
    acc = _diff_accounting(ta, tb)
    diff_alg = acc["bytes_no_keys"] + 8 * last["total_keys"]
    res = {
        "metric": "Merkle diff keys/s, config 4 (key-hash shard of 100M keys, 1 % differing)",
        "keys_per_gpu": n_keys, "depth": depth, "shard_bits": sbits,
        "value": 2 * n_keys / (2 * build_us * 1e-6 + med["diff"]), "unit": "keys/s",
        "note": "value = keys of both replicas / (hash both: two full builds + the diff)",
        "build_us": build_us,
        "roofline": {"bound": "hbm", "kernel": "merkle_chunk_kernel<BUILD> (one launch)",
                     "alg_bytes_per_launch": build_alg, "avg_launch_us": build_us,
                     "achieved": build_alg / (build_us * 1e-6) / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s",
                     "frac": build_alg / (build_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                     "launch_timing": "HIP events on the engine stream around the async builds"},
        "diff_roofline": {"bound": "hbm",
                          "kernel": "merkle_diff_count (subtree bounds + descent) + merkle_diff_write",
                          "alg_bytes_per_launch": diff_alg, "avg_launch_us": diff_us,
                          "achieved": diff_alg / (diff_us * 1e-6) / 1e9, "peak": HBM_PEAK_GBS,
                          "unit": "GB/s", "frac": diff_alg / (diff_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                          "sync_call_us": med["diff_ev"] * 1e6,
                          **acc,
                          "launch_timing": f"HIP events on the engine stream around {steps} "
                                           "back-to-back dg_merkle_diff_async launches (the "
                                           "scratch zeroing, count and write kernels); "
                                           "sync_call_us: one synchronous dg_merkle_diff with "
                                           "its count publish and host wait, median of 5 "
                                           "rounds"},
        "round_us": {k: v * 1e6 for k, v in med.items() if k not in ("diff_ev", "join_delta_ev")},
        "join_delta_device_us": med["join_delta_ev"] * 1e6,
        "join_delta_roofline": _join_delta_roofline(last, med["join_delta_ev"]),
        "join_delta_c_abi_us": join_delta_c_us,
        "diff_c_abi_us": diff_c_us,
        "diff_c_abi_note": "the synchronous dg_merkle_diff C-ABI call alone (count, write and "
                           "publish kernels, one host wait; arguments built beforehand, as the "
                           "NIF makes it), median of 7; round_us.diff is the Python call",
        "join_delta_note": "round_us.*: wall time of each synchronous Python call on the engine's "
                           "stream, to its return (the results on the host: its one host wait "
                           "included); join_delta_device_us: HIP events on the engine stream "
                           "around the same call (the host's launch work included); "
                           "join_delta_c_abi_us: the dg_join_delta C-ABI call alone, arguments "
                           "built beforehand, as the NIF makes it (median of 5)",
        "round_keys": last["keys"], "round_total_keys": last["total_keys"],
        "round_delta_rows": last["rows"], "round_changed_keys": last["changed"],
        "update_equals_rebuild": all(r["ok"] for r in rounds),
        "round_in_place": all(r["in_place"] for r in rounds),
        "resident_delta": resident,
        "partial": partial,
        "round_note": "synchronous calls: merkle_diff -> take_keys (the sync delta from B) -> "
                      "join_delta (update_state_with_delta on A: the keyed join in place, its "
                      "changed keys, the MerkleMap put/delete + update_hashes)",
    }
    if world > 1:
        # the round's collectives: the shard roots' all-gather + fold and the VV all-reduce.
        # The first call pays communicator setup (reported apart); then the median of 20.
        def coll():
            t0 = time.perf_counter()
            r = S.merkle_roots(ta.root())
            S.vv_allreduce_max_context(ca, len(N.dense))
            torch.cuda.synchronize()
            return r, (time.perf_counter() - t0) * 1e6
        (roots_a, root_a), cold = coll()
        warm = sorted(coll()[1] for _ in range(20))
        res["collectives_us"] = warm[len(warm) // 2]
        res["collectives_cold_us"] = cold
        res["collectives_note"] = ("merkle_roots (all-gather of one u64 per rank + fold) + "
                                   "vv_allreduce_max_context (all-reduce MAX of the dense VV); "
                                   "median of 20 after one warm-up call")
        res["replica_root"] = hex(root_a)
    return res, (2 * n_keys, 2 * build_us * 1e-6 + med["diff"])


def partial_round(eng, torch, ta, tb, levels=8, max_sync_size=200, reps=5):
    """CausalCrdt's anti-entropy message exchange as the reference runs it between two
    replicas that never hold each other's tree (causal_crdt.ex:91-110,252-270): the
    originator's prepare_partial_diff(mm, 8), then continue_partial_diff(cont, mm, 8)
    ping-pong, every {:continue, c} truncated to max_sync_size (default 200,
    delta_crdt.ex:32) before it is sent, until {:ok, keys} (truncated too, :105).  Per hop:
    wall time of the synchronous calls (continue + truncate) and the message the hop sends
    -- node form 16 B per entry (position, hash), leaf form 8 B per bucket + 16 B per
    (key, leaf) pair; keys 8 B each.  Median over reps."""
    hops_all = []
    for _ in range(reps + 1):
        hops = []
        t0 = time.perf_counter()
        cont = eng.merkle_prepare(ta, levels)
        hops.append({"call": "prepare", "us": (time.perf_counter() - t0) * 1e6, "level": cont.level,
                     "entries": cont.n, "bytes": 16 * cont.n})
        side = (tb, ta)
        i = 0
        while True:
            t = side[i % 2]
            t0 = time.perf_counter()
            res = eng.merkle_continue(t, cont, levels)
            if res[0] == "ok":
                keys = res[1][:max_sync_size] if max_sync_size else res[1]
                torch.cuda.synchronize()
                hops.append({"call": "continue -> ok", "us": (time.perf_counter() - t0) * 1e6,
                             "keys": int(keys.numel()), "total_keys": int(res[2]),
                             "bytes": 8 * int(keys.numel())})
                break
            cont = res[1]
            if max_sync_size:
                eng.merkle_truncate(t, cont, max_sync_size)
            el = (time.perf_counter() - t0) * 1e6
            h = {"call": "continue", "us": el, "level": cont.level, "entries": cont.n}
            if cont.leaf:
                h.update(buckets=cont.n_buckets, bytes=8 * cont.n_buckets + 16 * cont.n)
            else:
                h["bytes"] = 16 * cont.n
            hops.append(h)
            i += 1
        hops_all.append(hops)
    hops_all = hops_all[1:]
    out = []
    for j, h in enumerate(hops_all[0]):
        h = dict(h)
        h["us"] = float(np.median([hs[j]["us"] for hs in hops_all]))
        out.append(h)
    return {"max_sync_size": max_sync_size if max_sync_size else "infinite", "levels": levels,
            "hops": out, "total_us": sum(h["us"] for h in out),
            "total_bytes": sum(h["bytes"] for h in out)}


def resident_delta(eng, torch, sa, ca, cb, ta, tb, b, reps=7):
    """What a NIF caller pays per sync delta against a device-resident state
    (join_delta; the reference's update_state_with_delta,
    causal_crdt.ex:383-404), at wall time on the config-4 shard: H2D of the delta's rows
    and keyset from pinned host memory, dg_join_delta (the keyed join applied in place --
    every differing key keeps its one row -- its changed keys and the MerkleMap update),
    and D2H of the changed keys and their rows (returned by dg_join_delta_rows) for the
    on_diffs callback.
    The state is restored from a pristine copy before each rep (outside the clock)."""
    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Context, Store
    dev = sa.key.device
    keys_np = eng.merkle_diff(ta, tb).cpu().numpy().view(np.uint64)  # the differing keys
    d = W.sync_delta(b, keys_np)
    n, nk = len(d["rows"][0]), len(keys_np)
    # the delta as ONE pinned message (key | val | ts | cnt | keyset | node), one H2D copy;
    # the device store's columns are views into the landed buffer
    words = 4 * n + nk + (n + 1) // 2
    msg = torch.empty(words, dtype=torch.int64).pin_memory()
    m = msg.numpy()
    k_, v_, t_, nd_, c_ = d["rows"]
    for i, col in enumerate((k_, v_, t_, c_)):
        m[i * n:(i + 1) * n] = col.view(np.int64)
    m[4 * n:4 * n + nk] = keys_np.view(np.int64)
    m[4 * n + nk:].view(np.int32)[:n] = nd_.view(np.int32)
    dbuf = torch.empty(words, dtype=torch.int64, device=dev)
    dst = Store(dbuf[0:n], dbuf[n:2 * n], dbuf[2 * n:3 * n],
                dbuf[4 * n + nk:].view(torch.int32)[:n], dbuf[3 * n:4 * n], n)
    kd = dbuf[4 * n:4 * n + nk]
    # the changed keys' rows come back the same way: one device buffer, one D2H copy
    rcap = max(nk, 1)  # the changed keys and their rows (one per key here)
    rhost = torch.empty(5 * rcap + rcap, dtype=torch.int64).pin_memory()
    st = Store.empty(sa.n + n, dev)
    spare = Store.empty(sa.n + n, dev)
    sc = Context.empty(ca.kind, ca.n + cb.n, dev)
    # (rows: key | val | ts | cnt | node, then the changed keys)
    cbuf = torch.empty(5 * rcap + rcap, dtype=torch.int64, device=dev)
    rst = Store(cbuf[0:rcap], cbuf[rcap:2 * rcap], cbuf[2 * rcap:3 * rcap],
                cbuf[4 * rcap:5 * rcap].view(torch.int32)[:rcap], cbuf[3 * rcap:4 * rcap], 0)
    changed = cbuf[5 * rcap:]
    ph = {}
    swaps = 0
    for it in range(reps + 1):
        for f in ("key", "val", "ts", "node", "cnt"):
            getattr(st, f)[: sa.n].copy_(getattr(sa, f)[: sa.n])
        st.n = sa.n
        sc.node[: ca.n].copy_(ca.node[: ca.n])
        sc.cnt[: ca.n].copy_(ca.cnt[: ca.n])
        sc.n, sc.kind = ca.n, ca.kind
        tt = ta.clone()
        tt.store = st
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dbuf.copy_(msg, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        # dg_join_delta_rows: the changed keys' joined rows come back from the join's own
        # edit of the keyset (no dg_take_keys search of the 12.5M-row state afterwards)
        ch, sw = eng.join_delta(st, sc, dst, cb, kd, spare, tt, changed=changed, rows=rst)
        t2 = time.perf_counter()
        nr, nch = rst.n, int(ch.numel())
        rhost.copy_(cbuf, non_blocking=True)  # rows and changed keys: one D2H copy
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        swaps += int(sw)
        if it:
            for k, v in (("h2d", t1 - t0), ("join_delta", t2 - t1), ("d2h_changed_rows", t3 - t2),
                         ("total", t3 - t0)):
                ph.setdefault(k, []).append(v)
    med = {k: float(np.median(v)) * 1e6 for k, v in ph.items()}
    return {"metric": "sync delta applied to a device-resident state (config-4 shard), wall time",
            "us": med, "delta_rows": n, "keyset": int(len(keys_np)), "changed_keys": nch,
            "rows_back": int(nr), "state_rows": sa.n, "in_place": swaps == 0,
            "bytes_h2d": 8 * words, "bytes_d2h": 8 * (5 * rcap + rcap),
            "deltas_per_s": 1e6 / med["total"],
            "note": "synchronous calls; the delta travels as one pinned message (one H2D copy) "
                    "and the changed keys with their rows as one D2H copy; median of reps; join_delta = "
                    "dg_join_delta_rows: the state's rows of the keyset taken, joined with the delta, "
                    "written back in place (csrc/splice.hip), changed keys, MerkleMap update, the "
                    "changed keys' rows gathered from the join's edit"}


def _timed(torch, fn, reps):
    """Median wall time of `reps` synchronous calls (each call ends in a host sync)."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def config3_rate(eng, torch, dev, rank=0, world=1, n_keys=10_000_000, reps=3):
    """Config 3: 64 sync-shaped deltas (1 % of the keys each, 80 % adds / 20 % removes)
    applied to a 10M-key state with dg_apply_deltas (the fold of join/3 with each
    delta's keys; one pass over the state, csrc/kfold.hip).  At N ranks the state and
    every delta are split by key hash (strong scaling: each rank folds its shard).  Rate
    = (state rows + delta rows) / wall time, SURVEY §8(d)'s N_in ≈ 15M; at N = 1 the
    delta-by-delta fold is timed beside it (DG_APPLY_MODE=fold).  The call's device time
    comes from HIP events around back-to-back prepared calls."""
    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Context, Engine, Store
    base, deltas = W.config3_shard(rank, world, n_keys=n_keys)
    sb = Store.from_numpy(*base["rows"], device=dev)
    cb = Context.from_numpy(*base["ctx"], dev)
    ds = [Store.from_numpy(*d["rows"], device=dev) for d in deltas]
    dc = [Context.from_numpy(*d["ctx"], dev) for d in deltas]
    ks = [torch.from_numpy(d["keys"].view(np.int64)).to(dev) for d in deltas]
    out = Store.empty(sb.n + sum(d.n for d in ds), dev)
    octx = Context.empty(0, cb.n + sum(c.n for c in dc), dev)
    res = {}

    def run(e):
        o, c = e.apply_deltas(sb, cb, ds, dc, ks, out=out, out_ctx=octx)
        res["n"] = o.n

    call = eng.prepare_apply_deltas(sb, cb, ds, dc, ks, out, octx)  # marshalled once
    el = _timed(torch, call, reps)
    res["n"] = out.n
    # the call's device time: events around back-to-back calls (each ends in a host sync,
    # so this includes the synchronous call's gaps; rocprofv3 gives the kernels alone)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(eng.stream)
    for _ in range(reps):
        call()
    ev1.record(eng.stream)
    torch.cuda.synchronize()
    el_ev = ev0.elapsed_time(ev1) * 1e-3 / reps
    el_fold = None
    if world == 1:
        os.environ["DG_APPLY_MODE"] = "fold"
        try:
            fe = Engine(0)
        finally:
            del os.environ["DG_APPLY_MODE"]
        n_one = res["n"]
        el_fold = _timed(torch, lambda: run(fe), reps)
        fe.close()
        assert res["n"] == n_one
    d_rows = sum(d.n for d in ds)
    n_keys_total = sum(int(k.numel()) for k in ks)
    rows_in = sb.n + d_rows
    alg = 36 * (rows_in + res["n"]) + 8 * n_keys_total
    r = {"metric": "merged dots/s, config 3 (64 keyed sync deltas into a 10M-key state)",
         "value": rows_in / el, "unit": "merged dots/s", "ms_per_batch": el * 1e3,
         "alg_bytes": alg, "alg_GBps": alg / el / 1e9,
         "alg_frac": alg / el / 1e9 / HBM_PEAK_GBS,  # of the HBM peak, over the whole call
         "roofline": {"bound": "hbm", "kernel": "kfold_fill_kernel + kfold_kernel",
                      "alg_bytes_per_launch": alg, "avg_launch_us": el_ev * 1e6,
                      "achieved": alg / el_ev / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": alg / el_ev / 1e9 / HBM_PEAK_GBS,
                      "launch_timing": f"HIP events on the engine stream around {reps} "
                                       "back-to-back prepared dg_apply_deltas calls"},
         "state_rows": sb.n, "delta_rows": d_rows, "keyset_entries": n_keys_total,
         "rows_out": res["n"],
         "note": "dg_apply_deltas, synchronous (one host sync), arguments marshalled once "
                 "(prepare_apply_deltas); stepwise = 64 joins of join/3 back to back"}
    if el_fold is not None:
        r["stepwise_ms_per_batch"] = el_fold * 1e3
    return r, (rows_in, el)


def changes_rate(eng, torch, pr, reps=20):
    """SURVEY §8(f).1 on config 2: dg_join2_changes (the join plus the changed-key diff
    of update_state_with_delta) next to the plain synchronous dg_join2, same inputs."""
    res = {}

    def chg():
        _, _, c = eng.join2_changes(pr["sa"], pr["ca"], pr["sb"], pr["cb"], out=pr["out"],
                                    out_ctx=pr["octx"])
        res["n"] = int(c.numel())

    def plain():
        eng.join2(pr["sa"], pr["ca"], pr["sb"], pr["cb"], out=pr["out"], out_ctx=pr["octx"])

    el_c = _timed(torch, chg, reps)
    el_p = _timed(torch, plain, reps)
    return {"metric": "dg_join2_changes on config 2 (join + changed keys)",
            "us_per_call": el_c * 1e6, "join2_us_per_call": el_p * 1e6,
            "changed_keys": res["n"],
            "note": "synchronous calls (host sync each), median of reps"}


def e2e_rate(eng, torch, pr, reps=20):
    """SURVEY §8(d)'s end-to-end figure on config 2: the two replicas' host SoA columns
    copied to the device (pinned staging, as a NIF holding its marshalled rows would),
    joined, and the joined rows + context copied back -- wall time per call.  Not `value`
    (the bench contract's value is device-resident throughput)."""
    a, b = pr["a"], pr["b"]
    sa, sb, ca, cb, out, octx = pr["sa"], pr["sb"], pr["ca"], pr["cb"], pr["out"], pr["octx"]
    cols = [(np.asarray(x), t) for rows, st in ((a["rows"], sa), (b["rows"], sb))
            for x, t in zip(rows, (st.key, st.val, st.ts, st.node, st.cnt))]
    pinned = [torch.from_numpy(x.view(np.int64 if x.dtype.itemsize == 8 else np.int32)).pin_memory()
              for x, _ in cols]
    back = [torch.empty(t.shape, dtype=t.dtype).pin_memory() for t in (out.key, out.val, out.ts,
                                                                       out.node, out.cnt)]
    n_in = len(a["rows"][0]) + len(b["rows"][0])
    ph = {}

    def call():
        t0 = time.perf_counter()
        for (x, dst), h in zip(cols, pinned):
            dst[: len(x)].copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        eng.join2(sa, ca, sb, cb, out=out, out_ctx=octx)
        t2 = time.perf_counter()
        n = out.n
        for src, h in zip((out.key, out.val, out.ts, out.node, out.cnt), back):
            h[:n].copy_(src[:n], non_blocking=True)
        node, cnt = octx.to_numpy()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        ph.setdefault("h2d", []).append(t1 - t0)
        ph.setdefault("join", []).append(t2 - t1)
        ph.setdefault("d2h", []).append(t3 - t2)

    el = _timed(torch, call, reps)
    med = {k: float(np.median(v)) * 1e3 for k, v in ph.items()}
    return {"metric": "merged dots/s end to end (H2D + join + D2H), config 2",
            "value": n_in / el, "unit": "merged dots/s", "ms_per_call": el * 1e3,
            "ms_h2d": med["h2d"], "ms_join": med["join"], "ms_d2h": med["d2h"],
            "bytes_h2d": 36 * n_in, "bytes_d2h": 36 * out.n,
            "note": "pinned host staging reused across calls; synchronous join; "
                    "median of reps"}


def config5_rate(eng, torch, dev, rank=0, world=1, n_keys=12_500_000, reps=5, steps=20, settle_ms=0.0):
    """Config 5 at one GPU's share of 100M keys over 8 GPUs: full-state join of two
    remove-heavy replicas (50 % removes, 64 nodes, ts in [0,16): LWW ties everywhere),
    then read/1 of the result.  At N ranks each rank joins its key-hash shard of
    N x 12.5M keys (weak scaling: 100M keys at N = 8)."""
    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Context, Store
    a, b = W.config5_shard(rank, world, keys_per_rank=n_keys)
    sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
    ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
    del a, b
    out = Store.empty(sa.n + sb.n, dev)
    octx = Context.empty(0, ca.n + cb.n, dev)
    res = {}
    d_counts = torch.zeros(8, dtype=torch.int64, device=dev)
    launch = eng.prepare_join2(sa, ca, sb, cb, out, octx, d_counts)  # marshalled once

    def join():
        launch()
        eng.sync()

    t_settle = time.perf_counter()  # (optional) untimed joins first: the clocks up
    while (time.perf_counter() - t_settle) * 1e3 < settle_ms:
        for _ in range(8):
            launch()
        eng.sync()
    tj = _timed(torch, join, reps)
    # the kernels alone: `steps` launches back to back, HIP events on the engine stream
    launch()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(eng.stream)
    for _ in range(steps):
        launch()
    ev1.record(eng.stream)
    eng.sync()
    tk = ev0.elapsed_time(ev1) * 1e-3 / steps
    # the per-launch timeline of the same back-to-back loop: an event between every two
    # launches (config 5 reproducible without a profiler in the process)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    evs[0].record(eng.stream)
    for i in range(steps):
        launch()
        evs[i + 1].record(eng.stream)
    eng.sync()
    per_launch = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(steps)]
    out.n = int(d_counts[0].item())
    octx.n = int(d_counts[1].item())

    def read():
        k, _ = eng.read_lww(out)
        res["keys"] = int(k.numel())

    tr = _timed(torch, read, reps)
    n_in = sa.n + sb.n
    alg = 36 * (n_in + out.n)
    r = {"metric": "merged dots/s, config 5 (remove-heavy, LWW ties), 12.5M keys per GPU",
         "value": n_in / tj, "unit": "merged dots/s", "ms_per_join": tj * 1e3,
         "join_alg_GBps": alg / tj / 1e9,
         "roofline": {"bound": "hbm", "kernel": "join2_partition_kernel + join2_stream_kernel",
                      "alg_bytes_per_launch": alg, "avg_launch_us": tk * 1e6,
                      "achieved": alg / tk / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": alg / tk / 1e9 / HBM_PEAK_GBS,
                      "launch_timing": f"HIP events on the engine stream around {steps} "
                                       "back-to-back dg_join2_async launches",
                      "per_launch_us": [round(x, 2) for x in per_launch],
                      "per_launch_median_us": sorted(per_launch)[len(per_launch) // 2],
                      "per_launch_timing": "the same loop again with an event between every "
                                           "two launches (no profiler in the process)"},
         "rows_in": n_in, "rows_out": out.n, "ms_per_read": tr * 1e3,
         "read_rows_per_s": out.n / tr, "read_keys_per_s": res["keys"] / tr,
         "read_keys": res["keys"], "read_alg_GBps": (36 * out.n + 16 * res["keys"]) / tr / 1e9,
         "note": "value / ms_per_join: one dg_join2_async + host sync per join (arguments "
                 "marshalled once); roofline: the launches back to back; dg_read_lww "
                 "synchronous"}
    return r, (n_in, tj)


def read_runs_rate(eng, torch, dev, n_keys=1_000_000, max_entries=32, reps=5):
    """read/1 over key runs of 1..32 entries (uniform; SURVEY H2's reproducible regime
    at its widest), the shape where a per-lane serial walk would diverge: the segmented
    reduction of csrc/segred.hip.  Algorithmic bytes: key column twice (count and write
    passes) + val + ts per row, 16 B per key out."""
    from delta_crdt_ex_amd.store import Store
    rng = np.random.default_rng(32)
    keys = np.unique(rng.integers(0, 2**63, n_keys, dtype=np.uint64))
    lens = rng.integers(1, max_entries + 1, len(keys))
    n = int(lens.sum())
    starts = np.repeat(np.cumsum(lens) - lens, lens)
    rank = np.arange(n, dtype=np.int64) - starts
    rows = (np.repeat(keys, lens),
            (rank.astype(np.uint64) << np.uint64(20)) | rng.integers(0, 1 << 20, n, dtype=np.uint64),
            rng.integers(0, 4, n).astype(np.int64),          # ts ties everywhere
            rng.integers(0, 64, n).astype(np.uint32),
            np.arange(1, n + 1, dtype=np.uint64))
    s = Store.from_numpy(*rows, device=dev)
    res = {}

    def read():
        k, _ = eng.read_lww(s)
        res["keys"] = int(k.numel())

    tr = _timed(torch, read, reps)
    alg = 32 * n + 16 * res["keys"]
    return {"rows": n, "keys": res["keys"], "entries_per_key": f"uniform 1..{max_entries}",
            "ms_per_read": tr * 1e3, "alg_GBps": alg / tr / 1e9,
            "alg_frac": alg / tr / 1e9 / HBM_PEAK_GBS,
            "note": "dg_read_lww synchronous (three launches + one count readback)"}


MUTATE_EXE = os.path.join(ROOT, "c_src", "_build", "bench_mutate")


def _run_json(cmd, timeout=300):
    import subprocess
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"{cmd[0]} failed ({r.returncode}): {r.stderr[-2000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def mutate_rate(sizes=(1000, 10_000), reps=300):
    """The reference's own benchmark shape (bench/basic_operations.exs:25-41): per-op
    latency of read / add / update / remove on replicas of 1k and 10k keys, each mutation
    a one-key delta with a MapSet context joined into the GPU-resident state through the
    NIF's join_delta (c_src/replica.c: dg_join_delta_home -- the keyed join, changed keys,
    MerkleMap path update and the results written into page-locked memory by one kernel, a
    copy launch behind it when rows move, one host wait), timed from C (c_src/bench_mutate.c:
    no Python in the loop -- what a NIF pays).  `batch_us_per_op`: the trace workload (1000
    adds of new keys, :9-23) as ONE delta through the same call."""
    if not os.path.exists(MUTATE_EXE):
        raise RuntimeError(f"{MUTATE_EXE} is missing: built by __graft_entry__.build()")
    out = {"metric": "per-op latency of a local mutation on a GPU-resident replica "
                     "(basic_operations.exs shape), microseconds, median",
           "unit": "us"}
    for n in sizes:
        out[f"keys_{n}"] = _run_json([MUTATE_EXE, str(n), str(reps)])
    return out


HOP_EXE = os.path.join(ROOT, "c_src", "_build", "bench_hop")


def hop_rate(n_keys=12_500_000, depth=22, reps=20):
    """CausalCrdt's anti-entropy exchange (causal_crdt.ex:91-110,252-270) between two
    config-4-shaped replicas (12.5M keys each, 1 % differing, depth 22, 8 levels per
    message, max_sync_size 200) through the NIF's calls (c_src/replica.c:
    dgr_merkle_prepare / dgr_merkle_continue -> dg_merkle_continue_home, one launch and
    one wait per hop), each message copied between the calls as a send would; wall time
    per hop, median (c_src/bench_hop.c)."""
    if not os.path.exists(HOP_EXE):
        raise RuntimeError(f"{HOP_EXE} is missing: built by __graft_entry__.build()")
    out = _run_json([HOP_EXE, str(n_keys), str(depth), str(reps)], timeout=600)
    out["metric"] = "per-message latency of the partial-diff exchange, microseconds, median"
    out["unit"] = "us"
    return out


def mutate_cpu_baseline(sizes=(1000, 10_000), reps=300):
    """The same ops on the C restatement (oracle/deltaref.c ref_join2 + ref_store_diff per
    op on host rows, one thread; c_src/bench_mutate.c built with -DDG_REF)."""
    exe = MUTATE_EXE + "_ref"
    if not os.path.exists(exe):
        return None
    return {f"keys_{n}": _run_json([exe, str(n), str(reps)]) for n in sizes}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed joins for this long before the warm-up steps (clock ramp)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-merkle", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the secondary config-3 / config-5 measurements")
    ap.add_argument("--rotate", type=int, default=4,
                    help="distinct replica pairs joined round-robin (defeats cache residency)")
    ap.add_argument("--calibrate", action="store_true",
                    help="after timing, run dg_store_check once over every input store: a "
                         "read of exactly the key column (8 B/row on config-2 stores) that "
                         "tools/pmc_traffic.py uses to calibrate FETCH_SIZE for 8-B/lane loads")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Context, Engine, Store

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    # rehearsal of the N > 1 path on a one-GPU box: DG_BENCH_BACKEND=gloo and
    # DG_BENCH_SAME_GPU=1 put every rank on cuda:0 (RCCL refuses two ranks on one GPU)
    backend = os.environ.get("DG_BENCH_BACKEND", "nccl")
    if os.environ.get("DG_BENCH_SAME_GPU") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    # `--rotate R` distinct replica pairs (different seeds), joined round-robin: R x 112 MB
    # of inputs+outputs exceeds the 256 MB Infinity Cache, so every step streams its
    # inputs from HBM instead of re-reading the previous step's cache-resident copy.
    eng = Engine(local)
    stream = eng.stream
    pairs = []
    for r in range(args.rotate):
        a, b = W.config2_shard(rank, world, KEYS_PER_GPU, seed=2 + r)
        sa = Store.from_numpy(*a["rows"], device=dev)
        sb = Store.from_numpy(*b["rows"], device=dev)
        ca = Context.from_numpy(*a["ctx"], dev)
        cb = Context.from_numpy(*b["ctx"], dev)
        out = Store.empty(sa.n + sb.n, dev)
        octx = Context.empty(0, ca.n + cb.n, dev)
        d_counts = torch.zeros(8, dtype=torch.int64, device=dev)
        pairs.append(dict(a=a, b=b, sa=sa, sb=sb, ca=ca, cb=cb, out=out, octx=octx, d=d_counts,
                          launch=eng.prepare_join2(sa, ca, sb, cb, out, octx, d_counts)))
    torch.cuda.synchronize()
    launches = [pr["launch"] for pr in pairs]
    R = len(launches)
    a, b, ca, cb = pairs[0]["a"], pairs[0]["b"], pairs[0]["ca"], pairs[0]["cb"]
    n_in = len(a["rows"][0]) + len(b["rows"][0])
    n_in_all = [len(pr["a"]["rows"][0]) + len(pr["b"]["rows"][0]) for pr in pairs]

    # settle: untimed joins of the same pairs for --settle-ms of wall time before the W
    # warm-up steps, so that a short run (the driver's --steps 20 --warmup 5) times the
    # GPU at its steady clocks rather than the ramp out of idle
    t_settle = time.perf_counter()
    n_settle = 0
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        for i in range(16):
            launches[i % R]()
        eng.sync()
        n_settle += 16
    for i in range(args.warmup):
        launches[i % R]()
    eng.sync()
    n_out = int(pairs[0]["d"][0].item())
    n_ctx_out = int(pairs[0]["d"][1].item())

    # timed region: K back-to-back joins, barrier + sync on both sides
    if world > 1:
        dist.barrier()
    # HIP events on the engine stream bracket the timed region: the average launch
    # duration of the join (its kernels plus the gaps between back-to-back launches)
    # (ev0 goes in behind the FIRST timed step: it fires when that join ends, so the events
    # time steps 2..K back to back on the GPU and not the host's latency to submit step 1
    # into an idle stream; the wall clock below times all K)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.steps > 1:
        launches[0]()
    ev0.record(stream)
    for i in range(1 if args.steps > 1 else 0, args.steps):
        launches[i % R]()
    ev1.record(stream)
    host_submit_s = time.perf_counter() - t0
    eng.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ev_steps = args.steps - 1 if args.steps > 1 else 1
    avg_launch_s = ev0.elapsed_time(ev1) / 1e3 / ev_steps
    if world > 1:
        dist.barrier()

    # per-step event pairs in a separate pass (each pair adds its own record latency, so
    # this median is an upper bound; reported for reference)
    nev = min(args.steps, 100)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(nev + 1)]
    with torch.cuda.stream(stream):
        for i in range(nev):
            ev[i].record(stream)
            launches[i % R]()
        ev[nev].record(stream)
    eng.sync()
    torch.cuda.synchronize()
    step_event_median_us = float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(nev)])) * 1e3

    calib_rows = 0
    if args.calibrate:
        for pr in pairs:
            for st_ in (pr["sa"], pr["sb"]):
                eng.store_check(st_)
                calib_rows += st_.n
        eng.sync()

    rows_done = sum(n_in_all[i % R] for i in range(args.steps))  # input rows merged by K steps
    cdev = dev if backend == "nccl" else torch.device("cpu")  # the collectives' device
    el_t = torch.tensor([el], dtype=torch.float64, device=cdev)
    tot = torch.tensor([float(rows_done)], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    el_max = float(el_t.item())
    total_rows = float(tot.item())

    if rank == 0:
        alg_bytes = 36 * (n_in + n_out) + 12 * (ca.n + cb.n + n_ctx_out)
        achieved = alg_bytes / avg_launch_s / 1e9
        traffic = _traffic_from_profiles(n_in, n_out)
        res = {
            "metric": "merged dots/sec for AWLWWMap delta join + Merkle diff keys/sec at 1\u20138 GPUs",
            "value": total_rows / el_max,
            "unit": "merged dots/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "lib_digest": eng.lib.dg_build_digest().decode(),
            "data": "synthetic (seeded config-2 replicas, SURVEY.md §8(d))",
            "config": {
                "workload": "config2: 1M-key AWLWWMap full-state join of two replicas, 10% "
                            "concurrent-write conflicts, per GPU (key-hash range shards)",
                "keys_per_gpu": KEYS_PER_GPU,
                "rows_in_per_gpu": n_in,
                "rows_out_per_gpu": n_out,
                "parallelism": f"key-hash shards x{world}",
                "rotate": R,
            },
            **({"calib_rows": calib_rows} if args.calibrate else {}),
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "join2_stream_kernel (splits searched in-kernel at this size; joins "
                          "over 4 tiles per workgroup add a join2_partition_kernel launch, "
                          "and the events bracket both)",
                "alg_bytes_per_launch": alg_bytes,
                "avg_launch_us": avg_launch_s * 1e6,
                "launch_timing": "HIP events on the engine stream from the end of the timed "
                                 "region's first step to the end of its last, / (steps - 1)",
                "host_submit_us_per_step": host_submit_s / args.steps * 1e6,
                "per_step_event_median_us": step_event_median_us,
                "settle": {"ms": args.settle_ms, "joins": n_settle,
                           "note": "untimed joins before the warm-up steps"},
            },
        }
    def aggregate(r, units_secs):
        """Σ over ranks of the units, max over ranks of the time: the whole-job figure."""
        units, secs = units_secs
        if world > 1:
            u = torch.tensor([float(units)], dtype=torch.float64, device=cdev)
            t = torch.tensor([float(secs)], dtype=torch.float64, device=cdev)
            dist.all_reduce(u, op=dist.ReduceOp.SUM)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            units, secs = float(u.item()), float(t.item())
        r["aggregate"] = {"ranks": world, "value": units / secs, "units": units,
                          "max_rank_seconds": secs,
                          "note": "Σ units over ranks / max time over ranks (rank 0's own "
                                  "figures above)"}
        return r

    secondaries = {}
    if not args.no_merkle:  # every rank runs its shard's round
        secondaries["merkle"] = aggregate(*config4_round(eng, torch, dev, rank, world, cdev=cdev))
    if not args.no_configs:
        if world == 1:  # per-GPU secondaries of the config-2 pair: measured at N = 1
            secondaries["changes"] = changes_rate(eng, torch, pairs[0])
            secondaries["end_to_end"] = e2e_rate(eng, torch, pairs[0])
        for r in pairs:  # free the config-2 replicas before the larger configs
            r.clear()
        torch.cuda.empty_cache()
        secondaries["config3"] = aggregate(*config3_rate(eng, torch, dev, rank, world))
        torch.cuda.empty_cache()
        secondaries["config5"] = aggregate(*config5_rate(eng, torch, dev, rank, world))
        if world == 1:
            secondaries["read_runs32"] = read_runs_rate(eng, torch, dev)
            secondaries["mutate"] = mutate_rate()
            secondaries["anti_entropy_hops"] = hop_rate()
    if rank == 0:
        res.update(secondaries)
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(a, b)
            if not args.no_configs:
                res["cpu_baseline"]["mutate"] = mutate_cpu_baseline()
        elif not args.no_cpu_baseline:
            res["cpu_baseline"] = None
        import resource
        res["host_peak_rss_gb"] = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20  # (KiB)
        print(json.dumps(res), flush=True)
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
