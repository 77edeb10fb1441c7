import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.store import Engine
from test_gpu_configs import up, keys_dev
eng = Engine(0)
def fold_apply(n, seed):
    base, deltas = W.config3(n_keys=n, n_replicas=64, touch=0.01, seed=seed)
    sb, cb = up(base)
    ds, dc = zip(*[up(d) for d in deltas])
    ks = [keys_dev(d["keys"]) for d in deltas]
    out, octx = eng.apply_deltas(sb, cb, list(ds), list(dc), ks)
    return out.n, out.to_numpy()
def loop_join(n, seed):
    base, deltas = W.config3(n_keys=n, n_replicas=64, touch=0.01, seed=seed)
    cur, curc = up(base)
    for i, d in enumerate(deltas):
        sd, cd = up(d)
        cur, curc = eng.join2(cur, curc, sd, cd, keys=keys_dev(d["keys"]))
        if n > 100000: print("loop step", i, cur.n, file=sys.stderr)
    return cur.n, cur.to_numpy()
mode = sys.argv[1]
if mode.startswith("small_first"):
    print("small", fold_apply(3000, 1)[0])
if mode == "small_first_loop":
    n2, r2 = loop_join(2_000_000, 7)
    n1, r1 = fold_apply(2_000_000, 7)
else:
    n1, r1 = fold_apply(2_000_000, 7)
    n2, r2 = loop_join(2_000_000, 7)
n3, r3 = fold_apply(2_000_000, 7)
print(mode, "fold", n1, "loop", n2, "fold again", n3, "eq12", n1 == n2 and all(np.array_equal(a, b) for a, b in zip(r1, r2)),
      "eq23", n3 == n2 and all(np.array_equal(a, b) for a, b in zip(r3, r2)), flush=True)
if mode == "small_first" and n1 != n2:
    m = min(n1, n2)
    for c in range(5):
        bad = np.flatnonzero(r1[c][:m] != r2[c][:m])
        if len(bad):
            i = bad[0]
            print("col", c, "first diff", i, "of", m, "n1", n1, "n2", n2)
            print(" fold keys", r1[0][i-2:i+4])
            print(" loop keys", r2[0][i-2:i+4])
            # is the fold output a shifted copy of the loop output near i?
            j = np.searchsorted(r2[0], r1[0][i])
            print(" fold row i key found in loop at", j)
            break
    k = r1[0]
    uns = np.flatnonzero(k[1:] < k[:-1])
    print("unsorted positions", uns[:10], len(uns))
