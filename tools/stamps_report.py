"""Phase shares of the join stream kernel from a saved DG_STAMPS buffer (tools/prof_c5.py
with C5_STAMPS=<file.npy>).  Stamps (s_memrealtime, 100 MHz, lane 0 of each tile):
0 iteration start (a workgroup's first tile: the workgroup's entry), 1 iteration start, 2 tile committed to LDS, 7 next tile's loads issued, 3 merge done, 4 block scan + compaction
list (+ change events) done, 5 previous stripe's counts summed, 6 previous tile written.  Only shares
are meaningful (the stamps add barriers)."""
import sys

import numpy as np


def main(path):
    st = np.load(path).reshape(65536, 16).astype(np.int64)
    ntiles = int(np.nonzero(st[:, 0])[0].max()) + 1
    st = st[:ntiles]
    t0 = st[:, 0].min()
    names = ["commit", "issue", "merge", "scan", "sums", "write"]
    st[st[:, 5] == 0, 5] = st[st[:, 5] == 0, 4]  # first iteration: no previous tile
    d = np.diff(st[:, [1, 2, 7, 3, 4, 5, 6]], axis=1) * 10 / 1000.0
    print(f"tiles={ntiles} span={(st[:, 6].max() - t0) * 10 / 1000:.1f} us")
    for i, nm in enumerate(names):
        print(f"{nm:11s} median {np.median(d[:, i]):6.2f} us  p90 {np.percentile(d[:, i], 90):6.2f}"
              f"  mean {d[:, i].mean():6.2f}")
    it = np.diff(np.sort(st[:, 1]))
    print("per-tile total median", np.median((st[:, 6] - st[:, 1]) * 10 / 1000))
    first = st[:, 8] > 0  # a workgroup's first tile: slot 0 is its entry, 8 and 9 prologue stamps
    if first.any():
        pro = (st[first, 1] - st[first, 0]) * 10 / 1000
        ent = (st[first, 0] - st[first, 0].min()) * 10 / 1000
        for a, b, nm in ((0, 8, "split search"), (8, 9, "first tile issued"), (9, 1, "VV tables + tile landed")):
            x = (st[first, b] - st[first, a]) * 10 / 1000
            print(f"  prologue {nm:24s} median {np.median(x):5.2f} us  p90 {np.percentile(x, 90):5.2f}")
        print(f"prologue (entry -> first iteration) median {np.median(pro):.2f} us  p90 "
              f"{np.percentile(pro, 90):.2f}; entries spread over {ent.max():.2f} us; "
              f"last write {(st[:, 6].max() - st[first, 0].min()) * 10 / 1000:.1f} us after the first entry")
    first = (st[:, 1] - t0) * 10 / 1000  # iteration starts relative to the earliest one
    print("iteration start (us) at deciles:", np.percentile(first, np.arange(0, 101, 10)).round(1))
    print(f"last write done at {(st[:, 6].max() - t0) * 10 / 1000:.1f} us after the first iteration start")


if __name__ == "__main__":
    main(sys.argv[1])
