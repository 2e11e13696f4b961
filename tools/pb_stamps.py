"""Phase timing of the bucket build's main pass from a timing-probe build
(make OUT=build_stamps EXTRA=-DSA_PB_STAMPS=1; SA_PB_STAMPS_OUT=<file>):
8 u64 words per partition -- wall_clock64() at block start (0), records loaded
into LDS (1), LDS sort done (2), scans done (3), outputs issued (4), and
(smid | n << 32) (5).  wall_clock64 ticks at 100 MHz on MI355X (10 ns).

    python tools/pb_stamps.py stamps.bin [tick_ns]
"""
import sys

import numpy as np


def main(path, tick_ns=10.0):
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    ok = (a[:, 0] > 0) & (a[:, 4] >= a[:, 0])
    a = a[ok]
    t = a[:, :5].astype(np.int64)
    t0 = t[:, 0].min()
    rel = (t - t0) * tick_ns / 1000.0  # us
    n = (a[:, 5] >> np.uint64(32)).astype(np.int64)
    span = rel[:, 4].max()
    print(f"blocks {len(a)}  main-pass span {span:.1f} us  records/block mean {n.mean():.0f}")
    names = ["load", "sort", "scan", "out"]
    for i, nm in enumerate(names):
        d = rel[:, i + 1] - rel[:, i]
        print(f"  {nm:5s} mean {d.mean():6.2f} us  p50 {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f}  "
              f"p99 {np.percentile(d, 99):6.2f}")
    life = rel[:, 4] - rel[:, 0]
    print(f"  life  mean {life.mean():6.2f} us  p50 {np.median(life):6.2f}  p90 {np.percentile(life, 90):6.2f}")
    # concurrency: blocks alive per time bin
    bins = np.linspace(0, span, 41)
    alive = [int(((rel[:, 0] <= b) & (rel[:, 4] > b)).sum()) for b in bins[:-1]]
    print("  blocks alive over the pass (40 bins):", alive)
    starts = np.sort(rel[:, 0])
    print(f"  last block starts at {starts[-1]:.1f} us; first 2,048 blocks started by {starts[min(2047, len(starts) - 1)]:.1f} us")
    # per-CU: blocks handled
    cu = (a[:, 5] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    u, c = np.unique(cu, return_counts=True)
    print(f"  distinct smid {len(u)}; blocks per smid min {c.min()} mean {c.mean():.1f} max {c.max()}")
    # life vs records
    for lo, hi in [(0, 500), (500, 700), (700, 850), (850, 1025)]:
        m = (n >= lo) & (n < hi)
        if m.any():
            print(f"  n in [{lo},{hi}): {m.sum():6d} blocks, life mean {life[m].mean():6.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 10.0)
