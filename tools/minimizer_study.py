"""What owner-by-minimizer would give the sharded pair counter --
measured on the bench's own synthetic reads before building it.

Today every k-mer goes to the rank owning its hash range (top log2 P bits of
mix32(seqHash), multi.cpp).  The proposal: the owner of a k-mer is a hash of its
minimizer (the smallest, by a random order, of its k - m + 1 m-mers) -- still a function
of the k-mer alone, so every bucket stays whole on one rank, but a read's consecutive
k-mers share a minimizer over a super-k-mer and land on one rank together.

Per (k, m) on `--reads` reads of the bench workload (configs[1] shape, P ranks):
  run      mean run of consecutive k-mers of a read on one rank (what the counter would
           see as consecutive occurrences; hash owner: P / (P - 1))
  imb      the most loaded rank's k-mers / the mean (the rank's bucket build and
           pair count scale with it)
  x1       exchange-1 bytes per k-mer: 8 B records today; spans (read id 4 B, start 2 B,
           length 1 B + the run's bases at 2 bits) with minimizers
  x1_imb   the same imbalance for the received bytes

  python tools/minimizer_study.py --reads 20000
Writes profiles/r06/minimizer_study.json.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

CODE = np.zeros(256, np.uint64)
for i, ch in enumerate(b"ACGT"):
    CODE[ch] = i


def mix64(x):
    x = x.copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xFF51AFD7ED558CCD)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xC4CEB9FE1A85EC53)
        x ^= x >> np.uint64(33)
    return x


def window_codes(codes, w):
    """2-bit packed words of every w-mer of every read (rows: reads)."""
    n, L = codes.shape
    out = np.zeros((n, L - w + 1), np.uint64)
    for j in range(w):
        out = (out << np.uint64(2)) | codes[:, j:L - w + 1 + j]
    return out


def sliding_min(a, w):
    """min over windows of w along axis 1"""
    from numpy.lib.stride_tricks import sliding_window_view
    return sliding_window_view(a, w, axis=1).min(axis=2)


def runs(owner):
    same = owner[:, 1:] == owner[:, :-1]
    n_runs = owner.shape[0] + (~same).sum()
    return owner.size / n_runs, n_runs


def study(codes, k, m, P):
    kmers = window_codes(codes, k)
    rec = {"k": k, "m": m}
    if m is None:  # today: owner by the k-mer's hash
        owner = (mix64(kmers) >> np.uint64(64 - int(np.log2(P)))).astype(np.int64)
    else:
        mm = mix64(window_codes(codes, m) | np.uint64(1 << 62))  # random order of the m-mers
        mins = sliding_min(mm, k - m + 1)  # the k-mer's minimizer (by hash value)
        owner = (mix64(mins) >> np.uint64(64 - int(np.log2(P)))).astype(np.int64)
    rl, n_runs = runs(owner)
    load = np.bincount(owner.ravel(), minlength=P)
    rec["run"] = round(float(rl), 3)
    rec["imb"] = round(float(load.max() / load.mean()), 3)
    if m is None:
        rec["x1_bytes_per_kmer"] = 8.0
        rec["x1_imb"] = rec["imb"]
    else:
        # a run of r k-mers = r + k - 1 bases; span = 7 B header + 2 bits a base
        change = np.ones(owner.shape, bool)
        change[:, 1:] = owner[:, 1:] != owner[:, :-1]
        run_id = np.cumsum(change.ravel())
        run_len = np.bincount(run_id)[1:]
        run_owner = owner.ravel()[change.ravel()]
        span_bytes = 7 + np.ceil((run_len + k - 1) / 4.0)
        by_owner = np.bincount(run_owner, weights=span_bytes, minlength=P)
        rec["x1_bytes_per_kmer"] = round(float(span_bytes.sum() / owner.size), 3)
        rec["x1_imb"] = round(float(by_owner.max() / by_owner.mean()), 3)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=20000)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06", "minimizer_study.json"))
    a = ap.parse_args()
    # the bench's workload: 500 bp reads at 20x of a genome of reads x 25 bp (a sample of them)
    n_all = 100_000
    bases, off = bench.synth_workload(n_all, 500, n_all * 500 // 20, 0.5, 1)
    codes = CODE[bases[: a.reads * 500]].reshape(a.reads, 500)
    out = {"reads": a.reads, "read_len": 500, "ranks": a.ranks, "rows": []}
    for k, ms in ((15, (None, 7, 9, 11)), (12, (None, 7, 9))):
        for m in ms:
            r = study(codes, k, m, a.ranks)
            print(r)
            out["rows"].append(r)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
