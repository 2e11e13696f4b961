"""Golden vectors for `--quadratic-align` (BioLibs.generateLocalAlignmentSet,
BioLibs.scala:267-368) from the Scala-literal restatement (oracle/literal.py).

No output of the Scala program exists (no JVM here, none shipped), so -- as for
the banded aligner -- these come from the line-by-line Python transliteration.
They pin the C oracle's align_local (oracle/sa_oracle.c) and, through it, the
HIP kernels (local_align.hip).  Inputs:
  crp177.seq, k = 12                    the reference's small data set
  mutated_reads.seq (written here once)  90 reads of a 1,400 bp random genome,
                                         80-130 bp, with substitutions and indels
                                         (so gap moves occur), k = 10, under three
                                         gap settings
Writes quad_<name>.npz: lead, trail (dispatch order) and start_i, start_j,
end_i, end_j, correct, error for EVERY dispatched pair (valid or not), and
quad_<name>.ovl.  Runtime ~2 min (pure Python).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import literal as L  # noqa: E402

CASES = [
    ("crp177_k12", "crp177.seq", dict(k=12)),
    ("mut_k10_g200", "mutated_reads.seq", dict(k=10, min_coll=3, min_identity=0.9)),
    ("mut_k10_g40", "mutated_reads.seq", dict(k=10, min_coll=3, min_identity=0.9, gap_open=-40,
                                              gap_extend=-8)),
    ("mut_k10_g10", "mutated_reads.seq", dict(k=10, min_coll=3, min_identity=0.85, gap_open=-10,
                                              gap_extend=-1, min_overlap=30)),
]


def write_mutated(path):
    rng = np.random.default_rng(2024)
    genome = "".join(rng.choice(list("ACGT"), size=1400))
    out = []
    for r in range(90):
        ln = int(rng.integers(80, 131))
        s0 = int(rng.integers(0, len(genome) - ln + 1))
        s = list(genome[s0:s0 + ln])
        for _ in range(int(rng.integers(0, 5))):
            p = int(rng.integers(0, len(s)))
            op = int(rng.integers(0, 3))
            if op == 0:
                s[p] = "ACGT"[int(rng.integers(0, 4))]
            elif op == 1:
                del s[p]
            else:
                s.insert(p, "ACGT"[int(rng.integers(0, 4))])
        out.append(">m%d\n%s\n" % (r + 1, "".join(s)))
    with open(path, "w") as f:
        f.write("".join(out))


def main():
    mpath = os.path.join(HERE, "mutated_reads.seq")
    if not os.path.exists(mpath):
        write_mutated(mpath)
    for name, fn, kw in CASES:
        text = open(os.path.join(HERE, fn)).read()
        s = L.AlignSettings(**kw)
        seqs = L.read_seq(text)
        table = L.KmerTable()
        for idx, seq in enumerate(seqs):
            table.add_kmer_set(idx + 1, seq, L.generate_kmer_set(s.kmerSize, idx + 1, seq))
        rows, ovl = [], []
        for lead, trails in table.dispatch_blocks(s):  # genBlockMTAlign, Project4.scala:725-790
            A = table.SequenceData[lead]
            maxL = max(len(table.SequenceData[j]) for j in trails)
            block = L.local_alignment_set(maxL, lead, A, [(j, table.SequenceData[j]) for j in trails], s)
            for a in block:
                rows.append((a.idA, a.idB, a.start[0], a.start[1], a.end[0], a.end[1], a.correct, a.error))
                if a.valid(s) and a.overlap_valid(s):
                    ovl.append(a.ovl_text() + "\n")
        arr = np.array(rows, dtype=np.int32).reshape(-1, 8)
        np.savez_compressed(os.path.join(HERE, "quad_%s.npz" % name), lead=arr[:, 0], trail=arr[:, 1],
                            start_i=arr[:, 2], start_j=arr[:, 3], end_i=arr[:, 4], end_j=arr[:, 5],
                            correct=arr[:, 6], error=arr[:, 7])
        with open(os.path.join(HERE, "quad_%s.ovl" % name), "w") as f:
            f.write("".join(ovl))
        print(name, len(rows), len(ovl))


if __name__ == "__main__":
    main()
