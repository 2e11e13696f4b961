"""Shared test helpers: fixture loaders and synthetic read generators."""
import hashlib
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def crp177_path():
    return os.path.join(GOLDEN, "crp177.seq")


def c_ruddii_reads():
    """The 32,000 reconstructed c_ruddii reads, ids 1..32000 in .seq order."""
    z = np.load(os.path.join(GOLDEN, "c_ruddii_layout.npz"))
    contig = z["contig"].tobytes().decode()
    off = z["offset"]
    return [contig[o:o + 100] for o in off[1:]]


def reads_fasta_bytes(reads):
    return b"".join(b">r%d\n%s\n" % (i + 1, r.encode()) for i, r in enumerate(reads))


def splitmix64(seed):
    x = np.uint64(seed)
    while True:
        x = np.uint64(x + np.uint64(0x9E3779B97F4A7C15))
        z = x
        z = np.uint64((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9))
        z = np.uint64((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB))
        yield np.uint64(z ^ (z >> np.uint64(31)))


def synth_reads(n_reads, read_len, genome_len, gc=0.5, seed=1, mixed=None):
    """Synthetic error-free forward-strand reads of a random genome (numpy RNG,
    seeded): the test-size analogue of SURVEY.md 8(d)'s splitmix genomes."""
    rng = np.random.default_rng(seed)
    p_gc = gc / 2.0
    p_at = (1.0 - gc) / 2.0
    genome = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=genome_len,
                        p=[p_at, p_gc, p_gc, p_at]).tobytes().decode()
    reads = []
    for _ in range(n_reads):
        L = read_len if mixed is None else int(rng.integers(mixed[0], mixed[1] + 1))
        s = int(rng.integers(0, genome_len - L + 1))
        reads.append(genome[s:s + L])
    return reads


def sha256(b):
    return hashlib.sha256(b).hexdigest()


def mutate(reads, rng, max_ops):
    """Up to max_ops substitutions / deletions / insertions per read."""
    out = []
    for rd in reads:
        s = list(rd)
        for _ in range(int(rng.integers(0, max_ops + 1))):
            p = int(rng.integers(0, len(s)))
            op = int(rng.integers(0, 3))
            if op == 0:
                s[p] = "ACGT"[int(rng.integers(0, 4))]
            elif op == 1:
                del s[p]
            else:
                s.insert(p, "ACGT"[int(rng.integers(0, 4))])
        out.append("".join(s))
    return out


def read_fasta_seqs(path):
    """Sequences of a FASTA file (headers dropped), like BioLibs.readSeq."""
    seqs, cur = [], None
    for line in open(path).read().splitlines():
        if line.startswith(">"):
            if cur is not None:
                seqs.append("".join(cur))
            cur = []
        elif cur is not None:
            cur.append(line.upper())
    if cur is not None:
        seqs.append("".join(cur))
    return seqs
