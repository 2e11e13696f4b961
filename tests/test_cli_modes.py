"""The reference's developer modes on the `sa-overlap` CLI (Project4.scala:61-98):
--test-kmer-cover (KmerTable.uniqueKmers / kmerCollisionHistogram on the
device, KmerTable.scala:189-221), --test-dispatch-collisions,
--test-block-dispatch, --test-fasta-read and the --bench-* report lines.
Expected text is rebuilt here from the Scala-literal restatement
(oracle/literal.py) and the golden dispatch vectors.  GPU only (the CLI runs
the HIP path)."""
import collections
import os
import re
import subprocess

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "sequence-aligner_amd", "build", "sa-overlap")


def run_cli(*args):
    r = subprocess.run([CLI] + list(args), capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout.decode()


def java_float(x):
    """java.lang.Float.toString via numpy's shortest round-trip digits."""
    x = np.float32(x)
    if x == 0:
        return "0.0"
    if np.float32(1e-3) <= abs(x) < np.float32(1e7):
        s = np.format_float_positional(x, unique=True)
        return s + "0" if s.endswith(".") else s
    m, e = np.format_float_scientific(x, unique=True).split("e")
    if m.endswith("."):
        m += "0"
    return "%sE%d" % (m, int(e))


def test_java_float_rendering():
    assert java_float(1.0) == "1.0"
    assert java_float(0.25) == "0.25"
    assert java_float(np.float32(1164) / np.float32(16777216)) == "6.937981E-5"
    assert java_float(np.float32(3) / np.float32(4)) == "0.75"


def kmer_cover_text(seqs):
    import literal as L
    out = []
    for k in range(26):
        hist = collections.Counter()
        if k == 0:
            total = sum(len(s) + 1 for s in seqs)
            if total:
                hist[total] = 1
            uniques = 1 if total else 0
        else:
            buckets = collections.Counter()
            for s in seqs:
                for i in range(len(s) - k + 1):  # BioLibs.generateKmerSet
                    buckets[L.seq_hash(s[i:i + k])] += 1
            uniques = len(buckets)
            hist = collections.Counter(buckets.values())
        ratio = np.float32(uniques) / np.float32(4.0 ** k)
        out.append("Kmer Size : %d\n  uniques : %d\n  ratio   : %s\n" % (k, uniques, java_float(ratio)))
        out.append("  [ number of collisions -> count of seqs with that many collisions ] :\n")
        out.extend("          [%d -> %d]\n" % (s, hist[s]) for s in sorted(hist))
        out.append("\n")
    return "".join(out)


def test_test_kmer_cover_crp177():
    seqs = H.read_fasta_seqs(H.crp177_path())
    assert run_cli("-i", H.crp177_path(), "--test-kmer-cover") == kmer_cover_text(seqs)


def test_kmer_histogram_api_mixed_lengths():
    import literal as L
    import saoverlap as sao
    reads = H.synth_reads(300, 150, 3000, seed=91, mixed=(5, 150))
    for k in (1, 3, 11, 16, 17, 24):
        ov = sao.Overlapper(kmer_size=k)
        ov.add_reads(reads)
        uniques, hist = ov.kmer_histogram()
        buckets = collections.Counter(L.seq_hash(s[i:i + k]) for s in reads for i in range(len(s) - k + 1))
        assert uniques == len(buckets), k
        assert hist == dict(collections.Counter(buckets.values())), k
        ov.close()


@pytest.mark.parametrize("blocks", [False, True])
def test_dispatch_modes_match_golden(blocks):
    g = np.load(os.path.join(H.GOLDEN, "crp177_k12.npz"))
    flag = "--test-block-dispatch" if blocks else "--test-dispatch-collisions"
    text = run_cli("-i", H.crp177_path(), "-k", "12", flag)
    want = "".join(" Dispatched Coll : %d - %d <-> %d\n" % (i + 1, a, b)
                   for i, (a, b) in enumerate(zip(g["lead"], g["trail"])))
    if blocks:
        sizes = collections.Counter(collections.Counter(g["lead"].tolist()).values())
        want += "\n Histogram Of Relations : [Number of Aligns -> Number of Seqs w/ that many Aligns]\n"
        want += "".join("          [%d -> %d]\n" % (s, sizes[s]) for s in sorted(sizes)) + "\n"
    assert text == want


def test_test_fasta_read():
    seqs = H.read_fasta_seqs(H.crp177_path())
    want = "\n" + "".join("id : %d\nseq: %s\n\n" % (i + 1, s) for i, s in enumerate(seqs[:10]))
    assert run_cli("-i", H.crp177_path(), "--test-fasta-read") == want


def test_bench_report_lines():
    t = run_cli("-i", H.crp177_path(), "--bench-fasta-read")
    assert re.fullmatch(r" Read 223 sequences from \S+ in \d+ milliseconds\.\n", t)
    t = run_cli("-i", H.crp177_path(), "--bench-kmer-gen")
    assert re.fullmatch(r"\nGenerated 1164 unique kmers from 223 sequences from \S+ sequentially in \d+ milliseconds\.\n\n"
                        r"Generated 1164 unique kmers from 223 sequences from \S+ in parellel in \d+ milliseconds\.\n\n", t)
    t = run_cli("-i", H.crp177_path(), "--bench-kmer-analysis")
    assert re.fullmatch(r"Starting kmer gen\.\nFinished kmer gen\.\n\nCalculated pair data in \d+ milliseconds\.\n\n"
                        r"Calculated dispatch data in \d+ milliseconds\.\n\n", t)
    t = run_cli("-i", H.crp177_path(), "--bench-align")
    n = len(np.load(os.path.join(H.GOLDEN, "crp177_k12.npz"))["lead"])
    for name in ("single threaded quad single", "multi threaded quad block", "multi threaded linear block"):
        assert re.search(r"\nCalculated %d %s alignments in \d+ milliseconds\.\n\n" % (n, name), t), name
    t = run_cli("-i", H.crp177_path(), "--bench-align-quick")
    assert t.count("\nCalculated 0 ") == 8  # the reference's debugStop guard lets nothing through


def test_alignment_string_modes_are_refused():
    r = subprocess.run([CLI, "-i", H.crp177_path(), "--test-overlaps"], capture_output=True, timeout=60)
    assert r.returncode == 1 and b"alignment strings" in r.stderr
