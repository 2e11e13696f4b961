"""ASan + UBSan build of the library's host-side parsers and Trove replay
(a sanitizer build of the host C++).  CPU only.

tests/san/host_san.cpp links csrc/host/fasta.cpp (BioLibs.readSeq,
BioLibs.readHOXD restatements) and csrc/host/trove.h (GNU Trove 3.0.3 slot
layout) into one executable built with -fsanitize=address,undefined and no
recovery, then drives it over well-formed and malformed inputs.  A sanitizer
report makes the process exit non-zero.  The Trove order is also checked
against the C oracle's independent Trove emulator.
"""
import os
import subprocess

import numpy as np
import pytest

import helpers as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "san", "host_san.cpp")
FASTA_CPP = os.path.join(ROOT, "sequence-aligner_amd", "csrc", "host", "fasta.cpp")


@pytest.fixture(scope="module")
def san_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("san") / "host_san")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-o", out, SRC, FASTA_CPP]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


def run(san_bin, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([san_bin] + [str(a) for a in args], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


FASTAS = {
    "plain": b">a\nACGT\nacgt\n>b\nTTTT\n",
    "crlf": b">a\r\nACGT\r\nGG\r\n>b\r\nCC\r\n",
    "no_trailing_newline": b">a\nACGTACGT",
    "empty_records": b">a\n>b\n\n>c\nA\n",
    "header_only": b">only\n",
    "not_fasta": b"ACGT\n>a\nAC\n",
    "empty_file": b"",
    "long_line": b">a\n" + b"ACGT" * 50000 + b"\n",
    "binary": bytes(range(256)) * 4,
    "lone_cr": b">a\rAC\rgt\r>b\rT",
    "mixed_endings": b">x y\r\nAC\n\rgg\r\r\n>z\nTT\r",
}


def read_seq_model(data):
    """BioLibs.readSeq (BioLibs.scala:26-50) over java.io.BufferedReader.readLine
    (lines end at \\n, \\r or \\r\\n; a last line without terminator counts):
    the sequences, upper-cased, or None where the reference fails."""
    lines, cur, i, n = [], bytearray(), 0, len(data)
    while i < n:
        ch = data[i]
        if ch in (10, 13):
            lines.append(bytes(cur))
            cur = bytearray()
            i += 2 if ch == 13 and i + 1 < n and data[i + 1] == 10 else 1
        else:
            cur.append(ch)
            i += 1
    if cur:
        lines.append(bytes(cur))
    if not lines or not lines[0].startswith(b">"):
        return None
    seqs = [b""]
    for ln in lines[1:]:
        if ln.startswith(b">"):
            seqs.append(b"")
        else:
            seqs[-1] += bytes(c - 32 if 97 <= c <= 122 else c for c in ln)  # (ASCII a-z only)
    return seqs


def summary_line(seqs):
    """host_san's first output line for a parsed file."""
    allb, chk = b"".join(seqs), 0
    for c in allb:
        chk = (chk * 1000003 + c) & 0xFFFFFFFFFFFFFFFF
    return "n %d bases %d sum %d" % (len(seqs), len(allb), chk)


@pytest.mark.parametrize("name", sorted(FASTAS))
def test_fasta_reader_under_sanitizers(san_bin, tmp_path, name):
    p = tmp_path / "in.seq"
    p.write_bytes(FASTAS[name])
    out = run(san_bin, "fasta", p)
    if name == "plain":
        assert out.splitlines()[1:] == ["ACGTACGT", "TTTT"]
    want = read_seq_model(FASTAS[name])  # readLine semantics, every corpus
    if want is None:
        assert out.startswith("rc ")
    else:
        assert out.split("\n", 1)[0] == summary_line(want)


def test_fasta_reader_crp177(san_bin):
    out = run(san_bin, "fasta", H.crp177_path())
    assert out.splitlines()[1:] == H.read_fasta_seqs(H.crp177_path())


HOXDS = {
    "hoxd1": None,  # the reference's own amos/HOXD1.txt fixture
    "missing_rows": b"A,91,-114,-31,-123\nC,-114,100,-125,-31\n",
    "trailing_comma": b"A,1,2,3,4,\nC,5,6,7,8\nG,9,10,11,12\nT,13,14,15,16\n",
    "spaces": b" A, 1, 2, 3, 4\nC,5,6,7,8\n",
    "overflow": b"A,99999999999,0,0,0\n",
    "garbage": b"\x00\xff,,,\n,,\nZ,1\n",
    "empty": b"",
}


@pytest.mark.parametrize("name", sorted(HOXDS))
def test_hoxd_reader_under_sanitizers(san_bin, tmp_path, name):
    if HOXDS[name] is None:
        p = os.path.join(H.GOLDEN, "HOXD1.txt")
    else:
        p = tmp_path / "m.txt"
        p.write_bytes(HOXDS[name])
    out = run(san_bin, "hoxd", p).split()
    rc = int(out[1])
    costs = [int(x) for x in out[2:]]
    if rc != 0:
        assert costs == [12345] * 16  # the caller's matrix is left untouched on failure
    if name == "hoxd1":
        assert rc == 0 and costs == [91, -114, -31, -123, -114, 100, -125, -31, -31, -125, 100, -114,
                                     -123, -31, -114, 91]


@pytest.mark.parametrize("n,seed", [(0, 1), (1, 2), (25, 3), (3000, 4), (200000, 5)])
def test_trove_replay_under_sanitizers_matches_oracle(san_bin, oracle_mod, n, seed):
    out = run(san_bin, "trove", n, seed)
    got = np.array([int(x) for x in out.split()], dtype=np.int64)
    # the same key stream through the oracle's independent Trove emulator
    x = (seed * 0x9E3779B97F4A7C15 + 1) % (1 << 64)
    keys = []
    for _ in range(n):
        x ^= (x << 13) % (1 << 64)
        x ^= x >> 7
        x ^= (x << 17) % (1 << 64)
        k = ((x >> 40) % 1000) if x % 4 == 0 else (x >> 32)
        keys.append(k - (1 << 32) if k >= (1 << 31) else k)
    uniq = list(dict.fromkeys(keys))  # first-insertion order of distinct keys
    order, _ = oracle_mod.trove_order(np.array(uniq, dtype=np.int32))
    np.testing.assert_array_equal(got, order.astype(np.int64))
