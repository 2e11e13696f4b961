"""Rebuild the c_ruddii read set (32,000 x 100 bp) from data files the reference holds.

`amos/c_ruddii.seq` is a missing blob (.MISSING_LARGE_BLOBS).  The AMOS bank that
was built from it is present: `c_ruddii.bnk/LAY.0.0.var` holds one 24-byte tile
record per read (pad, iid, gapcount, offset, begin, end) starting at byte 1, and
`c_ruddii.fasta` is the assembled contig; every read is the forward-strand
substring contig[offset : offset+100].  Only data files are
read here; nothing under /root/reference is executed.

Writes tests/golden/c_ruddii_layout.npz = {contig: uint8[159659], offset: int32[32001]}
(offset[iid] for iid 1..32000; offset[0] unused), small enough to commit, from
which tests regenerate the reads (see tests/helpers.py: c_ruddii_reads()).
"""
import os
import struct

import numpy as np

REF = "/root/reference/amos"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_ruddii_layout.npz")


def main():
    lines = open(os.path.join(REF, "c_ruddii.fasta")).read().split("\n")
    assert lines[0].startswith(">")
    contig = "".join(lines[1:]).strip()
    lay = open(os.path.join(REF, "c_ruddii.bnk", "LAY.0.0.var"), "rb").read()
    n = (len(lay) - 1) // 24
    off = np.zeros(n + 1, dtype=np.int32)
    for r in range(n):
        pad, iid, gaps, o, b, e = struct.unpack("<6I", lay[1 + 24 * r: 25 + 24 * r])
        assert gaps == 0 and b == 0 and e == 100 and 1 <= iid <= n
        off[iid] = o
    assert (off[1:] + 100 <= len(contig)).all()
    np.savez_compressed(OUT, contig=np.frombuffer(contig.encode(), dtype=np.uint8), offset=off)
    print(n, len(contig), OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
