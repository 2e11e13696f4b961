"""Extract the read records of the reference's AMOS bank as a small fixture.

`amos/c_ruddii.bnk` is the bank `toAmos_new -s c_ruddii.seq -b c_ruddii.bnk`
built (amos/README:1-3, Rakefile.rb:174).  Two of its files say what a {RED}
message for these reads must load to:

* `RED.0.map`: a header line `RED <count>` then one line per read of three
  tab-separated ids (the bank's iid / bid / eid columns);
* `RED.0.0.fix`: one 55-byte fixed record per read (`RED.ifo`: bytes/index = 55).
  Across all 32,000 records only bytes 0-2 vary (the record's little-endian
  64-bit offset into the var blob, bytes 0-7); the rest is the same in every
  record: int32 100 at byte 10 (the sequence length), the int32 pair (0, 100) at
  bytes 14-21 (the clear range), zeros in bytes 22-50 (every other id and range
  of the record unset), int32 201 at byte 51.

Only data files are read; nothing under /root/reference is executed.  Writes
tests/golden/c_ruddii_bank_red.npz = {map: int32[n, 3], length, clr_begin,
clr_end: int32[n], rest_zero: bool[n]} in record order.
"""
import os

import numpy as np

BANK = "/root/reference/amos/c_ruddii.bnk"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_ruddii_bank_red.npz")


def main():
    lines = open(os.path.join(BANK, "RED.0.map")).read().split("\n")
    head = lines[0].split()
    assert head[0] == "RED"
    n = int(head[1])
    ids = np.array([[int(x) for x in ln.split("\t")] for ln in lines[1:1 + n]], dtype=np.int32)
    assert ids.shape == (n, 3) and lines[1 + n:] in ([], [""])
    fix = np.fromfile(os.path.join(BANK, "RED.0.0.fix"), dtype=np.uint8)
    assert fix.size == 55 * n
    fix = fix.reshape(n, 55)

    def i32(col):
        return fix[:, col:col + 4].copy().view("<i4").reshape(n)
    np.savez_compressed(OUT, map=ids, length=i32(10), clr_begin=i32(14), clr_end=i32(18),
                        rest_zero=(fix[:, 22:51] == 0).all(axis=1))
    print(n, OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
