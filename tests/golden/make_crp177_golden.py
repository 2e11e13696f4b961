"""Golden vectors for crp177 from the Scala-literal restatement (oracle/literal.py).

No output of the Scala program exists anywhere (no JVM here, and none shipped),
so these vectors come from the line-by-line Python transliteration of the Scala
code.  They pin the fast C oracle (oracle/sa_oracle.c) and, through it, the HIP
path.  Writes, for k in (12, 15):
  crp177_k{k}.ovl        the .ovl bytes of `-i crp177.seq -k {k} -o ...`
  crp177_k{k}.npz        PairData in Trove iteration order (fst, snd, count),
                         first-insertion order, DispatchData order (lead, trail),
                         KmerData iteration order (hashes)
Runtime ~25 s (pure Python).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import literal as L  # noqa: E402


def main():
    text = open(os.path.join(HERE, "crp177.seq")).read()
    for k in (12, 15):
        out, tab, _ = L.run(text, L.AlignSettings(k=k))
        with open(os.path.join(HERE, "crp177_k%d.ovl" % k), "w") as f:
            f.write(out)
        items = list(tab.PairData.items())
        keys = np.array([kk for kk, _ in items], dtype=np.int64)
        cnt = np.array([v for _, v in items], dtype=np.int32)
        first = np.array(tab.pair_first_order, dtype=np.int64)
        lead, trail = [], []
        for a, bs in tab.DispatchData.items():
            for b in bs:
                lead.append(a); trail.append(b)
        np.savez_compressed(os.path.join(HERE, "crp177_k%d.npz" % k),
                            pair_fst=(keys >> 16).astype(np.int32), pair_snd=(keys & 0xFFFF).astype(np.int32),
                            pair_cnt=cnt, first_fst=(first >> 16).astype(np.int32),
                            first_snd=(first & 0xFFFF).astype(np.int32),
                            lead=np.array(lead, dtype=np.int32), trail=np.array(trail, dtype=np.int32),
                            bucket_order=np.array([kk for kk, _ in tab.KmerData.items()], dtype=np.int32))
        print(k, len(keys), len(lead), out.count("{OVL"))


if __name__ == "__main__":
    main()
