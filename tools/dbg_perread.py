"""Debug: dispatch of the per-read pair mode vs the shared-region mode (keep_pairs)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sequence-aligner_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import saoverlap as sao
import helpers as H
reads = H.synth_reads(2000, 200, 20000, seed=61)
out = []
for kp in (False, True):
    ov = sao.Overlapper(keep_pairs=kp, id_mode=sao.SA_IDS_WIDE, kmer_size=15)
    ov.add_reads(reads)
    ov.build()
    out.append([np.asarray(x) for x in ov.dispatch()])
    print("keep_pairs", kp, "stats", ov.stats(), flush=True)
a, b = out
print("n", len(a[0]), len(b[0]))
m = min(len(a[0]), len(b[0]))
for name, x, y in zip(("lead", "trail", "count"), a, b):
    bad = np.nonzero(x[:m] != y[:m])[0]
    print(name, "mismatches", len(bad), "first", bad[:5], x[bad[:5]] if len(bad) else None, y[bad[:5]] if len(bad) else None)
print("a head", [v[:10] for v in a])
print("b head", [v[:10] for v in b])
