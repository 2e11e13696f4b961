"""Compare the PairData / dispatch of two library builds on one input (debug aid):
python tools/gpu/cmp_libs.py LIB_A LIB_B [k] -- crp177, wide ids, keep_pairs."""
import os, subprocess, sys, json
ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
if len(sys.argv) > 1 and sys.argv[1] == "--one":
    sys.path.insert(0, os.path.join(ROOT, "sequence-aligner_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import saoverlap as sao
    import helpers as H
    k = int(sys.argv[2])
    ov = sao.Overlapper(keep_pairs=True, id_mode=sao.SA_IDS_WIDE, kmer_size=k)
    ov.read_fasta(H.crp177_path())
    ov.build()
    pf, ps, pc = ov.pairs()
    st = ov.stats()
    np.savez(sys.argv[3], pf=pf, ps=ps, pc=pc)
    print(json.dumps({kk: int(v) for kk, v in st.items() if isinstance(v, int)}))
    sys.exit(0)
k = sys.argv[3] if len(sys.argv) > 3 else "12"
for tag, lib in (("a", sys.argv[1]), ("b", sys.argv[2])):
    env = dict(os.environ, SA_OVERLAP_LIB=lib)
    print(tag, subprocess.run([sys.executable, __file__, "--one", k, "/tmp/cmp_%s.npz" % tag], env=env,
                              capture_output=True, text=True, timeout=120).stdout.strip())
import numpy as np
A, B = np.load("/tmp/cmp_a.npz"), np.load("/tmp/cmp_b.npz")
da = {(int(f), int(s)): int(c) for f, s, c in zip(A["pf"], A["ps"], A["pc"])}
db = {(int(f), int(s)): int(c) for f, s, c in zip(B["pf"], B["ps"], B["pc"])}
diff = [(key, da.get(key), db.get(key)) for key in set(da) | set(db) if da.get(key) != db.get(key)]
print("pairs a", len(da), "b", len(db), "differ", len(diff))
diff.sort()
for d in diff[:40]:
    print(d)
