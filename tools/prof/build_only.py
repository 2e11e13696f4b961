"""Hash stage only (no alignment), for timing ablation libraries that break the
dispatch: python tools/prof/build_only.py [reads] [len] [k] -> stage ms per step."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sequence-aligner_amd"))
import bench
import saoverlap as sao
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
L = int(sys.argv[2]) if len(sys.argv) > 2 else 500
k = int(sys.argv[3]) if len(sys.argv) > 3 else 15
b, o = bench.synth_workload(n, L, int(n * L / 20.0), 0.5, seed=1)
ov = sao.Overlapper(timing=True, kmer_size=k, id_mode=sao.SA_IDS_WIDE)
ov.add_packed(b.tobytes(), o)
for _ in range(3):
    ov.device_build()
ov.sync()
ov.reset_stage_times()
t0 = time.perf_counter()
for _ in range(10):
    ov.device_build()
ov.sync()
dt = (time.perf_counter() - t0) / 10
st = ov.stage_times()
print(json.dumps({"ms": round(dt * 1e3, 3), "role_pairs": ov.stats()["role_pairs"], **{kk: round(v[0] / 10, 4) for kk, v in st.items() if v[1]}}))
