"""Bucket-build timing of several contexts created one after another in ONE
process (fresh allocations each): separates a per-process mode from a
per-allocation (placement) one.  Prints one line per context."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sequence-aligner_amd"))
import bench  # noqa: E402  (synthetic workload helpers)
import saoverlap as sao  # noqa: E402

# optional: hold a device buffer of SPACER_GB before the first context, so
# its arrays land elsewhere in VRAM (placement probe)
spacer_gb = float(os.environ.get("SPACER_GB", "0"))
if spacer_gb > 0:
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    sp = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(sp), ctypes.c_size_t(int(spacer_gb * (1 << 30)))) == 0
    print("spacer %.1f GB at 0x%x" % (spacer_gb, sp.value), flush=True)
n, L = 100000, 500
bases, offsets = bench.synth_workload(n, L, n * L // 20, 0.5, seed=1)
keep = []
# optional: DUMMY_CTX=1 creates one context (its streams) that never builds
# before the measured ones (queue probe)
if os.environ.get("DUMMY_CTX") == "1":
    keep.append(sao.Overlapper(timing=True, kmer_size=15, id_mode=sao.SA_IDS_WIDE))
    print("dummy context", flush=True)
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    ov = sao.Overlapper(timing=True, kmer_size=15, id_mode=sao.SA_IDS_WIDE)
    ov.add_packed(bases.tobytes(), offsets)
    ov.device_build()
    ov.reset_stage_times()
    for _ in range(6):
        ov.device_build()
    t = ov.stage_times()
    print("ctx %d buckets %.4f pairs %.4f sort %.4f" % (i, t["buckets"][0] / t["buckets"][1], t["pairs"][0] / t["pairs"][1],
                                                       t["sort"][0] / t["sort"][1]), flush=True)
    if i % 2:
        ov.close()   # odd contexts freed: the next one may reuse their memory
    else:
        keep.append(ov)
