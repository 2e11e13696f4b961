"""configs[4]-shape k = 12 on 8 virtual shards at 2M mixed reads (the test runs 1M): the sharded
dispatch against the single device's, element by element, with the pass count and timings.
  python tools/prof/r6_k12_2m.py [reads]   -> one JSON line"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sequence-aligner_amd"))
import bench  # noqa: E402
import saoverlap as sao  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
k = 12
b, o = bench.synth_workload(n, 1000, int(n * 550 / 20.0), 0.5, seed=12, min_len=100)
bases = b.tobytes()
del b
out = {"reads": n, "k": k, "shards": 8}
t0 = time.time()
one = sao.Overlapper(kmer_size=k, id_mode=sao.SA_IDS_WIDE)
one.add_packed(bases, o)
one.build()
out["single_build_s"] = round(time.time() - t0, 3)
ref = one.dispatch()
out["single_stats"] = one.stats()
one.close()
ov = sao.Overlapper(shards=8, kmer_size=k, id_mode=sao.SA_IDS_WIDE)
ov.add_packed(bases, o)
t0 = time.time()
ov.build()
out["sharded_first_build_s"] = round(time.time() - t0, 3)
out["shard_info_first"] = ov.shard_info()
t0 = time.time()
ov.build()
out["sharded_second_build_s"] = round(time.time() - t0, 3)
out["shard_info"] = ov.shard_info()
got = ov.dispatch()
out["sharded_stats"] = ov.stats()
ov.close()
out["dispatch_equal"] = all(np.array_equal(x, y) for x, y in zip(got, ref))
print(json.dumps(out, default=int))
