"""Parity at the per-GPU slice sizes of BASELINE configs[3] and [4].  GPU only.

configs[3] (8 GPUs, 10M x 500 bp, k = 15) and configs[4] (8 GPUs, 50M mixed
100-1,000 bp reads, k = 12 and k = 15) put 1.25M and 6.25M reads on each GPU.
Size-dependent faults live exactly there (round 3 found a 32-bit launch-grid
wrap that silently dropped 74 % of the pairs at 6.25M reads), so each test
builds a slice-sized read set on the device and compares it with the all-core
C oracle (oracle/sa_oracle.c: orc_run_wide_mt, KmerTable.scala:41-187 restated
on OpenMP threads, itself CPU-tested equal to the single-threaded restatement):

* the dispatch list (lead, trail) element by element, and every dispatched
  pair's collision count against the oracle's PairData count;
* the role-pair total and the distinct-pair total;
* 20,000 dispatched pairs sampled across the list, aligned by the oracle's
  generateFastDovetailAlignmentSet restatement (orc_align_batch), every tuple
  equal to the device's.

Sizes: configs[3]'s whole per-GPU slice (1.25M x 500 bp); a configs[4]-shaped
mixed set at k = 15 of 1M reads; at k = 12, 200k mixed reads (1.6e8 distinct
pairs, ~16 GB of oracle PairData maps) -- the 6.25M slice's 1.5e11 distinct
pairs do not fit host memory; 200k reads already send the long reads through
the recount tiers.
"""
import os
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sao = pytest.importorskip("saoverlap")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (the bench's workload generator)

ALIGN_CMP = ("start_i", "start_j", "end_i", "end_j", "correct", "error", "ahg", "bhg")
SAMPLE = 20000


def slice_vs_oracle(oracle_mod, n, read_len, min_len, k, shards=0):
    mean_len = read_len if min_len is None else (read_len + min_len) / 2.0
    G = int(n * mean_len / 20.0)  # bench.py's 20x coverage
    t0 = time.time()
    b, o = bench.synth_workload(n, read_len, G, 0.5, seed=1, min_len=min_len)
    bases = b.tobytes()
    del b
    ov = sao.Overlapper(kmer_size=k, id_mode=sao.SA_IDS_WIDE)
    ov.add_packed(bases, o)
    ov.device_build()
    ov.device_align()
    st = ov.stats()
    lead, trail, count = ov.dispatch()
    al = ov.alignments()
    ov.close()
    t_gpu = time.time() - t0
    if shards:
        # the sharded path (multi.cpp + dist.hip) on the same reads: the
        # single-device result, which is checked against the oracle below
        sv = sao.Overlapper(shards=shards, kmer_size=k, id_mode=sao.SA_IDS_WIDE)
        sv.add_packed(bases, o)
        sv.device_build()
        sv.device_align()
        ss = sv.stats()
        for key in ("kmers", "role_pairs", "pairs", "dispatched", "aligned", "ovl_records", "dp_cells"):
            assert ss[key] == st[key], key
        for x, y in zip(sv.dispatch(), (lead, trail, count)):
            np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(sv.alignments(), al)
        assert sv.exchanged_bytes() > 0
        sv.close()
    t0 = time.time()
    r = oracle_mod.Run(packed=(bases, o), settings=oracle_mod.default_settings(kmer_size=k), wide=True,
                       skip_align=True, threads=0)
    t_cpu = time.time() - t0
    print("slice n=%d L=%s k=%d: %d k-mers, %d role pairs, %d pairs, %d dispatched; device %.1f s, oracle %.1f s"
          % (n, read_len if min_len is None else "%d-%d" % (min_len, read_len), k, st["kmers"], st["role_pairs"],
             st["pairs"], st["dispatched"], t_gpu, t_cpu))
    assert st["kmers"] == int((np.diff(o.astype(np.int64)) - k + 1).clip(0).sum())
    assert st["role_pairs"] == r.role_pairs
    assert st["pairs"] == len(r.pair_fst)
    np.testing.assert_array_equal(lead, r.lead)
    np.testing.assert_array_equal(trail, r.trail)
    # each dispatched pair's count = the oracle's PairData count of that key
    okey = (r.pair_fst.astype(np.uint64) << np.uint64(32)) | r.pair_snd.astype(np.uint64)
    dkey = (lead.astype(np.uint64) << np.uint64(32)) | trail.astype(np.uint64)
    pos = np.searchsorted(okey, dkey)
    assert (pos < len(okey)).all() and (okey[np.minimum(pos, len(okey) - 1)] == dkey).all()
    np.testing.assert_array_equal(count, r.pair_cnt[pos])
    del okey, r
    # alignments of a sample spread over the whole list (both ends included)
    nd = len(lead)
    idx = np.unique(np.linspace(0, nd - 1, min(SAMPLE, nd)).astype(np.int64))
    ca = oracle_mod.align_batch(bases, o, lead[idx], trail[idx], settings=oracle_mod.default_settings(kmer_size=k),
                                threads=0)
    for name in ALIGN_CMP:
        np.testing.assert_array_equal(al[idx, sao.ALIGN_FIELDS.index(name)],
                                      ca[:, oracle_mod.ALIGN_FIELDS.index(name)], err_msg=name)
    flags = al[idx, sao.ALIGN_FIELDS.index("flags")]
    np.testing.assert_array_equal((flags & sao.FLAG_DUD) != 0, ca[:, oracle_mod.ALIGN_FIELDS.index("is_dud")] != 0)
    np.testing.assert_array_equal((flags & sao.FLAG_VALID) != 0, ca[:, oracle_mod.ALIGN_FIELDS.index("valid")] != 0)
    return st


def test_configs3_per_gpu_slice_matches_oracle(oracle_mod):
    """configs[3]'s whole per-GPU slice: 1.25M x 500 bp, k = 15 (607.5M k-mers,
    ~4e9 role pairs), 31.25 Mbp genome at 20x."""
    st = slice_vs_oracle(oracle_mod, 1250000, 500, None, 15)
    assert st["kmers"] == 1250000 * 486 and st["dispatched"] > 8000000


def test_configs4_shape_k15_matches_oracle(oracle_mod):
    """configs[4]'s read shape at k = 15: 1M mixed 100-1,000 bp reads, on one
    device and on 2 virtual shards x 500k reads (the sharded path with mixed
    lengths at size: every alignment equal to the single device's)."""
    st = slice_vs_oracle(oracle_mod, 1000000, 1000, 100, 15, shards=2)
    assert st["dispatched"] > 1000000


def test_configs4_shape_k12_matches_oracle(oracle_mod):
    """configs[4]'s k = 12 pass (the LDS-occupancy stress) at 200k mixed reads:
    12-mers in a 16.7M space collide at random, so long reads meet ~1,000
    distinct partners and overflow the first pass's 256-slot tables."""
    st = slice_vs_oracle(oracle_mod, 200000, 1000, 100, 12)
    assert st["flags"] & sao.SA_STATS_RECOUNTED
    assert st["pairs"] > 100000000
