"""Parity at the BASELINE configs' own sizes.  GPU only.

* configs[1]/[2]: the bench workload itself -- 100,000 synthetic 500 bp reads
  (bench.synth_workload, seed 1, 2.5 Mbp genome), k = 15, wide ids: dispatch,
  every alignment tuple and the .ovl bytes against the C oracle's full
  calc-overlaps run (one core, ~1 min on the box).
* configs[4]: mixed 100-1,000 bp reads at k = 12 and at k = 15 (its two
  passes), which exercise the float32 loc comparison across read lengths
  (KmerTable.scala:65) and the per-length band width (BioLibs.scala:619-620).
* README:164-175's sample record, pinned exactly.
* configs[3]'s sharding at the bench size: the 100k-read workload over 4 and 8
  virtual shards gives the single-device dispatch and .ovl exactly.
"""
import os
import sys

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

sao = pytest.importorskip("saoverlap")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (the bench's workload generator)

ALIGN_CMP = ("start_i", "start_j", "end_i", "end_j", "correct", "error", "ahg", "bhg")

# README:164-175 (the reference's documented calc-overlaps output sample)
README_RECORD = b"{OVL\nadj:N\nrds:18,22\nscr:0\nahg:20\nbhg:20\n}\n"


def compare(ov, r, pairs=True):
    lead, trail, count = ov.dispatch()
    np.testing.assert_array_equal(lead, r.lead)
    np.testing.assert_array_equal(trail, r.trail)
    # every dispatched pair's count = the oracle's PairData count of that key
    # (wide ids list PairData sorted by (fst, snd); strict ids in Trove order)
    okey = (r.pair_fst.astype(np.uint64) << np.uint64(32)) | r.pair_snd.astype(np.uint64)
    o = np.argsort(okey, kind="stable")
    okey, ocnt = okey[o], r.pair_cnt[o]
    dkey = (lead.astype(np.uint64) << np.uint64(32)) | trail.astype(np.uint64)
    pos = np.minimum(np.searchsorted(okey, dkey), max(len(okey) - 1, 0))
    assert (okey[pos] == dkey).all()
    np.testing.assert_array_equal(count, ocnt[pos])
    if pairs:
        pf, ps, pc = ov.pairs()
        np.testing.assert_array_equal(pf, r.pair_fst)
        np.testing.assert_array_equal(ps, r.pair_snd)
        np.testing.assert_array_equal(pc, r.pair_cnt)
    al = ov.alignments()
    for name in ALIGN_CMP:
        np.testing.assert_array_equal(al[:, sao.ALIGN_FIELDS.index(name)], r.align_field(name), err_msg=name)
    flags = al[:, sao.ALIGN_FIELDS.index("flags")]
    np.testing.assert_array_equal((flags & sao.FLAG_DUD) != 0, r.align_field("is_dud") != 0)
    np.testing.assert_array_equal((flags & sao.FLAG_VALID) != 0, r.align_field("valid") != 0)
    assert ov.ovl() == r.ovl


def test_bench_workload_matches_oracle(oracle_mod):
    """configs[1] + [2] at full size: 100k x 500 bp, k = 15, wide ids."""
    b, o = bench.synth_workload(100000, 500, 2500000, 0.5, seed=1)
    ov = sao.Overlapper(kmer_size=15, id_mode=sao.SA_IDS_WIDE)
    ov.add_packed(b.tobytes(), o)
    ov.build()
    ov.align()
    st = ov.stats()
    assert st["kmers"] == 48600000 and st["dispatched"] > 600000
    r = oracle_mod.Run(packed=(b.tobytes(), o), settings=oracle_mod.default_settings(kmer_size=15), wide=True)
    compare(ov, r, pairs=False)  # dispatch, its counts, every tuple, the .ovl
    assert st["pairs"] == len(r.pair_fst)
    _, _, count = ov.dispatch()
    assert ((count >= 7) & (count <= 222)).all()
    assert st["ovl_records"] == ov.ovl().count(b"{OVL") > 100000


@pytest.mark.parametrize("k", [15, 12])
def test_mixed_100_1000_matches_oracle(oracle_mod, k):
    """configs[4]'s read shape and both of its k values: 2,000 mixed 100-1,000 bp
    reads with indels/substitutions at ~20x coverage, wide ids, every stage."""
    rng = np.random.default_rng(400 + k)
    reads = H.mutate(H.synth_reads(2000, 1000, 55000, gc=0.5, seed=500 + k, mixed=(100, 1000)), rng, 2)
    st = dict(kmer_size=k, min_collisions=7)
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(**st), wide=True)
    ov = sao.Overlapper(keep_pairs=True, id_mode=sao.SA_IDS_WIDE, **st)
    ov.add_reads(reads)
    ov.build()
    ov.align()
    assert ov.stats()["dispatched"] > 5000
    compare(ov, r)


def test_mixed_lengths_dense_buckets_match_oracle(oracle_mod):
    """configs[4]'s k = 12 pass is a bucket-density stress (~1,600 occurrences
    per 12-mer at 50M reads).  At test size the same density comes from a
    smaller k: k = 8 on 1,200 mixed 100-1,000 bp reads of a 2 Mbp genome
    (~10 random collisions per 8-mer plus the true overlaps), strict ids."""
    reads = H.synth_reads(1200, 1000, 2000000, gc=0.5, seed=808, mixed=(100, 1000))
    st = dict(kmer_size=8, min_collisions=7, max_collisions=222)
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(**st))
    ov = sao.Overlapper(keep_pairs=True, id_mode=sao.SA_IDS_STRICT, **st)
    ov.add_reads(reads)
    ov.build()
    ov.align()
    assert ov.stats()["dispatched"] > 100
    compare(ov, r)


def test_readme_record_pinned():
    """The README's sample {OVL} record is produced exactly by crp177 at the
    reference defaults (k = 12), at the place the Trove order puts it."""
    ov = sao.Overlapper()
    ov.read_fasta(H.crp177_path())
    ov.build()
    ov.align()
    out = ov.ovl()
    assert out.count(README_RECORD) == 1
    golden = open(os.path.join(H.GOLDEN, "crp177_k12.ovl"), "rb").read()
    assert out.index(README_RECORD) == golden.index(README_RECORD)


@pytest.mark.parametrize("n_edge,max_coll", [(5000, 222), (12800, 222), (110000, 222), (12800, 300),
                                            (110000, 300)])
def test_many_partner_reads_recount_tiers(oracle_mod, n_edge, max_coll):
    """Reads with thousands to >98k distinct partners (configs[4]'s k = 12
    stress in miniature): 8 reads carry a 17 bp motif in their middle region,
    n_edge reads carry it at their start, so each middle read leads a pair with
    every edge read (the 15-mers inside the motif, plus those straddling its
    edges that share their few random bases).  max_collisions 222: the packed
    32,768-slot tier (5,000 and 12,800 partners in one pass, 110,000 in residue
    classes); max_collisions 300 (counts past 8 bits matter): the two-word
    16,384-slot tier, 12,800 partners in its 8-way residue split, 110,000 in the
    64-way split (which refines only the classes that overflowed).  Dispatch
    and counts vs the oracle, wide ids."""
    rng = np.random.default_rng(n_edge)
    motif = "".join("ACGT"[x] for x in rng.integers(0, 4, 17))
    n_mid = 8
    reads = []
    for i in range(n_mid + n_edge):
        s_ = "".join("ACGT"[x] for x in rng.integers(0, 4, 120))
        p_ = 55 if i < n_mid else 5   # loc 0.52 (md) vs 0.05 (st), L - k = 105
        reads.append(s_[:p_] + motif + s_[p_ + 17:])
    st = dict(kmer_size=15, min_collisions=3, max_collisions=max_coll)
    ov = sao.Overlapper(id_mode=sao.SA_IDS_WIDE, **st)
    ov.add_reads(reads)
    ov.build()
    lead, trail, count = ov.dispatch()
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(**st), wide=True, skip_align=True)
    np.testing.assert_array_equal(lead, r.lead)
    np.testing.assert_array_equal(trail, r.trail)
    assert (lead <= n_mid).sum() == n_mid * n_edge  # every middle read leads every edge read
    assert ov.stats()["role_pairs"] > 3 * n_mid * n_edge
    # the edge reads kept their per-read regions; only the middle reads were recounted
    assert ov.stats()["flags"] & 3 == sao.SA_STATS_PER_READ_REGIONS | sao.SA_STATS_RECOUNTED
    # item lists sliced into launches of 3 workgroups (the path taken where a
    # dispatch's 32-bit work-item count would wrap: configs[4]'s 6.25M-read
    # slice in the 1,024-thread tier and its residue classes): same dispatch
    sl = sao.Overlapper(id_mode=sao.SA_IDS_WIDE, launch_slice=3, **st)
    sl.add_reads(reads)
    sl.build()
    l2, t2, c2 = sl.dispatch()
    np.testing.assert_array_equal(l2, lead)
    np.testing.assert_array_equal(t2, trail)
    np.testing.assert_array_equal(c2, count)
    sl.close()


def test_packed_tier_count_saturation(oracle_mod):
    """The packed tier's 8-bit counts: a pair that collides hundreds of times (a
    40 bp poly-A run in the middle of one read and at the start of another) must
    stay above max_collisions although its count field wraps (e.g. 729 = 2 x 256
    + 217, inside [3, 222]); the lead has 3,000 other partners,
    so it is counted in the packed 32,768-slot tier.  Dispatch and counts vs
    the oracle."""
    rng = np.random.default_rng(676)
    motif = "".join("ACGT"[x] for x in rng.integers(0, 4, 17))
    reads = []
    for i in range(8 + 3000):
        s_ = "".join("ACGT"[x] for x in rng.integers(0, 4, 120))
        p_ = 55 if i < 8 else 5
        reads.append(s_[:p_] + motif + s_[p_ + 17:])
    # a 300 bp middle read: the motif at loc 0.53, the run at locs 0.32-0.40 (md)
    s_ = "".join("ACGT"[x] for x in rng.integers(0, 4, 300))
    reads[0] = s_[:90] + "A" * 40 + s_[130:150] + motif + s_[167:]
    reads.append("A" * 40 + reads[8][40:])  # a new edge read: the run at its start
    st = dict(kmer_size=15, min_collisions=3, max_collisions=222)
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(**st), wide=True, skip_align=True)
    okey = (r.pair_fst.astype(np.int64) << 32) | r.pair_snd
    big = r.pair_cnt[np.searchsorted(okey, (1 << 32) | len(reads))]
    assert big > 255  # the wrapping pair exists in the reference's counts
    ov = sao.Overlapper(id_mode=sao.SA_IDS_WIDE, **st)
    ov.add_reads(reads)
    ov.build()
    lead, trail, count = ov.dispatch()
    np.testing.assert_array_equal(lead, r.lead)
    np.testing.assert_array_equal(trail, r.trail)
    assert ov.stats()["flags"] & sao.SA_STATS_RECOUNTED
    assert not ((lead == 1) & (trail == len(reads))).any()
    ov.close()


@pytest.mark.parametrize("shards", [4, 8])
def test_bench_workload_sharded_matches_single(shards):
    """The sharded path at the bench's full size: the 100k x 500 bp workload over
    4 and 8 virtual shards gives the single-device dispatch and .ovl exactly
    (records carry source-local occurrence indices, the occurrence table rides
    through the partition sort, multi-read pair-count blocks, owner reduce)."""
    b, o = bench.synth_workload(100000, 500, 2500000, 0.5, seed=1)
    one = sao.Overlapper(kmer_size=15, id_mode=sao.SA_IDS_WIDE)
    one.add_packed(b.tobytes(), o)
    one.build()
    one.align()
    lead, trail, count = (np.array(x) for x in one.dispatch())
    ovl = one.ovl()
    one.close()
    sh = sao.Overlapper(kmer_size=15, id_mode=sao.SA_IDS_WIDE, shards=shards)
    sh.add_packed(b.tobytes(), o)
    sh.build()
    sh.align()
    l2, t2, c2 = sh.dispatch()
    np.testing.assert_array_equal(l2, lead)
    np.testing.assert_array_equal(t2, trail)
    np.testing.assert_array_equal(c2, count)
    assert sh.ovl() == ovl


@pytest.mark.parametrize("min_len", [None, 300])
def test_per_read_regions_match_shared_regions(min_len):
    """Dispatched pairs written into per-read regions (one scan + one copy, no
    sort; wide ids, keep_pairs off) equal the shared-region path's dispatch
    (every distinct pair kept, radix-sorted), for uniform and mixed lengths."""
    b, o = bench.synth_workload(20000, 500, 500000, 0.5, seed=3, min_len=min_len)
    out = []
    for kp in (False, True):
        ov = sao.Overlapper(kmer_size=15, id_mode=sao.SA_IDS_WIDE, keep_pairs=kp)
        ov.add_packed(b.tobytes(), o)
        ov.build()
        out.append([np.array(x) for x in ov.dispatch()])
        # the per-read mode really ran (and only without keep_pairs)
        assert bool(ov.stats()["flags"] & sao.SA_STATS_PER_READ_REGIONS) == (not kp)
        ov.close()
    assert len(out[0][0]) > 10000
    for x, y in zip(*out):
        np.testing.assert_array_equal(x, y)


def test_per_read_regions_with_recounted_reads_twice():
    """A read set where some reads overflow the first pass's table (> 192
    partners): 20k ordinary reads plus 1,200 reads sharing a motif (40 middle
    reads x 1,160 edge reads, so each middle read has > 1,000 partners).  Only
    the overflowed reads are recounted (their pairs sorted into the shared
    list), the rest keep their per-read regions; built twice on one context,
    both dispatches equal the keep_pairs (shared-region, sorted) path."""
    b, o = bench.synth_workload(20000, 500, 500000, 0.5, seed=5)
    reads = [b[int(o[i]):int(o[i + 1])].tobytes().decode() for i in range(len(o) - 1)]
    rng = np.random.default_rng(7)
    motif = "".join("ACGT"[x] for x in rng.integers(0, 4, 17))
    for i in range(1200):
        s_ = "".join("ACGT"[x] for x in rng.integers(0, 4, 120))
        p_ = 55 if i < 40 else 5
        reads.append(s_[:p_] + motif + s_[p_ + 17:])
    st = dict(kmer_size=15, min_collisions=3, id_mode=sao.SA_IDS_WIDE)
    ref = sao.Overlapper(keep_pairs=True, **st)
    ref.add_reads(reads)
    ref.build()
    want = [np.array(x) for x in ref.dispatch()]
    assert not ref.stats()["flags"] & sao.SA_STATS_PER_READ_REGIONS
    ref.close()
    ov = sao.Overlapper(**st)
    ov.add_reads(reads)
    for _ in range(2):
        ov.build()
        assert ov.stats()["flags"] & 3 == sao.SA_STATS_PER_READ_REGIONS | sao.SA_STATS_RECOUNTED
        got = [np.array(x) for x in ov.dispatch()]
        for x, y in zip(got, want):
            np.testing.assert_array_equal(x, y)
    assert len(want[0]) > 40 * 1000
    ov.close()
