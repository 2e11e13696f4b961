"""The 8-GPU configs at their per-rank sizes, against the oracle.  GPU only.

configs[3] (8 GPUs, 10M x 500 bp, k = 15) and configs[4] (8 GPUs, 50M mixed
100-1,000 bp reads, k = 12 and k = 15) run the SHARDED path (multi.cpp +
dist.hip): every rank sends its k-mer records to the hash-range owner,
receives ~1/P of all records (607.5M at configs[3]), counts partial pairs and
reduces its leads' partials (Project4.scala:531-563, KmerTable.scala:85-187).

* configs[3] per rank: 2 virtual shards x 1.25M x 500 bp reads (2.5M reads,
  62.5 Mbp genome at 20x) -- each shard receives a configs[3] rank's records --
  and the same 2.5M reads on 8 virtual shards (the 8-way plan at large
  counts).  Both against the all-core oracle (orc_run_wide_mt, itself
  CPU-tested equal to the single-threaded restatement): dispatch element by
  element, every dispatched pair's count, role-pair / distinct-pair totals,
  20,000 sampled alignments.  The 2-shard run's per-shard stage times are the
  first measurement of what a configs[3] rank does (SA_TEST_RECORD_DIR).
* configs[4]-shaped mixed lengths at k = 15 on 2 shards x 500k reads:
  test_gpu_slices.py (same oracle as its single-device check).
* configs[4]'s whole per-GPU slice, 6.25M mixed reads, at k = 12 and k = 15
  on one device: its PairData (1.5e11 distinct pairs at k = 12) does not fit
  host memory, so the checker is the sampled-lead oracle (orc_lead_rows,
  CPU-tested equal to the full restatement): ~2,000 leads' rows of PairData,
  filtered by [minCollisions, maxCollisions], against the device's dispatch
  rows of those leads, counts included; the whole dispatch's order (lead
  descending, trail ascending) is checked too.
"""
import json
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


def record(name, obj):
    d = os.environ.get("SA_TEST_RECORD_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".json"), "w") as f:
            json.dump(obj, f, indent=1)


class OracleRef:
    """The all-core oracle's PairData + dispatch for one read set, and its
    alignments of a fixed sample of the dispatch."""

    def __init__(self, oracle_mod, bases, o, k):
        t0 = time.time()
        self.settings = oracle_mod.default_settings(kmer_size=k)
        r = oracle_mod.Run(packed=(bases, o), settings=self.settings, wide=True, skip_align=True, threads=0)
        self.role_pairs, self.n_pairs = r.role_pairs, len(r.pair_fst)
        self.lead, self.trail = r.lead, r.trail
        okey = (r.pair_fst.astype(np.uint64) << np.uint64(32)) | r.pair_snd.astype(np.uint64)
        dkey = (self.lead.astype(np.uint64) << np.uint64(32)) | self.trail.astype(np.uint64)
        pos = np.searchsorted(okey, dkey)
        assert (okey[np.minimum(pos, len(okey) - 1)] == dkey).all()
        self.count = r.pair_cnt[pos]
        del okey, dkey, pos, r
        nd = len(self.lead)
        self.idx = np.unique(np.linspace(0, nd - 1, min(SAMPLE, nd)).astype(np.int64))
        self.aligns = oracle_mod.align_batch(bases, o, self.lead[self.idx], self.trail[self.idx],
                                             settings=self.settings, threads=0)
        self.oracle_mod = oracle_mod
        self.seconds = time.time() - t0

    def check(self, ov, st):
        assert st["role_pairs"] == self.role_pairs
        assert st["pairs"] == self.n_pairs
        lead, trail, count = ov.dispatch()
        np.testing.assert_array_equal(lead, self.lead)
        np.testing.assert_array_equal(trail, self.trail)
        np.testing.assert_array_equal(count, self.count)
        al = ov.alignments()
        om = self.oracle_mod
        for name in ALIGN_CMP:
            np.testing.assert_array_equal(al[self.idx, sao.ALIGN_FIELDS.index(name)],
                                          self.aligns[:, om.ALIGN_FIELDS.index(name)], err_msg=name)
        flags = al[self.idx, sao.ALIGN_FIELDS.index("flags")]
        np.testing.assert_array_equal((flags & sao.FLAG_DUD) != 0, self.aligns[:, om.ALIGN_FIELDS.index("is_dud")] != 0)
        np.testing.assert_array_equal((flags & sao.FLAG_VALID) != 0, self.aligns[:, om.ALIGN_FIELDS.index("valid")] != 0)


def run_sharded(bases, o, k, shards, timed_builds=0):
    """Build + align on `shards` virtual shards of one GPU; with timed_builds,
    that many more builds run one shard at a time (SA_OPT_SERIAL_SHARDS) with
    stage timing, so each stage time is one shard's."""
    ov = sao.Overlapper(shards=shards, kmer_size=k, id_mode=sao.SA_IDS_WIDE)
    ov.add_packed(bases, o)
    t0 = time.time()
    ov.device_build()
    first_build_s = time.time() - t0
    ov.device_align()
    st = ov.stats()
    times = None
    if timed_builds:
        ov.set_timing(True)
        ov._chk(sao.lib().sa_set_option(ov.h, sao.SA_OPT_SERIAL_SHARDS, 1))
        ov.device_build()  # warm, serial
        ov.reset_stage_times()
        for _ in range(timed_builds):
            ov.device_build()
        t = ov.stage_times()
        times = {s: round(ms / max(timed_builds, 1), 3) for s, (ms, n) in t.items() if n}
        ov._chk(sao.lib().sa_set_option(ov.h, sao.SA_OPT_SERIAL_SHARDS, 0))
        ov.set_timing(False)
        ov.device_build()
        ov.device_align()
        assert ov.stats()["dispatched"] == st["dispatched"]
    return ov, st, first_build_s, times


@pytest.fixture(scope="module")
def c3_rank_reads():
    n = 2500000
    b, o = bench.synth_workload(n, 500, n * 500 // 20, 0.5, seed=1)
    return b.tobytes(), o


@pytest.fixture(scope="module")
def c3_rank_oracle(oracle_mod, c3_rank_reads):
    bases, o = c3_rank_reads
    return OracleRef(oracle_mod, bases, o, 15)


def test_configs3_rank_size_two_shards_match_oracle(c3_rank_reads, c3_rank_oracle):
    """2 virtual shards x 1.25M x 500 bp: each shard receives a configs[3]
    rank's ~607.5M records and reduces ~half of the partials."""
    bases, o = c3_rank_reads
    ov, st, first_s, times = run_sharded(bases, o, 15, 2, timed_builds=2)
    ref = c3_rank_oracle
    assert st["kmers"] == 2500000 * 486
    ref.check(ov, st)
    xb = ov.exchanged_bytes()
    ov.close()
    print("c3 rank size, 2 shards: %d dispatched; first build %.1f s; per-shard stages %s; oracle %.1f s"
          % (st["dispatched"], first_s, times, ref.seconds))
    record("c3_rank_2shards", {"reads": 2500000, "read_len": 500, "k": 15, "shards": 2,
                               "records_per_shard": st["kmers"] // 2, "stats": st, "first_build_s": first_s,
                               "per_shard_stage_ms": times, "exchanged_bytes_total": xb,
                               "note": "stage ms = one shard (serial shards, mean of 2 timed builds)"})


def test_configs3_reads_eight_shards_match_oracle(c3_rank_reads, c3_rank_oracle):
    """The same 2.5M reads on 8 virtual shards (312.5k reads each)."""
    bases, o = c3_rank_reads
    ov, st, first_s, _ = run_sharded(bases, o, 15, 8)
    c3_rank_oracle.check(ov, st)
    ov.close()


# ---------------------------------------------------------------------------
# configs[4]'s whole per-GPU slice, sampled-lead oracle
# ---------------------------------------------------------------------------
C4_N = 6250000


@pytest.fixture(scope="module")
def c4_slice_reads():
    b, o = bench.synth_workload(C4_N, 1000, int(C4_N * 550 / 20.0), 0.5, seed=1, min_len=100)
    return b.tobytes(), o


def sampled_leads(n, lens, count=2000, seed=5):
    rng = np.random.default_rng(seed)
    longest = np.argsort(lens, kind="stable")[-8:] + 1
    shortest = np.argsort(lens, kind="stable")[:8] + 1
    return np.unique(np.concatenate([[1, 2, n - 1, n], rng.integers(1, n + 1, count), longest, shortest])).astype(np.int32)


@pytest.mark.parametrize("k", [15, 12])
def test_configs4_full_slice_sampled_leads(oracle_mod, c4_slice_reads, k):
    bases, o = c4_slice_reads
    lens = np.diff(o.astype(np.int64))
    t0 = time.time()
    ov = sao.Overlapper(kmer_size=k, id_mode=sao.SA_IDS_WIDE)
    ov.add_packed(bases, o)
    ov.device_build()
    st = ov.stats()
    lead, trail, count = ov.dispatch()
    ov.close()
    t_gpu = time.time() - t0
    assert st["kmers"] == int((lens - k + 1).clip(0).sum())
    # the whole dispatch is in the wide order: lead descending, trail ascending
    dl = np.diff(lead.astype(np.int64))
    assert (dl <= 0).all()
    assert (np.diff(trail.astype(np.int64))[dl == 0] > 0).all()
    assert len(lead) == st["dispatched"]
    leads = sampled_leads(C4_N, lens)
    t0 = time.time()
    s = oracle_mod.default_settings(kmer_size=k)
    ro, snd, cnt = oracle_mod.lead_rows(bases, o, leads, settings=s, threads=0)
    t_orc = time.time() - t0
    keep = (cnt >= s.min_collisions) & (cnt <= s.max_collisions)
    want_lead = np.repeat(leads, np.diff(ro))[keep]
    want_trail, want_cnt = snd[keep], cnt[keep]
    # the device's rows of the sampled leads, leads ascending (dispatch is descending)
    neg = -lead.astype(np.int64)
    lo = np.searchsorted(neg, -leads.astype(np.int64), "left")
    hi = np.searchsorted(neg, -leads.astype(np.int64), "right")
    sel = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)])
    np.testing.assert_array_equal(lead[sel], want_lead)
    np.testing.assert_array_equal(trail[sel], want_trail)
    np.testing.assert_array_equal(count[sel], want_cnt)
    print("configs[4] slice k=%d: %d k-mers, %d pairs, %d dispatched; %d sampled leads, %d of their PairData rows, "
          "%d dispatched rows; device %.1f s, sampled oracle %.1f s"
          % (k, st["kmers"], st["pairs"], st["dispatched"], len(leads), len(snd), len(sel), t_gpu, t_orc))
    assert len(sel) > 1000 and len(snd) > len(sel)
    record("c4_slice_k%d_sampled" % k, {"reads": C4_N, "k": k, "stats": st, "sampled_leads": int(len(leads)),
                                       "pairdata_rows": int(len(snd)), "dispatched_rows": int(len(sel)),
                                       "device_s": t_gpu, "oracle_s": t_orc})


# ---------------------------------------------------------------------------
# the dense path: first pass skipped, early-stopped big-tier reads
# ---------------------------------------------------------------------------
def test_dense_first_pass_modes_match_sampled_oracle(oracle_mod):
    """300k mixed 100-1,000 bp reads at k = 10 (a 1M hash space: buckets of
    ~150 occurrences, ~20-50k distinct partners per read -- past the 32,768-
    slot tier's 24,576, so reads stop early and go to partner classes).  The
    first pass run (SA_OPT_FIRST_PASS = 1), skipped (2) and left to the probe
    (0) give the same dispatch and stats, and the sampled leads' rows equal the
    oracle's PairData rows."""
    n, k = 300000, 10
    b, o = bench.synth_workload(n, 1000, int(n * 550 / 20.0), 0.5, seed=3, min_len=100)
    bases = b.tobytes()
    del b
    outs = []
    for mode in (1, 2, 0):
        ov = sao.Overlapper(kmer_size=k, id_mode=sao.SA_IDS_WIDE, first_pass=mode)
        ov.add_packed(bases, o)
        ov.device_build()
        st = ov.stats()
        outs.append((st, ov.dispatch()))
        ov.close()
    for st, d in outs[1:]:
        for key in ("kmers", "buckets", "role_pairs", "pairs", "dispatched"):
            assert st[key] == outs[0][0][key], key
        for x, y in zip(d, outs[0][1]):
            np.testing.assert_array_equal(x, y)
    st, (lead, trail, count) = outs[0]
    assert st["flags"] & sao.SA_STATS_RECOUNTED and st["pairs"] > 2000 * n
    leads = sampled_leads(n, np.diff(o.astype(np.int64)), count=1500, seed=7)
    s = oracle_mod.default_settings(kmer_size=k)
    ro, snd, cnt = oracle_mod.lead_rows(bases, o, leads, settings=s, threads=0)
    keep = (cnt >= s.min_collisions) & (cnt <= s.max_collisions)
    neg = -lead.astype(np.int64)
    lo = np.searchsorted(neg, -leads.astype(np.int64), "left")
    hi = np.searchsorted(neg, -leads.astype(np.int64), "right")
    sel = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)])
    np.testing.assert_array_equal(lead[sel], np.repeat(leads, np.diff(ro))[keep])
    np.testing.assert_array_equal(trail[sel], snd[keep])
    np.testing.assert_array_equal(count[sel], cnt[keep])
    # the sampled leads' distinct partners bound the device's distinct total from below
    print("dense k=10: %d pairs, %d dispatched; sampled leads %d rows (max %d partners)"
          % (st["pairs"], st["dispatched"], len(snd), int(np.diff(ro).max())))
    assert int(np.diff(ro).max()) > 24576  # some sampled lead is past one big table


# ---------------------------------------------------------------------------
# round 6: the 8-GPU configs at their REAL density
# ---------------------------------------------------------------------------
def sampled_rows_check(oracle_mod, bases, o, k, lead, trail, count, leads):
    """The dispatch rows of the sampled leads equal the oracle's PairData rows of
    those leads filtered by [7, 222]; the whole dispatch is lead-descending,
    trail-ascending.  Returns (PairData rows, dispatched rows) of the sample."""
    dl = np.diff(lead.astype(np.int64))
    assert (dl <= 0).all()
    assert (np.diff(trail.astype(np.int64))[dl == 0] > 0).all()
    s = oracle_mod.default_settings(kmer_size=k)
    ro, snd, cnt = oracle_mod.lead_rows(bases, o, leads, settings=s, threads=0)
    keep = (cnt >= s.min_collisions) & (cnt <= s.max_collisions)
    neg = -lead.astype(np.int64)
    lo = np.searchsorted(neg, -leads.astype(np.int64), "left")
    hi = np.searchsorted(neg, -leads.astype(np.int64), "right")
    sel = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)])
    np.testing.assert_array_equal(lead[sel], np.repeat(leads, np.diff(ro))[keep])
    np.testing.assert_array_equal(trail[sel], snd[keep])
    np.testing.assert_array_equal(count[sel], cnt[keep])
    return len(snd), sel


def test_configs3_real_density_eight_shards(oracle_mod):
    """configs[3]'s actual read set on one MI355X: 10M x 500 bp from a 250 Mbp
    genome (seed 4, 20x; 4.86e9 k-mers), k = 15, over 8 virtual shards -- each
    shard receives a configs[3] rank's 607.5M records at the config's own k-mer
    density (~1.3 random genomic occurrences per 15-mer code x 20x coverage).
    The shards run one after another with SA_OPT_LEAN_MEMORY (8 shards' bucket
    structures stay resident; sort and exchange scratch is freed between stages)
    and the count runs in lead-range passes sized from the free memory.  Checked:
    ~2,000 sampled leads' dispatch rows and counts against the oracle's PairData
    rows (orc_lead_rows), the dispatch order, the k-mer total, the sampled
    leads' alignments against orc_align_batch, and the partials the shards
    exchanged against the oracle's projection of the same read set
    (orc_lead_stats, tools/project_partials.py)."""
    n, G = 10_000_000, 250_000_000
    b, o = bench.synth_workload(n, 500, G, 0.5, seed=4)
    bases = b.tobytes()
    del b
    t0 = time.time()
    ov = sao.Overlapper(shards=8, kmer_size=15, id_mode=sao.SA_IDS_WIDE, serial_shards=True, lean_memory=True,
                        timing=True)
    ov.add_packed(bases, o)
    ov.device_build()
    t_first = time.time() - t0
    st = ov.stats()
    info = ov.shard_info()
    xb = ov.exchanged_bytes()
    # a second build, timed per shard (serial shards: each stage time is one shard's)
    ov.reset_stage_times()
    t0 = time.time()
    ov.device_build()
    t_second = time.time() - t0
    times = {s: round(ms, 3) for s, (ms, nl) in ov.stage_times().items() if nl}
    assert ov.stats()["dispatched"] == st["dispatched"]
    lead, trail, count = ov.dispatch()
    assert st["kmers"] == n * 486 and len(lead) == st["dispatched"]
    leads = sampled_leads(n, np.full(n, 500))
    t0 = time.time()
    rows, sel = sampled_rows_check(oracle_mod, bases, o, 15, lead, trail, count, leads)
    t_orc = time.time() - t0
    # the sampled leads' alignments (device) against the oracle's
    ov.device_align()
    al = ov.alignments()[sel]
    s = oracle_mod.default_settings(kmer_size=15)
    ref = oracle_mod.align_batch(bases, o, lead[sel], trail[sel], settings=s, threads=0)
    for name in ALIGN_CMP:
        np.testing.assert_array_equal(al[:, sao.ALIGN_FIELDS.index(name)], ref[:, oracle_mod.ALIGN_FIELDS.index(name)],
                                      err_msg=name)
    ov.close()
    # the projection's estimate of the same read set's partials (sampled leads, oracle)
    starts = bench.synth_layout(n, 500, G, 4)[0]
    proj = oracle_mod.lead_stats(oracle_mod.synth_genome(4, G, 0.5), starts, np.full(n, 500, np.int32), leads,
                                 settings=s, threads=0, log_ranks=3)
    est = proj[:, 2].mean() * n
    print("configs[3] real density, 8 shards: %d dispatched, %d passes, partials %d (projected %.4g), bound %d; "
          "first build %.1f s, second %.1f s; per-shard stages %s; sampled %d leads / %d rows / %d dispatched; "
          "oracle %.1f s" % (st["dispatched"], info["npass"], info["partials"], est, info["bound"], t_first, t_second,
                             times, len(leads), rows, len(sel), t_orc))
    assert abs(info["partials"] / est - 1) < 0.05
    assert len(sel) > 5000 and rows > len(sel)
    record("c3_real_density_8shards", {
        "reads": n, "read_len": 500, "genome_bp": G, "seed": 4, "k": 15, "shards": 8, "stats": st,
        "npass": info["npass"], "partials_total": info["partials"], "partials_per_shard": info["partials"] / 8,
        "partial_bound_total": info["bound"], "partials_projected_by_oracle": est,
        "exchanged_bytes_first_build": xb, "first_build_s": t_first, "second_build_s": t_second,
        "per_shard_stage_ms": times, "sampled_leads": int(len(leads)),
        "sampled_pairdata_rows": rows, "sampled_dispatched_rows": int(len(sel)),
        "note": "serial virtual shards, SA_OPT_LEAN_MEMORY, pass budget from free memory; stage times: per "
                "stage the slowest shard of the second build, summed over its passes (exchange: the host "
                "wall clock of every exchange)"})


def test_configs4_shape_k12_eight_shards_in_passes(oracle_mod):
    """configs[4]'s k = 12 pass on the sharded path (SA_E_NOMEM in round 5 from
    1M reads: every distinct partial was held at once): 1M mixed 100-1,000 bp
    reads, 8 virtual shards, the count in lead-range passes sized from the free
    memory.  The dispatch equals the single device's element for element, and
    the sampled leads' rows equal the oracle's PairData rows."""
    n, k = 1_000_000, 12
    b, o = bench.synth_workload(n, 1000, int(n * 550 / 20.0), 0.5, seed=12, min_len=100)
    bases = b.tobytes()
    del b
    one = sao.Overlapper(kmer_size=k, id_mode=sao.SA_IDS_WIDE)
    one.add_packed(bases, o)
    one.build()
    ref = one.dispatch()
    rst = one.stats()
    one.close()
    t0 = time.time()
    ov = sao.Overlapper(shards=8, kmer_size=k, id_mode=sao.SA_IDS_WIDE)
    ov.add_packed(bases, o)
    ov.build()
    t_sh = time.time() - t0
    st, info = ov.stats(), ov.shard_info()
    got = ov.dispatch()
    ov.close()
    for x, y in zip(got, ref):
        np.testing.assert_array_equal(x, y)
    for key in ("kmers", "role_pairs", "pairs", "dispatched"):
        assert st[key] == rst[key], key
    leads = sampled_leads(n, np.diff(o.astype(np.int64)), count=800, seed=9)
    rows, sel = sampled_rows_check(oracle_mod, bases, o, k, *got, leads)
    print("configs[4] shape k=12, 1M reads, 8 shards: %d passes, partials %d (bound %d), distinct %d, dispatched %d; "
          "sharded build %.1f s; sampled %d rows / %d dispatched" % (info["npass"], info["partials"], info["bound"],
                                                                    st["pairs"], st["dispatched"], t_sh, rows, len(sel)))
    assert info["partials"] > st["pairs"]
    record("c4shape_k12_1M_8shards", {"reads": n, "k": k, "shards": 8, "stats": st, "shard_info": info,
                                      "sharded_build_s": t_sh, "sampled_rows": rows, "sampled_dispatched": int(len(sel))})
