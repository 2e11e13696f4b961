"""Sharded contexts through the C ABI (SURVEY.md 8(b) `--gpus P`, 8(e)).  GPU only.

A sharded context splits the read ids into P ranges, exchanges k-mer records
and partial pair counts between shards and all-gathers the packed reads for
alignment -- all inside libsa_overlap (multi.cpp).  On one MI355X the shards are
virtual (exchanges are device copies) or a one-rank RCCL communicator (the RCCL
send/recv path to self); the bar is the single-device output, bit for bit,
for any P: dispatch, alignment tuples and .ovl bytes.
"""
import os
import subprocess

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

sao = pytest.importorskip("saoverlap")

CLI = os.path.join(os.path.dirname(sao.__file__), "build", "sa-overlap")


def run(reads, build_twice=False, **kw):
    ov = sao.Overlapper(**kw)
    ov.add_reads(reads)
    ov.build()
    if build_twice:
        ov.build()  # buffers reused, shards keep their reads
    ov.align()
    return ov


def assert_same(a, b):
    for x, y in zip(a.dispatch(), b.dispatch()):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a.alignments(), b.alignments())
    assert a.ovl() == b.ovl()
    sa, sb = a.stats(), b.stats()
    for k in ("kmers", "buckets", "role_pairs", "pairs", "dispatched", "aligned", "ovl_records", "dp_cells"):
        assert sa[k] == sb[k], k


def workload(seed, repeat=False):
    rng = np.random.default_rng(seed)
    reads = H.mutate(H.synth_reads(1500, 300, 20000, gc=0.5, seed=seed, mixed=(250, 340)), rng, 3)
    st = dict(kmer_size=15, min_collisions=5, id_mode=sao.SA_IDS_WIDE)
    if repeat:  # a 15-mer in 2,400 reads: multi-read pair-count blocks overflow and recount;
        # in 5,000 (repeat="big"): a partition past 4,096 records on its owner shard -- the
        # first pair-count pass aborts and the global bucket path runs (bucket_stage phase 2)
        motif = "ACGTTGCAACGTAGC"
        for i in range(5000 if repeat == "big" else 2400):
            s_ = "".join("ACGT"[x] for x in rng.integers(0, 4, 120))
            p_ = 5 if i % 2 == 0 else 55
            reads.append(s_[:p_] + motif + s_[p_ + 15:])
        st["min_collisions"] = 2
    return reads, st


@pytest.mark.parametrize("P,repeat", [(2, False), (4, False), (8, False), (4, True), (4, "big")])
def test_virtual_shards_match_single_gpu(P, repeat):
    reads, st = workload(90 + P, repeat)
    ref = run(reads, **st)
    assert ref.stats()["dispatched"] > 1000
    got = run(reads, shards=P, build_twice=True, **st)
    assert_same(got, ref)
    # the exchanges moved data between shards
    assert got.exchanged_bytes() > 0


@pytest.mark.parametrize("P,repeat,lean", [(4, False, False), (8, False, True), (4, "big", True)])
def test_virtual_shards_lead_range_passes(P, repeat, lean):
    """A 1 MiB partial budget (87k entries per shard and pass; the shards' bound
    is several times that) makes the sharded count run in lead-range passes:
    buckets built once, then per pass every shard counts the partials of 1/npass
    of every owner's leads, exchange 2 and the reduce append that slice of the
    dispatch.  Output = the single device's, bit for bit (dispatch, alignments,
    .ovl, stats), with and without SA_OPT_LEAN_MEMORY (scratch freed between
    stages), twice on one context."""
    reads, st = workload(110 + P, repeat)
    ref = run(reads, **st)
    got = run(reads, shards=P, build_twice=True, pass_budget_mb=1, lean_memory=lean, **st)
    info = got.shard_info()
    assert info["npass"] > 2 and info["bound"] > 3 * 87381, info
    assert info["partials"] >= ref.stats()["pairs"]  # every distinct pair met on >= 1 shard
    assert_same(got, ref)


def test_first_pass_modes_with_big_partition(oracle_mod):
    """One device, a 15-mer in 5,000 reads (a partition past 4,096 records: the
    global bucket path, bucket_stage phase 2): the pair counter's first pass run
    (SA_OPT_FIRST_PASS = 1), skipped (2) and probed (0) give the oracle's
    dispatch.  The skip mode must wait for the global path like the first pass
    does (it used to count from records not yet written)."""
    reads, st = workload(96, "big")
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(
        kmer_size=st["kmer_size"], min_collisions=st["min_collisions"]), wide=True, skip_align=True)
    outs = []
    for mode in (1, 2, 0):
        ov = sao.Overlapper(first_pass=mode, **st)
        ov.add_reads(reads)
        ov.build()
        lead, trail, _ = ov.dispatch()
        np.testing.assert_array_equal(lead, r.lead)
        np.testing.assert_array_equal(trail, r.trail)
        outs.append(ov.stats())
        ov.close()
    for s in outs[1:]:
        for k in ("kmers", "buckets", "role_pairs", "pairs", "dispatched"):
            assert s[k] == outs[0][k], k


def test_virtual_shards_device_only_path():
    """sa_device_build / sa_device_align on a sharded context, results fetched after."""
    reads, st = workload(97)
    ref = run(reads, **st)
    ov = sao.Overlapper(shards=4, timing=True, **st)
    ov.add_reads(reads)
    for _ in range(2):
        ov.device_build()
        ov.device_align()
    for x, y in zip(ov.dispatch(), ref.dispatch()):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(ov.alignments(), ref.alignments())
    t = ov.stage_times()
    assert t["exchange"][1] > 0 and t["pairs"][1] >= 2


def test_virtual_shards_reads_added_later():
    """Reads added after a build are re-split over the shards."""
    reads, st = workload(98)
    ov = sao.Overlapper(shards=2, **st)
    ov.add_reads(reads[:700])
    ov.build()
    ov.add_reads(reads[700:])
    ov.build()
    ov.align()
    assert_same(ov, run(reads, **st))


def test_sharded_strict_inputs_run_unsharded():
    """crp177 (the reference's own id domain): a 4-shard context reproduces the
    golden .ovl, Trove order included."""
    ov = sao.Overlapper(shards=4, kmer_size=12)
    ov.read_fasta(H.crp177_path())
    ov.build()
    ov.align()
    assert ov.stats()["id_mode"] == sao.SA_IDS_STRICT
    assert ov.ovl() == open(os.path.join(H.GOLDEN, "crp177_k12.ovl"), "rb").read()


def test_rank_mode_one_rank_rccl(tmp_path):
    """sa_ctx_create_rank with one rank: every exchange is an RCCL send/recv to
    self, so the RCCL code path (group calls, stream hand-off, count exchange,
    length all-gather, .ovl gather to rank 0) runs on the one GPU."""
    reads, st = workload(99)
    ref = run(reads, **st)
    uid = sao.rccl_unique_id()
    ov = sao.Overlapper(rank=0, nranks=1, rccl_id=uid, **st)
    ov.add_reads(reads)
    ov.build()
    # the collective writer fails on every rank (here: the only one) when a
    # rank has not aligned, instead of blocking in the gather
    with pytest.raises(sao.SAError) as ei:
        ov.write_ovl(str(tmp_path / "none.ovl"))
    assert ei.value.name == "SA_E_STATE"
    ov.build()
    ov.align()
    assert_same(ov, ref)
    path = str(tmp_path / "r.ovl")
    ov.write_ovl(path)
    assert open(path, "rb").read() == ref.ovl()
    # after a device-only align the writer formats this run's records (not
    # an earlier run's, and not an empty file)
    ov.device_align()
    path2 = str(tmp_path / "r2.ovl")
    ov.write_ovl(path2)
    assert open(path2, "rb").read() == ref.ovl()


def test_rank_mode_lead_range_passes():
    """One-rank RCCL context in lead-range passes: the pass count is agreed over
    RCCL (every rank's plan, the max) and every pass's partials go through the
    RCCL exchange to self."""
    reads, st = workload(105)
    ref = run(reads, **st)
    ov = sao.Overlapper(rank=0, nranks=1, rccl_id=sao.rccl_unique_id(), pass_budget_mb=1, **st)
    ov.add_reads(reads)
    ov.build()
    ov.align()
    assert ov.shard_info()["npass"] > 2
    assert_same(ov, ref)


@pytest.mark.parametrize("shards", [1, 4])
def test_device_align_then_results(shards):
    """sa_device_align leaves the records on the device; the getters read them
    back on first use and never return a previous run's (the quadratic
    aligner run in between gives different alignments)."""
    reads, st = workload(101)
    ov = sao.Overlapper(shards=shards, **st) if shards > 1 else sao.Overlapper(**st)
    ov.add_reads(reads)
    ov.build()
    ov.align()
    want_aln, want_ovl = ov.alignments(), ov.ovl()
    ov.set_aligner(sao.SA_ALIGNER_QUADRATIC)
    ov.align()
    quad_ovl = ov.ovl()
    ov.set_aligner(sao.SA_ALIGNER_LINEAR)
    ov.device_align()
    assert ov.ovl() == want_ovl
    np.testing.assert_array_equal(ov.alignments(), want_aln)
    assert ov.stats()["ovl_records"] == want_ovl.count(b"{OVL")
    assert len(quad_ovl) > 0


def test_multi_gpu_context_if_available():
    """gpus=2 (RCCL between devices 0 and 1) where the box has them."""
    reads, st = workload(100)
    try:
        ov = sao.Overlapper(gpus=2, **st)
    except sao.SAError as e:
        if e.name in ("SA_E_HIP", "SA_E_RCCL"):
            pytest.skip("one GPU on this box")
        raise
    ov.add_reads(reads)
    ov.build()
    ov.align()
    assert_same(ov, run(reads, **st))


def test_cli_shards_match_single(tmp_path):
    """`sa-overlap --shards 4` (and `--gpus 1`) writes the single-device bytes."""
    reads, _ = workload(101)
    fa = tmp_path / "reads.seq"
    fa.write_bytes(H.reads_fasta_bytes(reads))
    outs = []
    for extra in ([], ["--shards", "4"], ["--gpus", "1", "--shards", "2"]):
        o = tmp_path / ("o%d.ovl" % len(outs))
        r = subprocess.run([CLI, "-i", str(fa), "-o", str(o), "-k", "15", "--min-collisions", "5", "--wide-ids"]
                           + extra, capture_output=True, timeout=120)
        assert r.returncode == 0, r.stderr
        outs.append(o.read_bytes())
    assert outs[0].count(b"{OVL") > 100
    assert outs[1] == outs[0] and outs[2] == outs[0]
