"""HIP path vs the oracle, through the C ABI (libsa_overlap.so).  GPU only.

Bar: candidate pairs, dispatch order and the .ovl are bit-exact;
alignment tuples (start, end, c, e, flags, ahg, bhg) are bit-exact.  STRICT ids
(< 32,768 reads) reproduce the reference's Trove order; WIDE ids use the
canonical order (lead descending, trail ascending) defined in DESIGN.md.
"""
import os

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

sao = pytest.importorskip("saoverlap")

ALIGN_CMP = ("start_i", "start_j", "end_i", "end_j", "correct", "error", "ahg", "bhg")


def gpu_run(reads=None, fasta=None, wide=False, keep_pairs=True, **kw):
    ov = sao.Overlapper(keep_pairs=keep_pairs, id_mode=sao.SA_IDS_WIDE if wide else sao.SA_IDS_STRICT, **kw)
    if fasta:
        ov.read_fasta(fasta)
    else:
        ov.add_reads(reads)
    ov.build()
    ov.align()
    return ov


def oracle_settings(oracle_mod, **kw):
    return oracle_mod.default_settings(**kw)


def compare_with_oracle(oracle_mod, ov, r, wide):
    lead, trail, count = ov.dispatch()
    np.testing.assert_array_equal(lead, r.lead)
    np.testing.assert_array_equal(trail, r.trail)
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
    np.testing.assert_array_equal((flags & sao.FLAG_OVL_VALID) != 0,
                                  (r.align_field("ovl_valid") != 0) & (r.align_field("valid") != 0))
    assert ov.ovl() == r.ovl


@pytest.mark.parametrize("k", [12, 15])
def test_crp177_strict_golden(k):
    """crp177 against the Scala-literal golden vectors: .ovl, PairData and dispatch order."""
    g = np.load(os.path.join(H.GOLDEN, "crp177_k%d.npz" % k))
    ov = gpu_run(fasta=H.crp177_path(), kmer_size=k)
    assert ov.ovl() == open(os.path.join(H.GOLDEN, "crp177_k%d.ovl" % k), "rb").read()
    lead, trail, _ = ov.dispatch()
    np.testing.assert_array_equal(lead, g["lead"])
    np.testing.assert_array_equal(trail, g["trail"])
    pf, ps, pc = ov.pairs()
    np.testing.assert_array_equal(pf, g["pair_fst"])
    np.testing.assert_array_equal(ps, g["pair_snd"])
    np.testing.assert_array_equal(pc, g["pair_cnt"])
    st = ov.stats()
    assert st["id_mode"] == sao.SA_IDS_STRICT


@pytest.mark.parametrize("k", [12, 15])
def test_crp177_wide_matches_oracle(oracle_mod, k):
    r = oracle_mod.Run(fasta=H.crp177_path(), settings=oracle_settings(oracle_mod, kmer_size=k), wide=True)
    ov = gpu_run(fasta=H.crp177_path(), kmer_size=k, wide=True)
    compare_with_oracle(oracle_mod, ov, r, True)


@pytest.mark.parametrize("k", [15, 12])
def test_c_ruddii_strict_bit_exact(oracle_mod, k):
    """The reference's large data set (32,000 reads rebuilt from the AMOS bank)."""
    reads = H.c_ruddii_reads()
    r = oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, kmer_size=k))
    ov = gpu_run(reads=reads, kmer_size=k)
    compare_with_oracle(oracle_mod, ov, r, False)
    st = ov.stats()
    assert st["kmers"] == 32000 * (100 - k + 1)


def test_c_ruddii_wide_matches_oracle(oracle_mod):
    reads = H.c_ruddii_reads()
    r = oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, kmer_size=15), wide=True)
    ov = gpu_run(reads=reads, kmer_size=15, wide=True)
    compare_with_oracle(oracle_mod, ov, r, True)


SYNTH = [
    # (n, L, genome, gc, seed, mixed, settings)
    (400, 120, 3000, 0.5, 1, None, dict(kmer_size=12)),
    (300, 200, 4000, 0.3, 2, (80, 260), dict(kmer_size=15, min_collisions=3)),
    (250, 150, 2500, 0.17, 3, None, dict(kmer_size=10, min_identity=0.95, min_collisions=5)),
    (200, 90, 1200, 0.5, 4, (40, 140), dict(kmer_size=16)),
    (200, 120, 1500, 0.5, 5, None, dict(kmer_size=20, min_identity=0.9)),
    (300, 100, 2000, 0.45, 6, None, dict(kmer_size=13, kmer_edge=0.45, kmer_center=0.6)),
    (150, 300, 3000, 0.5, 7, None, dict(kmer_size=14, gap_open=-50, gap_extend=-5, min_overlap=20,
                                        max_ignore=250)),
]


@pytest.mark.parametrize("case", range(len(SYNTH)))
@pytest.mark.parametrize("wide", [False, True])
def test_synthetic_matches_oracle(oracle_mod, case, wide):
    n, L, G, gc, seed, mixed, st = SYNTH[case]
    reads = H.synth_reads(n, L, G, gc=gc, seed=seed, mixed=mixed)
    r = oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, **st), wide=wide)
    ov = gpu_run(reads=reads, wide=wide, **st)
    compare_with_oracle(oracle_mod, ov, r, wide)


@pytest.mark.parametrize("gaps", [(-60, -10, 0.9), (-20, -5, 0.95), (-200, -20, 0.9), (-35, -1, 0.85)])
def test_mutated_reads_with_indels(oracle_mod, gaps):
    """Reads with substitutions and indels exercise X/Y gap moves in both DP phases
    (small gap-open values make gap cells win and move the argmax)."""
    rng = np.random.default_rng(11 + abs(gaps[1]))
    base = H.synth_reads(300, 150, 3000, gc=0.5, seed=12)
    reads = []
    for rd in base:
        s = list(rd)
        for _ in range(int(rng.integers(0, 4))):
            p = int(rng.integers(0, len(s)))
            op = int(rng.integers(0, 3))
            if op == 0:
                s[p] = "ACGT"[int(rng.integers(0, 4))]
            elif op == 1:
                del s[p]
            else:
                s.insert(p, "ACGT"[int(rng.integers(0, 4))])
        reads.append("".join(s))
    st = dict(kmer_size=12, min_identity=gaps[2], min_collisions=4, gap_open=gaps[0], gap_extend=gaps[1])
    for wide in (False, True):
        r = oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, **st), wide=wide)
        ov = gpu_run(reads=reads, wide=wide, **st)
        compare_with_oracle(oracle_mod, ov, r, wide)


mutate = H.mutate


@pytest.mark.parametrize("gaps", [(-400, -30, 0.98), (-60, -10, 0.98), (-35, -1, 0.98)])
def test_full_width_band_500bp(oracle_mod, gaps):
    """k = 15 on 500-560 bp reads: every band is exactly 16 cells wide, the
    bench's shape (the lane kernel's EXACT variant), with substitutions and
    indels so gap moves, duds and invalid overlaps all occur."""
    rng = np.random.default_rng(abs(gaps[0]) + abs(gaps[1]))
    reads = mutate(H.synth_reads(500, 500, 25000, gc=0.5, seed=51), rng, 6)
    st = dict(kmer_size=15, min_identity=gaps[2], gap_open=gaps[0], gap_extend=gaps[1])
    r = oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, **st), wide=True)
    ov = gpu_run(reads=reads, wide=True, **st)
    assert ov.stats()["dispatched"] > 1000
    compare_with_oracle(oracle_mod, ov, r, True)


@pytest.mark.parametrize("k,L,minid", [(15, 500, 0.98), (12, 150, 0.92), (12, 300, 0.96), (9, 120, 0.9),
                                        (15, 1000, 0.98), (15, 1450, 0.98), (12, 500, 0.95)])
def test_align_kernels_agree(k, L, minid):
    """The lane-per-pair kernels (stored codes + walk, and forwarded path
    summaries) and the lane-group kernel give identical alignment tuples on the
    same dispatch (the default is also checked against the oracle elsewhere).
    Band widths 15 (16 registers), 21 (24), 26 and 29 (32)."""
    rng = np.random.default_rng(k * 1000 + L)
    reads = mutate(H.synth_reads(400, L, 20 * L, gc=0.5, seed=k + L), rng, 5)
    st = dict(kmer_size=k, min_identity=minid, min_collisions=3, gap_open=-60, gap_extend=-10)
    res = []
    for kern in (sao.ALIGN_GROUP, sao.ALIGN_LANE, sao.ALIGN_LANE_SUMMARY):
        ov = gpu_run(reads=reads, wide=True, align_kernel=kern, **st)
        res.append((ov.alignments(), ov.ovl(), ov.stats()["dp_cells"]))
    assert len(res[0][0]) > 100
    for r in res[1:]:
        np.testing.assert_array_equal(res[0][0], r[0])
        assert res[0][1] == r[1]
        assert res[0][2] == r[2]


def test_duplicate_reads_loc_ties(oracle_mod):
    """Identical reads give equal-loc k-mers: the tie rule fst = middle (KmerTable.scala:65-71)."""
    reads = H.synth_reads(60, 100, 700, seed=21)
    reads = reads + reads[:20] + [reads[5]] * 3
    for wide in (False, True):
        r = oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, kmer_size=11, min_collisions=2,
                                                                 max_collisions=400), wide=wide)
        ov = gpu_run(reads=reads, wide=wide, kmer_size=11, min_collisions=2, max_collisions=400)
        compare_with_oracle(oracle_mod, ov, r, wide)


def test_short_and_degenerate_reads(oracle_mod):
    """Reads shorter than k, exactly k (NaN loc: untagged), lowercase, tiny."""
    reads = H.synth_reads(80, 100, 600, seed=31)
    reads[3] = reads[3][:9]            # L < k
    reads[7] = reads[7][:12]           # L == k -> loc NaN
    reads[9] = reads[9].lower()        # readSeq upper-cases
    reads.append("")                   # empty sequence
    r = oracle_mod.Run(reads=[x.upper() for x in reads], settings=oracle_settings(oracle_mod, kmer_size=12))
    ov = gpu_run(reads=reads, kmer_size=12)
    compare_with_oracle(oracle_mod, ov, r, False)


@pytest.mark.parametrize("copies", [4000, 600, 1500, 3000])
def test_repeat_overflow_path(oracle_mod, copies):
    """A 12-mer repeated in `copies` reads (half in the leading edge, half in the
    middle) gives every middle-copy read copies/2 partners: 4,000 copies exceed
    both LDS pair tables (256 and 2,048 slots -> 64-way split pass), 600 only
    the first-pass table (-> the 2,048-slot re-run); counts must not change.
    The bucket build sees the motif's partition at 1,500 copies in its
    2,048-record pass, at 3,000 in the 4,096-record pass and at 4,000 on the
    global (big partition) path."""
    rng = np.random.default_rng(41)
    motif = "ACGTTGCAACGT"
    reads = []
    for i in range(copies):
        s = "".join("ACGT"[x] for x in rng.integers(0, 4, 100))
        p = 5 if i % 2 == 0 else 45
        reads.append(s[:p] + motif + s[p + 12:])
    reads += H.synth_reads(200, 100, 1500, seed=42)
    st = dict(kmer_size=12, min_collisions=2)
    for wide in (False, True):
        r = oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, **st), wide=wide)
        ov = gpu_run(reads=reads, wide=wide, **st)
        compare_with_oracle(oracle_mod, ov, r, wide)
        assert ov.stats()["pairs"] == len(r.pair_fst)


def test_literal_c_ruddii_fasta_is_one_read():
    """amos/c_ruddii.fasta as-is is a single sequence: every pair is same-read, the .ovl is empty (E7)."""
    z = np.load(os.path.join(H.GOLDEN, "c_ruddii_layout.npz"))
    contig = z["contig"].tobytes().decode()
    ov = gpu_run(reads=[contig], kmer_size=15)
    assert ov.ovl() == b""
    assert ov.stats()["dispatched"] == 0


def test_non_acgt_errors_like_matcherror(oracle_mod):
    reads = H.synth_reads(50, 100, 500, seed=51)
    reads = [r[:50] + "N" + r[51:] for r in reads]
    with pytest.raises(oracle_mod.OracleError):
        oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, kmer_size=12))
    with pytest.raises(sao.SAError) as e:
        gpu_run(reads=reads, kmer_size=12)
    assert e.value.name == "SA_E_NON_ACGT"


@pytest.mark.parametrize("wide", [False, True])
def test_failed_realign_leaves_no_stale_records(oracle_mod, wide):
    """A second align that fails must not leave the first run's records behind
    (ADVICE r3): 1,600 bp reads have 33-cell bands, so the first align runs the
    lane-group kernel; forcing the lane-per-pair kernel (SA_OPT_ALIGN_KERNEL=2,
    an option that does not reset the context) then fails the next align, and
    the getters and the .ovl writer report SA_E_STATE instead of the previous
    run's records.  Aligning again under the automatic choice gives them back."""
    rng = np.random.default_rng(77)
    g = "".join("ACGT"[x] for x in rng.integers(0, 4, 4000))
    reads = [g[s:s + 1600] for s in range(0, 2401, 40)]
    st = dict(kmer_size=15, min_collisions=3, max_ignore=2000)  # edge x middle offsets are ~1,000 bp
    r = oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, **st), wide=wide)
    ov = gpu_run(reads=reads, wide=wide, **st)
    assert ov.ovl() == r.ovl and r.ovl.count(b"{OVL") > 100
    ov._chk(sao.lib().sa_set_option(ov.h, sao.SA_OPT_ALIGN_KERNEL, sao.ALIGN_LANE))
    for align in (ov.align, ov.device_align):
        with pytest.raises(sao.SAError) as e:
            align()
        assert e.value.name == "SA_E_ARG"
        for getter in (ov.alignments, ov.ovl, ov.write_ovl):
            with pytest.raises(sao.SAError) as e:
                getter()
            assert e.value.name == "SA_E_STATE"
    ov._chk(sao.lib().sa_set_option(ov.h, sao.SA_OPT_ALIGN_KERNEL, sao.ALIGN_AUTO))
    ov.device_align()
    assert ov.ovl() == r.ovl
    ov.close()


def test_strict_rejects_aliasing_sizes():
    ov = sao.Overlapper(id_mode=sao.SA_IDS_STRICT)
    ov.add_reads(["ACGTACGTACGTACGT"] * 65536)
    with pytest.raises(sao.SAError) as e:
        ov.build()
    assert e.value.name == "SA_E_ID_RANGE"


def test_device_only_path_matches_readback():
    reads = H.synth_reads(2000, 200, 20000, seed=61)
    a = gpu_run(reads=reads, kmer_size=15, wide=True, keep_pairs=False)
    b = sao.Overlapper(kmer_size=15, id_mode=sao.SA_IDS_WIDE, timing=True)
    b.add_reads(reads)
    for _ in range(2):
        b.device_build()
        b.device_align()
    for x, y in zip(a.dispatch(), b.dispatch()):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a.alignments(), b.alignments())
    t = b.stage_times()
    assert t["pairs"][1] >= 2 and t["align"][1] == 2


def test_bench_scale_properties():
    """Bench-shaped input (wide ids, 20x coverage, 500 bp): determinism and the
    role-pair count against an independent numpy count over the k-mer buckets."""
    n, L, G, k = 20000, 500, 500000, 15
    reads = H.synth_reads(n, L, G, seed=71)
    ov = sao.Overlapper(kmer_size=k, id_mode=sao.SA_IDS_WIDE)
    ov.add_reads(reads)
    ov.build()
    d1 = ov.dispatch()
    st = ov.stats()
    ov.build()
    d2 = ov.dispatch()
    for x, y in zip(d1, d2):
        np.testing.assert_array_equal(x, y)
    # independent role-pair count: sum over buckets of (|st| + |en|) * |md| (incl. same-read pairs)
    arr = np.frombuffer("".join(reads).encode(), dtype=np.uint8).reshape(n, L)
    code = np.zeros(256, dtype=np.uint64)
    code[ord("C")], code[ord("T")], code[ord("G")] = 1, 2, 3
    c = code[arr]
    nk = L - k + 1
    h = np.zeros((n, nk), dtype=np.uint64)
    for t in range(k):
        h = (h << np.uint64(2)) | c[:, t:t + nk]
    loc = np.arange(nk, dtype=np.float32) / np.float32(L - k)
    stt = loc <= np.float32(0.4)
    en = np.float32(0.6) <= loc
    md = (np.float32(0.3) <= loc) & (loc <= np.float32(0.7))
    hh = h.reshape(-1)
    _, inv = np.unique(hh, return_inverse=True)
    w_edge = np.bincount(inv, weights=np.tile(stt.astype(np.float64) + en, n))
    w_md = np.bincount(inv, weights=np.tile(md.astype(np.float64), n))
    assert st["role_pairs"] == int(round(float((w_edge * w_md).sum())))
    assert st["kmers"] == n * nk
    assert st["buckets"] == len(w_md)
    # every dispatched pair has its count inside the collision window
    assert ((d1[2] >= 7) & (d1[2] <= 222)).all()
    # canonical order: lead descending, trail ascending within a lead
    assert (np.diff(d1[0]) <= 0).all()
    same = np.diff(d1[0]) == 0
    assert (np.diff(d1[1])[same] > 0).all()


def _hip_rank_main(rank, P, port, reads, starts, st, outdir, budget=None):
    import torch
    import torch.distributed as dist

    import saoverlap as sao_
    from sharded import HipWorker, ShardedOverlapper

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        torch.cuda.set_device(0)
        ov = sao_.Overlapper(id_mode=sao_.SA_IDS_WIDE, **st)
        ov.add_reads(reads[starts[rank]:starts[rank + 1]])
        so = ShardedOverlapper(HipWorker(ov), rank, P, starts, [len(r) for r in reads], "cuda:0")
        so.build(budget)
        so.build(budget)  # buffers reused
        lead, trail, count = ov.dispatch()
        so.gather_reads()
        ov.align()
        s = ov.stats()
        np.savez(os.path.join(outdir, "h%d.npz" % rank), lead=lead, trail=trail, count=count, al=ov.alignments(),
                 ovl=np.frombuffer(ov.ovl(), dtype=np.uint8), rp=np.int64(s["role_pairs"]),
                 npass=np.int64(so.npass))
        ov.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,repeat,budget", [(2, False, None), (4, False, None), (2, True, None),
                                             (4, False, 40000), (2, True, 40000)])
def test_sharded_hip_matches_single_gpu(P, repeat, budget, tmp_path):
    """P processes share the GPU (gloo, host-staged exchanges) and run the
    sharded stage on the HIP path: the ranks' dispatch, alignments and .ovl in
    descending rank order equal the single-context wide-id run exactly.  The
    repeat case (a 15-mer in 2,400 reads) overflows the multi-read blocks'
    tables, so those reads are recounted one per block.  With a budget the
    count runs in lead-range passes through the per-rank C ABI
    (sa_dist_buckets / _plan / _count_pass / _reduce_pass)."""
    import socket

    import torch.multiprocessing as mp
    rng = np.random.default_rng(70 + P)
    reads = mutate(H.synth_reads(1200, 300, 18000, gc=0.5, seed=71 + P, mixed=(250, 340)), rng, 3)
    st = dict(kmer_size=15, min_collisions=5)
    if repeat:
        motif = "ACGTTGCAACGTAGC"
        for i in range(2400):
            s_ = "".join("ACGT"[x] for x in rng.integers(0, 4, 120))
            p_ = 5 if i % 2 == 0 else 55
            reads.append(s_[:p_] + motif + s_[p_ + 15:])
        st = dict(kmer_size=15, min_collisions=2)
    cut = [0] + [int(len(reads) * f) for f in np.linspace(0.2, 0.75, P - 1)] + [len(reads)]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_hip_rank_main, args=(P, port, reads, cut, st, str(tmp_path), budget), nprocs=P)
    res = [np.load(os.path.join(str(tmp_path), "h%d.npz" % r)) for r in range(P)]
    order = list(range(P - 1, -1, -1))
    ref = gpu_run(reads=reads, wide=True, keep_pairs=False, **st)
    lead, trail, count = ref.dispatch()
    assert len(lead) > 1000
    np.testing.assert_array_equal(np.concatenate([res[r]["lead"] for r in order]), lead)
    np.testing.assert_array_equal(np.concatenate([res[r]["trail"] for r in order]), trail)
    np.testing.assert_array_equal(np.concatenate([res[r]["count"] for r in order]), count)
    np.testing.assert_array_equal(np.concatenate([res[r]["al"] for r in order]), ref.alignments())
    assert b"".join(res[r]["ovl"].tobytes() for r in order) == ref.ovl()
    assert sum(int(x["rp"]) for x in res) == ref.stats()["role_pairs"]
    npass = {int(x["npass"]) for x in res}
    assert len(npass) == 1 and (npass.pop() > 1) == (budget is not None)


@pytest.mark.parametrize("copies,force_sort", [(6000, False), (13000, False), (6000, True)])
def test_virtual_shards_reduce_tiers(copies, force_sort, monkeypatch):
    """The sharded reduce's lead tiers on 2 virtual shards: two 15-mers in `copies` short
    reads give leads up to ~copies distinct partners, every pair kept (2 collisions) --
    the 4,096- and 16,384-slot block tiers at 6,000, past the last tier (the whole pass
    to the (lead, trail) sort) at 13,000, and SA_LR_FORCE_SORT=1 sends every pass to the
    sort.  Dispatch equals the single context's exactly."""
    rng = np.random.default_rng(90 + copies)
    reads = mutate(H.synth_reads(600, 300, 9000, gc=0.5, seed=91, mixed=(250, 340)), rng, 3)
    ma, mb = "ACGTTGCAACGTAGC", "TTGACCGATGCAAGT"
    for i in range(copies):
        s_ = "".join("ACGT"[x] for x in rng.integers(0, 4, 80))
        p_ = 3 + i % 20
        reads.append(s_[:p_] + ma + s_[p_ + 15:p_ + 30] + mb + s_[p_ + 45:])
    st = dict(kmer_size=15, min_collisions=2)
    if force_sort:
        monkeypatch.setenv("SA_LR_FORCE_SORT", "1")
    ov = sao.Overlapper(shards=2, id_mode=sao.SA_IDS_WIDE, **st)
    ov.add_reads(reads)
    ov.build()
    got = ov.dispatch()
    ov.close()
    ref = sao.Overlapper(id_mode=sao.SA_IDS_WIDE, keep_pairs=False, **st)
    ref.add_reads(reads)
    ref.build()
    want = ref.dispatch()
    ref.close()
    assert len(want[0]) > copies * copies // 8  # (most motif pairs kept)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("mixed,k", [((100, 1000), 15), ((600, 1500), 14)])
def test_wide_band_lane_kernels_match_oracle(oracle_mod, mixed, k):
    """Reads up to 1,000-1,500 bp (configs[4]'s shape): bands of 16-31 cells run
    on the 24- and 32-register lane kernels; bit-exact against the oracle."""
    rng = np.random.default_rng(mixed[1] + k)
    reads = mutate(H.synth_reads(160, mixed[1], 12000, gc=0.5, seed=mixed[0] + k, mixed=mixed), rng, 4)
    st = dict(kmer_size=k, min_collisions=5, gap_open=-60, gap_extend=-10)
    r = oracle_mod.Run(reads=reads, settings=oracle_settings(oracle_mod, **st), wide=True)
    ov = gpu_run(reads=reads, wide=True, **st)
    assert ov.stats()["dispatched"] > 100
    compare_with_oracle(oracle_mod, ov, r, True)


@pytest.mark.parametrize("k", [15, 12])
def test_device_trove_layout_equals_host_replay(tmp_path, k):
    """The strict-id output order comes from GNU Trove layouts built on the device
    (trove_replay.hip: eviction-chain reservations per table of the rehash chain); the
    host replay (csrc/host/trove.h, one insert after another) is kept behind
    SA_HOST_TROVE=1.  On the c_ruddii reads (32,000 reads: ~2M KmerData and ~3M PairData
    keys, 15-17 tables each) both give the same .ovl bytes, and with SA_OPT_KEEP_PAIRS off
    only the dispatched pairs come back from the device."""
    import subprocess
    cli = os.path.join(os.path.dirname(sao.__file__), "build", "sa-overlap")
    fa = tmp_path / "c_ruddii.seq"
    fa.write_bytes(H.reads_fasta_bytes(H.c_ruddii_reads()))
    outs = []
    for host in ("0", "1"):
        o = tmp_path / ("o%s.ovl" % host)
        env = dict(os.environ, SA_HOST_TROVE=host)
        r = subprocess.run([cli, "-i", str(fa), "-o", str(o), "-k", str(k), "--strict-ids"], capture_output=True,
                           timeout=300, env=env)
        assert r.returncode == 0, r.stderr
        outs.append(o.read_bytes())
    assert outs[0].count(b"{OVL") > 1000
    assert outs[0] == outs[1]
