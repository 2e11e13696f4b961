"""Oracle pinning: the C restatement against every known answer available.

No output of the Scala reference exists (no JVM; none shipped), so the oracle is
pinned by (a) the Scala-literal Python transliteration's golden vectors for
crp177 (tests/golden/make_crp177_golden.py), (b) known answers taken from the
reference's own files (HOXD1.txt, the README record sample, Trove's prime
table read from lib/trove.jar as data), and (c) arithmetic facts derived from
the code (SURVEY.md E2 cut table, E5 widths, E1 capacity chain).
"""
import bisect
import json
import os
import re

import numpy as np
import pytest

import helpers as H

GOLD = H.GOLDEN


@pytest.mark.parametrize("k", [12, 15])
def test_crp177_matches_literal_restatement(oracle_mod, k):
    r = oracle_mod.Run(fasta=H.crp177_path(), settings=oracle_mod.default_settings(kmer_size=k),
                       keep_kmers=True)
    g = np.load(os.path.join(GOLD, "crp177_k%d.npz" % k))
    assert open(os.path.join(GOLD, "crp177_k%d.ovl" % k), "rb").read() == r.ovl
    np.testing.assert_array_equal(r.pair_fst, g["pair_fst"])
    np.testing.assert_array_equal(r.pair_snd, g["pair_snd"])
    np.testing.assert_array_equal(r.pair_cnt, g["pair_cnt"])
    np.testing.assert_array_equal(r.first_fst, g["first_fst"])
    np.testing.assert_array_equal(r.first_snd, g["first_snd"])
    np.testing.assert_array_equal(r.lead, g["lead"])
    np.testing.assert_array_equal(r.trail, g["trail"])
    np.testing.assert_array_equal(r.bucket_order, g["bucket_order"])


def test_small_random_matches_literal(oracle_mod):
    import literal as L
    reads = H.synth_reads(60, 80, 900, gc=0.4, seed=7)
    text = H.reads_fasta_bytes(reads).decode()
    for k, wid in ((10, 0.95), (13, 0.98)):
        s = oracle_mod.default_settings(kmer_size=k, min_identity=wid, min_collisions=3)
        r = oracle_mod.Run(reads=reads, settings=s)
        out, _, _ = L.run(text, L.AlignSettings(k=k, min_identity=wid, min_coll=3))
        assert r.ovl.decode() == out


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_all_core_hash_stage_equals_single_thread(oracle_mod, threads):
    """The all-core CPU baseline of the hash stage (orc_run_wide_mt: per-thread
    PairData maps over hash bins, merged by lead) gives the single-threaded
    restatement's PairData counts and wide dispatch exactly, for uniform and
    mixed lengths (float32 cross-length loc comparisons)."""
    for mixed, k in ((None, 15), ((60, 160), 12)):
        reads = H.synth_reads(900, 160, 12000, gc=0.45, seed=11 + threads, mixed=mixed)
        s = oracle_mod.default_settings(kmer_size=k, min_collisions=3)
        r1 = oracle_mod.Run(reads=reads, settings=s, wide=True, skip_align=True)
        r2 = oracle_mod.Run(reads=reads, settings=s, wide=True, skip_align=True, threads=threads)
        assert len(r1.lead) > 100
        for a in ("pair_fst", "pair_snd", "pair_cnt", "lead", "trail"):
            np.testing.assert_array_equal(getattr(r1, a), getattr(r2, a))
        assert r2.role_pairs > len(r1.pair_fst)


@pytest.mark.parametrize("case", ["uniform15", "mixed12", "k18", "edges", "degenerate"])
def test_lead_rows_equal_full_pairdata(oracle_mod, case):
    """The sampled-lead checker (orc_lead_rows: only the sampled leads' buckets
    are kept) gives, for every lead asked for, exactly its rows of the
    single-threaded restatement's PairData -- partners and counts -- including
    custom edges where one occurrence carries two roles, k > 16 (16-char
    seqHash), L == k (NaN loc), reads shorter than k and lowercase / non-ACGT
    characters."""
    kw = dict(min_collisions=3)
    if case == "uniform15":
        reads, k = H.synth_reads(700, 150, 9000, gc=0.5, seed=21), 15
    elif case == "mixed12":
        reads, k = H.synth_reads(900, 200, 12000, gc=0.45, seed=22, mixed=(40, 200)), 12
    elif case == "k18":
        reads, k = H.synth_reads(600, 160, 7000, gc=0.5, seed=23, mixed=(100, 160)), 18
    elif case == "edges":  # st and en overlap (edge 0.55), wide middle
        reads, k = H.synth_reads(600, 120, 6000, gc=0.5, seed=24), 11
        kw.update(kmer_edge=0.55, kmer_center=0.9)
    else:
        rng = np.random.default_rng(25)
        reads = H.mutate(H.synth_reads(500, 90, 3000, gc=0.3, seed=25, mixed=(8, 90)), rng, 2)
        reads = [r.lower() if i % 7 == 0 else (r[:5] + "N" + r[6:] if i % 11 == 0 else r) for i, r in enumerate(reads)]
        k = 10
        reads += ["ACGTACGTAC"] * 5 + ["ACG"]  # L == k (NaN loc), L < k
    s = oracle_mod.default_settings(kmer_size=k, **kw)
    full = oracle_mod.Run(reads=reads, settings=s, wide=True, skip_align=True)
    bases = "".join(reads).encode()
    off = np.zeros(len(reads) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r) for r in reads])
    for leads in (np.arange(1, len(reads) + 1), np.unique(np.random.default_rng(3).integers(1, len(reads) + 1, 50))):
        ro, snd, cnt = oracle_mod.lead_rows(bases, off, leads, settings=s, threads=3)
        sel = np.isin(full.pair_fst, leads)
        want_lead = full.pair_fst[sel]
        got_lead = np.repeat(leads.astype(np.int32), np.diff(ro))
        np.testing.assert_array_equal(got_lead, want_lead)
        np.testing.assert_array_equal(snd, full.pair_snd[sel])
        np.testing.assert_array_equal(cnt, full.pair_cnt[sel])
    assert len(full.pair_fst) > 100


def test_hoxd1_equals_default_matrix(oracle_mod):
    """amos/HOXD1.txt (readHOXD format) == defaultHOXD (BioLibs.scala:122-140)."""
    rows = [l.split(",") for l in open(os.path.join(GOLD, "HOXD1.txt")).read().strip().split("\n")[1:]]
    cols = [c.strip() for c in rows[0][1:]]
    idx = {"A": 0, "C": 1, "G": 2, "T": 3}
    m = np.zeros((4, 4), dtype=np.int32)
    for row in rows[1:]:
        for j, v in enumerate(row[1:]):
            m[idx[row[0].strip()], idx[cols[j]]] = int(v)
    s = oracle_mod.default_settings()
    np.testing.assert_array_equal(np.array(list(s.cost)).reshape(4, 4), m)


def test_trove_capacity_chain_and_order(oracle_mod):
    """E1: THash(10,0.5f) starts at nextPrime(20)=23, grows to nextPrime(cap<<1)."""
    primes = json.load(open(os.path.join(GOLD, "trove_primes.json")))["sorted"]
    assert len(primes) == 245
    np_ = lambda x: primes[bisect.bisect_left(primes, x)]
    chain = [np_(20)]
    for _ in range(20):
        chain.append(np_(chain[-1] << 1))
    assert chain[:21] == [23, 47, 97, 197, 397, 797, 1597, 3203, 6421, 12853, 25717, 51437, 102877,
                          205759, 411527, 823117, 1646237, 3292489, 6584983, 13169977, 26339969]
    # keys smaller than the capacity iterate in descending order
    order, cap = oracle_mod.trove_order(np.arange(1, 12, dtype=np.int32))
    assert cap == 23 and list(order) == list(range(11, 0, -1))
    # the 12th key overflows maxSize = min(22, (int)(23*0.5f)) = 11 -> rehash to 47
    order, cap = oracle_mod.trove_order(np.arange(1, 13, dtype=np.int32))
    assert cap == 47
    # collisions probe downward by 1 + h % (cap-2): keys 0 and 23 share slot 0
    order, cap = oracle_mod.trove_order(np.array([0, 23], dtype=np.int32))
    assert cap == 23 and list(order) == [23, 0]  # 23 lands at 0 - (1 + 23 % 21) + 23 = 20


def _cuts(L, k, edge=np.float32(0.4), center=np.float32(0.4)):
    d = np.float32(L - k)
    loc = np.arange(L - k + 1, dtype=np.float32) / d
    head, tail = edge, np.float32(1) - edge
    ml, mt = np.float32(0.5) - center * np.float32(0.5), np.float32(0.5) + center * np.float32(0.5)
    st = np.nonzero(loc <= head)[0]
    md = np.nonzero((ml <= loc) & (loc <= mt))[0]
    en = np.nonzero(tail <= loc)[0]
    return (st.min(), st.max()), (md.min(), md.max()), (en.min(), en.max())


@pytest.mark.parametrize("L,k,st,md,en", [
    (100, 12, (0, 35), (27, 61), (53, 88)), (100, 15, (0, 34), (26, 59), (51, 85)),
    (500, 15, (0, 194), (146, 339), (291, 485)), (500, 12, (0, 195), (147, 341), (293, 488)),
    (1000, 15, (0, 394), (296, 689), (591, 985))])
def test_region_cut_table(oracle_mod, L, k, st, md, en):
    """E2: float32 region tags; the oracle's k-mer locs reproduce the cuts."""
    assert _cuts(L, k) == (st, md, en)
    r = oracle_mod.Run(reads=["ACGT" * (L // 4)], settings=oracle_mod.default_settings(kmer_size=k),
                       keep_kmers=True)
    loc = r.kmer_loc
    np.testing.assert_array_equal(loc, np.arange(L - k + 1, dtype=np.float32) / np.float32(L - k))


@pytest.mark.parametrize("L,k,w", [(100, 12, 12), (100, 15, 15), (500, 15, 15), (1000, 15, 20)])
def test_band_width(L, k, w):
    """E5: width = max(k, floor(|A| * (1 - 0.98f)) + 1) with a float32 product."""
    prod = np.float32(L) * (np.float32(1) - np.float32(0.98))
    assert max(k, int(np.floor(prod)) + 1) == w


def test_record_format_matches_readme(oracle_mod):
    """README:164-175 sample record; every oracle record has exactly that shape."""
    r = oracle_mod.Run(fasta=H.crp177_path())
    recs = r.ovl.decode().split("}\n")[:-1]
    assert len(recs) == r.ovl.count(b"{OVL")
    pat = re.compile(r"^\{OVL\nadj:N\nrds:\d+,\d+\nscr:0\nahg:-?\d+\nbhg:-?\d+\n$")
    assert all(pat.match(x) for x in recs)


def test_readme_sample_record_is_produced(oracle_mod):
    """README:164-175's sample record, exactly: crp177 at the reference defaults
    (k = 12) produces it once, where the Scala-literal golden .ovl has it."""
    rec = b"{OVL\nadj:N\nrds:18,22\nscr:0\nahg:20\nbhg:20\n}\n"
    r = oracle_mod.Run(fasta=H.crp177_path())
    assert r.ovl.count(rec) == 1
    golden = open(os.path.join(GOLD, "crp177_k12.ovl"), "rb").read()
    assert r.ovl.index(rec) == golden.index(rec)


def test_recall_against_amos_hash_overlap(oracle_mod):
    """Set-level sanity only (not a parity gate): the AMOS overlapper's crp177.ovl
    pairs (a<b, ahg==bhg) vs ours (lead,trail) -- most true dovetails recovered."""
    amos = set(tuple(map(int, m)) for m in re.findall(r"rds:(\d+),(\d+)", open(
        os.path.join(GOLD, "crp177_amos.ovl")).read()))
    r = oracle_mod.Run(fasta=H.crp177_path(), settings=oracle_mod.default_settings(kmer_size=15))
    ours = set((min(a, b), max(a, b)) for a, b in re.findall(rb"rds:(\d+),(\d+)", r.ovl) for a, b in [(int(a), int(b))])
    recall = len(ours & amos) / len(amos)
    assert recall > 0.85, recall


def test_c_ruddii_reconstruction():
    reads = H.c_ruddii_reads()
    assert len(reads) == 32000 and all(len(x) == 100 for x in reads)
    assert H.sha256("".join(x + "\n" for x in reads).encode()).startswith("3d8724e6")


def test_degenerate_and_dud_cases(oracle_mod):
    # |B| < width -> StringIndexOutOfBounds in phase 1
    with pytest.raises(oracle_mod.OracleError):
        oracle_mod.align_pair("ACGT" * 25, "ACGTACG", settings=oracle_mod.default_settings(kmer_size=12))
    # no positive phase-1 cell -> degenerate backtrack (AIOOBE)
    with pytest.raises(oracle_mod.OracleError):
        oracle_mod.align_pair("A" * 50, "C" * 20, settings=oracle_mod.default_settings(kmer_size=12))
    # non-ACGT aligned -> MatchError
    with pytest.raises(oracle_mod.OracleError):
        oracle_mod.align_pair("ACGTN" * 10, "ACGTACGTACGTACGT", settings=oracle_mod.default_settings(kmer_size=12))
    # B's prefix absent from A's band -> dud
    a = oracle_mod.align_pair("ACGT" * 20, "GGGGACGTACGTACGT" * 2, settings=oracle_mod.default_settings(kmer_size=12))
    assert a["is_dud"] == 1 and a["valid"] == 0


def _mix32(h):
    h ^= h >> 16
    h = (h * 0x7FEB352D) & 0xFFFFFFFF
    h ^= h >> 15
    h = (h * 0x846CA68B) & 0xFFFFFFFF
    return h ^ (h >> 16)


def test_lead_stats_match_rows_and_brute_force(oracle_mod):
    """orc_lead_stats (the projection of configs[3] / [4]'s per-rank partials):
    on reads cut from one genome by (start, length) it gives, per lead, the
    number of its PairData rows, the sum of their counts (its role pairs as
    fst), its dispatched rows -- all equal to orc_lead_rows on the same reads
    materialised -- and its partials over 2^L hash-range owners, equal to a
    brute-force count of distinct (partner, owner of the k-mer) over its role
    pairs (owner = top L bits of mix32(seqHash), the device's record key)."""
    import bench
    G, n, k = 4000, 160, 11
    genome = oracle_mod.synth_genome(9, G, 0.5)
    starts, lens = bench.synth_layout(n, 120, G, 9, min_len=40)
    reads = [genome[int(a):int(a) + int(b)].decode() for a, b in zip(starts, lens)]
    s = oracle_mod.default_settings(kmer_size=k, min_collisions=2)
    leads = np.arange(1, n + 1, dtype=np.int32)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    ro, snd, cnt = oracle_mod.lead_rows("".join(reads).encode(), off, leads, settings=s, threads=2)
    rows = np.diff(ro)
    owner = np.repeat(np.arange(n), rows)

    def seg_sum(v):
        out = np.zeros(n, dtype=np.int64)
        np.add.at(out, owner, v.astype(np.int64))
        return out
    for L in (0, 1, 3):
        st = oracle_mod.lead_stats(genome, starts, lens, leads, settings=s, threads=2, log_ranks=L)
        np.testing.assert_array_equal(st[:, 0], rows)
        np.testing.assert_array_equal(st[:, 1], seg_sum(cnt))
        np.testing.assert_array_equal(st[:, 3], seg_sum((cnt >= 2) & (cnt <= 222)))
        if L == 0:
            np.testing.assert_array_equal(st[:, 2], rows)
    # brute force at L = 2 (KmerTable.scala:57-80 role pairs, keyed by the k-mer's owner)
    f32 = np.float32
    code = {"A": 0, "C": 1, "T": 2, "G": 3}
    occ = {}
    for r, rd in enumerate(reads):
        d = len(rd) - k
        for i in range(len(rd) - k + 1):
            h = 0
            for ch in rd[i:i + k]:
                h = ((h << 2) ^ code[ch]) & 0xFFFFFFFF
            loc = f32(i) / f32(d) if d > 0 else f32("nan")
            occ.setdefault(h, []).append((r, loc))
    parts = np.zeros(n, dtype=np.int64)
    seen = set()
    for h, lst in occ.items():
        own = _mix32(h) >> 30
        tag = [(r, l, l <= f32(0.4), f32(0.3) <= l <= f32(0.7), f32(0.6) <= l) for r, l in lst if not np.isnan(l)]
        for ra, la, sa, ma, ea in tag:
            for rb, lb, sb, mb, eb in tag:
                if ra == rb:
                    continue
                if ((sa or ea) and mb and la > lb) or (ma and (sb or eb) and not lb > la):
                    if (ra, rb, own) not in seen:
                        seen.add((ra, rb, own))
                        parts[ra] += 1
    st = oracle_mod.lead_stats(genome, starts, lens, leads, settings=s, threads=2, log_ranks=2)
    np.testing.assert_array_equal(st[:, 2], parts)
    assert (st[:, 2] > st[:, 0]).any()


def test_synth_genome_is_the_bench_genome(oracle_mod):
    import bench
    for seed, gc in ((1, 0.5), (5, 0.17)):
        assert oracle_mod.synth_genome(seed, 200000, gc) == bench.synth_genome(200000, gc, seed).tobytes()
