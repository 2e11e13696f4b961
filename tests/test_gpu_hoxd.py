"""Custom cost matrices on the device (BioLibs.readHOXD, BioLibs.scala:66-114;
`-m FILE`, Project4.scala:133-138, :243-247).  GPU only.

Both aligners -- the banded dovetail DP (generateFastDovetailAlignmentSet) and
--quadratic-align (generateLocalAlignmentSet) -- against the C oracle with:
an asymmetric matrix, HOXD70 scaled x10 with x10 gap costs (run as HOXD70
after the common-divisor reduction), and a matrix file with
missing rows (readHOXD starts from a zeroed 4x4).  Costs that do not fit 8
bits after that reduction run on int16 cost packs (every DP kernel: lane,
lane-group and quadratic); beyond 16 bits they fail with SA_E_OVERFLOW.
"""
import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

sao = pytest.importorskip("saoverlap")

ALIGN_CMP = ("start_i", "start_j", "end_i", "end_j", "correct", "error", "ahg", "bhg")
HOXD70 = [91, -114, -31, -123, -114, 100, -125, -31, -31, -125, 100, -114, -123, -31, -114, 91]


def reads_for(seed):
    rng = np.random.default_rng(seed)
    return H.mutate(H.synth_reads(220, 260, 4000, gc=0.45, seed=seed, mixed=(200, 300)), rng, 3)


def check(oracle_mod, reads, cost, quadratic, **st):
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(cost=cost, **st), quadratic=quadratic)
    ov = sao.Overlapper(cost=cost, aligner=sao.SA_ALIGNER_QUADRATIC if quadratic else sao.SA_ALIGNER_LINEAR, **st)
    ov.add_reads(reads)
    ov.build()
    ov.align()
    al = ov.alignments()
    assert len(al) == len(r.lead) > 100
    for name in ALIGN_CMP:
        np.testing.assert_array_equal(al[:, sao.ALIGN_FIELDS.index(name)], r.align_field(name), err_msg=name)
    assert ov.ovl() == r.ovl
    return ov


@pytest.mark.parametrize("quadratic", [False, True])
def test_asymmetric_matrix(oracle_mod, quadratic):
    cost = [60, -70, -20, -90, -80, 75, -95, -25, -15, -85, 70, -60, -100, -35, -65, 55]
    check(oracle_mod, reads_for(11), cost, quadratic, kmer_size=12, gap_open=-120, gap_extend=-15)


@pytest.mark.parametrize("quadratic", [False, True])
def test_hoxd70_scaled_by_ten(oracle_mod, quadratic):
    """A legal -m matrix outside int8: x10 costs and gaps give the same alignments."""
    reads = reads_for(12)
    big = check(oracle_mod, reads, [10 * c for c in HOXD70], quadratic, kmer_size=12, gap_open=-2000,
                gap_extend=-200)
    small = sao.Overlapper(aligner=sao.SA_ALIGNER_QUADRATIC if quadratic else sao.SA_ALIGNER_LINEAR, kmer_size=12)
    small.add_reads(reads)
    small.build()
    small.align()
    assert big.ovl() == small.ovl()


@pytest.mark.parametrize("quadratic", [False, True])
def test_matrix_file_with_missing_rows(oracle_mod, tmp_path, quadratic):
    """readHOXD fills a zeroed 4x4: rows the file lacks cost 0."""
    p = tmp_path / "m.txt"
    # readHOXD's format: a title line, the column header, then one row per base
    p.write_text("HOXD70 without its G row\n,A,C,G,T\nA,91,-114,-31,-123\nC,-114,100,-125,-31\n"
                 "T,-123,-31,-114,91\n")
    s = sao.settings(hoxd_file=str(p))
    cost = list(s.cost)
    assert cost[8:12] == [0, 0, 0, 0]  # the G row
    check(oracle_mod, reads_for(13), cost, quadratic, kmer_size=12)


@pytest.mark.parametrize("kernel", ["lane", "group", "quadratic"])
def test_costs_beyond_int8(oracle_mod, kernel):
    """A matrix whose reduced entries need 16 bits (gcd 1 with A:A = 1000):
    the int16 cost packs of each DP kernel against the oracle."""
    cost = list(HOXD70)
    cost[0] = 1000
    cost[15] = -777
    reads = reads_for(14)
    st = dict(kmer_size=12)
    quadratic = kernel == "quadratic"
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(cost=cost, **st), quadratic=quadratic)
    ov = sao.Overlapper(cost=cost, aligner=sao.SA_ALIGNER_QUADRATIC if quadratic else sao.SA_ALIGNER_LINEAR,
                        align_kernel=1 if kernel == "group" else 0, **st)
    ov.add_reads(reads)
    ov.build()
    ov.align()
    al = ov.alignments()
    assert len(al) == len(r.lead) > 100
    for name in ALIGN_CMP:
        np.testing.assert_array_equal(al[:, sao.ALIGN_FIELDS.index(name)], r.align_field(name), err_msg=name)
    assert ov.ovl() == r.ovl


def test_costs_beyond_int16_fail_exactly():
    cost = list(HOXD70)
    cost[0] = 40000  # gcd with the rest is 1: 40,000 does not fit the 16-bit cost packs
    ov = sao.Overlapper(cost=cost, kmer_size=12)
    ov.add_reads(reads_for(14))
    ov.build()
    with pytest.raises(sao.SAError) as e:
        ov.align()
    assert e.value.name == "SA_E_OVERFLOW"


@pytest.mark.parametrize("cost", ["hoxd70", "near_16bit"])
def test_two_pairs_per_lane_kernels(oracle_mod, cost):
    """Reads of 467..500 bp (every band exactly 16 cells) with int8 costs: both
    phases run two pairs per lane in packed 16-bit halves, pairs
    of different trail lengths side by side.  'near_16bit' puts the largest
    score (127 x 500 + bias) within 2,000 of the 16-bit limit."""
    c = list(HOXD70)
    if cost == "near_16bit":
        c[0] = c[15] = 127
        c[5] = c[10] = 113
    rng = np.random.default_rng(21)
    reads = H.mutate(H.synth_reads(200, 490, 4000, gc=0.45, seed=21, mixed=(470, 497)), rng, 3)
    assert 467 <= min(map(len, reads)) and max(map(len, reads)) <= 500
    check(oracle_mod, reads, c, False, kmer_size=12)


@pytest.mark.parametrize("segs", ["0", "1", "2", "5", "8"])
def test_phase1_row_segments(oracle_mod, monkeypatch, segs):
    """Phase 1 of the two-pairs-per-lane aligner in row segments (dovetail_p1x2_seg_kernel,
    DESIGN.md 4.6): the lanes' state handed between ticketed one-wave workgroups through
    device-scope atomics.  Every segment count -- 0 is the one-segment kernel -- gives the
    oracle's alignments, on reads of 467..500 bp (pairs of different lengths in one wave)."""
    monkeypatch.setenv("SA_P1_SEGS", segs)
    rng = np.random.default_rng(22)
    reads = H.mutate(H.synth_reads(240, 490, 4000, gc=0.45, seed=22, mixed=(467, 500)), rng, 3)
    check(oracle_mod, reads, HOXD70, False, kmer_size=12)
