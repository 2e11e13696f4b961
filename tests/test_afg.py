"""AMOS message-file writer (sa_write_afg, `sa-overlap --afg`).

The project pipeline builds the bank with `toAmos_new -s X.seq -b X.bnk` and loads
the overlapper's .ovl with `bank-transact -b X.bnk -m X.ovl` (Rakefile.rb:164-215,
amos/README:1-13).  `--afg` writes both halves as one AMOS message file for
`bank-transact -c -b X.bnk -m X.afg`: a {RED} per read, then the .ovl records.

Pins: the {OVL} half must equal the .ovl byte for byte (itself checked against the
oracle elsewhere).  The {RED} half is checked against the reference's own bank,
`amos/c_ruddii.bnk` (the 32,000 c_ruddii reads toAmos_new loaded), read as data into
tests/golden/c_ruddii_bank_red.npz by make_c_ruddii_bank_red.py: RED.0.map gives
every read's iid / bid / eid (all the ordinal; the eid RULE stays parity unpinned:
c_ruddii.seq's headers are a missing blob and may be the ordinals themselves, and
toAmos_new's source is absent, so the CLI's ordinal default and --afg-header-eids
are equally consistent with this map),
RED.0.0.fix every read's length and clear range (0, 100) with every other range
of the record unset (so the writer emits clr and no qcr).  toAmos_new's default
quality is not pinned (its var blob, RED.0.0.var, is absent from the fixture):
the writer takes it as a parameter (default 20).  The AMOS tools are prebuilt
binaries inside the reference and are not run here, so the bank load itself is
not exercised; the message grammar is checked by the parser below.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import helpers as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "sequence-aligner_amd", "build", "sa-overlap")


def parse_messages(text):
    """AMOS message grammar: '{TYPE' ... '}' blocks of 'key:value' fields; a field
    whose value is empty continues on the following lines up to a lone '.'."""
    lines = text.split("\n")
    assert lines[-1] == "", "file must end with a newline"
    msgs, i = [], 0
    while i < len(lines) - 1:
        m = re.fullmatch(r"\{([A-Z]{3})", lines[i])
        assert m, "line %d: %r" % (i, lines[i])
        kind, fields, i = m.group(1), {}, i + 1
        while lines[i] != "}":
            key, sep, val = lines[i].partition(":")
            assert sep and re.fullmatch(r"[a-z]{3}", key), "line %d: %r" % (i, lines[i])
            i += 1
            if val == "":
                body = []
                while lines[i] != ".":
                    body.append(lines[i])
                    i += 1
                i += 1
                val = "".join(body)
            assert key not in fields
            fields[key] = val
        msgs.append((kind, fields))
        i += 1
    return msgs


def test_parser_on_a_handwritten_message():
    text = "{RED\niid:1\neid:r1\nseq:\nAC\nGT\n.\nqlt:\nDD\nDD\n.\nclr:0,4\n}\n{OVL\nadj:N\nrds:1,2\n}\n"
    msgs = parse_messages(text)
    assert msgs == [("RED", {"iid": "1", "eid": "r1", "seq": "ACGT", "qlt": "DDDD", "clr": "0,4"}),
                    ("OVL", {"adj": "N", "rds": "1,2"})]
    with pytest.raises(AssertionError):
        parse_messages("{RED\niid:1\n")


def test_cli_rejects_bad_quality():
    if not os.path.exists(CLI):
        pytest.skip("CLI not built")
    r = subprocess.run([CLI, "-i", H.crp177_path(), "--afg", "/dev/null", "--afg-quality", "61"],
                       capture_output=True, timeout=60)
    assert r.returncode == 1 and b"afg-quality" in r.stderr


def check_afg(afg_text, ovl_bytes, seqs, eids, quality):
    red_part_end = afg_text.find("{OVL")
    red_part_end = len(afg_text) if red_part_end < 0 else red_part_end
    assert afg_text[red_part_end:].encode() == ovl_bytes
    msgs = parse_messages(afg_text[:red_part_end])
    assert len(msgs) == len(seqs)
    for i, (kind, f) in enumerate(msgs):
        assert kind == "RED"
        assert f["iid"] == str(i + 1)
        assert f["eid"] == eids[i]
        assert f["seq"] == seqs[i]
        assert f["qlt"] == chr(48 + quality) * len(seqs[i])
        assert f["clr"] == "0,%d" % len(seqs[i])
        assert set(f) == {"iid", "eid", "seq", "qlt", "clr"}


def bank_red():
    return np.load(os.path.join(H.GOLDEN, "c_ruddii_bank_red.npz"))


def test_bank_fixture_shape():
    """The fixture read from the reference's bank: 32,000 reads, iid = bid = eid =
    ordinal, 100 bp, clear range (0, 100), every other range unset."""
    z = bank_red()
    n = len(z["length"])
    assert n == 32000 == len(H.c_ruddii_reads())
    assert (z["map"] == np.arange(1, n + 1)[:, None]).all()
    assert (z["length"] == 100).all() and (z["clr_begin"] == 0).all() and (z["clr_end"] == 100).all()
    assert z["rest_zero"].all()


@pytest.mark.gpu
@pytest.mark.parametrize("header_eids", [False, True])
def test_cli_afg_crp177(tmp_path, header_eids):
    ovl, afg = tmp_path / "x.ovl", tmp_path / "x.afg"
    r = subprocess.run([CLI, "-i", H.crp177_path(), "-o", str(ovl), "--afg", str(afg)] +
                       (["--afg-header-eids"] if header_eids else []), capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr
    seqs = [s.upper() for s in H.read_fasta_seqs(H.crp177_path())]
    if header_eids:
        eids = [l[1:].split()[0] for l in open(H.crp177_path()) if l.startswith(">")]
        assert eids[0] == "r1_1-101"
    else:
        eids = [str(i + 1) for i in range(len(seqs))]
    check_afg(afg.read_text(), ovl.read_bytes(), seqs, eids, 20)
    assert ovl.read_bytes().count(b"{OVL") > 2000


@pytest.mark.gpu
def test_afg_c_ruddii_matches_reference_bank(tmp_path):
    """The c_ruddii reads' {RED} messages load to what the reference's bank holds:
    iid and eid from RED.0.map, sequence length and clear range from RED.0.0.fix."""
    import saoverlap as sao
    z = bank_red()
    reads = H.c_ruddii_reads()
    with sao.Overlapper(kmer_size=15) as ov:
        ov.add_reads(reads)
        ov.build()
        ov.align()
        p = tmp_path / "c.afg"
        ov.write_afg(str(p))
        text, ovl = p.read_text(), ov.ovl()
    red_end = text.find("{OVL")
    assert text[red_end:].encode() == ovl and ovl.count(b"{OVL") > 300000
    msgs = parse_messages(text[:red_end])
    assert len(msgs) == len(z["length"])
    iid = np.array([int(f["iid"]) for _, f in msgs])
    eid = np.array([int(f["eid"]) for _, f in msgs])
    clr = np.array([[int(x) for x in f["clr"].split(",")] for _, f in msgs])
    np.testing.assert_array_equal(iid, z["map"][:, 0])
    np.testing.assert_array_equal(eid, z["map"][:, 2])
    np.testing.assert_array_equal([len(f["seq"]) for _, f in msgs], z["length"])
    np.testing.assert_array_equal(clr[:, 0], z["clr_begin"])
    np.testing.assert_array_equal(clr[:, 1], z["clr_end"])
    assert all(set(f) == {"iid", "eid", "seq", "qlt", "clr"} for _, f in msgs)  # other ranges unset


@pytest.mark.gpu
def test_binding_afg_sharded_and_default_eids(tmp_path):
    import saoverlap as sao
    reads = H.synth_reads(3000, 300, 40_000, seed=5)
    out = {}
    for shards in (1, 4):
        with sao.Overlapper(shards=shards, kmer_size=15) as ov:
            ov.add_reads(reads)
            with pytest.raises(sao.SAError):
                ov.write_afg(str(tmp_path / "early.afg"))  # SA_E_STATE before an alignment
            ov.build()
            ov.align()
            p = tmp_path / ("s%d.afg" % shards)
            ov.write_afg(str(p), quality=30)
            out[shards] = (p.read_text(), ov.ovl())
    assert out[1] == out[4]
    assert out[1][1].count(b"{OVL") > 1000
    check_afg(out[1][0], out[1][1], reads, [str(i + 1) for i in range(len(reads))], 30)
    # eids: one per read, each one message-field token
    with sao.Overlapper(kmer_size=15) as ov:
        ov.add_reads(reads)
        ov.build()
        ov.align()
        with pytest.raises(ValueError):
            ov.write_afg(str(tmp_path / "short.afg"), eids=["x"] * 10)
        with pytest.raises(ValueError):
            ov.write_afg(str(tmp_path / "ws.afg"), eids=["r 1"] + ["x"] * (len(reads) - 1))
        # the C ABI refuses such an eid itself (callers other than this binding)
        import ctypes as C
        arr = (C.c_char_p * len(reads))(*([b"a:b"] + [b"x"] * (len(reads) - 1)))
        assert sao.lib().sa_write_afg(ov.h, str(tmp_path / "c.afg").encode(), arr, 20) == -1  # SA_E_ARG
        names = ["read_%d" % (i + 1) for i in range(len(reads))]
        ov.write_afg(str(tmp_path / "named.afg"), eids=names)
        check_afg((tmp_path / "named.afg").read_text(), ov.ovl(), reads, names, 20)
