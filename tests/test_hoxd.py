"""BioLibs.readHOXD (BioLibs.scala:66-114) at the boundary: sa_load_hoxd
(csrc/host/fasta.cpp) against the literal restatement (oracle/literal.py
read_hoxd) on crafted matrix files -- zeroed start, JVM split/trim/parseInt
rules, and failures that leave the caller's matrix untouched.  Host logic
only: no GPU call."""
import ctypes as C
import os

import pytest

import literal
import saoverlap as sao

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEAD = "#HOXD MATRIX\n-,A,C,G,T\n"

CASES = {
    "hoxd1": open(os.path.join(ROOT, "tests", "golden", "HOXD1.txt")).read(),
    # rows missing: the reference's matrix starts zeroed (Array.ofDim(4,4))
    "two_rows": HEAD + "A,10,-1,-2,-3\nT,-3,-2,-1,10\n",
    # a trailing comma is dropped by String.split; lower-case and padded labels
    "trailing_comma": HEAD + "a,5,-4,-4,-4,\n c ,-4,5,-4,-4\n",
    # column order permuted in the header
    "permuted_cols": "title\n-,T,G,C,A\nA,1,2,3,4\nG,5,6,7,8\n",
    # explicit '+' sign, CRLF line ends, stops at the first empty line
    "crlf_plus": "t\r\n-,A,C,G,T\r\nA,+7,-1,-1,-1\r\n\r\nC,9,9,9,9\r\n",
    # costs beyond int8 (a x10 HOXD70) and beyond int16
    "wide": HEAD + "A,910,-1140,-310,-1230\nC,-1140,1000,-1250,-310\nG,-310,-1250,1000,-1140\nT,-1230,-310,-1140,910\n",
    "huge": HEAD + "A,2147483647,-2147483648,0,0\n",
    # a label row with no values is never examined
    "label_only": HEAD + "X\nA,1,1,1,1\n",
    # CR-only line ends
    "cr_only": "t\r-,A,C,G,T\rG,3,3,3,3\r",
    # failures (the reference throws)
    "bad_space": HEAD + "A, 1,2,3,4\n",
    "bad_label": HEAD + "N,1,2,3,4\n",
    "bad_header": "t\n-,A,X,G,T\nA,1,2,3,4\n",
    "too_many": HEAD + "A,1,2,3,4,5\n",
    "overflow": HEAD + "A,2147483648,0,0,0\n",
    "empty_label": HEAD + ",1,2,3,4\n",
    "one_line": "#HOXD MATRIX\n",
    "empty_value": HEAD + "A,1,,3,4\n",
}


def literal_table(path):
    try:
        t = literal.read_hoxd(path)
    except literal.JvmError:
        return None
    return [t[a][b] for a in range(4) for b in range(4)]


@pytest.fixture(scope="module")
def lib():
    return sao.lib()


@pytest.mark.parametrize("name", sorted(CASES))
def test_load_hoxd_matches_literal(lib, tmp_path, name):
    p = tmp_path / (name + ".txt")
    p.write_bytes(CASES[name].encode())
    want = literal_table(str(p))
    s = sao.Settings()
    lib.sa_default_settings(C.byref(s))
    before = list(s.cost)
    rc = lib.sa_load_hoxd(C.byref(s), str(p).encode())
    if want is None:
        assert rc == -2, name  # SA_E_INPUT
        assert list(s.cost) == before, "a failed load must leave the matrix untouched"
    else:
        assert rc == 0, name
        assert list(s.cost) == want, name


def test_literal_expectations(tmp_path):
    """Spot values of the restatement itself (so the parity above means something)."""
    def tab(text):
        p = tmp_path / "m.txt"
        p.write_bytes(text.encode())
        return literal_table(str(p))
    assert tab(CASES["two_rows"])[4:12] == [0] * 8
    assert tab(CASES["permuted_cols"])[:4] == [4, 3, 2, 1]
    assert tab(CASES["crlf_plus"])[:4] == [7, -1, -1, -1] and tab(CASES["crlf_plus"])[4:8] == [0] * 4
    assert tab(CASES["trailing_comma"])[4:8] == [-4, 5, -4, -4]
    assert tab(CASES["bad_space"]) is None and tab(CASES["one_line"]) is None
