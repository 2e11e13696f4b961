"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports
every symbol include/sa_overlap.h declares, fails loudly without a GPU, and the
sa-overlap CLI keeps Project4.readArgs' exit codes.  No compute calls."""
import ctypes as C
import os
import re
import subprocess

import pytest

import saoverlap as sao

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "sa_overlap.h")
CLI = os.path.join(ROOT, "sequence-aligner_amd", "build", "sa-overlap")


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(sao.LIB_PATH) or not os.path.exists(CLI):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "sequence-aligner_amd")], check=True)
    return sao.lib()


def declared():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sa_[a-z_]+)\s*\(", txt)))


def test_header_and_exports_agree(built):
    names = declared()
    assert len(names) >= 20
    assert sorted(sao.EXPORTS) == names
    for n in names:
        assert hasattr(built, n), n


def test_default_settings_are_project4_defaults(built):
    s = sao.settings()
    assert (s.kmer_size, s.min_overlap, s.max_ignore, s.gap_open, s.gap_extend) == (12, 40, 90, -200, -20)
    assert (s.min_collisions, s.max_collisions) == (7, 222)
    assert abs(s.min_identity - 0.98) < 1e-7 and abs(s.kmer_edge - 0.4) < 1e-7 and abs(s.kmer_center - 0.4) < 1e-7
    assert list(s.cost) == [91, -114, -31, -123, -114, 100, -125, -31, -31, -125, 100, -114, -123, -31, -114, 91]


def test_hoxd_file_loader(built):
    s = sao.settings(hoxd_file=os.path.join(ROOT, "tests", "golden", "HOXD1.txt"))
    assert list(s.cost) == list(sao.settings().cost)


def test_struct_sizes_match_header(built):
    assert C.sizeof(sao.Settings) == 4 * 27
    assert C.sizeof(sao.Stats) == 8 * 8 + 8


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_no_gpu_fails_loudly(built):
    with pytest.raises(sao.SAError) as e:
        sao.Overlapper()
    assert e.value.name == "SA_E_HIP"


def test_cli_exit_codes(built):
    r = subprocess.run([CLI, "--help"], capture_output=True)
    assert r.returncode == 0 and b"Sequence Overlapper" in r.stdout
    r = subprocess.run([CLI, "--bogus"], capture_output=True)
    assert r.returncode == 1 and b"Invalid Argument : --bogus" in r.stderr
    r = subprocess.run([CLI, "-k", "15"], capture_output=True)
    assert r.returncode == 255 and b"No input file specified" in r.stderr
    r = subprocess.run([CLI, "-k"], capture_output=True)
    assert r.returncode == 1
