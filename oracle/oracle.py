"""ctypes wrapper for the C oracle (oracle/sa_oracle.c) -- TEST INFRASTRUCTURE.

Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() may import
this module, and only as the checker / CPU baseline.  The product path
(sequence-aligner_amd/) never links or calls it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liborc.so")

ORC_OK, ORC_E_INPUT, ORC_E_NPE, ORC_E_MATCH, ORC_E_INDEX = 0, -1, -2, -3, -4


class Settings(C.Structure):
    _fields_ = [("kmer_size", C.c_int32), ("min_overlap", C.c_int32), ("max_ignore", C.c_int32),
                ("gap_open", C.c_int32), ("gap_extend", C.c_int32), ("min_collisions", C.c_int32),
                ("max_collisions", C.c_int32), ("min_identity", C.c_float), ("kmer_edge", C.c_float),
                ("kmer_center", C.c_float), ("cost", C.c_int32 * 16)]


class Align(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("lead", "trail", "is_dud", "start_i", "start_j", "end_i", "end_j",
                                         "correct", "error", "len_a", "len_b", "valid", "ovl_valid",
                                         "ahg", "bhg")]


ALIGN_FIELDS = [f[0] for f in Align._fields_]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.POINTER
        L.orc_default_settings.argtypes = [P(Settings)]
        L.orc_create_from_fasta.argtypes = [C.c_char_p, P(C.c_void_p)]
        L.orc_create_from_buffers.argtypes = [C.c_char_p, P(C.c_uint64), C.c_uint32, P(C.c_void_p)]
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_num_reads.argtypes = [C.c_void_p]
        L.orc_num_reads.restype = C.c_uint32
        L.orc_run.argtypes = [C.c_void_p, P(Settings), C.c_int]
        L.orc_run_wide_mt.argtypes = [C.c_void_p, P(Settings), C.c_int, P(C.c_uint64)]
        for fn in ("orc_num_kmers", "orc_num_buckets", "orc_num_pairs", "orc_num_dispatch"):
            getattr(L, fn).argtypes = [C.c_void_p]
            getattr(L, fn).restype = C.c_size_t
        L.orc_kmers.argtypes = [C.c_void_p, P(P(C.c_int32)), P(P(C.c_int32)), P(P(C.c_float))]
        L.orc_bucket_order.argtypes = [C.c_void_p]
        L.orc_bucket_order.restype = P(C.c_int32)
        L.orc_pairs.argtypes = [C.c_void_p, P(P(C.c_int32)), P(P(C.c_int32)), P(P(C.c_int32))]
        L.orc_pairs_first_order.argtypes = [C.c_void_p, P(P(C.c_int32)), P(P(C.c_int32))]
        L.orc_dispatch.argtypes = [C.c_void_p, P(P(C.c_int32)), P(P(C.c_int32))]
        L.orc_aligns.argtypes = [C.c_void_p]
        L.orc_aligns.restype = P(Align)
        L.orc_ovl.argtypes = [C.c_void_p, P(C.c_char_p)]
        L.orc_ovl.restype = C.c_size_t
        L.orc_align_pair.argtypes = [C.c_char_p, C.c_int32, C.c_char_p, C.c_int32, C.c_int32, C.c_int32,
                                     P(Settings), P(Align)]
        L.orc_align_pair_local.argtypes = L.orc_align_pair.argtypes
        L.orc_trove_order.argtypes = [P(C.c_int32), C.c_size_t, P(C.c_int32), P(C.c_int32)]
        L.orc_align_batch.argtypes = [C.c_char_p, P(C.c_uint64), C.c_uint32, P(C.c_int32), P(C.c_int32), C.c_size_t,
                                      P(Settings), C.c_int, P(Align)]
        L.orc_max_threads.restype = C.c_int
        L.orc_lead_rows.argtypes = [C.c_char_p, P(C.c_uint64), C.c_uint32, P(Settings), P(C.c_int32), C.c_size_t,
                                    C.c_int, P(C.c_uint64), P(P(C.c_int32)), P(P(C.c_int32))]
        L.orc_lead_stats.argtypes = [C.c_char_p, P(C.c_uint64), P(C.c_int32), C.c_uint32, P(Settings), P(C.c_int32),
                                     C.c_size_t, C.c_int, C.c_int, P(C.c_uint64)]
        L.orc_synth_genome.argtypes = [C.c_uint64, C.c_uint64, C.c_double, C.c_void_p, C.c_int]
        L.orc_synth_genome.restype = None
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_free.restype = None
        _lib = L
    return _lib


def default_settings(**kw):
    s = Settings()
    lib().orc_default_settings(C.byref(s))
    for k, v in kw.items():
        if k == "cost":
            for i, x in enumerate(np.asarray(v).reshape(16)):
                s.cost[i] = int(x)
        else:
            setattr(s, k, v)
    return s


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


class OracleError(RuntimeError):
    def __init__(self, rc):
        super().__init__("oracle error %d" % rc)
        self.rc = rc


class Run:
    """Result of one calc-overlaps run of the oracle."""

    def __init__(self, reads=None, fasta=None, settings=None, wide=False, keep_kmers=False, skip_align=False,
                 packed=None, quadratic=False, threads=None):
        """threads (wide + skip_align only): the all-core hash stage
        (orc_run_wide_mt) on that many OpenMP threads (0 = all); self.role_pairs
        is then the role pairs it visited."""
        L = lib()
        h = C.c_void_p()
        if packed is not None:
            bases, off = packed
            off = np.ascontiguousarray(off, dtype=np.uint64)
            rc = L.orc_create_from_buffers(bases, off.ctypes.data_as(C.POINTER(C.c_uint64)), len(off) - 1,
                                           C.byref(h))
        elif fasta is not None:
            rc = L.orc_create_from_fasta(fasta.encode(), C.byref(h))
        else:
            bases = b"".join(r.encode() if isinstance(r, str) else bytes(r) for r in reads)
            off = np.zeros(len(reads) + 1, dtype=np.uint64)
            off[1:] = np.cumsum([len(r) for r in reads])
            rc = L.orc_create_from_buffers(bases, off.ctypes.data_as(C.POINTER(C.c_uint64)),
                                           len(reads), C.byref(h))
        if rc:
            raise OracleError(rc)
        self.settings = settings or default_settings()
        try:
            if threads is not None:
                if not (wide and skip_align and not keep_kmers):
                    raise ValueError("threads= runs the wide-id hash stage only")
                rp = C.c_uint64(0)
                rc = L.orc_run_wide_mt(h, C.byref(self.settings), int(threads), C.byref(rp))
                self.role_pairs = int(rp.value)
            else:
                rc = L.orc_run(h, C.byref(self.settings), (1 if wide else 0) | (2 if skip_align else 0) |
                             (4 if quadratic else 0))
            self.rc = rc
            self.n_reads = L.orc_num_reads(h)
            if keep_kmers:
                hp, ip, lp = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)(), C.POINTER(C.c_float)()
                L.orc_kmers(h, C.byref(hp), C.byref(ip), C.byref(lp))
                nk = L.orc_num_kmers(h)
                self.kmer_hash = _arr(hp, nk, np.int32)
                self.kmer_id = _arr(ip, nk, np.int32)
                self.kmer_loc = _arr(lp, nk, np.float32)
                nb = L.orc_num_buckets(h)
                self.bucket_order = _arr(L.orc_bucket_order(h), nb, np.int32)
            if rc:
                raise OracleError(rc)
            f, s_, c = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
            L.orc_pairs(h, C.byref(f), C.byref(s_), C.byref(c))
            n = L.orc_num_pairs(h)
            self.pair_fst, self.pair_snd, self.pair_cnt = (_arr(f, n, np.int32), _arr(s_, n, np.int32),
                                                           _arr(c, n, np.int32))
            if not wide:
                L.orc_pairs_first_order(h, C.byref(f), C.byref(s_))
                self.first_fst, self.first_snd = _arr(f, n, np.int32), _arr(s_, n, np.int32)
            d1, d2 = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
            L.orc_dispatch(h, C.byref(d1), C.byref(d2))
            nd = L.orc_num_dispatch(h)
            self.lead, self.trail = _arr(d1, nd, np.int32), _arr(d2, nd, np.int32)
            ap = L.orc_aligns(h)
            self.aligns = np.zeros((nd, len(ALIGN_FIELDS)), dtype=np.int32)
            if nd:
                raw = np.ctypeslib.as_array(C.cast(ap, C.POINTER(C.c_int32)), shape=(nd * len(ALIGN_FIELDS),))
                self.aligns[:] = raw.reshape(nd, len(ALIGN_FIELDS))
            t = C.c_char_p()
            ln = L.orc_ovl(h, C.byref(t))
            self.ovl = C.string_at(t, ln) if ln else b""
        finally:
            L.orc_destroy(h)

    def align_field(self, name):
        return self.aligns[:, ALIGN_FIELDS.index(name)]


def align_pair(A, B, id_a=1, id_b=2, settings=None, quadratic=False):
    s = settings or default_settings()
    out = Align()
    fn = lib().orc_align_pair_local if quadratic else lib().orc_align_pair
    rc = fn(A.encode(), len(A), B.encode(), len(B), id_a, id_b, C.byref(s), C.byref(out))
    if rc:
        raise OracleError(rc)
    return {n: getattr(out, n) for n in ALIGN_FIELDS}


def align_batch(bases, offsets, lead, trail, settings=None, threads=1):
    """Dovetail alignments of the given pairs (ids 1-based) on `threads` OpenMP
    threads (0 = all): the aligner leg of bench.py's CPU baseline."""
    s = settings or default_settings()
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ld = np.ascontiguousarray(lead, dtype=np.int32)
    tr = np.ascontiguousarray(trail, dtype=np.int32)
    out = (Align * max(len(ld), 1))()
    P = C.POINTER
    rc = lib().orc_align_batch(bases, off.ctypes.data_as(P(C.c_uint64)), len(off) - 1, ld.ctypes.data_as(P(C.c_int32)),
                               tr.ctypes.data_as(P(C.c_int32)), len(ld), C.byref(s), threads, out)
    if rc:
        raise OracleError(rc)
    raw = np.ctypeslib.as_array(C.cast(out, P(C.c_int32)), shape=(max(len(ld), 1) * len(ALIGN_FIELDS),))
    return raw.reshape(-1, len(ALIGN_FIELDS))[:len(ld)].copy()


def lead_rows(bases, offsets, leads, settings=None, threads=0):
    """PairData rows of the sampled leads (orc_lead_rows): returns (row_off,
    snd, cnt) with lead leads[i]'s partners (ascending) and counts in
    [row_off[i], row_off[i + 1]).  leads: 1-based, strictly ascending."""
    s = settings or default_settings()
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ld = np.ascontiguousarray(leads, dtype=np.int32)
    ro = np.zeros(len(ld) + 1, dtype=np.uint64)
    sp, cp = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
    P = C.POINTER
    rc = lib().orc_lead_rows(bases, off.ctypes.data_as(P(C.c_uint64)), len(off) - 1, C.byref(s),
                             ld.ctypes.data_as(P(C.c_int32)), len(ld), threads, ro.ctypes.data_as(P(C.c_uint64)),
                             C.byref(sp), C.byref(cp))
    if rc:
        raise OracleError(rc)
    n = int(ro[-1])
    snd, cnt = _arr(sp, n, np.int32), _arr(cp, n, np.int32)
    lib().orc_free(C.cast(sp, C.c_void_p))
    lib().orc_free(C.cast(cp, C.c_void_p))
    return ro.astype(np.int64), snd, cnt


def lead_stats(genome, starts, lens, leads, settings=None, threads=0, log_ranks=0):
    """Per sampled lead (orc_lead_stats), over reads genome[starts[r]:starts[r] +
    lens[r]]: an (n_leads, 4) int64 array of distinct partners, role pairs with the
    lead as fst, partials over 2^log_ranks hash-range owners, dispatched partners."""
    s = settings or default_settings()
    st = np.ascontiguousarray(starts, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.int32)
    ld = np.ascontiguousarray(leads, dtype=np.int32)
    out = np.zeros((len(ld), 4), dtype=np.uint64)
    P = C.POINTER
    rc = lib().orc_lead_stats(genome, st.ctypes.data_as(P(C.c_uint64)), ln.ctypes.data_as(P(C.c_int32)), len(st),
                              C.byref(s), ld.ctypes.data_as(P(C.c_int32)), len(ld), threads, log_ranks,
                              out.ctypes.data_as(P(C.c_uint64)))
    if rc:
        raise OracleError(rc)
    return out.astype(np.int64)


def synth_genome(seed, n, gc=0.5, threads=0):
    """bench.synth_workload's genome as bytes (orc_synth_genome: one C pass,
    not numpy's temporaries -- configs[4]'s 1.375 Gbp)."""
    buf = C.create_string_buffer(n)
    lib().orc_synth_genome(seed, n, gc, buf, threads)
    return buf.raw[:n]


def max_threads():
    return int(lib().orc_max_threads())


def trove_order(keys):
    keys = np.ascontiguousarray(keys, dtype=np.int32)
    out = np.zeros(len(keys), dtype=np.int32)
    cap = C.c_int32()
    rc = lib().orc_trove_order(keys.ctypes.data_as(C.POINTER(C.c_int32)), len(keys),
                               out.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(cap))
    if rc:
        raise OracleError(rc)
    return out, cap.value
