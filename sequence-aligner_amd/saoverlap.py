"""saoverlap -- Python binding of the MI355X hash-overlap stage (ctypes over libsa_overlap.so).

Mirrors the reference's calc-overlaps path (rohit507/Sequence-Aligner,
src/Project4.scala:56-60) through the C ABI in include/sa_overlap.h:

    ov = Overlapper(kmer_size=15)        # AlignSettings (ObjectStore.scala:17-36)
    ov.read_fasta("reads.seq")           # BioLibs.readSeq (BioLibs.scala:26-50)
    ov.build()                           # KmerTable.calcPairData + calcDispatchData
    lead, trail, count = ov.dispatch()   # DispatchData order (KmerTable.scala:251-271)
    ov.align()                           # genBlockMTAlign -> generateFastDovetailAlignmentSet
    ov.ovl()                             # Project4.calcOverlaps bytes

There is no CPU fallback: the HIP library must be built (make -C sequence-aligner_amd)
and a gfx950 device present, otherwise construction raises.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SA_OVERLAP_LIB") or os.path.join(HERE, "build", "libsa_overlap.so")  # env: experiments

SA_IDS_AUTO, SA_IDS_STRICT, SA_IDS_WIDE = 0, 1, 2
SA_OPT_KEEP_PAIRS, SA_OPT_TIMING, SA_OPT_ALIGN_KERNEL, SA_OPT_ALIGNER, SA_OPT_LOCAL_BATCH_MB = 1, 2, 3, 4, 5
SA_OPT_SERIAL_SHARDS, SA_OPT_LAUNCH_SLICE, SA_OPT_FIRST_PASS = 6, 7, 8
SA_OPT_PASS_BUDGET_MB, SA_OPT_LEAN_MEMORY = 9, 10   # sharded contexts: lead-range passes, scratch release
SA_ALIGNER_LINEAR, SA_ALIGNER_QUADRATIC = 0, 1   # --linear-align / --quadratic-align
SA_STATS_PER_READ_REGIONS, SA_STATS_RECOUNTED = 1, 2    # sa_stats.flags bits of the last build
ALIGN_AUTO, ALIGN_GROUP, ALIGN_LANE, ALIGN_LANE_SUMMARY = 0, 1, 2, 3
STAGES = ("pack", "emit", "sort", "buckets", "pairs", "order", "align", "exchange",
          "upload", "replay", "readback", "format", "write")  # (the last five: host wall clock)
ERRORS = {-1: "SA_E_ARG", -2: "SA_E_INPUT", -3: "SA_E_NON_ACGT", -4: "SA_E_ID_RANGE", -5: "SA_E_SHORT_READ",
          -6: "SA_E_DEGENERATE", -7: "SA_E_HIP", -8: "SA_E_NOMEM", -9: "SA_E_RCCL", -10: "SA_E_STATE",
          -11: "SA_E_OVERFLOW"}
FLAG_DUD, FLAG_VALID, FLAG_OVL_VALID = 1, 2, 4

# exported symbols declared in include/sa_overlap.h
EXPORTS = ("sa_default_settings", "sa_ctx_create", "sa_ctx_destroy", "sa_last_error", "sa_load_hoxd",
           "sa_add_reads", "sa_read_fasta", "sa_num_reads", "sa_get_read", "sa_build_candidates", "sa_get_dispatch",
           "sa_get_pairs", "sa_kmer_histogram", "sa_align", "sa_get_alignments", "sa_write_ovl", "sa_get_ovl", "sa_write_afg", "sa_set_option",
           "sa_get_stats", "sa_get_stage_times", "sa_reset_stage_times", "sa_device_build", "sa_device_align",
           "sa_sync", "sa_dist_init", "sa_dist_local_kmers", "sa_dist_emit", "sa_dist_count", "sa_dist_partials",
           "sa_dist_reduce", "sa_dist_codes", "sa_dist_set_reads", "sa_ctx_create_multi", "sa_rccl_unique_id",
           "sa_ctx_create_rank", "sa_exchanged_bytes", "sa_dist_buckets", "sa_dist_plan", "sa_dist_count_pass",
           "sa_dist_reduce_pass", "sa_get_shard_info")
RCCL_ID_BYTES = 128


class Settings(C.Structure):
    _fields_ = [("kmer_size", C.c_int32), ("min_overlap", C.c_int32), ("max_ignore", C.c_int32),
                ("gap_open", C.c_int32), ("gap_extend", C.c_int32), ("min_collisions", C.c_int32),
                ("max_collisions", C.c_int32), ("min_identity", C.c_float), ("kmer_edge", C.c_float),
                ("kmer_center", C.c_float), ("cost", C.c_int32 * 16), ("id_mode", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("kmers", "buckets", "role_pairs", "pairs", "dispatched", "aligned",
                                           "ovl_records", "dp_cells")] + [("id_mode", C.c_int32),
                                                                          ("flags", C.c_int32)]


ALIGN_FIELDS = ("lead", "trail", "start_i", "start_j", "end_i", "end_j", "correct", "error", "ahg", "bhg",
                "flags", "reserved")

_lib = None


def lib():
    """Load libsa_overlap.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libsa_overlap.so not built: run `make -C %s`" % HERE)
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        vp = C.c_void_p
        L.sa_default_settings.argtypes = [P(Settings)]
        L.sa_default_settings.restype = None
        L.sa_ctx_create.argtypes = [P(Settings), C.c_int, P(vp)]
        L.sa_ctx_destroy.argtypes = [vp]
        L.sa_ctx_destroy.restype = None
        L.sa_last_error.argtypes = [vp]
        L.sa_last_error.restype = C.c_char_p
        L.sa_load_hoxd.argtypes = [P(Settings), C.c_char_p]
        L.sa_add_reads.argtypes = [vp, C.c_char_p, P(C.c_uint64), C.c_uint32]
        L.sa_read_fasta.argtypes = [vp, C.c_char_p]
        L.sa_num_reads.argtypes = [vp]
        L.sa_num_reads.restype = C.c_uint32
        for fn in ("sa_build_candidates", "sa_align", "sa_device_build", "sa_device_align", "sa_sync",
                   "sa_reset_stage_times"):
            getattr(L, fn).argtypes = [vp]
        L.sa_get_dispatch.argtypes = [vp, P(P(C.c_int32)), P(P(C.c_int32)), P(P(C.c_int32)), P(C.c_size_t)]
        L.sa_get_pairs.argtypes = [vp, P(P(C.c_int32)), P(P(C.c_int32)), P(P(C.c_int32)), P(C.c_size_t)]
        L.sa_get_alignments.argtypes = [vp, P(vp), P(C.c_size_t)]
        L.sa_get_read.argtypes = [vp, C.c_uint32, P(C.c_char_p), P(C.c_size_t)]
        L.sa_kmer_histogram.argtypes = [vp, P(C.c_uint64), P(P(C.c_uint64)), P(P(C.c_uint64)), P(C.c_size_t)]
        L.sa_write_ovl.argtypes = [vp, C.c_char_p]
        L.sa_get_ovl.argtypes = [vp, P(C.c_char_p), P(C.c_size_t)]
        L.sa_write_afg.argtypes = [vp, C.c_char_p, P(C.c_char_p), C.c_int]
        L.sa_set_option.argtypes = [vp, C.c_int, C.c_int64]
        L.sa_get_stats.argtypes = [vp, P(Stats)]
        L.sa_get_stage_times.argtypes = [vp, P(C.c_double), P(C.c_uint64), C.c_int]
        L.sa_dist_init.argtypes = [vp, C.c_int, C.c_int, P(C.c_uint32), P(C.c_int32)]
        L.sa_dist_local_kmers.argtypes = [vp, P(C.c_uint64)]
        L.sa_dist_emit.argtypes = [vp, vp, P(C.c_uint64)]
        L.sa_dist_count.argtypes = [vp, vp, P(C.c_uint64), P(C.c_uint64)]
        L.sa_dist_partials.argtypes = [vp, vp, vp, vp]
        L.sa_dist_reduce.argtypes = [vp, vp, vp, vp, C.c_uint64]
        L.sa_dist_codes.argtypes = [vp, vp, vp, P(C.c_uint64)]
        L.sa_dist_set_reads.argtypes = [vp, vp, vp, C.c_uint64]
        L.sa_ctx_create_multi.argtypes = [P(Settings), C.c_int, C.c_int, P(vp)]
        L.sa_rccl_unique_id.argtypes = [C.c_char_p, C.c_size_t]
        L.sa_ctx_create_rank.argtypes = [P(Settings), C.c_int, C.c_int, C.c_int, C.c_char_p, P(vp)]
        L.sa_exchanged_bytes.argtypes = [vp]
        L.sa_exchanged_bytes.restype = C.c_uint64
        # (round 6 entry points; a library built from an older tree -- SA_OVERLAP_LIB,
        # same-box A/B runs -- lacks them and the bindings stay unset)
        if hasattr(L, "sa_get_shard_info"):
            L.sa_dist_buckets.argtypes = [vp, vp, P(C.c_uint64), P(C.c_uint64)]
            L.sa_dist_plan.argtypes = [vp, C.c_uint64, P(C.c_uint32)]
            L.sa_dist_count_pass.argtypes = [vp, C.c_uint32, C.c_uint32, P(C.c_uint64)]
            L.sa_dist_reduce_pass.argtypes = [vp, vp, vp, vp, C.c_uint64, C.c_uint32, C.c_uint32]
            L.sa_get_shard_info.argtypes = [vp, P(C.c_uint32), P(C.c_uint64), P(C.c_uint64)]
        _lib = L
    return _lib


def rccl_unique_id():
    """An RCCL unique id (bytes) for Overlapper(rank=..., nranks=..., rccl_id=...):
    create it on one rank and broadcast it to the others."""
    buf = C.create_string_buffer(RCCL_ID_BYTES)
    rc = lib().sa_rccl_unique_id(buf, RCCL_ID_BYTES)
    if rc:
        raise SAError(rc, "ncclGetUniqueId failed")
    return buf.raw


class SAError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__("%s (%d): %s" % (ERRORS.get(code, "?"), code, msg))
        self.code = code
        self.name = ERRORS.get(code, "?")


def settings(**kw):
    """AlignSettings with Project4.readArgs defaults; keyword overrides use the C field names."""
    s = Settings()
    lib().sa_default_settings(C.byref(s))
    for k, v in kw.items():
        if k == "cost":
            for i, x in enumerate(np.asarray(v).reshape(16)):
                s.cost[i] = int(x)
        elif k == "hoxd_file":
            rc = lib().sa_load_hoxd(C.byref(s), v.encode())
            if rc:
                raise SAError(rc, "cannot read " + v)
        else:
            setattr(s, k, v)
    return s


def _arr(ptr, n):
    if n == 0:
        return np.zeros(0, dtype=np.int32)
    return np.ctypeslib.as_array(ptr, shape=(n,)).copy()


class Overlapper:
    """One context = one AlignSettings + one KmerTable, on one GPU or sharded:
    gpus=P (devices 0..P-1, RCCL exchanges), shards=S (virtual shards on one
    device), or rank/nranks/rccl_id (one process per GPU, collective calls)."""

    def __init__(self, device=0, timing=False, keep_pairs=False, align_kernel=ALIGN_AUTO,
                 aligner=SA_ALIGNER_LINEAR, local_batch_mb=None, gpus=1, shards=1, rank=None, nranks=None,
                 rccl_id=None, serial_shards=False, launch_slice=0, first_pass=0, pass_budget_mb=0,
                 lean_memory=False, **kw):
        self.s = settings(**kw)
        h = C.c_void_p()
        if rank is not None:
            rc = lib().sa_ctx_create_rank(C.byref(self.s), device, rank, nranks, rccl_id, C.byref(h))
        elif gpus > 1 or shards > 1:
            rc = lib().sa_ctx_create_multi(C.byref(self.s), gpus, max(gpus, shards), C.byref(h))
        else:
            rc = lib().sa_ctx_create(C.byref(self.s), device, C.byref(h))
        if rc:
            raise SAError(rc, "cannot create the context (device %d, gpus %d, shards %d, rank %s)"
                          % (device, gpus, shards, rank))
        self.h = h
        if timing:
            self._chk(lib().sa_set_option(h, SA_OPT_TIMING, 1))
        if keep_pairs:
            self._chk(lib().sa_set_option(h, SA_OPT_KEEP_PAIRS, 1))
        if align_kernel != ALIGN_AUTO:
            self._chk(lib().sa_set_option(h, SA_OPT_ALIGN_KERNEL, align_kernel))
        if aligner != SA_ALIGNER_LINEAR:
            self._chk(lib().sa_set_option(h, SA_OPT_ALIGNER, aligner))
        if local_batch_mb is not None:
            self._chk(lib().sa_set_option(h, SA_OPT_LOCAL_BATCH_MB, local_batch_mb))
        if serial_shards:
            self._chk(lib().sa_set_option(h, SA_OPT_SERIAL_SHARDS, 1))
        if launch_slice:
            self._chk(lib().sa_set_option(h, SA_OPT_LAUNCH_SLICE, launch_slice))
        if first_pass:
            self._chk(lib().sa_set_option(h, SA_OPT_FIRST_PASS, first_pass))
        if pass_budget_mb:
            self._chk(lib().sa_set_option(h, SA_OPT_PASS_BUDGET_MB, pass_budget_mb))
        if lean_memory:
            self._chk(lib().sa_set_option(h, SA_OPT_LEAN_MEMORY, 1))

    def kmer_histogram(self):
        """(uniques, {bucket size: number of hashes}) -- KmerTable.uniqueKmers /
        kmerCollisionHistogram (KmerTable.scala:189-221)."""
        u = C.c_uint64()
        sp, cp = C.POINTER(C.c_uint64)(), C.POINTER(C.c_uint64)()
        n = C.c_size_t()
        self._chk(lib().sa_kmer_histogram(self.h, C.byref(u), C.byref(sp), C.byref(cp), C.byref(n)))
        return u.value, {int(sp[i]): int(cp[i]) for i in range(n.value)}

    def set_timing(self, on):
        """SA_OPT_TIMING: HIP events around every stage (sa_get_stage_times)."""
        self._chk(lib().sa_set_option(self.h, SA_OPT_TIMING, 1 if on else 0))

    def set_aligner(self, aligner):
        """SA_OPT_ALIGNER: SA_ALIGNER_LINEAR (--linear-align) or SA_ALIGNER_QUADRATIC."""
        self._chk(lib().sa_set_option(self.h, SA_OPT_ALIGNER, aligner))

    def close(self):
        if getattr(self, "h", None):
            lib().sa_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc):
        if rc:
            raise SAError(rc, (lib().sa_last_error(self.h) or b"").decode())
        return rc

    # -- input -------------------------------------------------------------
    def add_reads(self, reads):
        bs = [r.encode() if isinstance(r, str) else bytes(r) for r in reads]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        if bs:
            off[1:] = np.cumsum([len(b) for b in bs])
        self._chk(lib().sa_add_reads(self.h, b"".join(bs), off.ctypes.data_as(C.POINTER(C.c_uint64)), len(bs)))

    def add_packed(self, bases, offsets):
        """bases: bytes/uint8 array of all reads back to back; offsets: uint64[n+1]."""
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        b = bases if isinstance(bases, bytes) else np.ascontiguousarray(bases, dtype=np.uint8).tobytes()
        self._chk(lib().sa_add_reads(self.h, b, off.ctypes.data_as(C.POINTER(C.c_uint64)), len(off) - 1))

    def read_fasta(self, path):
        self._chk(lib().sa_read_fasta(self.h, path.encode()))

    @property
    def n_reads(self):
        return lib().sa_num_reads(self.h)

    # -- the hot path ------------------------------------------------------
    def build(self):
        self._chk(lib().sa_build_candidates(self.h))

    def device_build(self):
        self._chk(lib().sa_device_build(self.h))

    def align(self):
        self._chk(lib().sa_align(self.h))

    def device_align(self):
        self._chk(lib().sa_device_align(self.h))

    def sync(self):
        self._chk(lib().sa_sync(self.h))

    # -- results -----------------------------------------------------------
    def dispatch(self):
        a, b, c = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
        n = C.c_size_t()
        self._chk(lib().sa_get_dispatch(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(n)))
        return _arr(a, n.value), _arr(b, n.value), _arr(c, n.value)

    def pairs(self):
        a, b, c = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
        n = C.c_size_t()
        self._chk(lib().sa_get_pairs(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(n)))
        return _arr(a, n.value), _arr(b, n.value), _arr(c, n.value)

    def alignments(self):
        p, n = C.c_void_p(), C.c_size_t()
        self._chk(lib().sa_get_alignments(self.h, C.byref(p), C.byref(n)))
        if n.value == 0:
            return np.zeros((0, len(ALIGN_FIELDS)), dtype=np.int32)
        raw = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int32)), shape=(n.value * len(ALIGN_FIELDS),))
        return raw.reshape(n.value, len(ALIGN_FIELDS)).copy()

    def ovl(self):
        t, n = C.c_char_p(), C.c_size_t()
        self._chk(lib().sa_get_ovl(self.h, C.byref(t), C.byref(n)))
        return C.string_at(t, n.value) if n.value else b""

    def write_ovl(self, path=None):
        self._chk(lib().sa_write_ovl(self.h, path.encode() if path else None))

    def write_afg(self, path, eids=None, quality=20):
        """AMOS {RED} + {OVL} message file (sa_write_afg); eids: one name per read
        (no whitespace, ':' or braces) or None for the read ordinals."""
        arr = None
        if eids is not None:
            if len(eids) != self.n_reads:
                raise ValueError("write_afg: %d eids for %d reads" % (len(eids), self.n_reads))
            bad = [e for e in eids if e and any(ch.isspace() or ch in ":{}" for ch in e)]
            if bad:
                raise ValueError("write_afg: eid %r is not one token" % bad[0])
            arr = (C.c_char_p * len(eids))(*[e.encode() if e else None for e in eids])
        self._chk(lib().sa_write_afg(self.h, path.encode(), arr, quality))

    def stats(self):
        st = Stats()
        self._chk(lib().sa_get_stats(self.h, C.byref(st)))
        return {f[0]: getattr(st, f[0]) for f in Stats._fields_}

    def stage_times(self):
        ms = (C.c_double * len(STAGES))()
        nl = (C.c_uint64 * len(STAGES))()
        self._chk(lib().sa_get_stage_times(self.h, ms, nl, len(STAGES)))
        return {s: (ms[i], nl[i]) for i, s in enumerate(STAGES)}

    def reset_stage_times(self):
        self._chk(lib().sa_reset_stage_times(self.h))

    def exchanged_bytes(self):
        """Bytes sent to other shards so far (sharded contexts)."""
        return int(lib().sa_exchanged_bytes(self.h))

    def shard_info(self):
        """The last sharded build: {npass, partials, bound} (sa_get_shard_info) --
        its lead-range passes, the partial entries counted over all shards and passes
        (exchange 2's volume, 12 B each) and their upper bound."""
        npass, parts, bound = C.c_uint32(), C.c_uint64(), C.c_uint64()
        self._chk(lib().sa_get_shard_info(self.h, C.byref(npass), C.byref(parts), C.byref(bound)))
        return {"npass": npass.value, "partials": parts.value, "bound": bound.value}

    # ---- sharded hash stage (include/sa_overlap.h, sa_dist_*); buffers are
    # device pointers (ints), e.g. torch_tensor.data_ptr() on this context's GPU
    def dist_init(self, rank, nranks, starts, lengths):
        st = np.ascontiguousarray(starts, dtype=np.uint32)
        ln = np.ascontiguousarray(lengths, dtype=np.int32)
        self._chk(lib().sa_dist_init(self.h, rank, nranks, st.ctypes.data_as(C.POINTER(C.c_uint32)),
                                     ln.ctypes.data_as(C.POINTER(C.c_int32))))
        self.nranks = nranks

    def dist_local_kmers(self):
        n = C.c_uint64()
        self._chk(lib().sa_dist_local_kmers(self.h, C.byref(n)))
        return n.value

    def _counts(self):
        return (C.c_uint64 * self.nranks)()

    def dist_emit(self, send_recs):
        cnt = self._counts()
        self._chk(lib().sa_dist_emit(self.h, send_recs, cnt))
        return np.array(cnt[:], dtype=np.int64)

    def dist_count(self, recv_recs, recv_counts):
        """recv_counts[s]: records received from rank s (concatenated in rank order)."""
        cnt = self._counts()
        rc = (C.c_uint64 * self.nranks)(*[int(x) for x in recv_counts])
        self._chk(lib().sa_dist_count(self.h, recv_recs, rc, cnt))
        return np.array(cnt[:], dtype=np.int64)

    def dist_partials(self, fst, snd, cnt):
        self._chk(lib().sa_dist_partials(self.h, fst, snd, cnt))

    def dist_reduce(self, fst, snd, cnt, n):
        self._chk(lib().sa_dist_reduce(self.h, fst, snd, cnt, n))

    # lead-range passes (bounded partials): buckets once, then per pass (npass - 1 down
    # to 0) count -> partials -> exchange 2 -> reduce_pass
    def dist_buckets(self, recv_recs, recv_counts):
        """Returns the upper bound of this rank's partials."""
        rc = (C.c_uint64 * self.nranks)(*[int(x) for x in recv_counts])
        b = C.c_uint64()
        self._chk(lib().sa_dist_buckets(self.h, recv_recs, rc, C.byref(b)))
        return b.value

    def dist_plan(self, budget):
        n = C.c_uint32()
        self._chk(lib().sa_dist_plan(self.h, int(budget), C.byref(n)))
        return n.value

    def dist_count_pass(self, p, npass):
        cnt = self._counts()
        self._chk(lib().sa_dist_count_pass(self.h, p, npass, cnt))
        return np.array(cnt[:], dtype=np.int64)

    def dist_reduce_pass(self, fst, snd, cnt, n, p, npass):
        self._chk(lib().sa_dist_reduce_pass(self.h, fst, snd, cnt, n, p, npass))

    def dist_codes(self, codes=None, bad=None):
        nw = C.c_uint64()
        self._chk(lib().sa_dist_codes(self.h, codes, bad, C.byref(nw)))
        return nw.value

    def dist_set_reads(self, codes, bad, nwords):
        self._chk(lib().sa_dist_set_reads(self.h, codes, bad, nwords))

