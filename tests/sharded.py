"""sharded.py -- TEST HARNESS for the sharded hash stage's per-rank C ABI
(sa_dist_*): the product path is the library's own orchestration (multi.cpp:
sa_ctx_create_multi / sa_ctx_create_rank, RCCL inside libsa_overlap), which
bench.py and the CLI use.  This module drives the same per-rank steps from
Python so the tests can run them over gloo on CPU (with a numpy model worker)
and compare the HIP worker against it; nothing in the product imports it.

The multi-GPU hash stage: one process and one
context per GPU, exchanges over torch.distributed (backend "nccl" is RCCL on
ROCm and moves device tensors over xGMI; "gloo" stages through host memory,
used by the CPU tests and single-GPU multi-process checks).

Rank r holds reads [starts[r], starts[r+1]) of the global set (global id =
index + 1).  One build step:

  emit       local k-mer records, grouped by owner rank = top log2(P) bits of
             the mixed seqHash (whole buckets per owner)
  exchange 1 all-to-all of the 8-byte records (mixed hash << 32 | the
             occurrence index local to the source rank; the owner re-derives
             read and loc rank from the source's segment of its receive buffer)
  count      owner builds its buckets and counts partial (lead, trail) pairs
             for every read over ITS buckets (KmerTable.calcPairData,
             KmerTable.scala:85-149, restricted to a hash range)
  exchange 2 all-to-all of the partials (u32 lead, trail, count) to the rank
             owning the lead
  reduce     sum the partials, apply [minCollisions, maxCollisions]
             (calcDispatchData, KmerTable.scala:155-187): this rank's
             dispatch in the wide canonical order (lead desc, trail asc)

Alignment: the packed reads are all-gathered once (2 bits/base), then each
rank aligns its own leads.  Concatenating the ranks' dispatch / .ovl in
descending rank order gives the single-GPU wide-id output exactly.

A worker implements the per-rank compute on buffers the orchestrator owns:
`HipWorker` wraps saoverlap.Overlapper (device pointers of torch tensors on
this rank's GPU); tests/dist_model.py is a numpy model with the same methods.

Lead-range passes (build(budget=...)): for read sets whose partials do not fit
at once, each pass p of npass counts, exchanges and reduces only the leads
[s_r + len_r * p // npass, s_r + len_r * (p + 1) // npass) of every owner r;
the ranks agree on npass (the largest of their plans) and run the passes from
the last to the first, so each rank's dispatch stays lead-descending.
"""
import numpy as np
import torch
import torch.distributed as dist


class HipWorker:
    """Per-rank compute on the GPU (libsa_overlap.so, sa_dist_*)."""

    device_kind = "cuda"

    def __init__(self, overlapper):
        self.ov = overlapper

    def init(self, rank, nranks, starts, lengths):
        self.ov.dist_init(rank, nranks, starts, lengths)

    def local_kmers(self):
        return self.ov.dist_local_kmers()

    def emit(self, send_recs):
        return self.ov.dist_emit(send_recs.data_ptr())

    def count(self, recv_recs, recv_counts):
        return self.ov.dist_count(recv_recs.data_ptr(), recv_counts)

    def partials(self, fst, snd, cnt):
        self.ov.dist_partials(fst.data_ptr(), snd.data_ptr(), cnt.data_ptr())

    def reduce(self, fst, snd, cnt, n):
        self.ov.dist_reduce(fst.data_ptr(), snd.data_ptr(), cnt.data_ptr(), n)

    # lead-range passes (sa_dist_buckets / _plan / _count_pass / _reduce_pass)
    def buckets(self, recv_recs, recv_counts):
        return self.ov.dist_buckets(recv_recs.data_ptr(), recv_counts)

    def plan(self, budget):
        return self.ov.dist_plan(budget)

    def count_pass(self, p, npass):
        return self.ov.dist_count_pass(p, npass)

    def reduce_pass(self, fst, snd, cnt, n, p, npass):
        self.ov.dist_reduce_pass(fst.data_ptr(), snd.data_ptr(), cnt.data_ptr(), n, p, npass)

    def code_words(self):
        return self.ov.dist_codes()

    def codes(self, codes, bad):
        self.ov.dist_codes(codes.data_ptr(), bad.data_ptr())

    def set_reads(self, codes, bad, nwords):
        self.ov.dist_set_reads(codes.data_ptr(), bad.data_ptr(), nwords)

    def align(self):
        self.ov.device_align()

    def stats(self):
        return self.ov.stats()


class ShardedOverlapper:
    """Orchestrates one rank of the sharded hash stage and alignment."""

    def __init__(self, worker, rank, nranks, starts, lengths, device, group=None):
        self.w = worker
        self.rank, self.P = rank, nranks
        self.starts = np.asarray(starts, dtype=np.int64)
        self.lengths = np.asarray(lengths, dtype=np.int32)
        self.dev = torch.device(device)
        self.group = group
        backend = dist.get_backend(group)
        # gloo exchanges host tensors; nccl (RCCL) exchanges device tensors
        self.xdev = torch.device("cpu") if backend == "gloo" else self.dev
        self._bufs = {}
        self.exchanged_bytes = 0
        worker.init(rank, nranks, self.starts, self.lengths)

    # -- buffers reused across steps (grown, never shrunk) --------------------
    def _buf(self, name, n, dtype):
        b = self._bufs.get(name)
        if b is None or b.numel() < max(n, 1):
            b = torch.empty(max(n, 1) + max(n, 1) // 8, dtype=dtype, device=self.dev)
            self._bufs[name] = b
        return b[:n] if n else b[:0]

    # -- collectives ----------------------------------------------------------
    def _a2a_counts(self, counts):
        t = torch.as_tensor(np.asarray(counts, dtype=np.int64), device=self.xdev)
        r = torch.empty_like(t)
        dist.all_to_all_single(r, t, group=self.group)
        return r.cpu().numpy().astype(np.int64)

    def _ready(self):
        """Device collectives (RCCL) complete on torch's current stream, but the
        library runs its kernels on its own non-blocking HIP stream: wait for the
        current stream before handing received buffers to the worker."""
        if self.dev.type == "cuda":
            torch.cuda.current_stream(self.dev).synchronize()

    def _a2a(self, recv, send, recv_counts, send_counts):
        rs = [int(x) for x in recv_counts]
        ss = [int(x) for x in send_counts]
        self.exchanged_bytes += int(send.element_size()) * (sum(ss) - ss[self.rank])
        if self.xdev == self.dev:
            dist.all_to_all_single(recv, send, rs, ss, group=self.group)
            return
        s_h = send.to(self.xdev)
        r_h = torch.empty(recv.shape, dtype=recv.dtype, device=self.xdev)
        dist.all_to_all_single(r_h, s_h, rs, ss, group=self.group)
        recv.copy_(r_h)

    # -- one build step ---------------------------------------------------------
    def build(self, budget=None):
        """One step; with `budget` (partial entries per rank and pass) the count runs
        in lead-range passes: buckets once, every rank plans its passes, the ranks
        take the largest pass count, then per pass (npass - 1 down to 0) count ->
        exchange 2 -> reduce, each appending its leads' dispatch."""
        w = self.w
        n = w.local_kmers()
        sk = self._buf("sk", n, torch.int64)
        counts = w.emit(sk)
        rcounts = self._a2a_counts(counts)
        nr = int(rcounts.sum())
        rk = self._buf("rk", nr, torch.int64)
        self._a2a(rk, sk, rcounts, counts)
        self._ready()
        if budget is None:
            self._exchange2(w.count(rk, rcounts), w.reduce)
            self.npass = 1
            return
        self.bound = w.buckets(rk, rcounts)
        mine = w.plan(budget)
        self.npass = npass = int(self._a2a_counts([mine] * self.P).max())  # every rank's plan: the max
        for p in range(npass - 1, -1, -1):
            self._exchange2(w.count_pass(p, npass),
                            lambda qf, qs, qc, nq, p=p: w.reduce_pass(qf, qs, qc, nq, p, npass))

    def _exchange2(self, pcounts, reduce):
        w = self.w
        npart = int(np.sum(pcounts))
        pf = self._buf("pf", npart, torch.int32)
        ps = self._buf("ps", npart, torch.int32)
        pc = self._buf("pc", npart, torch.int32)
        w.partials(pf, ps, pc)
        rp = self._a2a_counts(pcounts)
        nq = int(rp.sum())
        qf = self._buf("qf", nq, torch.int32)
        qs = self._buf("qs", nq, torch.int32)
        qc = self._buf("qc", nq, torch.int32)
        self._a2a(qf, pf, rp, pcounts)
        self._a2a(qs, ps, rp, pcounts)
        self._a2a(qc, pc, rp, pcounts)
        self._ready()
        reduce(qf, qs, qc, nq)

    # -- reads for alignment: all-gather of the packed words ---------------------
    def gather_reads(self):
        w = self.w
        nw = w.code_words()
        nl = int(self.starts[self.rank + 1] - self.starts[self.rank])
        words = (self.lengths.astype(np.int64) + 15) // 16
        per_rank_words = [int(words[self.starts[r]:self.starts[r + 1]].sum()) for r in range(self.P)]
        per_rank_reads = [int(self.starts[r + 1] - self.starts[r]) for r in range(self.P)]
        assert per_rank_words[self.rank] == nw
        mw, mr = max(max(per_rank_words), 1), max(max(per_rank_reads), 1)
        codes = self._buf("lc", mw, torch.int32)
        bad = self._buf("lb", mr, torch.int32)
        w.codes(codes[:nw], bad[:nl])
        # equal-size all-gather of padded slices, then compact in rank order
        send_c = codes[:mw].to(self.xdev)
        send_b = bad[:mr].to(self.xdev)
        gc = torch.empty(self.P * mw, dtype=torch.int32, device=self.xdev)
        gb = torch.empty(self.P * mr, dtype=torch.int32, device=self.xdev)
        dist.all_gather_into_tensor(gc, send_c, group=self.group)
        dist.all_gather_into_tensor(gb, send_b, group=self.group)
        self.exchanged_bytes += 4 * (mw + mr) * (self.P - 1)
        allc = torch.cat([gc[r * mw:r * mw + per_rank_words[r]] for r in range(self.P)]).to(self.dev)
        allb = torch.cat([gb[r * mr:r * mr + per_rank_reads[r]] for r in range(self.P)]).to(self.dev)
        self._ready()
        w.set_reads(allc, allb, int(sum(per_rank_words)))

    def align(self):
        self.w.align()

    def stats(self):
        return self.w.stats()
