"""dist_model.py -- a numpy model of one rank of the sharded hash stage, with the
same worker interface as sharded.HipWorker (test infrastructure only).

It restates the reference semantics the sharded protocol has to preserve:
seqHash over min(16, k) chars (ObjectStore.scala:48-67), float32 loc = i/(L-k)
and the st / md / en tags (BioLibs.scala:56-58, KmerTable.scala:106-115),
role pairs st x md and en x md per bucket with fst = the larger loc, ties to
the md occurrence, same-read pairs skipped (KmerTable.scala:57-80, :118-128),
and the [min, max] collision filter (:155-187), in wide-id form.  Records are
owned by a hash of the bucket; the orchestrator moves them between ranks.
"""
import numpy as np

CODE = {"A": 0, "C": 1, "T": 2, "G": 3}


def seq_hash(s):
    h = 0
    for ch in s:
        h = ((h << 2) ^ CODE.get(ch, 0)) & 0xFFFFFFFF
    return h


class NumpyWorker:
    device_kind = "cpu"

    def __init__(self, reads, k=15, edge=0.4, center=0.4, min_c=7, max_c=222):
        self.reads = [r.upper() for r in reads]
        self.k, self.m = k, min(16, k)
        f32 = np.float32
        self.head, self.tail = f32(edge), f32(1.0) - f32(edge)
        half = f32(center) * f32(0.5)
        self.mid_lo, self.mid_hi = f32(0.5) - half, f32(0.5) + half
        self.min_c, self.max_c = min_c, max_c
        self.lead = self.trail = self.dcount = np.zeros(0, dtype=np.int32)
        self.role_pairs = 0

    def init(self, rank, nranks, starts, lengths):
        self.rank, self.P = rank, nranks
        self.starts = np.asarray(starts, dtype=np.int64)
        lengths = np.asarray(lengths, dtype=np.int64)
        self.lengths = lengths
        self.gocc = np.concatenate([[0], np.cumsum(np.maximum(lengths - self.k + 1, 0))]).astype(np.int64)
        self.logp = int(nranks).bit_length() - 1

    def _owner(self, h):
        return 0 if self.logp == 0 else ((h * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - self.logp)

    def local_kmers(self):
        return int(sum(max(len(r) - self.k + 1, 0) for r in self.reads))

    def emit(self, send_recs):
        # 8-byte records: hash << 32 | occurrence index local to this rank (the
        # owner re-derives read, position and loc from it and the source rank)
        recs = []
        g = 0
        for r in self.reads:
            for i in range(len(r) - self.k + 1):
                h = seq_hash(r[i:i + self.m])
                recs.append((self._owner(h), (h << 32) | g))
                g += 1
        recs.sort(key=lambda x: x[0])  # stable: occurrence order within an owner
        n = len(recs)
        if n:
            send_recs[:n].copy_(_t(np.array([x[1] for x in recs], dtype=np.uint64).view(np.int64)))
        counts = np.zeros(self.P, dtype=np.int64)
        for o, _ in recs:
            counts[o] += 1
        return counts

    def _tags(self, loc):
        st = loc <= self.head
        md = (self.mid_lo <= loc) and (loc <= self.mid_hi)
        en = self.tail <= loc
        return st, md, en

    def buckets(self, recv_recs, recv_counts):
        """This rank's buckets and their partial pairs (all leads), plus every
        read's upper bound of the partials it leads here: its role pairs as fst,
        same-read ones included (>= its distinct partials)."""
        n = int(np.sum(recv_counts))
        recs = recv_recs[:n].numpy().view(np.uint64)
        src = np.repeat(np.arange(self.P), np.asarray(recv_counts, dtype=np.int64))
        g = (recs & np.uint64(0xFFFFFFFF)).astype(np.int64) + self.gocc[self.starts[src]]
        rid = np.searchsorted(self.gocc, g, side="right") - 1
        pos = g - self.gocc[rid]
        d = self.lengths[rid] - self.k
        buckets = {}
        for key, r, p, dd in zip(recs.tolist(), rid.tolist(), pos.tolist(), d.tolist()):
            h = key >> 32
            loc = np.float32(p) / np.float32(dd) if dd > 0 else np.float32("nan")
            buckets.setdefault(h, []).append((r, loc))
        pairs = {}
        rp = 0
        self.rbound = np.zeros(len(self.lengths), dtype=np.int64)
        for occ in buckets.values():
            st, md, en = [], [], []
            for r, loc in occ:
                if np.isnan(loc):
                    continue
                s_, m_, e_ = self._tags(loc)
                if s_:
                    st.append((r, loc))
                if m_:
                    md.append((r, loc))
                if e_:
                    en.append((r, loc))
            for edge_list in (st, en):
                for ra, la in edge_list:
                    for rb, lb in md:
                        rp += 1
                        fst, snd = (ra, rb) if la > lb else (rb, ra)  # tie: md occurrence first
                        self.rbound[fst] += 1
                        if ra == rb:
                            continue
                        pairs[(fst, snd)] = pairs.get((fst, snd), 0) + 1
        self.role_pairs = rp
        self._pairs = sorted(pairs.items())
        return int(self.rbound.sum())

    def _range(self, r, p, npass):
        s, ln = int(self.starts[r]), int(self.starts[r + 1] - self.starts[r])
        return s + ln * p // npass, s + ln * (p + 1) // npass

    def plan(self, budget):
        """The fewest passes whose every pass's bound on this rank is <= budget
        (sa_dist_plan)."""
        total = int(self.rbound.sum())
        if total <= budget:
            return 1
        cum = np.concatenate([[0], np.cumsum(self.rbound)])
        maxlen = max(1, int(np.max(np.diff(self.starts))))

        def worst(np_):
            return max(sum(int(cum[b] - cum[a]) for a, b in (self._range(r, p, np_) for r in range(self.P)))
                       for p in range(np_))
        np_ = min(maxlen, -(-total // budget))
        while np_ < maxlen and worst(np_) > budget:
            np_ = min(maxlen, np_ + max(1, np_ // 8))
        return np_

    def count_pass(self, p, npass):
        rg = [self._range(r, p, npass) for r in range(self.P)]
        items = [(k, c) for k, c in self._pairs if any(a <= k[0] < b for a, b in rg)]
        self._pf = np.array([a for (a, _), _ in items], dtype=np.int32)
        self._ps = np.array([b for (_, b), _ in items], dtype=np.int32)
        self._pc = np.array([c for _, c in items], dtype=np.int32)
        owner = np.searchsorted(self.starts, self._pf, side="right") - 1
        return np.bincount(owner, minlength=self.P).astype(np.int64)

    def count(self, recv_recs, recv_counts):
        self.buckets(recv_recs, recv_counts)
        return self.count_pass(0, 1)

    def partials(self, fst, snd, cnt):
        n = len(self._pf)
        if n:
            fst[:n].copy_(_t(self._pf))
            snd[:n].copy_(_t(self._ps))
            cnt[:n].copy_(_t(self._pc))

    def reduce_pass(self, fst, snd, cnt, n, p, npass):
        """This rank's leads of pass p, appended (passes run npass - 1 down to 0)."""
        f, s, c = fst[:n].numpy(), snd[:n].numpy(), cnt[:n].numpy()
        a0, a1 = self._range(self.rank, p, npass)
        tot = {}
        for a, b, x in zip(f.tolist(), s.tolist(), c.tolist()):
            assert a0 <= a < a1, "a partial outside this pass's leads"
            tot[(a, b)] = tot.get((a, b), 0) + x
        keep = sorted(((a, b, x) for (a, b), x in tot.items() if self.min_c <= x <= self.max_c),
                      key=lambda t: (-t[0], t[1]))
        if p == npass - 1:
            self.lead = self.trail = self.dcount = np.zeros(0, dtype=np.int32)
            self.distinct = 0
        self.lead = np.concatenate([self.lead, np.array([a + 1 for a, _, _ in keep], dtype=np.int32)])
        self.trail = np.concatenate([self.trail, np.array([b + 1 for _, b, _ in keep], dtype=np.int32)])
        self.dcount = np.concatenate([self.dcount, np.array([x for _, _, x in keep], dtype=np.int32)])
        self.distinct += len(tot)

    def reduce(self, fst, snd, cnt, n):
        self.reduce_pass(fst, snd, cnt, n, 0, 1)

    def stats(self):
        return {"role_pairs": self.role_pairs, "dispatched": len(self.lead)}


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a))
