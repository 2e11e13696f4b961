// multi.cpp -- sharded contexts: one sa_ctx over P shards of the read set
// (SURVEY.md 8(b) `--gpus P`, 8(e)), behind the same C ABI as a single device.
//
// The reference is one JVM process (KmerTable.scala:41-187 builds one table;
// Project4.scala:725-790 aligns its blocks on one actor pool).  Here the read
// ids are split into P contiguous ranges, one per shard, and one build is
//
//   emit        every shard: k-mer records of its reads, grouped by the shard
//               owning their hash range (sa_dist_emit)
//   exchange 1  all-to-all of the 8-byte records
//   count       every shard: buckets of its hash range, partial (lead, trail,
//               count) for every read (sa_dist_count / sa_dist_partials)
//   exchange 2  all-to-all of the partials to the shard owning the lead
//   reduce      every shard: sum, [minCollisions, maxCollisions] filter, its
//               leads' dispatch in the wide order (sa_dist_reduce)
//
// and alignment all-gathers the 2-bit packed reads once, then every shard aligns
// its own leads.  The shards' outputs concatenated in descending shard order
// are the single-device output exactly (lead descending), for any P.
//
// Shards and exchanges:
//   sa_ctx_create_multi(s, P, P)   one process, devices 0..P-1, one shard each,
//                                  exchanges = RCCL send/recv groups (xGMI),
//                                  shard compute on one host thread per device;
//   sa_ctx_create_multi(s, 1, P)   P virtual shards on device 0, exchanges =
//                                  device copies (the sharded path on one GPU);
//   sa_ctx_create_rank(...)        one process per GPU (e.g. torchrun), one
//                                  shard here, RCCL communicator from a shared
//                                  unique id; build / align / write_ovl collective.
// Each shard is a plain single-device child context driven through the
// sa_dist_* entry points of include/sa_overlap.h.
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>

#include "ctx.h"

namespace {

struct Shard {
    sa_ctx *child = nullptr;
    int device = 0;
    int rank = 0;                 // shard index in the job
    ncclComm_t comm = nullptr;
    hipStream_t xs = nullptr;     // exchange stream
    DBuf sk, rk, pf, ps, pc, qf, qs, qc, codes, bad, xbuf;
    std::vector<uint64_t> cnt, rcnt;  // per peer: elements sent / received
    uint64_t n_recv = 0, n_part = 0;
    uint64_t bound = 0;               // upper bound of this shard's partials (sa_dist_buckets)
    uint64_t mem_total = 0;           // its device's memory (hipDeviceProp_t::totalGlobalMem)
    uint32_t npass = 1;               // this shard's pass plan (sa_dist_plan)
    std::string err;
};

}  // namespace

struct sa_multi {
    int P = 1;
    bool rank_mode = false;
    bool rccl = false;
    std::vector<Shard> sh;          // the shards this process drives
    std::vector<uint32_t> starts;   // [P + 1] first global read of every shard
    std::vector<int32_t> lens;      // every global read's length
    uint64_t dist_gen = ~0ull;      // reads generation the shards hold
    bool reads_gathered = false;    // packed reads all-gathered for alignment
    bool sharded = false;           // the last build ran sharded
    bool serial = false;            // SA_OPT_SERIAL_SHARDS: shard compute one after another
    DBuf gcodes, gbad;              // virtual shards: one all-gathered copy on the device
    double x_ms = 0;                // exchange wall time (SA_STAGE_EXCHANGE)
    uint64_t x_n = 0, x_bytes = 0;
    // lead-range passes (SA_OPT_PASS_BUDGET_MB; 0 = from the free device memory) and
    // one pool of the shards' transients (SA_OPT_LEAN_MEMORY, virtual shards)
    uint64_t budget_mb = 0;
    bool lean = false;
    std::vector<DBuf> pool;         // one buffer per kPooled member (lean virtual shards)
    // the last sharded build: passes, partial entries over every shard and pass, and
    // their upper bound (sa_get_shard_info)
    uint32_t npass = 1;
    uint64_t partials = 0, bound = 0;
};

namespace {

// The per-shard transients (sort / bucket-build scratch, pair-counter regions, reduce
// scratch): with SA_OPT_LEAN_MEMORY on virtual shards -- which then run one after another --
// the shards borrow them from one pool for the length of a call instead of holding P
// copies (configs[3]'s real read set on 8 virtual shards: ~15 GB of sort scratch once, not
// 8x).  Nothing is freed between builds: HIP allocations of this size cost ~1 s per 7 GB,
// which a build that released and re-allocated them paid every time.
DBuf sa_ctx::*const kPooled[] = {&sa_ctx::d_keys,   &sa_ctx::d_keys2,  &sa_ctx::d_vals,   &sa_ctx::d_vals2,
                                 &sa_ctx::d_sorttmp, &sa_ctx::d_rl,    &sa_ctx::d_srl,    &sa_ctx::d_srl2,
                                 &sa_ctx::d_pf,     &sa_ctx::d_ps,     &sa_ctx::d_pc,     &sa_ctx::d_okeys,
                                 &sa_ctx::d_okeys2, &sa_ctx::d_ovals,  &sa_ctx::d_ovals2, &sa_ctx::d_osort,
                                 &sa_ctx::d_psum,   &sa_ctx::d_pkeep,  &sa_ctx::d_ppos,   &sa_ctx::d_tb,
                                 &sa_ctx::d_p1st,   &sa_ctx::d_ltb,    &sa_ctx::d_lmax};
constexpr size_t kNPooled = sizeof(kPooled) / sizeof(kPooled[0]);

int set_err(sa_ctx *c, int code, const std::string &msg) {
    c->err = msg;
    return code;
}

int grow(DBuf &b, size_t bytes, int device) {
    if (b.bytes >= bytes && b.p) return SA_OK;
    (void)hipSetDevice(device);
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    const size_t a = std::max<size_t>(bytes + bytes / 8, 256);
    if (hipMalloc(&b.p, a) != hipSuccess) return SA_E_NOMEM;
    b.bytes = a;
    return SA_OK;
}

void release(DBuf &b, int device) {
    if (b.p) {
        (void)hipSetDevice(device);
        (void)hipFree(b.p);
    }
    b.p = nullptr;
    b.bytes = 0;
}

bool pooled(const sa_multi *m) { return m->lean && !m->rccl && m->sh.size() > 1; }

// the pool's buffers into shard k for one call (a buffer the shard still owns -- e.g. the
// aligner's sort scratch -- goes to the pool if larger, else is freed)
void lend(sa_multi *m, sa_ctx *k) {
    if (m->pool.size() != kNPooled) m->pool.assign(kNPooled, DBuf{});
    for (size_t i = 0; i < kNPooled; ++i) {
        DBuf &cb = k->*kPooled[i], &pb = m->pool[i];
        if (cb.p && !cb.borrowed) {
            if (cb.bytes > pb.bytes) {
                if (pb.p) (void)hipFree(pb.p);
                pb = cb;
            } else {
                (void)hipFree(cb.p);
            }
        }
        cb = pb;
        cb.borrowed = pb.p != nullptr;
    }
}
// ... and back: a buffer the shard had to grow during the call replaces the pool's
void reclaim(sa_multi *m, sa_ctx *k) {
    for (size_t i = 0; i < kNPooled; ++i) {
        DBuf &cb = k->*kPooled[i], &pb = m->pool[i];
        if (cb.p && !cb.borrowed) {
            if (pb.p) (void)hipFree(pb.p);
            pb = cb;
            pb.borrowed = false;
        }
        cb = DBuf{};
    }
}

// Run f on every local shard (one host thread per shard when there are several),
// each thread bound to its shard's device.  The first failure is reported.
// lend_pool: the calls use the pooled transients (lean virtual shards; they then run one
// after another)
template <class F>
int for_shards(sa_ctx *c, F f, bool lend_pool = false) {
    sa_multi *m = c->multi;
    std::vector<int> rcs(m->sh.size(), SA_OK);
    const bool pool = pooled(m) && lend_pool;
    auto run = [&](size_t i) {
        Shard &s = m->sh[i];
        s.err.clear();
        if (hipSetDevice(s.device) != hipSuccess) { rcs[i] = SA_E_HIP; s.err = "hipSetDevice"; return; }
        if (pool) lend(m, s.child);
        rcs[i] = f(s);
        if (rcs[i] && s.err.empty()) s.err = s.child ? sa_last_error(s.child) : "";
        if (pool) {
            (void)sa_sync(s.child);
            reclaim(m, s.child);
        }
    };
    if (m->sh.size() == 1 || m->serial || pool) {
        for (size_t i = 0; i < m->sh.size(); ++i) {
            run(i);
            if (m->serial && m->sh[i].child) (void)sa_sync(m->sh[i].child);
        }
    } else {
        std::vector<std::thread> th;
        for (size_t i = 0; i < m->sh.size(); ++i) th.emplace_back(run, i);
        for (auto &t : th) t.join();
    }
    for (size_t i = 0; i < m->sh.size(); ++i)
        if (rcs[i]) return set_err(c, rcs[i], "shard " + std::to_string(m->sh[i].rank) + ": " + m->sh[i].err);
    return SA_OK;
}

std::vector<uint64_t> prefix(const std::vector<uint64_t> &v) {
    std::vector<uint64_t> o(v.size(), 0);
    uint64_t a = 0;
    for (size_t i = 0; i < v.size(); ++i) { o[i] = a; a += v[i]; }
    return o;
}

// One exchange step: local shard l sends scnt[q] elements from send + soff[q]
// to shard q and receives rcnt[q] elements from shard q into recv + roff[q].
struct Plan {
    const void *send = nullptr;
    void *recv = nullptr;
    std::vector<uint64_t> soff, scnt, roff, rcnt;
};

// One exchange of several arrays that share a plan's counts and offsets
// (parts[a] = array a's send / recv buffers per local shard): every send and
// receive of every array goes into ONE RCCL group, so the arrays travel
// together instead of one group (and one wait) per array.
struct Part {
    std::vector<const void *> send;
    std::vector<void *> recv;
};

int exchange_parts(sa_ctx *c, std::vector<Plan> &pl, const std::vector<Part> &parts, size_t elem) {
    sa_multi *m = c->multi;
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t moved = 0;
    if (m->rccl) {
        // RCCL point-to-point: over xGMI every pair of MI355X has its own link,
        // so the P - 1 sends of a shard proceed in parallel (no ring)
        ncclResult_t r = ncclGroupStart();
        for (const Part &pa : parts)
            for (size_t l = 0; l < m->sh.size() && r == ncclSuccess; ++l) {
                Shard &s = m->sh[l];
                for (int q = 0; q < m->P && r == ncclSuccess; ++q) {
                    if (pl[l].scnt[q]) {
                        r = ncclSend((const char *)pa.send[l] + pl[l].soff[q] * elem, pl[l].scnt[q] * elem, ncclUint8,
                                     q, s.comm, s.xs);
                        if (q != s.rank) moved += pl[l].scnt[q] * elem;
                    }
                    if (r == ncclSuccess && pl[l].rcnt[q])
                        r = ncclRecv((char *)pa.recv[l] + pl[l].roff[q] * elem, pl[l].rcnt[q] * elem, ncclUint8, q,
                                     s.comm, s.xs);
                }
            }
        const ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess || r2 != ncclSuccess)
            return set_err(c, SA_E_RCCL, std::string("RCCL send/recv: ") +
                                             ncclGetErrorString(r != ncclSuccess ? r : r2));
    } else {
        // virtual shards, all in this process on one device: device copies
        for (const Part &pa : parts)
            for (size_t q = 0; q < m->sh.size(); ++q)
                for (size_t l = 0; l < m->sh.size(); ++l) {
                    const uint64_t n = pl[l].scnt[q];
                    if (n != pl[q].rcnt[l]) return set_err(c, SA_E_STATE, "exchange counts disagree");
                    if (!n) continue;
                    if (hipMemcpyAsync((char *)pa.recv[q] + pl[q].roff[l] * elem,
                                       (const char *)pa.send[l] + pl[l].soff[q] * elem, n * elem,
                                       hipMemcpyDeviceToDevice, m->sh[q].xs) != hipSuccess)
                        return set_err(c, SA_E_HIP, "exchange copy");
                    if (q != l) moved += n * elem;
                }
    }
    for (Shard &s : m->sh) {
        (void)hipSetDevice(s.device);
        if (hipStreamSynchronize(s.xs) != hipSuccess) return set_err(c, SA_E_HIP, "exchange stream");
    }
    m->x_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    m->x_n += 1;
    m->x_bytes += moved;
    return SA_OK;
}

int exchange(sa_ctx *c, std::vector<Plan> &pl, size_t elem) {
    std::vector<Part> parts(1);
    for (const Plan &p : pl) {
        parts[0].send.push_back(p.send);
        parts[0].recv.push_back(p.recv);
    }
    return exchange_parts(c, pl, parts, elem);
}

// per-peer element counts: cnt[l][q] (shard l -> q) becomes rcnt[l][q] (q -> l)
int exchange_counts(sa_ctx *c) {
    sa_multi *m = c->multi;
    const int P = m->P;
    if (!m->rank_mode) {
        for (Shard &d : m->sh) {
            d.rcnt.assign(P, 0);
            for (Shard &s : m->sh) d.rcnt[s.rank] = s.cnt[d.rank];
        }
        return SA_OK;
    }
    Shard &s = m->sh[0];
    if (grow(s.xbuf, 2 * (size_t)P * 8, s.device)) return set_err(c, SA_E_NOMEM, "exchange buffer");
    uint64_t *d = (uint64_t *)s.xbuf.p;
    if (hipMemcpy(d, s.cnt.data(), (size_t)P * 8, hipMemcpyHostToDevice) != hipSuccess)
        return set_err(c, SA_E_HIP, "counts upload");
    std::vector<Plan> pl(1);
    pl[0].send = d;
    pl[0].recv = d + P;
    pl[0].soff.resize(P); pl[0].roff.resize(P);
    for (int q = 0; q < P; ++q) pl[0].soff[q] = pl[0].roff[q] = q;
    pl[0].scnt.assign(P, 1);
    pl[0].rcnt.assign(P, 1);
    int rc = exchange(c, pl, 8);
    if (rc) return rc;
    s.rcnt.assign(P, 0);
    if (hipMemcpy(s.rcnt.data(), d + P, (size_t)P * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return set_err(c, SA_E_HIP, "counts download");
    return SA_OK;
}

bool is_pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }

// Partial entries (counted by their upper bound) one shard may produce per lead-range
// pass: SA_OPT_PASS_BUDGET_MB, or from the free memory of its device after the bucket
// build.  A partial takes ~15 B of pair-counter regions, 12 B of send and 12 B of
// receive buffer and ~28 B of reduce scratch on every shard of the device, all held
// across the passes; per bound entry that is 67 B x rho, rho = 1.5 x the partials /
// bound ratio of the last build of these reads (1 before one ran: the bound counts
// partner-list elements, ~20x the partials at the bench shape).  Within [2^16, 2^31].
// (The free memory is asked for only when the shards' bounds come near it: hipMemGetInfo
// costs ~2 ms a call -- 8 serial shards of the bench shape took 35.6 -> 52.1 ms per step
// with one query per shard and build, profiles/r06/ab/ab_sharded8_meminfo.txt.)
uint64_t pass_budget(const sa_multi *m, const Shard &s) {
    uint64_t b;
    const uint64_t cap = 1ull << 31;
    if (m->budget_mb) {
        b = (m->budget_mb << 20) / 12;
    } else {
        const uint64_t per_dev = m->rccl ? 1 : m->sh.size();  // shards sharing this device
        const double rho = s.child->dist_rho_ok ? std::min(1.0, 1.5 * s.child->dist_rho + 0.01) : 1.0;
        // (pooled: every shard holds its send and receive buffers, one the regions and scratch)
        const double per_entry = rho * (pooled(m) ? 24.0 * (double)per_dev + 43.0 : 67.0 * (double)per_dev);
        if ((double)s.bound * per_entry <= 0.15 * (double)s.mem_total) return cap;  // far from the memory: one pass
        (void)hipSetDevice(s.device);
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
        b = (uint64_t)((double)fr * 0.6 / per_entry);
    }
    return std::min<uint64_t>(std::max<uint64_t>(b, 1ull << 16), cap);
}

void clear_child_reads(sa_ctx *k) {
    k->bases.clear();
    k->boff.assign(1, 0);
    k->reads_dirty = true;
    k->built = k->aligned = false;
    k->dist = false;
    k->dist_reads = false;
}

// Give every shard its id range of the current reads (single process: split
// the top context's reads; rank mode: this rank's reads, global lengths
// all-gathered) and sa_dist_init it.
int distribute(sa_ctx *c) {
    sa_multi *m = c->multi;
    if (m->dist_gen == c->reads_gen) return SA_OK;
    const int P = m->P;
    const uint32_t nl = (uint32_t)(c->boff.size() - 1);
    if (!m->rank_mode) {
        const uint64_t N = nl;
        m->starts.assign(P + 1, 0);
        for (int r = 0; r <= P; ++r) m->starts[r] = (uint32_t)(N * (uint64_t)r / (uint64_t)P);
        m->lens.resize(N);
        for (uint32_t i = 0; i < nl; ++i) m->lens[i] = (int32_t)(c->boff[i + 1] - c->boff[i]);
    } else {
        // all-gather the read counts, then the lengths, over RCCL
        Shard &s = m->sh[0];
        s.cnt.assign(P, nl);
        int rc = exchange_counts(c);
        if (rc) return rc;
        m->starts.assign(P + 1, 0);
        for (int q = 0; q < P; ++q) m->starts[q + 1] = m->starts[q] + (uint32_t)s.rcnt[q];
        const uint32_t N = m->starts[P];
        std::vector<int32_t> mine(nl);
        for (uint32_t i = 0; i < nl; ++i) mine[i] = (int32_t)(c->boff[i + 1] - c->boff[i]);
        if (grow(s.xbuf, ((size_t)nl + N + 2) * 4, s.device)) return set_err(c, SA_E_NOMEM, "exchange buffer");
        int32_t *d = (int32_t *)s.xbuf.p;
        if (nl && hipMemcpy(d, mine.data(), (size_t)nl * 4, hipMemcpyHostToDevice) != hipSuccess)
            return set_err(c, SA_E_HIP, "lengths upload");
        std::vector<Plan> pl(1);
        pl[0].send = d;
        pl[0].recv = d + nl;
        pl[0].soff.assign(P, 0);
        pl[0].scnt.assign(P, nl);
        pl[0].roff.resize(P); pl[0].rcnt.resize(P);
        for (int q = 0; q < P; ++q) { pl[0].roff[q] = m->starts[q]; pl[0].rcnt[q] = m->starts[q + 1] - m->starts[q]; }
        rc = exchange(c, pl, 4);
        if (rc) return rc;
        m->lens.resize(N);
        if (N && hipMemcpy(m->lens.data(), d + nl, (size_t)N * 4, hipMemcpyDeviceToHost) != hipSuccess)
            return set_err(c, SA_E_HIP, "lengths download");
    }
    int rc = for_shards(c, [&](Shard &s) {
        sa_ctx *k = s.child;
        clear_child_reads(k);
        const uint32_t a = m->rank_mode ? 0 : m->starts[s.rank];
        const uint32_t b = m->rank_mode ? nl : m->starts[s.rank + 1];
        std::vector<uint64_t> off(b - a + 1);
        for (uint32_t i = a; i <= b; ++i) off[i - a] = c->boff[i] - c->boff[a];
        int r = sa_add_reads(k, c->bases.data() + c->boff[a], off.data(), b - a);
        if (r) return r;
        return sa_dist_init(k, s.rank, P, m->starts.data(), m->lens.data());
    });
    if (rc) return rc;
    m->dist_gen = c->reads_gen;
    m->reads_gathered = false;
    return SA_OK;
}

int resolved_mode(sa_ctx *c) {
    if (c->multi->rank_mode) return SA_IDS_WIDE;
    const int mode = c->set.id_mode;
    if (mode != SA_IDS_AUTO) return mode;
    return (c->boff.size() - 1) < 32768 ? SA_IDS_STRICT : SA_IDS_WIDE;
}

template <class T>
void concat_desc(sa_ctx *c, std::vector<T> &out, const std::vector<std::vector<T>> &parts) {
    (void)c;
    out.clear();
    for (size_t i = parts.size(); i-- > 0;) out.insert(out.end(), parts[i].begin(), parts[i].end());
}

}  // namespace

// ---------------------------------------------------------------------------
// hooks called by api.cpp
// ---------------------------------------------------------------------------
namespace sa {

bool multi_sharded(const sa_ctx *c) { return c->multi && c->multi->sharded; }

void multi_destroy(sa_ctx *c) {
    sa_multi *m = c->multi;
    if (!m) return;
    for (Shard &s : m->sh) {
        (void)hipSetDevice(s.device);
        if (s.comm) (void)ncclCommDestroy(s.comm);
        DBuf *bs[] = {&s.sk, &s.rk, &s.pf, &s.ps, &s.pc, &s.qf, &s.qs, &s.qc, &s.codes, &s.bad, &s.xbuf};
        for (DBuf *b : bs) release(*b, s.device);
        if (s.xs) (void)hipStreamDestroy(s.xs);
        sa_ctx_destroy(s.child);
    }
    release(m->gcodes, m->sh.empty() ? 0 : m->sh[0].device);
    release(m->gbad, m->sh.empty() ? 0 : m->sh[0].device);
    for (DBuf &b : m->pool) release(b, m->sh.empty() ? 0 : m->sh[0].device);
    delete m;
    c->multi = nullptr;
}

int multi_build(sa_ctx *c, bool readback, int (*single_build)(sa_ctx *, bool)) {
    sa_multi *m = c->multi;
    const int mode = resolved_mode(c);
    if (mode == SA_IDS_STRICT) {
        // the reference's own id domain (< 32,768 reads): its PairData / Trove
        // order needs every pair in one table -- run unsharded on the first device
        m->sharded = false;
        return single_build(c, readback);
    }
    if (c->keep_pairs) return set_err(c, SA_E_ARG, "SA_OPT_KEEP_PAIRS is not available on a sharded context");
    int rc = distribute(c);
    if (rc) return rc;
    const int P = m->P;
    c->built = c->aligned = false;
    m->sharded = true;
    // (SA_DEBUG_PHASES=1: host wall clock of each phase of the build on stderr, diagnostics)
    static const bool dbg = getenv("SA_DEBUG_PHASES") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    std::string phases;
    auto mark = [&](const char *name) {
        if (!dbg) return;
        const auto t = std::chrono::steady_clock::now();
        char b[64];
        snprintf(b, sizeof(b), " %s %.3f", name, std::chrono::duration<double, std::milli>(t - tp).count());
        phases += b;
        tp = t;
    };
    // ---- emit: records grouped by owner shard
    rc = for_shards(c, [&](Shard &s) {
        uint64_t n = 0;
        int r = sa_dist_local_kmers(s.child, &n);
        if (r) return r;
        if (grow(s.sk, n * 8 + 8, s.device)) return (int)SA_E_NOMEM;
        s.cnt.assign(P, 0);
        return sa_dist_emit(s.child, s.sk.p, s.cnt.data());
    }, true);
    if (rc) return rc;
    mark("emit");
    // ---- exchange 1: k-mer records to the shard owning their hash range
    if ((rc = exchange_counts(c))) return rc;
    std::vector<Plan> pl(m->sh.size());
    for (size_t l = 0; l < m->sh.size(); ++l) {
        Shard &s = m->sh[l];
        s.n_recv = 0;
        for (uint64_t v : s.rcnt) s.n_recv += v;
        if (grow(s.rk, s.n_recv * 8 + 8, s.device)) return set_err(c, SA_E_NOMEM, "receive buffer");
        pl[l].send = s.sk.p; pl[l].recv = s.rk.p;
        pl[l].scnt = s.cnt; pl[l].soff = prefix(s.cnt);
        pl[l].rcnt = s.rcnt; pl[l].roff = prefix(s.rcnt);
    }
    if ((rc = exchange(c, pl, 8))) return rc;
    mark("x1");
    // ---- buckets of this hash range (built once), the partials' upper bounds
    rc = for_shards(c, [&](Shard &s) { return sa_dist_buckets(s.child, s.rk.p, s.rcnt.data(), &s.bound); }, true);
    if (rc) return rc;
    // ---- lead-range passes: every pass holds the partials of 1/npass of every
    // owner's leads, within the budget on every shard (all ranks agree on npass)
    mark("buckets");
    // (the first build of a read set: its partials / bound ratio from a probe, api.cpp)
    rc = for_shards(c, [&](Shard &s) { return sa::dist_probe_rho(s.child); }, true);
    if (rc) return rc;
    mark("probe");
    std::vector<uint64_t> budget(m->sh.size());
    for (size_t l = 0; l < m->sh.size(); ++l) budget[l] = pass_budget(m, m->sh[l]);
    uint32_t npass = 1;
    rc = for_shards(c, [&](Shard &s) { return sa_dist_plan(s.child, budget[&s - m->sh.data()], &s.npass); });
    if (rc) return rc;
    for (Shard &s : m->sh) npass = std::max(npass, s.npass);
    if (m->rank_mode) {  // the max over ranks
        Shard &s = m->sh[0];
        s.cnt.assign(P, npass);
        if ((rc = exchange_counts(c))) return rc;
        for (uint64_t v : s.rcnt) npass = std::max<uint32_t>(npass, (uint32_t)v);
    }
    mark("plan");
    m->npass = npass;
    m->partials = 0;
    m->bound = 0;
    for (Shard &s : m->sh) m->bound += s.bound;
    DBuf Shard::*src[3] = {&Shard::pf, &Shard::ps, &Shard::pc};
    DBuf Shard::*dst[3] = {&Shard::qf, &Shard::qs, &Shard::qc};
    for (uint32_t pass = npass; pass-- > 0;) {
        // ---- count: partial pairs of this pass's leads, grouped by lead owner
        rc = for_shards(c, [&](Shard &s) {
            s.cnt.assign(P, 0);
            int r = sa_dist_count_pass(s.child, pass, npass, s.cnt.data());
            if (r) return r;
            s.n_part = 0;
            for (uint64_t v : s.cnt) s.n_part += v;
            if (grow(s.pf, s.n_part * 4 + 4, s.device) || grow(s.ps, s.n_part * 4 + 4, s.device) ||
                grow(s.pc, s.n_part * 4 + 4, s.device))
                return (int)SA_E_NOMEM;
            return sa_dist_partials(s.child, s.pf.p, s.ps.p, s.pc.p);
        }, true);
        if (rc) return rc;
        mark("count");
        for (Shard &s : m->sh) m->partials += s.n_part;
        // ---- exchange 2: partials to the shard owning the lead
        if ((rc = exchange_counts(c))) return rc;
        for (size_t l = 0; l < m->sh.size(); ++l) {
            Shard &s = m->sh[l];
            s.n_recv = 0;
            for (uint64_t v : s.rcnt) s.n_recv += v;
            if (grow(s.qf, s.n_recv * 4 + 4, s.device) || grow(s.qs, s.n_recv * 4 + 4, s.device) ||
                grow(s.qc, s.n_recv * 4 + 4, s.device))
                return set_err(c, SA_E_NOMEM, "receive buffer");
            pl[l].scnt = s.cnt; pl[l].soff = prefix(s.cnt);
            pl[l].rcnt = s.rcnt; pl[l].roff = prefix(s.rcnt);
        }
        // (lead, trail, count) arrays in one RCCL group
        std::vector<Part> parts(3);
        for (int a = 0; a < 3; ++a)
            for (size_t l = 0; l < m->sh.size(); ++l) {
                parts[a].send.push_back((m->sh[l].*src[a]).p);
                parts[a].recv.push_back((m->sh[l].*dst[a]).p);
            }
        if ((rc = exchange_parts(c, pl, parts, 4))) return rc;
        mark("x2");
        // ---- reduce + filter: this shard's leads of the pass, appended
        rc = for_shards(c, [&](Shard &s) {
            return sa_dist_reduce_pass(s.child, s.qf.p, s.qs.p, s.qc.p, s.n_recv, pass, npass);
        }, true);
        if (rc) return rc;
        mark("reduce");
    }
    if (dbg) fprintf(stderr, "[sa phases ms]%s\n", phases.c_str());
    c->stats = sa_stats{};
    uint64_t nd = 0;
    for (Shard &s : m->sh) {
        sa_stats st;
        sa_get_stats(s.child, &st);
        c->stats.kmers += st.kmers;
        c->stats.buckets += st.buckets;
        c->stats.role_pairs += st.role_pairs;
        c->stats.pairs += st.pairs;
        c->stats.dispatched += st.dispatched;
        nd += st.dispatched;
    }
    c->stats.id_mode = SA_IDS_WIDE;
    c->mode = SA_IDS_WIDE;
    c->n_disp = nd;
    c->lead.clear(); c->trail.clear(); c->count.clear();
    c->alns.clear();
    c->ovl.clear();
    c->built = true;
    if (readback) {
        const int32_t *x;
        return sa_get_dispatch(c, &x, &x, &x, &nd);
    }
    return SA_OK;
}

// lead / trail / count of every local shard, descending shard order
int multi_dispatch(sa_ctx *c) {
    sa_multi *m = c->multi;
    if (c->lead.size() == c->n_disp) return SA_OK;
    std::vector<std::vector<int32_t>> L(m->sh.size()), T(m->sh.size()), K(m->sh.size());
    int rc = for_shards(c, [&](Shard &s) {
        const int32_t *a, *b, *k;
        size_t n = 0;
        int r = sa_get_dispatch(s.child, &a, &b, &k, &n);
        if (r) return r;
        const size_t i = &s - m->sh.data();
        L[i].assign(a, a + n); T[i].assign(b, b + n); K[i].assign(k, k + n);
        return (int)SA_OK;
    });
    if (rc) return rc;
    concat_desc(c, c->lead, L);
    concat_desc(c, c->trail, T);
    concat_desc(c, c->count, K);
    return SA_OK;
}

int multi_align(sa_ctx *c, bool readback, int (*single_align)(sa_ctx *, bool)) {
    sa_multi *m = c->multi;
    if (!m->sharded) return single_align(c, readback);
    if (!c->built) return set_err(c, SA_E_STATE, "sa_align before sa_build_candidates");
    c->aligned = false;  // as device_align: no previous run's records after a failure
    c->host_valid = false;
    const int P = m->P;
    int rc;
    if (!m->reads_gathered) {
        // all-gather the 2-bit packed reads (0.25 B/base) and first-invalid positions
        const uint32_t N = m->starts[P];
        std::vector<uint64_t> wo(P + 1, 0);  // first packed word of every shard's reads
        for (int q = 0; q < P; ++q) {
            uint64_t w = 0;
            for (uint32_t i = m->starts[q]; i < m->starts[q + 1]; ++i) w += (uint64_t)((m->lens[i] + 15) / 16);
            wo[q + 1] = wo[q] + w;
        }
        const uint64_t total_w = wo[P];
        rc = for_shards(c, [&](Shard &s) {
            uint64_t nw = 0;
            int r = sa_dist_codes(s.child, nullptr, nullptr, &nw);
            if (r) return r;
            const uint32_t nl = m->starts[s.rank + 1] - m->starts[s.rank];
            if (grow(s.codes, nw * 4 + 4, s.device) || grow(s.bad, (size_t)nl * 4 + 4, s.device))
                return (int)SA_E_NOMEM;
            return sa_dist_codes(s.child, s.codes.p, s.bad.p, &nw);
        });
        if (rc) return rc;
        // destinations: one copy per device (virtual shards share theirs)
        std::vector<Plan> pc(m->sh.size()), pb(m->sh.size());
        if (!m->rccl) {
            if (grow(m->gcodes, total_w * 4 + 8, m->sh[0].device) || grow(m->gbad, (size_t)N * 4 + 4, m->sh[0].device))
                return set_err(c, SA_E_NOMEM, "read all-gather buffer");
        }
        for (size_t l = 0; l < m->sh.size(); ++l) {
            Shard &s = m->sh[l];
            const uint64_t nw = wo[s.rank + 1] - wo[s.rank];
            const uint64_t nl = m->starts[s.rank + 1] - m->starts[s.rank];
            void *gc = m->gcodes.p, *gb = m->gbad.p;
            if (m->rccl) {
                // every device gets its own copy: received into the child's buffers
                // through the generic exchange, then handed to sa_dist_set_reads
                if (grow(s.xbuf, (total_w + N) * 4 + 16, s.device)) return set_err(c, SA_E_NOMEM, "read all-gather");
                gc = s.xbuf.p;
                gb = (char *)s.xbuf.p + total_w * 4 + 8;
            }
            pc[l].send = s.codes.p; pc[l].recv = gc;
            pb[l].send = s.bad.p; pb[l].recv = gb;
            pc[l].soff.assign(P, 0); pb[l].soff.assign(P, 0);
            pc[l].scnt.assign(P, nw); pb[l].scnt.assign(P, nl);
            pc[l].roff.resize(P); pc[l].rcnt.resize(P); pb[l].roff.resize(P); pb[l].rcnt.resize(P);
            for (int q = 0; q < P; ++q) {
                pc[l].roff[q] = wo[q]; pc[l].rcnt[q] = wo[q + 1] - wo[q];
                pb[l].roff[q] = m->starts[q]; pb[l].rcnt[q] = m->starts[q + 1] - m->starts[q];
            }
            if (!m->rccl && l > 0) {  // virtual shards: only shard 0 receives (one copy per device)
                pc[l].rcnt.assign(P, 0); pb[l].rcnt.assign(P, 0);
            }
        }
        if (!m->rccl) {  // virtual: shard 0 "receives" from every shard; others send only to it
            for (size_t l = 0; l < m->sh.size(); ++l)
                for (int q = 1; q < P; ++q) { pc[l].scnt[q] = 0; pb[l].scnt[q] = 0; }
        }
        if ((rc = exchange(c, pc, 4))) return rc;
        if ((rc = exchange(c, pb, 4))) return rc;
        rc = for_shards(c, [&](Shard &s) {
            const void *gc = m->rccl ? s.xbuf.p : m->gcodes.p;
            const void *gb = m->rccl ? (const void *)((const char *)s.xbuf.p + total_w * 4 + 8) : m->gbad.p;
            if (!m->rccl) {  // virtual shards read the one all-gathered copy (no P copies of it)
                for (DBuf sa_ctx::*mb : {&sa_ctx::d_gcodes, &sa_ctx::d_gbad}) {
                    DBuf &cb = s.child->*mb;
                    if (cb.p && !cb.borrowed) release(cb, s.device);
                }
                s.child->d_gcodes = DBuf{m->gcodes.p, m->gcodes.bytes, true};
                s.child->d_gbad = DBuf{m->gbad.p, m->gbad.bytes, true};
            }
            return sa_dist_set_reads(s.child, gc, gb, total_w);
        });
        if (rc) return rc;
        m->reads_gathered = true;
    }
    rc = for_shards(c, [&](Shard &s) { return readback ? sa_align(s.child) : sa_device_align(s.child); }, true);
    if (rc) return rc;
    c->stats.aligned = c->stats.ovl_records = c->stats.dp_cells = 0;
    for (Shard &s : m->sh) {
        sa_stats st;
        sa_get_stats(s.child, &st);
        c->stats.aligned += st.aligned;
        c->stats.ovl_records += st.ovl_records;
        c->stats.dp_cells += st.dp_cells;
    }
    c->alns.clear();
    c->ovl.clear();
    c->aligned = true;
    c->host_valid = false;
    return readback ? multi_host_results(c) : SA_OK;
}

// every local shard's alignments and .ovl records (read back and formatted by
// the shard on first use), concatenated in descending shard order
int multi_host_results(sa_ctx *c) {
    if (c->host_valid) return SA_OK;
    sa_multi *m = c->multi;
    std::vector<std::vector<sa_alignment>> A(m->sh.size());
    std::vector<std::string> O(m->sh.size());
    uint64_t recs = 0;
    for (size_t i = 0; i < m->sh.size(); ++i) {
        (void)hipSetDevice(m->sh[i].device);
        const sa_alignment *p;
        size_t n;
        int rc = sa_get_alignments(m->sh[i].child, &p, &n);
        if (rc) return set_err(c, rc, sa_last_error(m->sh[i].child));
        A[i].assign(p, p + n);
        const char *t;
        size_t tl;
        if ((rc = sa_get_ovl(m->sh[i].child, &t, &tl))) return set_err(c, rc, sa_last_error(m->sh[i].child));
        O[i].assign(t, tl);
        sa_stats st;
        sa_get_stats(m->sh[i].child, &st);
        recs += st.ovl_records;
    }
    concat_desc(c, c->alns, A);
    c->ovl.clear();
    for (size_t i = O.size(); i-- > 0;) c->ovl += O[i];
    c->stats.ovl_records = recs;
    c->host_valid = true;
    return SA_OK;
}

// rank mode, collective: every rank learns whether every rank is ok
int multi_all_ok(sa_ctx *c, bool ok) {
    sa_multi *m = c->multi;
    Shard &s = m->sh[0];
    s.cnt.assign(m->P, ok ? 1 : 0);
    int rc = exchange_counts(c);
    if (rc) return rc;
    for (int q = 0; q < m->P; ++q)
        if (!s.rcnt[q]) return set_err(c, SA_E_STATE, "rank " + std::to_string(q) + " has no alignments to write");
    return SA_OK;
}

// rank mode: every rank's .ovl bytes gathered on rank 0 (descending rank order)
int multi_gather_ovl(sa_ctx *c, std::string &all) {
    sa_multi *m = c->multi;
    const int P = m->P;
    Shard &s = m->sh[0];
    s.cnt.assign(P, 0);
    s.cnt[0] = c->ovl.size();
    // sizes to rank 0 (an all-to-all of counts where only rank 0's column is used)
    int rc = exchange_counts(c);
    if (rc) return rc;
    const uint64_t mine = c->ovl.size();
    uint64_t total = 0;
    std::vector<uint64_t> sz(P, 0);
    if (s.rank == 0)
        for (int q = 0; q < P; ++q) { sz[q] = s.rcnt[q]; total += sz[q]; }
    if (grow(s.xbuf, mine + total + 16, s.device)) return set_err(c, SA_E_NOMEM, "ovl gather buffer");
    char *d = (char *)s.xbuf.p;
    if (mine && hipMemcpy(d, c->ovl.data(), mine, hipMemcpyHostToDevice) != hipSuccess)
        return set_err(c, SA_E_HIP, "ovl upload");
    std::vector<Plan> pl(1);
    pl[0].send = d;
    pl[0].recv = d + mine;
    pl[0].soff.assign(P, 0);
    pl[0].scnt.assign(P, 0);
    pl[0].scnt[0] = mine;
    pl[0].rcnt = sz;
    pl[0].roff = prefix(sz);
    if ((rc = exchange(c, pl, 1))) return rc;
    all.clear();
    if (s.rank == 0) {
        std::string buf(total, '\0');
        if (total && hipMemcpy(&buf[0], d + mine, total, hipMemcpyDeviceToHost) != hipSuccess)
            return set_err(c, SA_E_HIP, "ovl download");
        for (int q = P; q-- > 0;) all.append(buf, pl[0].roff[q], sz[q]);
    }
    return SA_OK;
}

bool multi_rank_mode(const sa_ctx *c) { return c->multi && c->multi->rank_mode; }
int multi_rank(const sa_ctx *c) { return c->multi && c->multi->rank_mode ? c->multi->sh[0].rank : 0; }

int multi_set_option(sa_ctx *c, int option, int64_t value) {
    if (option == SA_OPT_SERIAL_SHARDS) {
        c->multi->serial = value != 0;
        return SA_OK;
    }
    if (option == SA_OPT_PASS_BUDGET_MB) {
        c->multi->budget_mb = (uint64_t)value;
        return SA_OK;
    }
    if (option == SA_OPT_LEAN_MEMORY) {
        c->multi->lean = value != 0;
        return SA_OK;
    }
    for (Shard &s : c->multi->sh) {
        int rc = sa_set_option(s.child, option, value);
        if (rc) return set_err(c, rc, sa_last_error(s.child));
    }
    return SA_OK;
}

void multi_stage_times(const sa_ctx *c, double *ms, uint64_t *n) {
    // the critical path: per stage the slowest shard; exchanges on the host clock
    for (const Shard &s : c->multi->sh) {
        double m[SA_NUM_STAGES];
        uint64_t k[SA_NUM_STAGES];
        sa_get_stage_times(s.child, m, k, SA_NUM_STAGES);
        for (int i = 0; i < SA_NUM_STAGES; ++i) {
            if (m[i] > ms[i]) ms[i] = m[i];
            if (k[i] > n[i]) n[i] = k[i];
        }
    }
    ms[SA_STAGE_EXCHANGE] += c->multi->x_ms;
    n[SA_STAGE_EXCHANGE] += c->multi->x_n;
}

void multi_reset_stage_times(sa_ctx *c) {
    for (Shard &s : c->multi->sh) sa_reset_stage_times(s.child);
    c->multi->x_ms = 0;
    c->multi->x_n = 0;
}

int multi_sync(sa_ctx *c) {
    for (Shard &s : c->multi->sh) {
        int rc = sa_sync(s.child);
        if (rc) return set_err(c, rc, sa_last_error(s.child));
    }
    return SA_OK;
}

uint64_t multi_exchanged_bytes(const sa_ctx *c) { return c->multi ? c->multi->x_bytes : 0; }

}  // namespace sa

// ---------------------------------------------------------------------------
// C ABI: constructors
// ---------------------------------------------------------------------------
extern "C" {

int sa_get_shard_info(const sa_ctx *c, uint32_t *npass, uint64_t *partials, uint64_t *bound) {
    if (!c || !c->multi) return SA_E_ARG;
    if (npass) *npass = c->multi->npass;
    if (partials) *partials = c->multi->partials;
    if (bound) *bound = c->multi->bound;
    return SA_OK;
}

int sa_rccl_unique_id(void *id, size_t cap) {
    if (!id || cap < sizeof(ncclUniqueId)) return SA_E_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return SA_E_RCCL;
    memcpy(id, &u, sizeof(u));
    return SA_OK;
}

int sa_ctx_create_multi(const sa_settings *s, int n_gpus, int n_shards, sa_ctx **out) {
    if (!s || !out) return SA_E_ARG;
    *out = nullptr;
    if (!is_pow2(n_shards) || n_shards > 256 || n_gpus < 1 || (n_gpus != 1 && n_gpus != n_shards)) return SA_E_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < n_gpus) return SA_E_HIP;
    sa_ctx *c = nullptr;
    int rc = sa_ctx_create(s, 0, &c);
    if (rc) return rc;
    sa_multi *m = new sa_multi();
    c->multi = m;
    m->P = n_shards;
    m->rccl = n_gpus > 1;
    m->sh.resize(n_shards);
    std::vector<int> devs(n_shards);
    for (int r = 0; r < n_shards; ++r) {
        Shard &sh = m->sh[r];
        sh.rank = r;
        sh.device = n_gpus > 1 ? r : 0;
        devs[r] = sh.device;
        rc = sa_ctx_create(s, sh.device, &sh.child);
        if (rc) { sa_ctx_destroy(c); return rc; }
        (void)hipSetDevice(sh.device);
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, sh.device) == hipSuccess) sh.mem_total = prop.totalGlobalMem;
        if (hipStreamCreateWithFlags(&sh.xs, hipStreamNonBlocking) != hipSuccess) { sa_ctx_destroy(c); return SA_E_HIP; }
    }
    if (m->rccl) {
        std::vector<ncclComm_t> comms(n_shards);
        if (ncclCommInitAll(comms.data(), n_shards, devs.data()) != ncclSuccess) { sa_ctx_destroy(c); return SA_E_RCCL; }
        for (int r = 0; r < n_shards; ++r) m->sh[r].comm = comms[r];
    }
    (void)hipSetDevice(0);
    *out = c;
    return SA_OK;
}

int sa_ctx_create_rank(const sa_settings *s, int device, int rank, int nranks, const void *id, sa_ctx **out) {
    if (!s || !out || !id) return SA_E_ARG;
    *out = nullptr;
    if (!is_pow2(nranks) || nranks > 256 || rank < 0 || rank >= nranks) return SA_E_ARG;
    if (s->id_mode == SA_IDS_STRICT) return SA_E_ARG;  // ranks run the wide-id path
    sa_ctx *c = nullptr;
    int rc = sa_ctx_create(s, device, &c);
    if (rc) return rc;
    sa_multi *m = new sa_multi();
    c->multi = m;
    m->P = nranks;
    m->rank_mode = true;
    m->rccl = true;
    m->sh.resize(1);
    Shard &sh = m->sh[0];
    sh.rank = rank;
    sh.device = device;
    rc = sa_ctx_create(s, device, &sh.child);
    if (rc) { sa_ctx_destroy(c); return rc; }
    (void)hipSetDevice(device);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) sh.mem_total = prop.totalGlobalMem;
    if (hipStreamCreateWithFlags(&sh.xs, hipStreamNonBlocking) != hipSuccess) { sa_ctx_destroy(c); return SA_E_HIP; }
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&sh.comm, nranks, u, rank) != ncclSuccess) { sa_ctx_destroy(c); return SA_E_RCCL; }
    *out = c;
    return SA_OK;
}

}  // extern "C"
