// api.cpp -- C ABI (include/sa_overlap.h) and host orchestration of the
// MI355X hash-overlap stage.
//
// Pipeline (one HIP stream; bulk data never leaves HBM between stages):
//   pack_reads      ASCII -> 2-bit words                       (BioLibs.readSeq output)
//   kmer_emit       (seqHash << lb | locrank, g) per k-mer     (BioLibs.generateKmerSet)
//   radix_sort      group by hash, loc order, g-stable          (KmerData, KmerTable.scala:41-53)
//   build_buckets   middle / edge lists + partner ranges        (calcPairData split, :97-115)
//   pair_count      per-read LDS aggregation + [min,max] filter (addKmerPair / calcDispatchData)
//   order           wide: lead desc / trail asc; strict: first-occurrence rank -> Trove layouts (device)
//   dovetail        banded two-phase DP + validity             (generateFastDovetailAlignmentSet)
// then the .ovl writer (Project4.calcOverlaps) on the host.
#include "../../../include/sa_overlap.h"

#include <hip/hip_runtime.h>
#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include "../sa_internal.h"
#include "ctx.h"
#include "trove.h"

namespace sa {
int read_fasta(const char *path, std::vector<char> &bases, std::vector<uint64_t> &offsets);
int read_hoxd(const char *path, int32_t cost[16]);
size_t pair_count_lds_bytes(bool strict);
hipError_t launch_bucket_first(const uint64_t *skeys, const uint32_t *svals, const Buckets &b, int lb,
                               uint32_t *hash_out, uint32_t *first_out, hipStream_t s);
}  // namespace sa

using namespace sa;

namespace {

int fail(sa_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(expr)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(c, SA_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
    } while (0)

template <class T>
int ensure(sa_ctx *c, DBuf &b, size_t count, T **out) {
    const size_t need = std::max<size_t>(count, 1) * sizeof(T);
    if (b.bytes < need) {
        if (b.p && !b.borrowed) (void)hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
        b.borrowed = false;
        const size_t alloc = need + need / 8;
        hipError_t e = hipMalloc(&b.p, alloc);
        if (e != hipSuccess) return fail(c, SA_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        b.bytes = alloc;
    }
    *out = (T *)b.p;
    return SA_OK;
}

#define ENSURE(buf, n, ptr)                          \
    do {                                             \
        int r_ = ensure(c, (buf), (size_t)(n), ptr); \
        if (r_) return r_;                           \
    } while (0)

hipEvent_t get_event(sa_ctx *c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

struct StageScope {
    sa_ctx *c;
    int stage;
    hipEvent_t a = nullptr;
    StageScope(sa_ctx *c_, int s) : c(c_), stage(s) {
        if (c->timing) {
            a = get_event(c);
            (void)hipEventRecord(a, c->stream);
        }
    }
    ~StageScope() {
        if (c->timing && a) {
            hipEvent_t b = get_event(c);
            (void)hipEventRecord(b, c->stream);
            c->pending.push_back({stage, a, b});
        }
    }
};

// host wall-clock stage (SA_STAGE_UPLOAD .. SA_STAGE_WRITE): the calc-overlaps path's
// host work around the device stages, recorded whatever SA_OPT_TIMING says
struct HostScope {
    sa_ctx *c;
    int stage;
    std::chrono::steady_clock::time_point t0;
    HostScope(sa_ctx *c_, int s) : c(c_), stage(s), t0(std::chrono::steady_clock::now()) {}
    ~HostScope() {
        c->stage_ms[stage] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        c->stage_n[stage] += 1;
    }
};

// the side stream (ctx.h) and its events, created on first use on the
// context's (current) device
hipError_t ensure_side(sa_ctx *c) {
    if (c->side) return hipSuccess;
    hipError_t e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
    for (hipEvent_t *ev : {&c->ev_fork, &c->ev_join, &c->ev_fork2, &c->ev_join2})
        if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    return e;
}

// the pinned counter copy (ctx.h), allocated on first use
int pinned_counters(sa_ctx *c, Counters **out) {
    if (!c->hcnt) {
        void *p = nullptr;
        hipError_t e = hipHostMalloc(&p, sizeof(Counters), hipHostMallocDefault);
        if (e != hipSuccess) return fail(c, SA_E_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        c->hcnt = (Counters *)p;
    }
    *out = c->hcnt;
    return SA_OK;
}

// fork: the side stream waits for everything queued on the main stream so far
hipError_t fork_side(sa_ctx *c, hipEvent_t ev) {
    hipError_t e = hipEventRecord(ev, c->stream);
    return e == hipSuccess ? hipStreamWaitEvent(c->side, ev, 0) : e;
}

// join: the main stream waits for everything queued on the side stream so far
hipError_t join_side(sa_ctx *c, hipEvent_t ev) {
    hipError_t e = hipEventRecord(ev, c->side);
    return e == hipSuccess ? hipStreamWaitEvent(c->stream, ev, 0) : e;
}

void resolve_timing(sa_ctx *c) {
    for (auto &p : c->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            c->stage_ms[p.stage] += ms;
            c->stage_n[p.stage] += 1;
        }
        c->ev_pool.push_back(p.a);
        c->ev_pool.push_back(p.b);
    }
    c->pending.clear();
}

int bits_for(uint64_t v) {  // bits to represent 0..v
    int b = 1;
    while (b < 64 && (v >> b)) ++b;
    return b;
}

// ---------------------------------------------------------------------------
// host-side read metadata: lengths, word/occurrence offsets, loc ranks, tags
// ---------------------------------------------------------------------------
int prepare_reads(sa_ctx *c) {
    const uint32_t n = (uint32_t)(c->boff.size() - 1);
    const int k = c->set.kmer_size;
    if (k < 1) return fail(c, SA_E_ARG, "kmer size must be >= 1");
    c->m = k < 16 ? k : 16;
    c->len.resize(n);
    c->woff.resize(n + 1);
    c->occ_off.resize(n + 1);
    c->woff[0] = 0;
    c->occ_off[0] = 0;
    c->maxL = 0;
    c->minL = n ? INT32_MAX : 0;
    c->max_occ = 0;
    std::vector<char> has_d;
    int maxd = -1;
    int32_t uni = -1;
    bool uniform = true;
    for (uint32_t r = 0; r < n; ++r) {
        const uint64_t L64 = c->boff[r + 1] - c->boff[r];
        if (L64 > (1u << 20) - 2) return fail(c, SA_E_OVERFLOW, "read longer than 1,048,574 bases");
        const int32_t L = (int32_t)L64;
        c->len[r] = L;
        c->maxL = std::max(c->maxL, L);
        c->minL = std::min(c->minL, L);
        c->woff[r + 1] = c->woff[r] + (uint64_t)((L + 15) / 16);
        const int32_t nk = L - k + 1 > 0 ? L - k + 1 : 0;
        c->occ_off[r + 1] = c->occ_off[r] + (uint64_t)nk;
        c->max_occ = std::max<uint32_t>(c->max_occ, (uint32_t)nk);
        if (uni < 0) uni = L;
        if (L != uni || L < k) uniform = false;
        if (L >= k) {
            const int d = L - k;
            if (d > maxd) { maxd = d; has_d.resize(d + 1, 0); }
            has_d[d] = 1;
        }
    }
    c->n_occ = c->occ_off[n];
    // occurrence indices are u32 (records: mix << 32 | occurrence)
    if (c->n_occ >= 0xFFFFFFF0ull) return fail(c, SA_E_OVERFLOW, "more than 2^32 - 16 k-mers on one device");
    if (c->dist) {
        // loc ranks / tags / sort-key width must agree on every rank: derive
        // them from the lengths of ALL reads, not just this rank's
        has_d.clear();
        maxd = -1;
        for (int32_t L : c->dlen) {
            if (L < k) continue;
            const int d = L - k;
            if (d > maxd) { maxd = d; has_d.resize(d + 1, 0); }
            has_d[d] = 1;
        }
    }
    c->n_words = c->woff[n] + 2;  // pad: windows read one word past a read
    c->uniform_npr = (uniform && n > 0) ? (uint32_t)(uni - k + 1) : 0;
    c->maxd = maxd < 0 ? 0 : maxd;
    // distinct float32 locs i/d (BioLibs.scala:56-58) -> ranks; NaN (d == 0) ranks last, untagged
    std::vector<float> vals;
    bool nan_loc = false;
    for (int d = 0; d <= maxd; ++d) {
        if (!has_d[d]) continue;
        if (d == 0) { nan_loc = true; continue; }
        const float fd = (float)d;
        for (int i = 0; i <= d; ++i) vals.push_back((float)i / fd);
    }
    std::sort(vals.begin(), vals.end());
    vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
    const uint32_t nan_rank = (uint32_t)vals.size();
    c->lbase.assign((size_t)c->maxd + 1, 0);
    c->lrank.clear();
    for (int d = 0; d <= maxd; ++d) {
        c->lbase[d] = (uint32_t)c->lrank.size();
        if (!has_d[d]) continue;
        if (d == 0) { c->lrank.push_back(nan_rank); continue; }
        const float fd = (float)d;
        for (int i = 0; i <= d; ++i) {
            const float v = (float)i / fd;
            c->lrank.push_back((uint32_t)(std::lower_bound(vals.begin(), vals.end(), v) - vals.begin()));
        }
    }
    if (c->lrank.empty()) c->lrank.push_back(0);
    // AlignSettings edges (ObjectStore.scala:32-35), float32
    const float head = c->set.kmer_edge;
    const float tail = 1.0f - c->set.kmer_edge;
    const float half_c = c->set.kmer_center * 0.5f;
    const float midLead = 0.5f - half_c;
    const float midTail = 0.5f + half_c;
    c->tagtab.assign(vals.size() + 1 + (nan_loc ? 1 : 0), 0);
    for (size_t q = 0; q < vals.size(); ++q) {
        const float v = vals[q];
        uint8_t t = 0;
        if (v <= head) t |= TAG_ST;  // KmerTable.scala:106-115
        if (midLead <= v && v <= midTail) t |= TAG_MD;
        if (tail <= v) t |= TAG_EN;
        c->tagtab[q] = t;
    }
    c->lb = bits_for(nan_rank);
    if (2 * c->m + c->lb > 64) return fail(c, SA_E_OVERFLOW, "sort key wider than 64 bits");
    // tag table indexed by (key & lbmask): pad to 1 << lb
    c->tagtab.resize((size_t)1 << c->lb, 0);
    return SA_OK;
}

int upload_reads(sa_ctx *c) {
    const uint32_t n = (uint32_t)(c->boff.size() - 1);
    uint8_t *ascii; uint64_t *boff, *woff, *occ; int32_t *len; uint32_t *codes; int32_t *bad;
    uint32_t *lbase, *lrank; uint8_t *tag;
    ENSURE(c->d_ascii, c->bases.size() + 32, &ascii);  // pack_reads reads 20 bytes past a word start
    ENSURE(c->d_boff, n + 1, &boff);
    ENSURE(c->d_woff, n + 1, &woff);
    ENSURE(c->d_len, n + 1, &len);
    ENSURE(c->d_codes, c->n_words, &codes);
    ENSURE(c->d_bad, n + 1, &bad);
    ENSURE(c->d_occ_off, n + 1, &occ);
    ENSURE(c->d_lbase, c->lbase.size(), &lbase);
    ENSURE(c->d_lrank, c->lrank.size(), &lrank);
    ENSURE(c->d_tagtab, c->tagtab.size(), &tag);
    if (!c->bases.empty()) HIPCHK(hipMemcpyAsync(ascii, c->bases.data(), c->bases.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(boff, c->boff.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(woff, c->woff.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    if (n) HIPCHK(hipMemcpyAsync(len, c->len.data(), n * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(occ, c->occ_off.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(lbase, c->lbase.data(), c->lbase.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(lrank, c->lrank.data(), c->lrank.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(tag, c->tagtab.data(), c->tagtab.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(codes, 0, c->n_words * 4, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->uploaded = true;
    return SA_OK;
}

DevReads dev_reads(sa_ctx *c) {
    DevReads r;
    r.n = (uint32_t)(c->boff.size() - 1);
    r.ascii = (const uint8_t *)c->d_ascii.p;
    r.boff = (const uint64_t *)c->d_boff.p;
    r.woff = (const uint64_t *)c->d_woff.p;
    r.len = (const int32_t *)c->d_len.p;
    r.codes = (uint32_t *)c->d_codes.p;
    r.bad = (int32_t *)c->d_bad.p;
    return r;
}

EmitParams emit_params(sa_ctx *c) {
    EmitParams e{};
    e.k = c->set.kmer_size;
    e.m = c->m;
    e.lb = c->lb;
    e.occ_off = (const uint64_t *)c->d_occ_off.p;
    e.npr = c->uniform_npr;
    e.lbase = (const uint32_t *)c->d_lbase.p;
    e.lrank = (const uint32_t *)c->d_lrank.p;
    e.maxd = c->maxd;
    e.rkey = nullptr;
    e.rord = nullptr;
    e.pos_bits = 0;
    e.occ_rl = nullptr;
    return e;
}

int ensure_prepared(sa_ctx *c) {
    if (c->reads_dirty || !c->uploaded) {
        HostScope hs(c, SA_STAGE_UPLOAD);
        if (c->reads_dirty) {
            int rc = prepare_reads(c);
            if (rc) return rc;
            c->reads_dirty = false;
            c->uploaded = false;
        }
        int rc = upload_reads(c);
        if (rc) return rc;
    }
    const uint32_t n = (uint32_t)(c->boff.size() - 1);
    int mode = c->set.id_mode;
    if (mode == SA_IDS_AUTO) mode = n < 32768 ? SA_IDS_STRICT : SA_IDS_WIDE;
    if (c->dist) mode = SA_IDS_WIDE;
    if (mode == SA_IDS_STRICT && n >= 65536)
        return fail(c, SA_E_ID_RANGE, "strict ids: >= 65,536 reads alias in the reference's (fst<<16)^snd keys; use wide ids");
    c->mode = mode;
    return SA_OK;
}

// Uniform lengths (one packed-word count per read, records carrying their
// occurrence index): the first radix pass over the records generates them from
// the packed reads (radix_sort_gen), so they are never written and re-read
// unsorted, and pack_emit only packs and writes the locality keys.
// SA_KEYGEN=0 keeps the stored records (A/B)
// the pack kernel counts the first radix pass's digits (SA_HIST_IN_PACK=0: the upsweep does)
static bool hist_in_pack() {
    static const bool on = !getenv("SA_HIST_IN_PACK") || atoi(getenv("SA_HIST_IN_PACK")) != 0;  // (A/B)
    return on;
}

static bool make_keygen(const sa_ctx *c, const EmitParams &E, uint64_t n, KeyGen &kg) {
    static const bool env_on = !getenv("SA_KEYGEN") || atoi(getenv("SA_KEYGEN")) != 0;
    const size_t nr = c->woff.empty() ? 0 : c->woff.size() - 1;
    // (up to 2^27 records: at configs[3]'s slice, 607.5M records, generating the
    // first pass's keys twice -- upsweep and downsweep -- cost more than storing
    // them: hash step 48.4 -> 49.1 ms, profiles/r04/ab/ab_c3_keygen_vs_old.txt)
    if (!env_on || !E.npr || E.pos_bits || E.occ_rl || nr == 0 || n >= (1ull << 27)) return false;
    const uint64_t nw = c->woff[1] - c->woff[0];
    for (size_t r = 1; r < nr; ++r)
        if (c->woff[r + 1] - c->woff[r] != nw) return false;
    kg.codes = (const uint32_t *)c->d_codes.p;
    kg.nw = (uint32_t)nw;
    kg.npr = E.npr;
    kg.npr_magic = E.npr >= 2 ? ~0ull / E.npr + 1 : 0ull;
    kg.shift = 32 - 2 * c->m;
    return true;
}

// PartArgs' two shortcuts around table lookups (checked against the tables,
// off when they do not hold): loc rank = position for uniform lengths, and the
// tags as three loc-rank intervals
static void set_part_shortcuts(const sa_ctx *c, PartArgs &PA, uint32_t npr) {
    PA.lr_ident = 0;
    if (npr >= 2 && (size_t)npr - 1 < c->lbase.size()) {
        const uint32_t b = c->lbase[npr - 1];
        bool id = (size_t)b + npr <= c->lrank.size();
        for (uint32_t i = 0; id && i < npr; ++i) id = c->lrank[b + i] == i;
        PA.lr_ident = id ? 1 : 0;
    }
    const std::vector<uint8_t> &t = c->tagtab;
    const uint32_t T = (uint32_t)t.size();
    auto run = [&](uint8_t bit, uint32_t &lo, uint32_t &cnt) {
        lo = 0;
        while (lo < T && !(t[lo] & bit)) ++lo;
        uint32_t hi = lo;
        while (hi < T && (t[hi] & bit)) ++hi;
        cnt = hi - lo;
        if (lo == T) lo = 0;
    };
    uint32_t st0, stn;
    run(TAG_ST, st0, stn);
    run(TAG_MD, PA.tg_md0, PA.tg_mdn);
    run(TAG_EN, PA.tg_en0, PA.tg_enn);
    PA.tg_st = stn ? st0 + stn : 0;
    PA.tg_on = stn == 0 || st0 == 0;
    for (uint32_t q = 0; PA.tg_on && q < T; ++q) {
        const uint32_t v = (q < PA.tg_st ? (uint32_t)TAG_ST : 0u) | (q - PA.tg_md0 < PA.tg_mdn ? (uint32_t)TAG_MD : 0u) |
                           (q - PA.tg_en0 < PA.tg_enn ? (uint32_t)TAG_EN : 0u);
        PA.tg_on = v == t[q];
    }
}

// Bucket build over one device's k-mer records (keys = mix << lb | locrank,
// vals = occurrence index): partition radix sort on the top PB bits of the
// mix, then one LDS workgroup per partition (part_build), the global scan path
// for partitions too large for LDS.  Read ids come from rid[val] when given
// (distributed mode), else from the occurrence offsets.
// partition bits of the bucket build for n records (see bucket_stage)
static int part_bits(uint64_t n) {
    const uint64_t part_target = 700;
    int PB = 1;
    while (PB < 24 && (part_target << PB) < n) ++PB;
    if (PB > 16 && (n >> 16) <= 900) PB = 16;
    return PB;
}

int bucket_stage(sa_ctx *c, uint64_t *&keys, uint64_t *&keys2, uint32_t *vals, uint32_t *vals2, uint64_t n,
                 const uint64_t *occ_off, uint32_t n_reads, uint32_t npr, const uint2 *rl,
                 const int32_t *len, bool strict, void *stmp, Counters *cnt, PartArgs &PA,
                 unsigned long long &big_buckets, int skip_bits = 0, int phase = 0, const uint32_t *pv = nullptr,
                 const KeyGen *kgen = nullptr, const RecvGen *recv = nullptr, bool counters_zeroed = false) {
    // counters_zeroed: the caller cleared the whole Counters block just before (its
    // partition-list counts then need no clear of their own)
    // phase 0: everything; 1: sort + LDS tiers, no readback (the caller's
    // first pair-count pass aborts on big_n); 2: only the global path of the
    // partitions phase 1 listed (keys / PA as phase 1 left them)
    // keys: 8-byte records (mix32 << 32 | occurrence index); vals / vals2: u32
    // scratch for the big-partition path.  skip_bits: top bits of the mix every
    // record here shares (the owner rank's bits in distributed mode);
    // partitions use the PB bits below them
    // ---- partition by the top P bits of mix(seqHash): whole buckets per partition
    // ~700 records per partition (LDS capacity 1,024); up to 2^24 partitions
    // (1.25M reads of 500 bp = 607M k-mers per GPU -> 2^20), but stay at 16 bits
    // (two radix passes) while the average still fits the 1,024-record kernel
    // (round 4, same-box A/B at the bench shape: ~1,100-1,400-record partitions
    // with the 2,048-record tier as the main pass -- 8 waves per block -- built
    // buckets in 1.53-1.55 ms against 1.15 for ~700-record ones on the 1,024 tier)
    const int PB = part_bits(n);
    const uint32_t nparts = 1u << PB;
    const int kbits = 32 + c->lb;  // LDS sort key: mix << lb | loc rank
    uint2 *srl = nullptr;
    const uint32_t *spv = nullptr;
    uint32_t *pstart, *biglist;
    ENSURE(c->d_pstart, nparts + 1, &pstart);
    ENSURE(c->d_biglist, 4 * ((size_t)nparts + 1), &biglist);  // big list, mid list, mid2 list, fb list
    const uint8_t *tagtab = (const uint8_t *)c->d_tagtab.p;
    if (phase != 2) {
        {
            StageScope st(c, SA_STAGE_SORT);
            if (pv) {
                // the occurrence table packed into 4 bytes (read << lb | loc rank)
                // rides along as the sort's value: 12-byte records through the
                // passes instead of 16 (vals / vals2 are free until the global path)
                uint32_t *v0 = vals, *v1 = vals2;
                if (recv) {  // received records: relabelled and decoded by the first pass
                    // (source-relative records carry their source in the key's top bits, which a
                    // last pass of fewer than 8 bits would read with its digit: the range is
                    // widened downwards to whole passes -- the same pass count, a finer order)
                    const int lo_r = recv->src_shift ? 64 - skip_bits - 8 * ((PB + 7) / 8) : 64 - skip_bits - PB;
                    HIPCHK(radix_sort_recv(*recv, &keys, &v0, &keys2, &v1, n, lo_r, 64 - skip_bits,
                                           stmp, c->stream));
                } else {
                    if (n && v0 != pv) HIPCHK(hipMemcpyAsync(v0, pv, n * 4, hipMemcpyDeviceToDevice, c->stream));
                    HIPCHK(radix_sort(&keys, &v0, &keys2, &v1, n, 64 - skip_bits - PB, 64 - skip_bits, stmp,
                                      c->stream));
                }
                spv = v0;
            } else if (rl) {
                // an occurrence table rides along as the sort's 8-byte value, so the
                // bucket build reads each record's {read, loc rank} coalesced instead
                // of gathering it (16-byte records through the two passes)
                uint64_t *v0, *v1;
                ENSURE(c->d_srl, n + 1, &v0);
                ENSURE(c->d_srl2, n + 1, &v1);
                if (n) HIPCHK(hipMemcpyAsync(v0, rl, n * 8, hipMemcpyDeviceToDevice, c->stream));
                HIPCHK(radix_sort_kv64(&keys, &v0, &keys2, &v1, n, 64 - skip_bits - PB, 64 - skip_bits, stmp,
                                       c->stream));
                srl = (uint2 *)v0;
            } else {
                uint32_t *nv = nullptr, *nv2 = nullptr;  // key-only: the payload rides in the record
                if (kgen)  // records generated by the first pass, never stored unsorted
                    HIPCHK(radix_sort_gen(*kgen, &keys, &keys2, n, 64 - skip_bits - PB, 64 - skip_bits, stmp,
                                          c->stream));
                else
                    HIPCHK(radix_sort(&keys, &nv, &keys2, &nv2, n, 64 - skip_bits - PB, 64 - skip_bits, stmp,
                                      c->stream));
            }
        }
        PA = PartArgs{};
        PA.sk = keys; PA.sv = nullptr; PA.start = pstart; PA.np = nparts; PA.lb = c->lb; PA.sort_bits = kbits - skip_bits - PB;
        PA.tagtab = (const uint8_t *)c->d_tagtab.p;
        PA.occ_off = occ_off;
        PA.n_reads = n_reads; PA.npr = npr; PA.rl = rl; PA.srl = srl; PA.pv = pv; PA.spv = spv;
        if (pv && c->dist_src_shift) {  // (sharded, source-relative packed values: RecvGen::src_shift)
            PA.src_shift = c->dist_src_shift;
            PA.src_own = (uint32_t)c->rank << (c->dist_src_shift - 32);
            PA.src_starts = (const uint32_t *)c->d_starts.p;
        }
            PA.npr_magic = npr >= 2 ? ~0ull / npr + 1 : 0;
        PA.len = len;
        PA.lbase = (const uint32_t *)c->d_lbase.p;
        PA.lrank = (const uint32_t *)c->d_lrank.p;
        PA.k = c->set.kmer_size;
        set_part_shortcuts(c, PA, npr);
        PA.pos_bits = rl || pv ? 0 : c->pos_bits;  // (occurrence indices + the {read, loc rank} table)
        PA.meta = (const uint2 *)c->d_meta.p;
        ENSURE(c->d_md, 3 * n + 3, &PA.lst);
        ENSURE(c->d_rec, n + 1, &PA.rec);
        PA.xrec = nullptr;
        PA.xrec_n = &cnt->xrec_n;
        PA.big_list = biglist; PA.big_n = &cnt->big_n;
        PA.mid_list = biglist + nparts + 1; PA.mid_n = &cnt->mid_n;
        PA.mid2_list = biglist + 2 * ((size_t)nparts + 1); PA.mid2_n = &cnt->mid2_n;
        PA.fb_list = biglist + 3 * ((size_t)nparts + 1); PA.fb_n = &cnt->fb_n;
        static const bool split_env = !getenv("SA_SPLIT_TIER") || atoi(getenv("SA_SPLIT_TIER")) != 0;  // (A/B)
        PA.split = split_env && !strict && !srl && !spv ? 1 : 0;
        PA.counts = cnt->bkt_counts;
#ifdef SA_PB_PROBE_DUP
        {   // bandwidth probe builds: a second record array the bucket build also scatters to
            static uint2 *dup = nullptr;
            static uint64_t dup_n = 0;
            if (dup_n < n + 1) {
                if (dup) (void)hipFree(dup);
                HIPCHK(hipMalloc(&dup, (n + 1) * sizeof(uint2)));
                dup_n = n + 1;
            }
            PA.rec_dup = dup;
        }
#endif
#ifdef SA_PB_STAMPS
        {   // timing probe builds: SA_PB_STAMPS_OUT=<path> gets the last build's stamps
            static uint64_t *stamps = nullptr;
            static uint32_t stamps_np = 0;
            if (stamps_np < nparts) {
                if (stamps) (void)hipFree(stamps);
                HIPCHK(hipMalloc(&stamps, 8 * sizeof(uint64_t) * nparts));
                stamps_np = nparts;
            }
            HIPCHK(hipMemsetAsync(stamps, 0, 8 * sizeof(uint64_t) * nparts, c->stream));
            PA.stamps = stamps;
            c->stamps_dev = stamps;
            c->stamps_np = nparts;
        }
#endif
        if (strict) {
            ENSURE(c->d_mdidx, 3 * n + 3, &PA.lidx);
            ENSURE(c->d_srec, n + 1, &PA.srec);
            ENSURE(c->d_bnst, n + 1, &PA.bkt_nst);
            ENSURE(c->d_bnmd, n + 1, &PA.bkt_nmd);
            ENSURE(c->d_bfirst, n + 1, &PA.bkt_first);
            ENSURE(c->d_ishead, n + 1, &PA.is_head);
            ENSURE(c->d_brank, n + 1, &c->bkt_rank_dev);
            HIPCHK(hipMemsetAsync(PA.is_head, 0, n + 1, c->stream));
        }
        if (!counters_zeroed)
            HIPCHK(hipMemsetAsync(&cnt->mid_n, 0, 3 * sizeof(uint32_t), c->stream));  // mid_n, mid2_n, fb_n
        {
            // the bounds kernel lists the partitions above 1,024 records; their
            // 2,048 / 4,096-record tiers (~1 % of partitions, a few blocks' latency)
            // run on the side stream beside the 1,024-record pass
            StageScope st(c, SA_STAGE_BUCKETS);
            HIPCHK(launch_part_starts(PA, n, 64 - skip_bits - PB, c->stream));
            HIPCHK(ensure_side(c));
            HIPCHK(fork_side(c, c->ev_fork2));
            // (the same tiers in line on one stream, before or after the main
            // pass, measured the same: profiles/r04/ab/ab_tier_order_pair_build.txt)
            if (PA.split) HIPCHK(launch_part_build(PA, strict, 1, c->side));  // (then 2,048: fb_list only)
            HIPCHK(launch_part_build(PA, strict, 2048, c->side));
            HIPCHK(launch_part_build(PA, strict, 4096, c->side));
            HIPCHK(launch_part_build(PA, strict, 1024, c->stream));
            HIPCHK(join_side(c, c->ev_join2));
        }
#ifdef SA_PB_STAMPS
        if (const char *path = getenv("SA_PB_STAMPS_OUT")) {
            std::vector<uint64_t> h(8 * (size_t)c->stamps_np);
            HIPCHK(hipMemcpyAsync(h.data(), c->stamps_dev, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            if (FILE *f = fopen(path, "wb")) {
                fwrite(h.data(), 8, h.size(), f);
                fclose(f);
            }
        }
#endif
        if (phase == 1) return SA_OK;
    }
    uint32_t big_n = 0;
    HIPCHK(hipMemcpyAsync(&big_n, &cnt->big_n, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    big_buckets = 0;
    unsigned long long big_groups = 0;
    if (big_n) {
        // partitions too large for LDS (high-copy repeats): sort the rest of the
        // key in place, then the global scan build of buckets.hip on the range
        std::vector<uint32_t> bl(big_n), starts(nparts + 1);
        HIPCHK(hipMemcpy(bl.data(), biglist, big_n * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(starts.data(), pstart, (nparts + 1) * 4, hipMemcpyDeviceToHost));
        std::sort(bl.begin(), bl.end());
        uint32_t maxn = 0;
        uint64_t big_recs = 0;
        for (uint32_t p : bl) {
            maxn = std::max(maxn, starts[p + 1] - starts[p]);
            big_recs += starts[p + 1] - starts[p];
        }
        Buckets B{};
        // the scan's ascending partition-relative lists (moved into the combined
        // layout per partition) and the escape records of high-copy repeats
        ENSURE(c->d_tmd, (size_t)maxn + 1, &B.md_list);
        ENSURE(c->d_ted, 2 * (size_t)maxn + 2, &B.ed_list);
        if (strict) {
            ENSURE(c->d_tmdi, (size_t)maxn + 1, &B.md_idx);
            ENSURE(c->d_tedi, 2 * (size_t)maxn + 2, &B.ed_idx);
        }
        ENSURE(c->d_xrec, big_recs + 1, &PA.xrec);
        ENSURE(c->d_bmdo, maxn + 2, &B.bkt_mdo);
        ENSURE(c->d_bedo, maxn + 2, &B.bkt_edo);
        ENSURE(c->d_bstart, maxn + 2, &B.bkt_start);
        ENSURE(c->d_gbid, maxn + 1, &B.grp_bid);
        ENSURE(c->d_gmds, maxn + 1, &B.grp_mds);
        ENSURE(c->d_gede, maxn + 1, &B.grp_ede);
        ENSURE(c->d_ogid, n + 1, &B.occ_gid);
        uint8_t *btmp;
        ENSURE(c->d_bkttmp, std::max(radix_sort_temp_bytes(maxn), buckets_temp_bytes(maxn)), &btmp);
        if (strict) {
            ENSURE(c->d_occidx, 3 * n + 3, &B.occ_idx);
            ENSURE(c->d_bnst2, maxn + 1, &B.bkt_nst);
        }
        uint32_t *bigtot;
        ENSURE(c->d_bigtot, 4 * (size_t)big_n, &bigtot);
        uint32_t bi = 0;
        StageScope st(c, SA_STAGE_BUCKETS);
        for (uint32_t p : bl) {
            const uint32_t ps = starts[p], pn = starts[p + 1] - starts[p];
            // (mix << lb | loc rank, g) pairs of the range into keys2 / vals, then
            // sort the bits below the partition id (the records in keys are spent)
            HIPCHK(launch_convert_records(keys + ps, pn, PA, keys2 + ps, vals + ps, ps, c->stream));
            uint64_t *k0 = keys2 + ps, *k1 = keys + ps;
            uint32_t *v0 = vals + ps, *v1 = vals2 + ps;
            HIPCHK(radix_sort(&k0, &v0, &k1, &v1, pn, 0, kbits - skip_bits - PB, btmp, c->stream));
            if (k0 != keys2 + ps) {  // odd number of passes: copy the sorted range back
                HIPCHK(hipMemcpyAsync(keys2 + ps, k0, (size_t)pn * 8, hipMemcpyDeviceToDevice, c->stream));
                HIPCHK(hipMemcpyAsync(vals + ps, v0, (size_t)pn * 4, hipMemcpyDeviceToDevice, c->stream));
            }
            B.n_occ = pn;
            HIPCHK(build_buckets(keys2 + ps, vals + ps, pn, c->lb, tagtab, PA.occ_off, n_reads, npr, rl, B,
                                 bigtot + 4 * (size_t)bi, btmp, c->stream));
            if (strict) HIPCHK(build_strict_index(keys2 + ps, vals + ps, pn, c->lb, tagtab, B, c->stream));
            HIPCHK(launch_relayout_lists(B, ps, pn, bigtot + 4 * (size_t)bi, PA, strict, c->stream));
            HIPCHK(launch_records_from_tables(keys2, vals, ps, pn, c->lb, tagtab, B, PA, strict ? 1 : 0, c->stream));
            ++bi;
        }
        // per-partition totals read back once (no host sync inside the loop)
        std::vector<uint32_t> tots(4 * (size_t)big_n);
        HIPCHK(hipMemcpyAsync(tots.data(), bigtot, tots.size() * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (uint32_t i = 0; i < big_n; ++i) {
            big_buckets += tots[4 * (size_t)i];
            big_groups += tots[4 * (size_t)i + 1];
        }
    }
    (void)big_groups;
    return SA_OK;
}

// Pair counting (pair_count.hip) with output-capacity growth and the
// partner-residue split pass for reads whose LDS table overflows.  Leaves np
// entries in the NSHARD output regions of cap_s_out entries each -- or, with
// owners > 1 (sharded path), in owners x NSHARD regions grouped by the rank
// owning the lead (owner_starts, device), their fill in c->d_ocur / c->ocur.
int pair_stage(sa_ctx *c, const EmitParams &E, const PairIn &PI, bool strict, bool emit_all,
               const uint32_t *read_order, uint32_t n_items, Counters *cnt, uint64_t &np, uint64_t &cap_s_out,
               const uint32_t *item_start = nullptr, uint32_t n_multi = 0, const uint32_t *abort_flag = nullptr,
               bool *aborted = nullptr, bool *per_read = nullptr, uint64_t *distinct_ub = nullptr,
               uint32_t owners = 1, const uint32_t *owner_starts = nullptr, const uint32_t *item_owner = nullptr,
               bool counters_zeroed = false, const uint32_t *item_end = nullptr) {
    // counters_zeroed: the caller cleared the whole Counters block and nothing has counted
    // since (the cursors and the overflow count then need no clear of their own)
    // per_read (in: allowed; out: used): the first pass writes each read's
    // dispatched pairs, trail-ascending, into a fixed region of PC_RREG slots
    // (wide ids, dispatched pairs only, one device); a read whose table
    // overflows is recounted by the tiers below into the shared regions (np
    // entries), and only those reads' pairs are sorted afterwards (device_build).
    // distinct_ub: an upper bound of the dispatched pairs (first-pass distinct
    // pairs + the tiers' kept pairs)
    // abort_flag (device): the first pass exits when it is set (big partitions
    // still to build, bucket_stage phase 1); *aborted then tells the caller
    // ---- pair counting -------------------------------------------------
    PairParams P;
    P.min_coll = c->set.min_collisions;
    P.max_coll = c->set.max_collisions;
    P.emit_all = emit_all ? 1 : 0;
    P.strict = strict ? 1 : 0;
    P.split = 1;
    P.coded = 0;
    P.max_occ = c->max_occ;
    P.n_items = n_items;
    P.xcd_swizzle = read_order ? 1 : 0;
    P.table = 256;
    P.abort = abort_flag;
    if (aborted) *aborted = false;
    P.per_read = per_read && *per_read ? 1 : 0;
    P.max_blocks = c->launch_slice;
    P.early = 0;
    if (per_read) *per_read = false;
    uint2 *rreg = nullptr;
    uint32_t *rcnt = nullptr;
    if (P.per_read) {
        ENSURE(c->d_rreg, (uint64_t)n_items * PC_RREG, &rreg);
        ENSURE(c->d_rcnt, (uint64_t)n_items + 1, &rcnt);
    }
    if (c->pair_cap == 0) c->pair_cap = std::max<uint64_t>(1 << 16, (uint64_t)n_items * (P.emit_all ? 64 : 24));
    // output regions: NSHARD (x owners) of cap_s entries (a block appends to
    // region blockIdx % NSHARD, of its lead's owner)
    const uint32_t R = NSHARD * std::max(owners, 1u);
    unsigned long long *dcur = cnt->cursor;
    if (owners > 1) ENSURE(c->d_ocur, R, &dcur);
    std::vector<unsigned long long> cur(R, 0);
    auto cur_max = [&]() { unsigned long long m = 0; for (auto v : cur) m = std::max(m, v); return m; };
    auto read_cur = [&]() -> int {  // (stream work up to here complete)
        if (owners > 1) HIPCHK(hipMemcpy(cur.data(), dcur, (size_t)R * 8, hipMemcpyDeviceToHost));
        return SA_OK;
    };
    uint32_t ovn = 0;
    uint64_t cap_s = (c->pair_cap + R - 1) / R;
    // Dense read sets (configs[4]'s k = 12 slice: 12-mers collide at random, and
    // every read meets ~24k partners): every 256-slot table of the first pass
    // overflows, and the pass costs its whole launch (0.49 s of ~7 s there) for
    // nothing.  Every 64th read runs it first, counting only (dummy counters,
    // no output room); when >= 95 % of that sample overflows, every read goes
    // straight to the big tier in the shared-region mode, whose split-1 pass then
    // sums the role pairs (SA_SKIP_PROBE=0: no probe, A/B runs).
    bool skip_first = false;
    static const bool probe_on = !getenv("SA_SKIP_PROBE") || atoi(getenv("SA_SKIP_PROBE")) != 0;
    const bool dense_ok = !strict && !item_start && !P.emit_all;
    if (dense_ok && c->first_pass == 2) {
        skip_first = true;
        P.per_read = 0;
    } else if (probe_on && dense_ok && c->first_pass == 0 && n_items >= (1u << 18)) {
        constexpr uint32_t stride = 64;
        const uint32_t ns = n_items / stride;
        std::vector<uint32_t> sample(ns);
        for (uint32_t i = 0; i < ns; ++i) sample[i] = i * stride + stride / 2;
        uint32_t *sl;
        ENSURE(c->d_tier, ns, &sl);
        PairOut OS{};
        OS.cursor = cnt->role_pairs_dummy;  // (claims only: cap_s = 0, nothing is written)
        OS.cap_s = 0;
        OS.role_pairs = cnt->role_pairs_dummy;
        OS.distinct = cnt->role_pairs_dummy;
        OS.overflow_n = &cnt->overflow_n;
        ENSURE(c->d_ovl, (uint64_t)n_items + 3, &OS.overflow_list);
        ENSURE(c->d_ovlrp, (uint64_t)n_items + 3, &OS.overflow_rp);
        PairParams PS = P;
        PS.n_items = ns;
        PS.xcd_swizzle = 0;
        PS.per_read = 0;  // (the one-read workgroup: its emission claims land in the dummy)
        uint32_t nov = 0;
        HIPCHK(hipMemcpyAsync(sl, sample.data(), (size_t)ns * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemsetAsync(&cnt->overflow_n, 0, sizeof(uint32_t), c->stream));
        {
            StageScope st(c, SA_STAGE_PAIRS);
            HIPCHK(launch_pair_count(E, PI, PS, OS, sl, ns, c->stream));
        }
        HIPCHK(hipMemcpyAsync(&nov, &cnt->overflow_n, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemsetAsync(&cnt->overflow_n, 0, sizeof(uint32_t), c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        // (a pending big-partition build makes the sample exit at once: nov = 0)
        skip_first = (uint64_t)nov * 20 >= (uint64_t)ns * 19 && ns > 0;
        if (skip_first) P.per_read = 0;
    }
    for (int attempt = 0; attempt < 4; ++attempt) {
        PairOut O{};
        const uint64_t tot_cap = cap_s * R;
        ENSURE(c->d_pf, tot_cap, &O.fst);
        ENSURE(c->d_ps, tot_cap, &O.snd);
        ENSURE(c->d_pc, tot_cap, &O.cnt);
        O.rank = nullptr;
        if (strict) ENSURE(c->d_pr, tot_cap, &O.rank);
        ENSURE(c->d_ovl, (uint64_t)n_items + 3, &O.overflow_list);  // reads whose table overflowed
        ENSURE(c->d_ovlrp, (uint64_t)n_items + 3, &O.overflow_rp);  // and their role pairs
        if (item_start) O.overflow_rp = nullptr;  // multi-read blocks: the host routes by table
        O.cursor = dcur;
        O.owners = owners;
        O.owner_starts = owner_starts;
        O.item_owner = item_owner;
        O.item_end = item_end;
        O.cap_s = cap_s;
        O.role_pairs = cnt->role_pairs;
        O.overflow_n = &cnt->overflow_n;
        O.distinct = cnt->distinct;
        O.rreg = rreg;
        O.rcnt = rcnt;
        // (cursor, role pairs, dummy, distinct: a pass re-run after an abort or
        // in the shared-region mode counts from zero)
        if (!counters_zeroed || attempt > 0) {  // (a re-run attempt counts from zero)
            HIPCHK(hipMemsetAsync(cnt->cursor, 0, 4 * NSHARD * sizeof(unsigned long long), c->stream));
            HIPCHK(hipMemsetAsync(&cnt->overflow_n, 0, sizeof(uint32_t), c->stream));
        }
        if (owners > 1) HIPCHK(hipMemsetAsync(dcur, 0, (size_t)R * 8, c->stream));
        if (!skip_first) {
            StageScope st(c, SA_STAGE_PAIRS);
            if (item_start) {  // multi-read blocks (sharded path)
                PairParams PM = P;
                PM.n_items = n_multi;
                PM.table = 1024;
                HIPCHK(launch_pair_count_multi_wave(E, PI, PM, O, item_start, n_multi, n_items, c->stream));
            } else {
                HIPCHK(launch_pair_count(E, PI, P, O, read_order, read_order ? ((n_items + 7) & ~7u) : n_items,
                                         c->stream));
            }
        }
        // one pinned copy of the counters: cursors, overflow count, distinct
        // pairs and the abort flag (P.abort is cnt->big_n)
        Counters *hp;
        if (int rc_p = pinned_counters(c, &hp)) return rc_p;
        HIPCHK(hipMemcpyAsync(hp, cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (owners > 1) { if (int rc_c = read_cur()) return rc_c; }
        else memcpy(cur.data(), hp->cursor, NSHARD * 8);
        ovn = skip_first ? n_items : hp->overflow_n;
        // big partitions still to build: the first pass exited at once -- and with the
        // first pass skipped (SA_OPT_FIRST_PASS = 2) the tiers below would read records
        // the global path has not written yet, so the skip mode aborts the same way
        const uint32_t abv = P.abort ? hp->big_n : 0u;
        unsigned long long dist_h[NSHARD];
        memcpy(dist_h, hp->distinct, sizeof(dist_h));
        if (abv) {
            *aborted = true;
            return SA_OK;
        }
        P.abort = nullptr;
        c->first_overflow = ovn;  // reads the first pass handed to the recount tiers
        const uint64_t first_distinct = shard_sum(dist_h);
        if (P.per_read && ovn == 0) {
            *per_read = true;
            if (distinct_ub) *distinct_ub = first_distinct;
            np = 0;
            cap_s_out = cap_s;
            return SA_OK;
        }
        // Reads whose 256-slot table overflowed (> 192 partners) are recounted
        // one per block in bigger tables: 2,048 slots unless their partner count
        // -- extrapolated from how fast the first pass filled -- is far beyond it,
        // 16,384 slots (128 KB of
        // LDS, wide ids) for the rest and for 2,048-slot failures, then in 8 and
        // 64 partner-residue classes -- refining only the classes that
        // overflowed.  Strict ids: 2,048 slots, then 64 classes.  Items are
        // codes (read << 6 | residue class).
        if (ovn > 0 && n_items >= (1u << 26))
            return fail(c, SA_E_OVERFLOW, "recount tiers address reads with 26 bits");
        std::vector<uint32_t> q_big, q_huge;
        if (skip_first) {  // every read, straight to the big tier, in the locality order
            q_huge.resize(n_items);
            if (read_order) {
                // blocks are dealt round-robin over the 8 XCDs: item i runs on XCD
                // i % 8, so XCD x is given a contiguous run of the locality order
                // (as the first pass's swizzle does) and shares its partner lists in L2
                std::vector<uint32_t> ro(n_items);
                HIPCHK(hipMemcpyAsync(ro.data(), read_order, (size_t)n_items * 4, hipMemcpyDeviceToHost, c->stream));
                HIPCHK(hipStreamSynchronize(c->stream));
                const uint32_t per = n_items / 8, rem = n_items % 8;  // XCD x: per + (x < rem) reads
                uint32_t i = 0;
                for (uint32_t j = 0; j <= per; ++j)
                    for (uint32_t x = 0; x < 8; ++x) {
                        if (j == per && x >= rem) break;
                        const uint32_t base = x * per + std::min(x, rem);
                        q_huge[i++] = ro[base + j] << 6;
                    }
            } else {
                for (uint32_t i = 0; i < n_items; ++i) q_huge[i] = i << 6;
            }
        } else if (ovn > 0) {
            std::vector<uint32_t> codes(ovn), rps(ovn, 0);
            HIPCHK(hipMemcpy(codes.data(), O.overflow_list, (size_t)ovn * 4, hipMemcpyDeviceToHost));
            if (O.overflow_rp) HIPCHK(hipMemcpy(rps.data(), O.overflow_rp, (size_t)ovn * 4, hipMemcpyDeviceToHost));
            for (uint32_t i = 0; i < ovn; ++i)
                // rps: the partner estimate, a linear extrapolation of the
                // first pass's fill rate -- partners are met early and then
                // recur, so it over-reads (estimate >= partners).  Past 1.5x the
                // 2,048-slot table's 1,536 a read goes straight to 16,384 slots:
                // on configs[4]'s k = 12 shape (~3,900 partners per read) 86 % of
                // the reads the 2,048-slot tier took filled it and were re-run
                // anyway (57 ms of 221 ms of pair counting, 1M reads)
                (strict || rps[i] <= pc_fill_max(2048) * 3u / 2u ? q_big : q_huge).push_back(codes[i]);
        }
        // one tier over host-side items; returns its failures (codes)
        auto run_tier = [&](int table, int split, const std::vector<uint32_t> &items, std::vector<uint32_t> &failed,
                            std::vector<uint32_t> *fest = nullptr) -> int {
            failed.clear();
            if (fest) fest->clear();
            if (items.empty() || cur_max() > cap_s) return SA_OK;
            uint32_t *tl, *fl;
            ENSURE(c->d_tier, items.size(), &tl);
            ENSURE(c->d_ovl, items.size() + 3, &fl);  // at most one failure per item
            HIPCHK(hipMemcpy(tl, items.data(), items.size() * 4, hipMemcpyHostToDevice));
            PairParams PT = P;
            PT.abort = nullptr;
            PT.per_read = 0;  // the tiers emit into the shared regions
            PT.table = table;
            PT.split = split;
            PT.coded = 1;
            PT.n_items = (uint32_t)items.size();
            PT.xcd_swizzle = 0;
            // big tiers: stop a read whose projected partners pass the fill limit
            // (SA_EARLY_STOP=n: n/8 of it, default 8; 0 turns it off, A/B runs)
            // after at least 1/SA_EARLY_FRAC of its role pairs (default 8).
            // configs[4]'s k = 12 slice, pairs stage: no early stop 7.00 s; 9/8
            // after 1/4 5.79; 8/8 after 1/8 5.48 s (profiles/r05/c4ab)
            static const int early_env = getenv("SA_EARLY_STOP") ? atoi(getenv("SA_EARLY_STOP")) : 8;
            static const int early_frac = getenv("SA_EARLY_FRAC") ? std::max(1, atoi(getenv("SA_EARLY_FRAC"))) : 8;
            // (not at the finest split: with no finer class left, a projection that
            // over-reads would push a read that fits into `failed` -> SA_E_OVERFLOW)
            PT.early = table >= 16384 && fest && split < 64 && early_env > 0 ? (early_env & 255) | (early_frac << 8)
                                                                             : 0;
            PairOut OT = O;
            // (skip mode: the split-1 big-tier pass is every read's first pass)
            OT.role_pairs = skip_first && split == 1 && table >= 16384 ? cnt->role_pairs : cnt->role_pairs_dummy;
            OT.overflow_list = fl;
            OT.overflow_rp = nullptr;
            uint32_t *fe = nullptr;
            if (fest) {  // the failures' partner estimates (this class's partners)
                ENSURE(c->d_ovlrp, items.size() + 3, &fe);
                OT.overflow_rp = fe;
            }
            HIPCHK(hipMemsetAsync(&cnt->overflow_n, 0, sizeof(uint32_t), c->stream));
            {
                StageScope st(c, SA_STAGE_PAIRS);
                HIPCHK(launch_pair_count(E, PI, PT, OT, tl, PT.n_items, c->stream));
            }
            uint32_t nf = 0;
            HIPCHK(hipMemcpyAsync(cur.data(), dcur, (size_t)R * 8, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(&nf, &cnt->overflow_n, 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            failed.resize(nf);
            if (nf) HIPCHK(hipMemcpy(failed.data(), fl, (size_t)nf * 4, hipMemcpyDeviceToHost));
            static const bool dbg_tiers = getenv("SA_DEBUG_TIERS") != nullptr;  // (diagnostics: stderr)
            if (dbg_tiers)
                fprintf(stderr, "[sa tiers] table %d split %d items %zu failed %u\n", table, split, items.size(), nf);
            if (fest) {
                fest->resize(nf);
                if (nf) HIPCHK(hipMemcpy(fest->data(), fe, (size_t)nf * 4, hipMemcpyDeviceToHost));
            }
            return SA_OK;
        };
        // the failed classes of a tier at split s, refined into f sub-classes
        auto refine = [](const std::vector<uint32_t> &codes_, uint32_t s_, uint32_t f) {
            std::vector<uint32_t> out;
            out.reserve(codes_.size() * f);
            for (uint32_t cd : codes_)
                for (uint32_t j = 0; j < f; ++j) out.push_back(cd + s_ * j);
            return out;
        };
        std::vector<uint32_t> failed;
        int rc_t;
        uint64_t wide_limit = 64ull * pc_fill_max(16384);  // distinct partners per read the tiers can count
        if ((rc_t = run_tier(2048, 1, q_big, failed))) return rc_t;
        if (strict) {
            if ((rc_t = run_tier(2048, 64, refine(failed, 1, 64), failed))) return rc_t;
        } else {
            // 16,384 slots (12,288 partners) per block; a read that overflows is
            // recounted in partner-residue classes (split s: partners with
            // partner % s == residue, each class re-enumerating the read), as
            // many as its partner estimate from the overflowed 16,384-slot
            // pass asks for (12,288 partners found in the first x role pairs;
            // that sample is large enough to trust -- the first pass's is not:
            // classes chosen from it ran 1M k=12 reads 172 -> 219 ms):
            // configs[4]'s k = 12 slice has ~24k partners per read -> 2-4
            // classes, not 8; a class that still overflows is refined again
            // The packed form (one word per slot: 32,768 slots, 24,576 partners, in
            // the same 128 KB) whenever its 8-bit counts and 24-bit partner ids
            // hold: every count that matters is <= max_coll <= 255, and only the
            // dispatched pairs are emitted.  (SA_PACKED_TIER=0: the two-word
            // table, for A/B runs.)
            static const bool packed_ok = !getenv("SA_PACKED_TIER") || atoi(getenv("SA_PACKED_TIER")) != 0;
            const bool packed = packed_ok && !P.emit_all && P.max_coll <= 255 && n_items < 0xFFFFFFu;
            const int htab = packed ? 32768 : 16384;
            const uint32_t hcap = pc_fill_max((uint32_t)htab);
            wide_limit = 64ull * hcap;
            std::vector<uint32_t> lv[7];  // split 1, 2, 4, ..., 64
            lv[0] = q_huge;
            lv[0].insert(lv[0].end(), failed.begin(), failed.end());  // the 2,048-slot tier's overflow
            failed.clear();
            for (int e = 0; e <= 6; ++e) {
                std::vector<uint32_t> fest;
                if ((rc_t = run_tier(htab, 1 << e, lv[e], failed, &fest))) return rc_t;
                if (failed.empty() || e == 6) continue;
                for (size_t i = 0; i < failed.size(); ++i) {
                    // classes so that each holds <= hcap of this class's
                    // estimated partners (at least 2x finer, at most 64 in all)
                    int ne = e + 1;
                    while (ne < 6 && (uint64_t)fest[i] > (uint64_t)hcap << (ne - e)) ++ne;
                    for (uint32_t j = 0; j < (1u << (ne - e)); ++j) lv[ne].push_back(failed[i] + (1u << e) * j);
                }
                failed.clear();
            }
        }
        if (!failed.empty() && cur_max() <= cap_s)
            return fail(c, SA_E_OVERFLOW, "a read has more than " +
                                              std::to_string(strict ? 64ull * pc_fill_max(2048) : wide_limit) +
                                              " distinct partners");
        if (cur_max() <= cap_s) {
            if (P.per_read) {  // regions kept; the recounted reads' pairs are in the shared regions
                *per_read = true;
                uint64_t ns = 0;
                for (auto v : cur) ns += v;
                if (distinct_ub) *distinct_ub = first_distinct + ns;
            }
            break;
        }
        cap_s = cur_max() + cur_max() / 4 + 1024;  // grow and recount
        c->pair_cap = cap_s * R;
        if (attempt == 3) return fail(c, SA_E_OVERFLOW, "pair output did not fit");
    }
    np = 0;
    for (auto v : cur) np += v;
    if (owners > 1) c->ocur = cur;
    cap_s_out = cap_s;
    return SA_OK;
}


// The per-read regions (pair_stage's per_read mode) as one (lead, trail, count)
// list, lead descending, trail ascending, ids 1-based: the regions in order of
// an exclusive scan of their counts, with the reads the tiers recounted (np
// pairs in the shared regions, their regions empty) taken from those pairs
// sorted lead-descending / trail-ascending -- each such read's segment start in
// rsh[read] (+1), its length in rcnt[read].  The total lands in cnt->rtotal.
int assemble_read_regions(sa_ctx *c, uint32_t nr, uint64_t np, uint64_t np_ub, uint64_t cap_s, Counters *cnt,
                          int32_t **dlead, int32_t **dtrail, int32_t **dcount) {
    uint32_t *rex; uint8_t *stmp2;
    uint64_t *ok, *ok2; uint32_t *ov, *ov2; uint8_t *otmp;
    ENSURE(c->d_lead, np_ub, dlead);
    ENSURE(c->d_trail, np_ub, dtrail);
    ENSURE(c->d_count, np_ub, dcount);
    ENSURE(c->d_rex, (uint64_t)nr + 1, &rex);
    uint32_t *rcnt = (uint32_t *)c->d_rcnt.p;
    const int32_t *stl = nullptr, *scn = nullptr;
    uint32_t *rsh = nullptr;
    if (np) {
        int32_t *shl, *sht, *shc;
        ENSURE(c->d_okeys, np, &ok);
        ENSURE(c->d_okeys2, np, &ok2);
        ENSURE(c->d_ovals, np, &ov);
        ENSURE(c->d_ovals2, np, &ov2);
        ENSURE(c->d_osort, std::max(radix_sort_temp_bytes(np), scan_temp_bytes(nr)), &otmp);
        ENSURE(c->d_shl, np, &shl);
        ENSURE(c->d_sht, np, &sht);
        ENSURE(c->d_shc, np, &shc);
        ENSURE(c->d_rsh, nr, &rsh);
        const int idb = bits_for(nr ? nr - 1 : 0);
        HIPCHK(launch_make_order_keys((const uint32_t *)c->d_pf.p, (const uint32_t *)c->d_ps.p, nullptr,
                                      cnt->cursor, cap_s, 0, idb, ok, ov, cnt->shard_off, c->stream));
        HIPCHK(radix_sort(&ok, &ov, &ok2, &ov2, np, 0, 2 * idb, otmp, c->stream));
        HIPCHK(launch_gather_pairs(ov, np, (const uint32_t *)c->d_pf.p, (const uint32_t *)c->d_ps.p,
                                   (const uint32_t *)c->d_pc.p, shl, sht, shc, c->stream));
        HIPCHK(hipMemsetAsync(rsh, 0, (size_t)nr * 4, c->stream));
        HIPCHK(launch_mark_segments(shl, np, rsh, rcnt, c->stream));
        stl = sht; scn = shc;
        stmp2 = otmp;
    } else {
        ENSURE(c->d_osort, scan_temp_bytes(nr), &stmp2);
    }
    HIPCHK(exclusive_scan_u32(rcnt, rex, nr, &cnt->rtotal, stmp2, c->stream));
    HIPCHK(launch_copy_read_regions((const uint2 *)c->d_rreg.p, rcnt, rex, &cnt->rtotal, nr, rsh, stl, scn,
                                    *dlead, *dtrail, *dcount, c->stream));
    return SA_OK;
}

// ---------------------------------------------------------------------------
// candidate build (device), optional host readback
// ---------------------------------------------------------------------------
int device_build(sa_ctx *c, bool readback) {
    if (c->dist) return fail(c, SA_E_STATE, "distributed context: use sa_dist_emit / sa_dist_count / sa_dist_reduce");
    int rc = ensure_prepared(c);
    if (rc) return rc;
    c->built = false;
    c->aligned = false;
    const bool strict = c->mode == SA_IDS_STRICT;
    const uint32_t nr = (uint32_t)(c->boff.size() - 1);
    const uint64_t n = c->n_occ;
    DevReads R = dev_reads(c);
    EmitParams E = emit_params(c);
    Counters *cnt;
    ENSURE(c->d_cnt, 1, &cnt);
    HIPCHK(hipMemsetAsync(cnt, 0, sizeof(Counters), c->stream));  // (the first bucket and pair stages rely on it)

    uint64_t *keys, *keys2; uint32_t *vals, *vals2; void *stmp;
    ENSURE(c->d_keys, n, &keys);
    ENSURE(c->d_keys2, n, &keys2);
    ENSURE(c->d_vals, n, &vals);
    ENSURE(c->d_vals2, n, &vals2);
    uint8_t *stmp8;
    ENSURE(c->d_sorttmp, std::max(radix_sort_temp_bytes(n), buckets_temp_bytes(n)), &stmp8);
    stmp = stmp8;
    // reads of <= 1,024 bases: packing and emission in one kernel (pack_emit.hip),
    // timed as the emit stage
    const bool fused = c->maxL <= 1024;
    if (!fused) {
        StageScope st(c, SA_STAGE_PACK);
        HIPCHK(launch_pack_reads(R, c->stream));
    }
    uint64_t *rk0, *rk1; uint32_t *ro0, *ro1; uint8_t *rtmp;
    ENSURE(c->d_rkey, nr, &rk0);
    ENSURE(c->d_rkey2, nr, &rk1);
    ENSURE(c->d_rord, nr, &ro0);
    ENSURE(c->d_rord2, nr, &ro1);
    ENSURE(c->d_rtmp, radix_sort_temp_bytes(nr), &rtmp);
    E.rkey = rk0;
    E.rord = ro0;
    // mixed read lengths, wide ids: records carry (read, pos) and the bucket
    // build finds a k-mer's occurrence index and loc rank with one meta load
    c->pos_bits = 0;
    if (!strict && c->uniform_npr == 0 && nr > 0) {
        const int pb = bits_for((uint64_t)std::max(c->maxd, 1));
        if (pb < 32 && (uint64_t)nr < (1ull << (32 - pb))) {
            if (c->meta_gen != c->reads_gen || c->meta_k != c->set.kmer_size) {
                std::vector<uint32_t> meta(2 * (size_t)nr);
                for (uint32_t r = 0; r < nr; ++r) {
                    meta[2 * r] = (uint32_t)c->occ_off[r];
                    const int32_t d = c->len[r] - c->set.kmer_size;
                    meta[2 * r + 1] = d >= 0 ? c->lbase[d] : 0u;
                }
                uint32_t *dm;
                ENSURE(c->d_meta, 2 * (size_t)nr, &dm);
                HIPCHK(hipMemcpyAsync(dm, meta.data(), meta.size() * 4, hipMemcpyHostToDevice, c->stream));
                HIPCHK(hipStreamSynchronize(c->stream));
                c->meta_gen = c->reads_gen;
                c->meta_k = c->set.kmer_size;
            }
            c->pos_bits = pb;
        }
    }
    E.pos_bits = c->pos_bits;
    // mixed lengths without (read, pos) codes (too many reads, or strict ids):
    // the emit kernel also writes each occurrence's read and loc rank, so the
    // bucket build looks both up with one load each instead of a search
    uint2 *orl = nullptr;
    if (c->uniform_npr == 0 && c->pos_bits == 0) {
        ENSURE(c->d_rl, n + 1, &orl);
        E.occ_rl = orl;
    }
    KeyGen kg{};
    const bool use_kgen = fused && make_keygen(c, E, n, kg);
    {
        StageScope st(c, SA_STAGE_EMIT);
        if (use_kgen && hist_in_pack()) {  // + the first radix pass's tile histogram
            E.hist = (uint32_t *)stmp;
            E.hist_shift = kg.hist_shift = 64 - part_bits(n);
            HIPCHK(launch_pack_emit_hist(R, E, n, c->stream));
        } else if (fused) HIPCHK(launch_pack_emit(R, E, use_kgen ? nullptr : keys, c->stream));
        else HIPCHK(launch_kmer_emit(R, E, keys, vals, c->stream));
    }
    // reads in locality order (overlapping reads adjacent) for pair_count: by
    // their minimum k-mer mix (reads sharing it stay adjacent), on the side
    // stream beside the partition sort and the bucket build.  The minimum of
    // a read's ~500 mixes sits far below 2^32 (mean 2^32 / 487 ~ 2^23), so
    // the sort must reach below the top 16 bits to separate distinct minima
#ifndef SA_LOCALITY_LO
#define SA_LOCALITY_LO 8  // (A/B: 16 -> 8, pairs 0.595-0.608 -> 0.578-0.588 ms)
#endif
    HIPCHK(ensure_side(c));
    HIPCHK(fork_side(c, c->ev_fork));
    HIPCHK(radix_sort(&rk0, &ro0, &rk1, &ro1, nr, SA_LOCALITY_LO, 32, rtmp, c->side));
    HIPCHK(hipEventRecord(c->ev_join, c->side));
    static const bool no_loc = getenv("SA_NO_LOCALITY") && atoi(getenv("SA_NO_LOCALITY")) != 0;  // (A/B)
    const uint32_t *read_order = no_loc ? nullptr : ro0;
    PartArgs PA{};
    unsigned long long big_buckets = 0;
    // wide ids: no readback between the bucket build and the pair counter (its
    // first pass aborts if a partition needs the global path, see below)
    const int bphase = strict ? 0 : 1;
    rc = bucket_stage(c, keys, keys2, vals, vals2, n, (const uint64_t *)c->d_occ_off.p, nr, c->uniform_npr,
                      orl, (const int32_t *)c->d_len.p, strict, stmp, cnt, PA, big_buckets, 0, bphase, nullptr,
                      use_kgen ? &kg : nullptr, nullptr, true);
    if (rc) return rc;
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
    if (strict) {
        // KmerData iteration rank of every bucket: replay its Trove layout over the
        // distinct hashes in first-occurrence order (KmerTable.scala:45-50).  A
        // bucket is named by the sorted position of its head record.
        HostScope hs(c, SA_STAGE_REPLAY);
        static const bool host_replay = getenv("SA_HOST_TROVE") && atoi(getenv("SA_HOST_TROVE")) != 0;  // (A/B)
        if (!host_replay) {
            // on the device (trove_replay.hip): heads by first occurrence, their seqHash from
            // the packed reads, the layout, the ranks -- no readback of the 5 B per k-mer of
            // head flags and first occurrences
            uint8_t *kt;
            ENSURE(c->d_trove, kmerdata_temp_bytes(n), &kt);
            uint32_t heads = 0;
            HIPCHK(kmerdata_rank_device(PA.is_head, PA.bkt_first, n, dev_reads(c), (const uint64_t *)c->d_occ_off.p, nr,
                                        c->m, c->bkt_rank_dev, kt, c->stream, &heads));
            if (heads >= (1u << 26)) return fail(c, SA_E_OVERFLOW, "strict ids: more than 2^26 distinct k-mers");
        } else {
            std::vector<uint8_t> head(n);
            std::vector<uint32_t> first(n);
            if (n) {
                HIPCHK(hipMemcpy(head.data(), PA.is_head, n, hipMemcpyDeviceToHost));
                HIPCHK(hipMemcpy(first.data(), PA.bkt_first, n * 4, hipMemcpyDeviceToHost));
            }
            // the buckets in first-occurrence order: first occurrences are distinct indices < n,
            // so each head lands at its own slot of a g-indexed table and one ascending walk
            // reads them in order -- with the read of g advancing monotonically (no sort of the
            // ~2M heads, no binary search per head)
            std::vector<uint32_t> by_g(n, 0);  // head position + 1 of the bucket first met at g
            for (uint64_t i = 0; i < n; ++i)
                if (head[i]) by_g[first[i]] = (uint32_t)i + 1;
            TroveLayout kd;
            const int k = c->set.kmer_size, mm = c->m;
            uint32_t r = 0;
            for (uint64_t g = 0; g < n; ++g) {
                const uint32_t hp = by_g[g];
                if (!hp) continue;
                while (c->occ_off[r + 1] <= g) ++r;  // the last read with occ_off[r] <= g
                const char *sq = c->bases.data() + c->boff[r] + (g - c->occ_off[r]);
                uint32_t h = 0;  // Kmer.seqHash (ObjectStore.scala:48-67)
                for (int q = 0; q < mm; ++q) {
                    char ch = sq[q];
                    if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
                    h <<= 2;
                    h ^= ch == 'C' ? 1u : ch == 'T' ? 2u : ch == 'G' ? 3u : 0u;
                }
                (void)k;
                kd.insert((int32_t)h, (int32_t)(hp - 1));  // (distinct hashes: every insert is fresh)
            }
            std::vector<uint32_t> rank(n, 0);
            uint32_t rk = 0;
            kd.for_each_kv([&](int32_t, int32_t pos) { rank[(uint32_t)pos] = rk++; });
            if (rk >= (1u << 26)) return fail(c, SA_E_OVERFLOW, "strict ids: more than 2^26 distinct k-mers");
            if (n) HIPCHK(hipMemcpy(c->bkt_rank_dev, rank.data(), n * 4, hipMemcpyHostToDevice));
        }
    }
    PairIn PI{};
    PI.rec = PA.rec; PI.xrec = PA.xrec; PI.lst = PA.lst;
    if (strict) {
        PI.srec = PA.srec; PI.lidx = PA.lidx;
        PI.bkt_nst = PA.bkt_nst; PI.bkt_nmd = PA.bkt_nmd; PI.bkt_rank = c->bkt_rank_dev;
    }

    uint64_t np = 0, cap_s = 0;
    bool aborted = false;
    const bool emit_all = strict || c->keep_pairs;
    // dispatched pairs straight into per-read regions (pair_stage) when the
    // regions stay within 4 GB: the lead-descending order is then a scan and
    // a copy instead of a 34-bit radix sort (of the recounted reads' pairs only)
    const bool per_read_ok = !emit_all && (uint64_t)nr * PC_RREG * sizeof(uint2) <= (4ull << 30);
    bool per_read = per_read_ok;
    uint64_t np_ub = 0;
    rc = pair_stage(c, E, PI, strict, emit_all, read_order, nr, cnt, np, cap_s, nullptr, 0,
                    bphase == 1 ? &cnt->big_n : nullptr, &aborted, &per_read, &np_ub, 1, nullptr, nullptr, true);
    if (rc) return rc;
    if (aborted) {  // partitions above 4,096 records (high-copy repeats): build them, count again
        rc = bucket_stage(c, keys, keys2, vals, vals2, n, (const uint64_t *)c->d_occ_off.p, nr, c->uniform_npr,
                          orl, (const int32_t *)c->d_len.p, strict, stmp, cnt, PA, big_buckets, 0, 2);
        if (rc) return rc;
        PI.xrec = PA.xrec;
        per_read = per_read_ok;
        rc = pair_stage(c, E, PI, strict, emit_all, read_order, nr, cnt, np, cap_s, nullptr, 0, nullptr, nullptr,
                        &per_read, &np_ub);
        if (rc) return rc;
    }
    c->recounted = per_read ? np : 0;
    c->used_per_read = per_read;

    // ---- ordering --------------------------------------------------------
    int32_t *dlead, *dtrail, *dcount;
    uint64_t *ok, *ok2; uint32_t *ov, *ov2; uint8_t *otmp;
    if (per_read) {
        StageScope st(c, SA_STAGE_ORDER);
        if ((rc = assemble_read_regions(c, nr, np, np_ub, cap_s, cnt, &dlead, &dtrail, &dcount))) return rc;
    }
    if (!per_read) {
        ENSURE(c->d_okeys, np, &ok);
        ENSURE(c->d_okeys2, np, &ok2);
        ENSURE(c->d_ovals, np, &ov);
        ENSURE(c->d_ovals2, np, &ov2);
        ENSURE(c->d_osort, radix_sort_temp_bytes(np), &otmp);
        ENSURE(c->d_lead, np, &dlead);
        ENSURE(c->d_trail, np, &dtrail);
        ENSURE(c->d_count, np, &dcount);
        {
            StageScope st(c, SA_STAGE_ORDER);
            const int idb = bits_for(nr ? nr - 1 : 0);
            HIPCHK(launch_make_order_keys((const uint32_t *)c->d_pf.p, (const uint32_t *)c->d_ps.p,
                                          (const uint64_t *)c->d_pr.p, cnt->cursor, cap_s, strict ? 1 : 0, idb, ok, ov,
                                          cnt->shard_off, c->stream));
            const int hi = strict ? 64 : 2 * idb;
            HIPCHK(radix_sort(&ok, &ov, &ok2, &ov2, np, 0, hi, otmp, c->stream));
            HIPCHK(launch_gather_pairs(ov, np, (const uint32_t *)c->d_pf.p, (const uint32_t *)c->d_ps.p,
                                       (const uint32_t *)c->d_pc.p, dlead, dtrail, dcount, c->stream));
        }
    }
    Counters *hp;
    if ((rc = pinned_counters(c, &hp))) return rc;
    HIPCHK(hipMemcpyAsync(hp, cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const Counters hc = *hp;
    if (per_read) np = hc.rtotal;
    resolve_timing(c);
    c->stats = sa_stats{};
    c->stats.kmers = n;
    c->stats.buckets = shard_sum(hc.bkt_counts) + big_buckets;
    c->stats.role_pairs = shard_sum(hc.role_pairs);
    c->stats.pairs = shard_sum(hc.distinct);
    c->stats.id_mode = c->mode;
    c->stats.flags = (per_read ? SA_STATS_PER_READ_REGIONS : 0) | (c->first_overflow ? SA_STATS_RECOUNTED : 0);

    c->lead.clear(); c->trail.clear(); c->count.clear();
    c->pfst.clear(); c->psnd.clear(); c->pcnt.clear();
    if (!strict && !emit_all) {
        c->n_disp = np;
        if (readback && np) {
            HostScope hs(c, SA_STAGE_READBACK);
            c->lead.resize(np); c->trail.resize(np); c->count.resize(np);
            HIPCHK(hipMemcpy(c->lead.data(), dlead, np * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(c->trail.data(), dtrail, np * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(c->count.data(), dcount, np * 4, hipMemcpyDeviceToHost));
        }
    } else {
        // every distinct pair came back (strict: in first-insertion order; wide: lead desc)
        HostScope hs(c, SA_STAGE_REPLAY);
        // strict: PairData's Trove layout of the keys (fst << 16) ^ snd inserted in
        // first-occurrence order is built on the device (trove_replay.hip: the host replay,
        // one insert after another at DRAM latency, was ~170 ms of configs[0]'s 0.2 s end to
        // end), and the pairs come back permuted into its iteration order
        static const bool host_replay = getenv("SA_HOST_TROVE") && atoi(getenv("SA_HOST_TROVE")) != 0;  // (A/B)
        const bool dev_replay = strict && !host_replay && np > 0;
        const int32_t *rf = dlead, *rs = dtrail, *rk = dcount;
        if (dev_replay) {
            uint8_t *tb;
            // keys, fo / so / ko, order, then the layout's scratch -- which the dispatched pairs'
            // compaction reuses afterwards (3 n + n + 64 words + a scan's scratch: within it)
            const size_t need = 5 * (size_t)np * 4 +
                                std::max(trove_temp_bytes((uint32_t)np), (4 * (size_t)np + 64) * 4 + scan_temp_bytes(np)) +
                                256;
            ENSURE(c->d_trove, need, &tb);
            int32_t *keys = (int32_t *)tb, *fo = keys + np, *so = fo + np, *ko = so + np;
            uint32_t *order = (uint32_t *)(ko + np);
            void *ttmp = (void *)(order + np);
            HIPCHK(launch_trove_pair_keys(dlead, dtrail, (uint32_t)np, keys, c->stream));
            uint32_t tcap = 0;
            HIPCHK(trove_layout_device(keys, (uint32_t)np, order, ttmp, c->stream, &tcap));
            HIPCHK(launch_trove_gather3(order, (uint32_t)np, dlead, dtrail, dcount, fo, so, ko, c->stream));
            rf = fo; rs = so; rk = ko;
        }
        // (device layout without SA_OPT_KEEP_PAIRS: only the dispatched pairs come back --
        // the filter and the compaction run on the device, in iteration order)
        uint64_t nb = np;
        if (dev_replay && !c->keep_pairs) {
            int32_t *keys = (int32_t *)c->d_trove.p, *fo = keys + np, *so = fo + np, *ko = so + np;
            uint32_t *order = (uint32_t *)(ko + np), *flag = (uint32_t *)keys, *tot = order;
            int32_t *fk = (int32_t *)(order + np), *sk = fk + np, *kk = sk + np;
            uint32_t *ex = (uint32_t *)(kk + np);
            void *stmp = (void *)(ex + np + 64);
            HIPCHK(launch_trove_keep(fo, so, ko, (uint32_t)np, c->set.min_collisions, c->set.max_collisions, flag, ex,
                                     tot, stmp, fk, sk, kk, c->stream));
            uint32_t nk = 0;
            HIPCHK(hipMemcpyAsync(&nk, tot, 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            nb = nk;
            rf = fk; rs = sk; rk = kk;
        }
        std::vector<int32_t> f(nb), s(nb), k(nb);
        if (nb) {
            HIPCHK(hipMemcpyAsync(f.data(), rf, nb * 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(s.data(), rs, nb * 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(k.data(), rk, nb * 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
        }
        if (strict) {
            // PairData: Trove layout of keys (fst<<16)^snd inserted in first-occurrence
            // order, each slot carrying its pair's index (the count without a lookup);
            // with the device layout the pairs already are in its iteration order
            TroveLayout pd;
            if (!dev_replay)
                for (uint64_t i = 0; i < np; ++i)
                    pd.insert((int32_t)(((uint32_t)f[i] << 16) ^ (uint32_t)s[i]), (int32_t)i);
            // calcDispatchData (KmerTable.scala:155-187) over PairData iteration order:
            // DispatchData's Trove layout over the leads, each lead's (trail, count)
            // list in that order.  Decoded leads are 16-bit (key >> 16, E4): a lead's
            // list slot is looked up in a 65,536-entry table
            TroveLayout dd;
            std::vector<std::vector<std::pair<int32_t, int32_t>>> lists;
            std::vector<int32_t> list_of(1 << 16, -1);  // lead + 32,768 -> list index
            bool id_err = false;
            auto each_pair = [&](int32_t key, int32_t ix) {
                const int32_t cnt_ = k[(uint32_t)ix];
                const int32_t a = key >> 16;
                const int32_t b = (int32_t)((uint32_t)key << 16) >> 16;
                if (c->keep_pairs) { c->pfst.push_back(a); c->psnd.push_back(b); c->pcnt.push_back(cnt_); }
                if (c->set.min_collisions <= cnt_ && cnt_ <= c->set.max_collisions) {
                    int32_t &li = list_of[(uint32_t)(a + 32768) & 0xFFFFu];
                    if (li < 0) {
                        dd.insert(a, (int32_t)lists.size());
                        li = (int32_t)lists.size();
                        lists.emplace_back();
                    }
                    lists[(size_t)li].push_back({b, cnt_});
                    if (a < 1 || a > (int32_t)nr || b < 1 || b > (int32_t)nr) id_err = true;
                }
            };
            if (dev_replay) {
                for (uint64_t j = 0; j < nb; ++j)
                    each_pair((int32_t)(((uint32_t)f[j] << 16) ^ (uint32_t)s[j]), (int32_t)j);
            } else {
                pd.for_each_kv(each_pair);
            }
            if (id_err)
                return fail(c, SA_E_ID_RANGE, "strict ids: a dispatched pair decodes to an id outside 1..N "
                                              "(reference NullPointerException, KmerTable.scala:263-265)");
            size_t nd_ = 0;
            for (const auto &v : lists) nd_ += v.size();
            c->lead.reserve(nd_); c->trail.reserve(nd_); c->count.reserve(nd_);
            dd.for_each_kv([&](int32_t a, int32_t li) {
                for (const auto &bc : lists[(size_t)li]) {
                    c->lead.push_back(a);
                    c->trail.push_back(bc.first);
                    c->count.push_back(bc.second);
                }
            });
        } else {
            // wide + keep_pairs: PairData sorted (fst, snd); dispatch = filter, lead desc
            std::vector<uint32_t> ix(np);
            for (uint64_t i = 0; i < np; ++i) ix[i] = (uint32_t)i;
            std::sort(ix.begin(), ix.end(), [&](uint32_t x, uint32_t y) {
                return f[x] != f[y] ? f[x] < f[y] : s[x] < s[y];
            });
            for (uint32_t i : ix) { c->pfst.push_back(f[i]); c->psnd.push_back(s[i]); c->pcnt.push_back(k[i]); }
            for (uint64_t i = 0; i < np; ++i)
                if (c->set.min_collisions <= k[i] && k[i] <= c->set.max_collisions) {
                    c->lead.push_back(f[i]); c->trail.push_back(s[i]); c->count.push_back(k[i]);
                }
        }
        c->n_disp = c->lead.size();
        if (c->n_disp) {
            HIPCHK(hipMemcpy(dlead, c->lead.data(), c->n_disp * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(dtrail, c->trail.data(), c->n_disp * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(dcount, c->count.data(), c->n_disp * 4, hipMemcpyHostToDevice));
        }
    }
    c->stats.dispatched = c->n_disp;
    c->built = true;
    return SA_OK;
}

int host_results(sa_ctx *c);

int device_align(sa_ctx *c, bool readback) {
    if (!c->built) return fail(c, SA_E_STATE, "sa_align before sa_build_candidates");
    // this run's records or none: a failure below must not leave the previous
    // run's alignments / .ovl readable through the getters
    c->aligned = false;
    c->host_valid = false;
    const uint64_t nd = c->n_disp;
    // reads the aligner sees: this device's, or (distributed) the all-gathered set
    DevReads AR = dev_reads(c);
    int32_t maxL = c->maxL, minL = c->minL;
    if (c->dist) {
        if (!c->dist_reads) return fail(c, SA_E_STATE, "distributed align before sa_dist_set_reads");
        AR.n = (uint32_t)c->dlen.size();
        AR.ascii = nullptr;
        AR.boff = nullptr;
        AR.woff = (const uint64_t *)c->d_gwoff.p;
        AR.len = (const int32_t *)c->d_glen.p;
        AR.codes = (uint32_t *)c->d_gcodes.p;
        AR.bad = (int32_t *)c->d_gbad.p;
        maxL = c->gmaxL;
        minL = c->gminL;
    }
    const float omm = 1.0f - c->set.min_identity;
    const float prod = (float)maxL * omm;
    const int32_t wmax = std::max(c->set.kmer_size, (int32_t)floor((double)prod) + 1);
    // Lane groups and LDS traceback are sized for the longest read; a pair whose
    // band (w > 63) or lead (> ~2,500 bp) exceeds what this build holds fails in
    // the kernel with SA_E_OVERFLOW -- only if such a pair is actually dispatched.
    const int G = wmax <= 15 ? 16 : (wmax <= 31 ? 32 : 64);
    const uint32_t rw_fit = (160u * 1024u / (256u * 4u) - 1u) | 1u;
    const uint32_t rw = std::min<uint32_t>((uint32_t)((maxL + 1 + 15) / 16) | 1u, rw_fit);
    // The DP kernels hold the cost matrix as int8 bytes (HOXD70 spans -125..100),
    // or as int16 halves for other matrices (one extra select per lookup).
    // Every recurrence (BioLibs.scala:645-668, :725-764; :171-263 for the
    // quadratic aligner) is max-plus and linear in (costs, gO, gE) with 0, so
    // dividing all of them by their common divisor g scales every cell by 1/g
    // exactly: argmax, walk codes and the alignment are unchanged (a x10 HOXD
    // matrix with gap costs -200 / -20 runs as HOXD70 in int8).
    int32_t cost[16], gap_open = c->set.gap_open, gap_extend = c->set.gap_extend;
    int32_t cost_bits = 8;
    {
        auto gcd = [](int64_t a, int64_t b) { a = a < 0 ? -a : a; b = b < 0 ? -b : b; while (b) { int64_t t = a % b; a = b; b = t; } return a; };
        int64_t g = gcd(gap_open, gap_extend);
        for (int x = 0; x < 16; ++x) g = gcd(g, c->set.cost[x]);
        if (g <= 1) g = 1;
        for (int x = 0; x < 16; ++x) {
            cost[x] = (int32_t)(c->set.cost[x] / g);
            if (cost[x] < -32768 || cost[x] > 32767)
                return fail(c, SA_E_OVERFLOW, "cost matrix entries (divided by their common divisor with the gap "
                                              "costs) must lie in [-32768, 32767]");
            if (cost[x] < -128 || cost[x] > 127) cost_bits = 16;
        }
        gap_open = (int32_t)(gap_open / g);
        gap_extend = (int32_t)(gap_extend / g);
    }
    // lane-per-pair kernels: band <= 31 columns (16 / 24 / 32 registers per row),
    // reads <= 30,000 bp (c << 16 | e packing)
    const int lw = dovetail_lane_width(wmax);
    const bool lane_fits = lw > 0 && maxL <= 30000;
    if (c->aligner == SA_ALIGNER_LINEAR && c->align_kernel == 2 && !lane_fits)
        return fail(c, SA_E_ARG, "SA_OPT_ALIGN_KERNEL=2 but a band or read exceeds the lane kernel");
    if (c->aligner == SA_ALIGNER_LINEAR && c->align_kernel == 3 && !lane_fits)
        return fail(c, SA_E_ARG, "SA_OPT_ALIGN_KERNEL=3 but a band or read exceeds the lane kernel");
    if (c->aligner == SA_ALIGNER_QUADRATIC && (c->set.gap_open > 0 || c->set.gap_extend > 0))
        return fail(c, SA_E_ARG, "--quadratic-align needs gap costs <= 0 (Project4.readArgs negates them)");
    if (c->aligner == SA_ALIGNER_QUADRATIC) {
        // its row argmax key packs (T << 5 | column): scores stay below 2^26
        int64_t cmax = 0;
        for (int x = 0; x < 16; ++x) cmax = std::max<int64_t>(cmax, cost[x]);
        if (cmax * (int64_t)maxL >= (1ll << 26))
            return fail(c, SA_E_OVERFLOW, "--quadratic-align: largest cost x read length reaches 2^26");
    }
    const bool use_lane = c->align_kernel >= 2 || (c->align_kernel == 0 && lane_fits);
    const int32_t wmin = std::max(c->set.kmer_size, (int32_t)floor((double)((float)minL * omm)) + 1);
    const bool exact = wmin == 15 && wmax == 15 && lw == 16;  // every band exactly 16 cells wide
    AlignParams P;
    P.k = c->set.kmer_size;
    P.gap_open = gap_open;
    P.gap_extend = gap_extend;
    P.min_overlap = c->set.min_overlap;
    P.one_minus_minid = omm;
    P.min_identity = c->set.min_identity;
    P.max_ignore = (float)c->set.max_ignore;
    memcpy(P.cost, cost, sizeof(P.cost));
    P.cost_bits = cost_bits;
    P.rw = rw;
    Counters *cnt = (Counters *)c->d_cnt.p;
    DevAlignment *out;
    ENSURE(c->d_aln, nd, &out);
    HIPCHK(hipMemsetAsync(&cnt->err, 0, 4, c->stream));
    HIPCHK(hipMemsetAsync(cnt->cells, 0, sizeof(cnt->cells), c->stream));
    {
        StageScope st(c, SA_STAGE_ALIGN);
        if (c->aligner == SA_ALIGNER_QUADRATIC) {
            // generateLocalAlignmentSet (BioLibs.scala:267-368): one wave per pair,
            // codes for the greedy walk in HBM, in launches of <= local_batch_bytes
            const int stripe = local_align_stripe(maxL);
            const uint32_t wpl = local_align_wpl(stripe, maxL);
            const uint64_t per_pair = (uint64_t)64 * wpl * 4;
            uint64_t chunk = std::max<uint64_t>(64, c->local_batch_bytes / per_pair);
            chunk = std::min<uint64_t>(chunk, std::max<uint64_t>(nd, 1));
            uint32_t *tb;
            int4 *lmax;
            ENSURE(c->d_ltb, chunk * 64 * (uint64_t)wpl, &tb);
            ENSURE(c->d_lmax, chunk, &lmax);
            const int32_t *dl = (const int32_t *)c->d_lead.p, *dt = (const int32_t *)c->d_trail.p;
            for (uint64_t p0 = 0; p0 < nd; p0 += chunk)
                HIPCHK(launch_local_align(AR, dl, dt, p0, std::min(chunk, nd - p0), P, stripe, wpl, tb, lmax, out,
                                          &cnt->err, cnt->cells, c->stream));
        } else if (use_lane) {
            // phase 1, then pairs grouped by phase-2 row count, then phase 2
            int32_t *p1; uint64_t *k0, *k1; uint32_t *v0, *v1; uint8_t *tmp;
            ENSURE(c->d_p1, nd, &p1);
            ENSURE(c->d_okeys, nd, &k0);
            ENSURE(c->d_okeys2, nd, &k1);
            ENSURE(c->d_ovals, nd, &v0);
            ENSURE(c->d_ovals2, nd, &v1);
            ENSURE(c->d_osort, radix_sort_temp_bytes(nd), &tmp);
            const int32_t *dl = (const int32_t *)c->d_lead.p, *dt = (const int32_t *)c->d_trail.p;
            // phase 1 two pairs per lane (packed 16-bit) when every score fits 16 bits
            int64_t cmax = 0;
            for (int x = 0; x < 16; ++x) cmax = std::max<int64_t>(cmax, P.cost[x]);
            const bool x2 = lw == 16 && exact && P.cost_bits == 8 && P.gap_open <= 0 && P.gap_extend <= 0 &&
                            -(int64_t)P.gap_open < 65536 && -(int64_t)P.gap_extend < 65536 &&
                            cmax * (int64_t)maxL + 255 < 65536;
            if (x2) {
                // row segments when the waves are few enough for the last round to matter: units of
                // 1 / nseg of a wave, ~20+ per SIMD (1,024 SIMDs), at most 8, rows >= 32 per segment
                const uint32_t ng = dovetail_p1x2_groups(nd);
                int32_t nseg = (int32_t)std::min<uint64_t>(8, (20 * 1024 + ng - 1) / ng);
                nseg = std::max(1, std::min(nseg, (int32_t)(maxL / 32)));
                if (const char *e = getenv("SA_P1_SEGS")) nseg = atoi(e);  // A/B: 0 = one-segment kernel
                if (nseg >= 1) {
                    uint32_t *tf, *st = nullptr;
                    ENSURE(c->d_p1tf, (uint64_t)ng + 1, &tf);
                    if (nseg > 1) ENSURE(c->d_p1st, dovetail_p1x2_state_words(nd), &st);
                    HIPCHK(launch_dovetail_p1x2_seg(AR, dl, dt, nd, P, p1, k0, v0, &cnt->err, cnt->cells, nseg, tf, st,
                                                    c->stream));
                } else
                    HIPCHK(launch_dovetail_p1x2(AR, dl, dt, nd, P, p1, k0, v0, &cnt->err, cnt->cells, c->stream));
            } else
                HIPCHK(launch_dovetail_p1(AR, dl, dt, nd, P, lw, exact, p1, k0, v0, &cnt->err, cnt->cells,
                                          c->stream));
            HIPCHK(radix_sort(&k0, &v0, &k1, &v1, nd, 0, 20, tmp, c->stream));
            if (c->align_kernel == 3) {  // path summaries forwarded per cell
                HIPCHK(launch_dovetail_p2(AR, dl, dt, nd, P, lw, exact, p1, v0, out, &cnt->err, c->stream));
            } else {  // 2-bit traceback codes in HBM + per-lane walk, in launches of <= 4 GiB of codes
                // two pairs per lane as in phase 1 when the argmax row also fits (u << 4 | k in 16 bits)
                const bool x2tb = x2 && maxL < 4096;
                const uint64_t per_2 = x2tb ? dovetail_tbx2_words(2, maxL) : dovetail_tb_words(2, maxL, lw);
                uint64_t chunk = std::max<uint64_t>(512, (2 * ((1ull << 30) / per_2)) & ~511ull);
                chunk = std::min<uint64_t>(chunk, (nd + 511) & ~511ull);
                uint32_t *tb;
                ENSURE(c->d_tb, x2tb ? dovetail_tbx2_words(chunk, maxL) : dovetail_tb_words(chunk, maxL, lw), &tb);
                for (uint64_t t0 = 0; t0 < nd; t0 += chunk) {
                    if (x2tb)
                        HIPCHK(launch_dovetail_p2tbx2(AR, dl, dt, nd, t0, chunk, P, p1, v0, out, &cnt->err, tb,
                                                      c->stream));
                    else
                        HIPCHK(launch_dovetail_p2tb(AR, dl, dt, nd, t0, chunk, P, lw, exact, p1, v0, out, &cnt->err,
                                                    tb, c->stream));
                }
            }
        } else
            HIPCHK(launch_dovetail(AR, (const int32_t *)c->d_lead.p, (const int32_t *)c->d_trail.p, nd, P,
                                   G, out, &cnt->err, cnt->cells, c->stream));
    }
    int32_t err = 0;
    unsigned long long cells_s[NSHARD];
    HIPCHK(hipMemcpyAsync(&err, &cnt->err, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(cells_s, cnt->cells, sizeof(cells_s), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    resolve_timing(c);
    c->stats.aligned = nd;
    c->stats.ovl_records = 0;  // (set when the records are formatted: host_results)
    c->stats.dp_cells = shard_sum(cells_s);
    if (err) {
        const char *msg = err == SA_E_NON_ACGT ? "non-ACGT base in an aligned region (HOXD MatchError)"
                        : err == SA_E_SHORT_READ ? "trail shorter than the band width (StringIndexOutOfBounds)"
                        : err == SA_E_DEGENERATE ? "no positive phase-1 cell (degenerate backtrack)"
                        : err == SA_E_HIP ? "phase-1 row-segment hand-off timed out or read inconsistent state"
                        : "alignment limit exceeded";
        return fail(c, err, msg);
    }
    c->aligned = true;
    c->host_valid = false;
    if (readback) return host_results(c);
    return SA_OK;
}

// alignments read back and the .ovl records formatted (calcOverlaps,
// Project4.scala:795-825; Overlap.print, ObjectStore.scala:127-135) for the
// last alignment, once: sa_align does it at once, after sa_device_align the
// getters / writer do it on first use (never a previous run's records)
// decimal text of v at p (Integer.toString), returns the end
static inline char *put_int(char *p, int32_t v) {
    uint32_t u = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
    if (v < 0) *p++ = '-';
    char t[12];
    int n = 0;
    do { t[n++] = (char)('0' + u % 10); u /= 10; } while (u);
    while (n) *p++ = t[--n];
    return p;
}

int host_results(sa_ctx *c) {
    if (c->host_valid) return SA_OK;
    const uint64_t nd = c->n_disp;
    {
        HostScope hs(c, SA_STAGE_READBACK);
        c->alns.resize(nd);
        if (nd) HIPCHK(hipMemcpy(c->alns.data(), c->d_aln.p, nd * sizeof(sa_alignment), hipMemcpyDeviceToHost));
    }
    HostScope hs(c, SA_STAGE_FORMAT);
    // "{OVL\nadj:N\nrds:" + lead + "," + trail + "\nscr:0\nahg:" + ahg + "\nbhg:" + bhg + "\n}" + "\n"
    // (Overlap.print, ObjectStore.scala:127-135; Project4.scala:814-818).  In chunks on up to 8
    // host threads: each chunk's exact byte count first, then every chunk formats straight into
    // its place (round 6: 7 ms for configs[0]'s 366k records on one thread)
    static const char H1[] = "{OVL\nadj:N\nrds:", H2[] = "\nscr:0\nahg:", H3[] = "\nbhg:", H4[] = "\n}\n";
    constexpr size_t FIXED = (sizeof(H1) - 1) + 1 + (sizeof(H2) - 1) + (sizeof(H3) - 1) + (sizeof(H4) - 1);
    auto ndig = [](int32_t v) {
        uint32_t u = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
        size_t n = v < 0 ? 2 : 1;
        while (u >= 10) { u /= 10; ++n; }
        return n;
    };
    auto fields = [&](const sa_alignment &a, int &ra, int &rb) {
        ra = (a.flags & SA_ALN_DUD) ? 0 : a.lead;
        rb = (a.flags & SA_ALN_DUD) ? 0 : a.trail;
    };
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const uint64_t T = std::max<uint64_t>(1, std::min<uint64_t>({8ull, (uint64_t)hw, nd / 20000 + 1}));
    std::vector<uint64_t> cbytes(T + 1, 0), crec(T, 0);
    auto chunk = [&](uint64_t t, uint64_t &a0, uint64_t &a1) { a0 = nd * t / T; a1 = nd * (t + 1) / T; };
    auto run = [&](auto f) {
        if (T == 1) { f(0); return; }
        std::vector<std::thread> th;
        for (uint64_t t = 0; t < T; ++t) th.emplace_back(f, t);
        for (auto &x : th) x.join();
    };
    run([&](uint64_t t) {
        uint64_t a0, a1, b = 0, r = 0;
        chunk(t, a0, a1);
        for (uint64_t i = a0; i < a1; ++i) {
            const sa_alignment &a = c->alns[i];
            if (!(a.flags & SA_ALN_OVL_VALID)) continue;
            int ra, rb;
            fields(a, ra, rb);
            b += FIXED + ndig(ra) + ndig(rb) + ndig(a.ahg) + ndig(a.bhg);
            ++r;
        }
        cbytes[t + 1] = b;
        crec[t] = r;
    });
    uint64_t rec = 0;
    for (uint64_t t = 0; t < T; ++t) { cbytes[t + 1] += cbytes[t]; rec += crec[t]; }
    c->ovl.resize(cbytes[T]);
    char *const base = &c->ovl[0];
    run([&](uint64_t t) {
        uint64_t a0, a1;
        chunk(t, a0, a1);
        char *p = base + cbytes[t];
        for (uint64_t i = a0; i < a1; ++i) {
            const sa_alignment &a = c->alns[i];
            if (!(a.flags & SA_ALN_OVL_VALID)) continue;
            int ra, rb;
            fields(a, ra, rb);
            memcpy(p, H1, sizeof(H1) - 1); p += sizeof(H1) - 1;
            p = put_int(p, ra);
            *p++ = ',';
            p = put_int(p, rb);
            memcpy(p, H2, sizeof(H2) - 1); p += sizeof(H2) - 1;
            p = put_int(p, a.ahg);
            memcpy(p, H3, sizeof(H3) - 1); p += sizeof(H3) - 1;
            p = put_int(p, a.bhg);
            memcpy(p, H4, sizeof(H4) - 1); p += sizeof(H4) - 1;
        }
    });
    c->stats.ovl_records = rec;
    c->host_valid = true;
    return SA_OK;
}

}  // namespace

int single_build(sa_ctx *c, bool readback) {
    (void)hipSetDevice(c->device);
    return device_build(c, readback);
}

int single_align(sa_ctx *c, bool readback) {
    (void)hipSetDevice(c->device);
    return device_align(c, readback);
}


// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

void sa_default_settings(sa_settings *s) {
    static const int32_t hoxd[16] = {91, -114, -31, -123, -114, 100, -125, -31,
                                     -31, -125, 100, -114, -123, -31, -114, 91};
    memset(s, 0, sizeof(*s));
    s->kmer_size = 12;
    s->min_overlap = 40;
    s->max_ignore = 90;
    s->gap_open = -200;
    s->gap_extend = -20;
    s->min_collisions = 7;
    s->max_collisions = 222;
    s->min_identity = 0.98f;
    s->kmer_edge = 0.4f;
    s->kmer_center = 0.4f;
    memcpy(s->cost, hoxd, sizeof(hoxd));
    s->id_mode = SA_IDS_AUTO;
}

int sa_ctx_create(const sa_settings *s, int device, sa_ctx **out) {
    if (!s || !out) return SA_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return SA_E_HIP;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SA_E_HIP;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SA_E_HIP;  // code objects are gfx950 only
    if (hipSetDevice(device) != hipSuccess) return SA_E_HIP;
    sa_ctx *c = new sa_ctx();
    c->set = *s;
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return SA_E_HIP;
    }
    *out = c;
    return SA_OK;
}

void sa_ctx_destroy(sa_ctx *c) {
    if (!c) return;
    if (c->multi) multi_destroy(c);
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    DBuf *bufs[] = {&c->d_ascii, &c->d_boff, &c->d_woff, &c->d_len, &c->d_codes, &c->d_bad, &c->d_occ_off,
                    &c->d_lbase, &c->d_lrank, &c->d_tagtab, &c->d_keys, &c->d_vals, &c->d_keys2, &c->d_vals2,
                    &c->d_sorttmp, &c->d_md, &c->d_ed, &c->d_bmdo, &c->d_bedo, &c->d_bstart, &c->d_gbid,
                    &c->d_gmds, &c->d_gede, &c->d_ogid, &c->d_bkttmp, &c->d_mdidx, &c->d_edidx, &c->d_occidx,
                    &c->d_bnst, &c->d_brank, &c->d_bhash, &c->d_bfirst, &c->d_pf, &c->d_ps, &c->d_pc, &c->d_pr,
                    &c->d_ovl, &c->d_cnt, &c->d_okeys, &c->d_ovals, &c->d_okeys2, &c->d_ovals2, &c->d_osort,
                    &c->d_lead, &c->d_trail, &c->d_count, &c->d_aln, &c->d_p1, &c->d_p1tf, &c->d_p1st, &c->d_tb, &c->d_rkey, &c->d_rkey2, &c->d_rord, &c->d_rord2, &c->d_rtmp, &c->d_gocc, &c->d_seg, &c->d_rl, &c->d_srl, &c->d_srl2, &c->d_loff, &c->d_starts, &c->d_bounds, &c->d_gcodes, &c->d_gwoff, &c->d_glen, &c->d_gbad, &c->d_psum, &c->d_pkeep, &c->d_ppos, &c->d_scan, &c->d_pstart, &c->d_biglist, &c->d_rec,
                    &c->d_srec, &c->d_bnmd, &c->d_ishead, &c->d_bnst2, &c->d_tmd, &c->d_ted, &c->d_tmdi,
                    &c->d_tedi, &c->d_xrec, &c->d_tier, &c->d_ovlrp, &c->d_meta, &c->d_items, &c->d_pq, &c->d_ocur, &c->d_lr, &c->d_bigtot, &c->d_hk0, &c->d_hk1, &c->d_hflag,
                    &c->d_hidx, &c->d_hpos, &c->d_htmp, &c->d_hist, &c->d_hovf, &c->d_hsmall,
                    &c->d_ltb, &c->d_lmax, &c->d_rreg, &c->d_rcnt, &c->d_rex,
                    &c->d_shl, &c->d_sht, &c->d_shc, &c->d_rsh, &c->d_pbound, &c->d_pbown, &c->d_trove, &c->d_prange,
                    &c->d_pioff, &c->d_pitems};
    for (DBuf *b : bufs)
        if (b->p && !b->borrowed) (void)hipFree(b->p);
    for (auto &p : c->pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->hcnt) (void)hipHostFree(c->hcnt);
    if (c->side) {
        (void)hipStreamSynchronize(c->side);
        (void)hipStreamDestroy(c->side);
    }
    for (hipEvent_t e : {c->ev_fork, c->ev_join, c->ev_fork2, c->ev_join2})
        if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *sa_last_error(const sa_ctx *c) { return c ? c->err.c_str() : "null context"; }

int sa_add_reads(sa_ctx *c, const char *bases, const uint64_t *offsets, uint32_t n) {
    if (!c || (n && (!bases || !offsets))) return SA_E_ARG;
    const uint64_t base0 = c->bases.size();
    for (uint32_t r = 0; r < n; ++r) {
        if (offsets[r + 1] < offsets[r]) return fail(c, SA_E_ARG, "offsets must be non-decreasing");
    }
    c->bases.insert(c->bases.end(), bases + offsets[0], bases + offsets[n]);
    c->boff.reserve(c->boff.size() + n);
    for (uint32_t r = 0; r < n; ++r) c->boff.push_back(base0 + (offsets[r + 1] - offsets[0]));
    c->reads_dirty = true;
    c->built = c->aligned = false;
    ++c->reads_gen;
    return SA_OK;
}

int sa_read_fasta(sa_ctx *c, const char *path) {
    if (!c || !path) return SA_E_ARG;
    std::vector<char> b;
    std::vector<uint64_t> off;
    if (read_fasta(path, b, off) != 0) return fail(c, SA_E_INPUT, std::string("Invalid Sequence File: ") + path);
    if (off.size() - 1 > 0xFFFFFFFFull) return fail(c, SA_E_OVERFLOW, "more than 2^32 - 1 reads");
    if (c->bases.empty() && c->boff.size() == 1) {  // the first reads: taken over, not copied
        c->bases.swap(b);
        c->boff.swap(off);
        c->reads_dirty = true;
        c->built = c->aligned = false;
        ++c->reads_gen;
        return SA_OK;
    }
    return sa_add_reads(c, b.data(), off.data(), (uint32_t)(off.size() - 1));
}

uint32_t sa_num_reads(const sa_ctx *c) { return c ? (uint32_t)(c->boff.size() - 1) : 0; }

int sa_get_read(const sa_ctx *c, uint32_t id, const char **seq, size_t *len) {
    if (!c || !seq || !len) return SA_E_ARG;
    const uint32_t n = (uint32_t)(c->boff.size() - 1);
    if (id < 1 || id > n) return SA_E_ARG;
    *seq = c->bases.data() + c->boff[id - 1];
    *len = (size_t)(c->boff[id] - c->boff[id - 1]);
    return SA_OK;
}

int sa_build_candidates(sa_ctx *c) {
    if (!c) return SA_E_ARG;
    if (c->multi) return multi_build(c, true, single_build);
    return single_build(c, true);
}

int sa_device_build(sa_ctx *c) {
    if (!c) return SA_E_ARG;
    if (c->multi) return multi_build(c, false, single_build);
    return single_build(c, false);
}

int sa_get_dispatch(sa_ctx *c, const int32_t **lead, const int32_t **trail, const int32_t **count, size_t *n) {
    if (!c || !n) return SA_E_ARG;
    if (!c->built) return fail(c, SA_E_STATE, "no candidates built");
    if (multi_sharded(c)) {
        int rc = multi_dispatch(c);
        if (rc) return rc;
    } else if (c->lead.size() != c->n_disp) {  // device-only build: fetch now
        c->lead.resize(c->n_disp); c->trail.resize(c->n_disp); c->count.resize(c->n_disp);
        if (c->n_disp) {
            HIPCHK(hipMemcpy(c->lead.data(), c->d_lead.p, c->n_disp * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(c->trail.data(), c->d_trail.p, c->n_disp * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(c->count.data(), c->d_count.p, c->n_disp * 4, hipMemcpyDeviceToHost));
        }
    }
    if (lead) *lead = c->lead.data();
    if (trail) *trail = c->trail.data();
    if (count) *count = c->count.data();
    *n = c->n_disp;
    return SA_OK;
}

int sa_kmer_histogram(sa_ctx *c, uint64_t *uniques, const uint64_t **size, const uint64_t **count, size_t *n) {
    if (!c || !uniques || !n) return SA_E_ARG;
    (void)hipSetDevice(c->device);
    int rc = ensure_prepared(c);
    if (rc) return rc;
    const uint64_t nk = c->n_occ;
    DevReads R = dev_reads(c);
    EmitParams E = emit_params(c);
    uint64_t *k0, *k1;
    uint32_t *flag, *idx, *pos, *small;
    uint8_t *tmp;
    unsigned long long *hist, *ovf;
    ENSURE(c->d_hk0, nk + 1, &k0);
    ENSURE(c->d_hk1, nk + 1, &k1);
    ENSURE(c->d_hflag, nk + 1, &flag);
    ENSURE(c->d_hidx, nk + 1, &idx);
    ENSURE(c->d_hpos, nk + 1, &pos);
    ENSURE(c->d_htmp, std::max(radix_sort_temp_bytes(nk), scan_temp_bytes(nk)), &tmp);
    ENSURE(c->d_hist, KMER_HIST_CAP, &hist);
    ENSURE(c->d_hovf, nk / KMER_HIST_CAP + 2, &ovf);  // at most n / CAP buckets that large
    ENSURE(c->d_hsmall, 2, &small);
    // generateKmerSet + addKmerSet (BioLibs.scala:54-61, KmerTable.scala:41-53) as
    // records, fully sorted on the mixed hash, then run lengths
    HIPCHK(launch_pack_reads(R, c->stream));
    HIPCHK(launch_kmer_emit(R, E, k0, nullptr, c->stream));
    uint32_t *nv = nullptr, *nv2 = nullptr;
    HIPCHK(radix_sort(&k0, &nv, &k1, &nv2, nk, 32, 64, tmp, c->stream));
    HIPCHK(launch_kmer_hist(k0, nk, flag, idx, pos, small, tmp, hist, ovf, small + 1, c->stream));
    uint32_t hs[2] = {0, 0};
    std::vector<unsigned long long> h(KMER_HIST_CAP);
    HIPCHK(hipMemcpyAsync(hs, small, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(h.data(), hist, KMER_HIST_CAP * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    std::vector<unsigned long long> big(hs[1]);
    if (hs[1]) HIPCHK(hipMemcpy(big.data(), ovf, (size_t)hs[1] * 8, hipMemcpyDeviceToHost));
    std::sort(big.begin(), big.end());
    c->hsize.clear();
    c->hcount.clear();
    for (uint32_t q = 1; q < KMER_HIST_CAP; ++q)
        if (h[q]) { c->hsize.push_back(q); c->hcount.push_back(h[q]); }
    for (size_t q = 0; q < big.size(); ++q) {
        if (!c->hsize.empty() && c->hsize.back() == big[q]) ++c->hcount.back();
        else { c->hsize.push_back(big[q]); c->hcount.push_back(1); }
    }
    *uniques = hs[0];
    if (size) *size = c->hsize.data();
    if (count) *count = c->hcount.data();
    *n = c->hsize.size();
    return SA_OK;
}

int sa_get_pairs(sa_ctx *c, const int32_t **fst, const int32_t **snd, const int32_t **count, size_t *n) {
    if (!c || !n) return SA_E_ARG;
    if (!c->built || !c->keep_pairs) return fail(c, SA_E_STATE, "pairs not kept (SA_OPT_KEEP_PAIRS)");
    if (fst) *fst = c->pfst.data();
    if (snd) *snd = c->psnd.data();
    if (count) *count = c->pcnt.data();
    *n = c->pfst.size();
    return SA_OK;
}

int sa_align(sa_ctx *c) {
    if (!c) return SA_E_ARG;
    if (c->multi) return multi_align(c, true, single_align);
    return single_align(c, true);
}

int sa_device_align(sa_ctx *c) {
    if (!c) return SA_E_ARG;
    if (c->multi) return multi_align(c, false, single_align);
    return single_align(c, false);
}

int sa_get_alignments(sa_ctx *c, const sa_alignment **out, size_t *n) {
    if (!c || !out || !n) return SA_E_ARG;
    if (!c->aligned) return fail(c, SA_E_STATE, "no alignments");
    const int rc = multi_sharded(c) ? multi_host_results(c) : host_results(c);
    if (rc) return rc;
    *out = c->alns.data();
    *n = c->alns.size();
    return SA_OK;
}

int sa_get_ovl(sa_ctx *c, const char **text, size_t *len) {
    if (!c || !text || !len) return SA_E_ARG;
    if (!c->aligned) return fail(c, SA_E_STATE, "no alignments");
    const int rc = multi_sharded(c) ? multi_host_results(c) : host_results(c);
    if (rc) return rc;
    *text = c->ovl.data();
    *len = c->ovl.size();
    return SA_OK;
}

int sa_write_ovl(sa_ctx *c, const char *path) {
    if (!c) return SA_E_ARG;
    const std::string *text = &c->ovl;
    std::string all;
    if (multi_rank_mode(c)) {
        // collective: rank 0 writes every rank's records.  Every rank takes part
        // in the status exchange whatever its own state, so one rank that has
        // not aligned fails them all instead of leaving the others blocked in
        // the gather; records after sa_device_align are formatted first
        int rc = c->aligned ? multi_host_results(c) : SA_E_STATE;
        const int rc_all = multi_all_ok(c, rc == SA_OK);
        if (rc_all) return rc_all;
        if (rc) return fail(c, rc, "no alignments");
        rc = multi_gather_ovl(c, all);
        if (rc) return rc;
        if (multi_rank(c) != 0) return SA_OK;
        text = &all;
    } else {
        if (!c->aligned) return fail(c, SA_E_STATE, "no alignments");
        const int rc = multi_sharded(c) ? multi_host_results(c) : host_results(c);
        if (rc) return rc;
    }
    HostScope hs(c, SA_STAGE_WRITE);
    FILE *f = path ? fopen(path, "wb") : stdout;  // the file is deleted and recreated (Project4.scala:797-805)
    if (!f) return fail(c, SA_E_INPUT, std::string("cannot write ") + path);
    const size_t w = fwrite(text->data(), 1, text->size(), f);
    if (path) fclose(f); else fflush(f);
    return w == text->size() ? SA_OK : fail(c, SA_E_INPUT, "short write");
}

// AMOS message file: what toAmos_new puts in the bank (Rakefile.rb:174) as
// {RED} messages, then the .ovl records bank-transact -m loads (Rakefile.rb:180-184)
int sa_write_afg(sa_ctx *c, const char *path, const char *const *eids, int quality) {
    if (!c || !path) return SA_E_ARG;
    if (quality < 0 || quality > 60) return fail(c, SA_E_ARG, "afg quality must be 0..60");
    if (multi_rank_mode(c)) return fail(c, SA_E_ARG, "sa_write_afg: one-process contexts only");
    if (!c->aligned) return fail(c, SA_E_STATE, "no alignments");
    const int rc = multi_sharded(c) ? multi_host_results(c) : host_results(c);
    if (rc) return rc;
    FILE *f = fopen(path, "wb");
    if (!f) return fail(c, SA_E_INPUT, std::string("cannot write ") + path);
    const uint32_t n = (uint32_t)(c->boff.size() - 1);
    // an eid is one message-field token: no whitespace, no ':' / '{' / '}'
    for (uint32_t id = 1; eids && id <= n; ++id)
        for (const char *e = eids[id - 1]; e && *e; ++e)
            if (isspace((unsigned char)*e) || *e == ':' || *e == '{' || *e == '}')
                return fail(c, SA_E_ARG, "afg eid of read " + std::to_string(id) + " is not one token");
    constexpr size_t LINE = 60;  // sequence / quality line width
    std::string m;
    bool ok = true;
    for (uint32_t id = 1; id <= n && ok; ++id) {
        const char *seq = c->bases.data() + c->boff[id - 1];
        const size_t len = (size_t)(c->boff[id] - c->boff[id - 1]);
        m.clear();
        m += "{RED\niid:" + std::to_string(id) + "\neid:";
        if (eids && eids[id - 1] && *eids[id - 1]) m += eids[id - 1];
        else m += std::to_string(id);
        m += "\nseq:\n";
        for (size_t p = 0; p < len; p += LINE) {
            m.append(seq + p, std::min(LINE, len - p));
            m += '\n';
        }
        m += ".\nqlt:\n";
        for (size_t p = 0; p < len; p += LINE) {
            m.append(std::min(LINE, len - p), (char)('0' + quality));
            m += '\n';
        }
        // clr only: the reference bank's RED records hold the clear range (0, len)
        // and leave every other range unset (RED.0.0.fix, tests/golden/c_ruddii_bank_red.npz)
        m += ".\nclr:0," + std::to_string(len) + "\n}\n";
        ok = fwrite(m.data(), 1, m.size(), f) == m.size();
    }
    if (ok) ok = fwrite(c->ovl.data(), 1, c->ovl.size(), f) == c->ovl.size();
    ok = (fclose(f) == 0) && ok;
    return ok ? SA_OK : fail(c, SA_E_INPUT, "short write");
}

int sa_set_option(sa_ctx *c, int option, int64_t value) {
    if (!c) return SA_E_ARG;
    switch (option) {
    case SA_OPT_KEEP_PAIRS: c->keep_pairs = value != 0; break;
    case SA_OPT_TIMING: c->timing = value != 0; break;
    case SA_OPT_ALIGN_KERNEL:
        if (value < 0 || value > 3) return fail(c, SA_E_ARG, "SA_OPT_ALIGN_KERNEL must be 0..3");
        c->align_kernel = (int)value;
        break;
    case SA_OPT_ALIGNER:
        if (value != SA_ALIGNER_LINEAR && value != SA_ALIGNER_QUADRATIC)
            return fail(c, SA_E_ARG, "SA_OPT_ALIGNER must be SA_ALIGNER_LINEAR or SA_ALIGNER_QUADRATIC");
        c->aligner = (int)value;
        c->aligned = false;
        break;
    case SA_OPT_LOCAL_BATCH_MB:
        if (value < 1) return fail(c, SA_E_ARG, "SA_OPT_LOCAL_BATCH_MB must be >= 1");
        c->local_batch_bytes = (uint64_t)value << 20;
        break;
    case SA_OPT_LAUNCH_SLICE:
        if (value < 0 || value > 0x7FFFFFFF) return fail(c, SA_E_ARG, "SA_OPT_LAUNCH_SLICE must be 0..2^31-1");
        c->launch_slice = (uint32_t)value;
        break;
    case SA_OPT_FIRST_PASS:
        if (value < 0 || value > 2) return fail(c, SA_E_ARG, "SA_OPT_FIRST_PASS must be 0..2");
        c->first_pass = (int)value;
        break;
    case SA_OPT_SERIAL_SHARDS:
    case SA_OPT_PASS_BUDGET_MB:
    case SA_OPT_LEAN_MEMORY:
        if (!c->multi) return fail(c, SA_E_ARG, "this option needs a sharded context");
        if (value < 0) return fail(c, SA_E_ARG, "option value must be >= 0");
        return multi_set_option(c, option, value);
    default: return fail(c, SA_E_ARG, "unknown option");
    }
    return c->multi ? multi_set_option(c, option, value) : SA_OK;
}

int sa_get_stats(const sa_ctx *c, sa_stats *out) {
    if (!c || !out) return SA_E_ARG;
    *out = c->stats;
    return SA_OK;
}

int sa_get_stage_times(const sa_ctx *c, double *ms, uint64_t *launches, int n) {
    if (!c) return SA_E_ARG;
    double m[SA_NUM_STAGES];
    uint64_t k[SA_NUM_STAGES];
    for (int i = 0; i < SA_NUM_STAGES; ++i) { m[i] = c->stage_ms[i]; k[i] = c->stage_n[i]; }
    if (c->multi) multi_stage_times(c, m, k);
    for (int i = 0; i < n && i < SA_NUM_STAGES; ++i) {
        if (ms) ms[i] = m[i];
        if (launches) launches[i] = k[i];
    }
    return SA_OK;
}

int sa_reset_stage_times(sa_ctx *c) {
    if (!c) return SA_E_ARG;
    for (int i = 0; i < SA_NUM_STAGES; ++i) { c->stage_ms[i] = 0; c->stage_n[i] = 0; }
    if (c->multi) multi_reset_stage_times(c);
    return SA_OK;
}

int sa_sync(sa_ctx *c) {
    if (!c) return SA_E_ARG;
    (void)hipSetDevice(c->device);
    HIPCHK(hipStreamSynchronize(c->stream));
    return c->multi ? multi_sync(c) : SA_OK;
}

uint64_t sa_exchanged_bytes(const sa_ctx *c) { return c ? multi_exchanged_bytes(c) : 0; }

// ---------------------------------------------------------------------------
// sharded hash stage; the exchanges are the caller's
// ---------------------------------------------------------------------------
int sa_dist_init(sa_ctx *c, int rank, int nranks, const uint32_t *starts, const int32_t *lengths) {
    if (!c || !starts || !lengths) return SA_E_ARG;
    if (c->multi) return fail(c, SA_E_STATE, "a sharded context exchanges internally (sa_dist_* are per-shard calls)");
    if (nranks < 1 || nranks > 256 || (nranks & (nranks - 1)) || rank < 0 || rank >= nranks)
        return fail(c, SA_E_ARG, "nranks must be a power of two <= 256 and 0 <= rank < nranks");
    if (c->set.id_mode == SA_IDS_STRICT) return fail(c, SA_E_ARG, "the sharded path runs in wide-id mode only");
    const uint32_t N = starts[nranks];
    for (int r = 0; r < nranks; ++r)
        if (starts[r + 1] < starts[r]) return fail(c, SA_E_ARG, "rank starts must be non-decreasing");
    const uint32_t nl = (uint32_t)(c->boff.size() - 1);
    if (starts[0] != 0 || starts[rank + 1] - starts[rank] != nl)
        return fail(c, SA_E_ARG, "this rank's read count does not match starts[rank+1] - starts[rank]");
    for (uint32_t i = 0; i < nl; ++i)
        if ((int64_t)(c->boff[i + 1] - c->boff[i]) != (int64_t)lengths[starts[rank] + i])
            return fail(c, SA_E_ARG, "lengths[] disagrees with this rank's reads");
    const int k = c->set.kmer_size;
    c->dist = true;
    c->dist_reads = false;
    c->rank = rank;
    c->nranks = nranks;
    c->log_ranks = 0;
    while ((1 << c->log_ranks) < nranks) ++c->log_ranks;
    c->dstarts.assign(starts, starts + nranks + 1);
    c->dlen.assign(lengths, lengths + N);
    c->gocc.assign((size_t)N + 1, 0);
    c->gmaxL = 0;
    c->gminL = N ? INT32_MAX : 0;
    int32_t uni = -1;
    bool uniform = N > 0;
    for (uint32_t i = 0; i < N; ++i) {
        const int32_t L = lengths[i];
        if (L < 0) return fail(c, SA_E_ARG, "negative read length");
        c->gocc[i + 1] = c->gocc[i] + (uint64_t)(L - k + 1 > 0 ? L - k + 1 : 0);
        c->gmaxL = std::max(c->gmaxL, L);
        c->gminL = std::min(c->gminL, L);
        if (uni < 0) uni = L;
        if (L != uni || L < k) uniform = false;
    }
    // records carry occurrence indices local to their source rank
    for (int r = 0; r < nranks; ++r)
        if (c->gocc[starts[r + 1]] - c->gocc[starts[r]] >= 0xFFFFFFF0ull)
            return fail(c, SA_E_OVERFLOW, "more than 2^32 k-mers on one rank");
    c->gnpr = uniform ? (uint32_t)(uni - k + 1) : 0;
    c->dist_rho_ok = false;  // (a new read set: its partials / bound ratio is unknown)
    c->reads_dirty = true;  // loc tables come from all lengths now
    c->built = c->aligned = false;
    (void)hipSetDevice(c->device);
    uint64_t *gocc;
    uint32_t *st;
    int32_t *glen;
    ENSURE(c->d_gocc, (size_t)N + 1, &gocc);
    ENSURE(c->d_starts, (size_t)nranks + 1, &st);
    ENSURE(c->d_glen, (size_t)N + 1, &glen);
    HIPCHK(hipMemcpy(gocc, c->gocc.data(), ((size_t)N + 1) * 8, hipMemcpyHostToDevice));
    if (N) HIPCHK(hipMemcpy(glen, lengths, (size_t)N * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(st, c->dstarts.data(), ((size_t)nranks + 1) * 4, hipMemcpyHostToDevice));
    return SA_OK;
}

int sa_dist_local_kmers(sa_ctx *c, uint64_t *n) {
    if (!c || !n) return SA_E_ARG;
    if (!c->dist) return fail(c, SA_E_STATE, "sa_dist_init first");
    (void)hipSetDevice(c->device);
    int rc = ensure_prepared(c);
    if (rc) return rc;
    *n = c->n_occ;
    return SA_OK;
}

int sa_dist_emit(sa_ctx *c, void *send_recs, uint64_t *counts) {
    if (!c || !counts) return SA_E_ARG;
    if (!c->dist) return fail(c, SA_E_STATE, "sa_dist_init first");
    (void)hipSetDevice(c->device);
    int rc = ensure_prepared(c);
    if (rc) return rc;
    c->built = c->aligned = false;
    const uint64_t n = c->n_occ;
    if (n && !send_recs) return SA_E_ARG;
    DevReads R = dev_reads(c);
    EmitParams E = emit_params(c);
    uint64_t *keys, *keys2; uint8_t *stmp;
    ENSURE(c->d_keys, n, &keys);
    ENSURE(c->d_sorttmp, std::max(radix_sort_temp_bytes(n), buckets_temp_bytes(n)), &stmp);
    // reads of <= 1,024 bases: packing and emission in one kernel, as on one device
    const bool fused = c->maxL <= 1024;
    if (!fused) {
        StageScope st(c, SA_STAGE_PACK);
        HIPCHK(launch_pack_reads(R, c->stream));
    }
    KeyGen kg{};
    const bool use_kgen = fused && make_keygen(c, E, n, kg);
    {
        StageScope st(c, SA_STAGE_EMIT);
        if (use_kgen && c->log_ranks > 0 && hist_in_pack()) {  // + the owner pass's tile histogram
            E.hist = (uint32_t *)stmp;
            E.hist_shift = kg.hist_shift = 64 - c->log_ranks;
            HIPCHK(launch_pack_emit_hist(R, E, n, c->stream));
        } else if (fused) HIPCHK(launch_pack_emit(R, E, use_kgen ? nullptr : keys, c->stream));
        else HIPCHK(launch_kmer_emit(R, E, keys, nullptr, c->stream));
    }
    // owner = top log2(P) bits of the mixed hash: one stable radix pass groups
    // the 8-byte records by owner and keeps them in occurrence order within each
    {
        StageScope st(c, SA_STAGE_SORT);
        if (use_kgen) {  // generated straight into the send buffer
            uint64_t *out = (uint64_t *)send_recs;
            HIPCHK(radix_sort_gen(kg, &out, &keys, n, 64 - c->log_ranks, 64, stmp, c->stream));
            if (out != (uint64_t *)send_recs && n)
                HIPCHK(hipMemcpyAsync(send_recs, out, n * 8, hipMemcpyDeviceToDevice, c->stream));
        } else {
            keys2 = (uint64_t *)send_recs;
            uint32_t *nv = nullptr, *nv2 = nullptr;
            if (c->log_ranks > 0)
                HIPCHK(radix_sort(&keys, &nv, &keys2, &nv2, n, 64 - c->log_ranks, 64, stmp, c->stream));
            if (keys != (uint64_t *)send_recs && n)
                HIPCHK(hipMemcpyAsync(send_recs, keys, n * 8, hipMemcpyDeviceToDevice, c->stream));
        }
    }
    uint64_t *bounds;
    ENSURE(c->d_bounds, (size_t)c->nranks + 1, &bounds);
    std::vector<uint64_t> b((size_t)c->nranks + 1, 0);
    if (n) {
        HIPCHK(launch_owner_bounds((const uint64_t *)send_recs, n, 64 - c->log_ranks, (uint32_t)c->nranks, bounds,
                                   c->stream));
        HIPCHK(hipMemcpyAsync(b.data(), bounds, b.size() * 8, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    b[c->nranks] = n;
    for (int o = 0; o < c->nranks; ++o) counts[o] = b[o + 1] - b[o];
    c->stats = sa_stats{};
    c->stats.kmers = n;
    c->stats.id_mode = SA_IDS_WIDE;
    return SA_OK;
}

extern "C++" {  // (host helpers of the pass functions below: C++ linkage)
// Owner r's leads in pass `pass` of npass (lead-range passes): [s + len * pass / npass,
// s + len * (pass + 1) / npass) of its reads [s, s + len).  Every rank derives the same
// ranges from the same starts, so the partials of a pass meet at their owners complete.
static void pass_range(const sa_ctx *c, int r, uint32_t pass, uint32_t npass, uint32_t &a, uint32_t &b) {
    const uint32_t s = c->dstarts[r];
    const uint64_t len = c->dstarts[r + 1] - s;
    a = s + (uint32_t)(len * pass / npass);
    b = s + (uint32_t)(len * (pass + 1) / npass);
}

// the partial bounds prefix-summed on the host: per read up to 2^20 reads, else per block
// of 64 reads (round 6: the per-read bounds of configs[3]'s 10M reads -- 80 MB read back and
// summed on every shard -- cost 28 ms per shard and build)
static int ensure_pbcum(sa_ctx *c) {
    if (!c->pbcum.empty()) return SA_OK;
    const uint32_t N = (uint32_t)c->dlen.size();
    c->pb_gran = N <= (1u << 20) ? 1 : 64;
    const size_t nb = ((size_t)N + c->pb_gran - 1) / c->pb_gran;
    std::vector<uint64_t> b(nb);
    const uint64_t *src = (const uint64_t *)c->d_pbound.p + (c->pb_gran == 1 ? 0 : (size_t)N + 1);
    if (nb) HIPCHK(hipMemcpy(b.data(), src, nb * 8, hipMemcpyDeviceToHost));
    c->pbcum.assign(nb + 1, 0);
    for (size_t i = 0; i < nb; ++i) c->pbcum[i + 1] = c->pbcum[i] + b[i];
    return SA_OK;
}

// an upper bound of the partials of leads [a, b): the bounds of the blocks of pb_gran reads
// it touches (exact per read)
static uint64_t bound_sum(const sa_ctx *c, uint32_t a, uint32_t b) {
    if (a >= b) return 0;
    const size_t g = c->pb_gran;
    return c->pbcum[((size_t)b + g - 1) / g] - c->pbcum[a / g];
}

// grow a device buffer keeping its first `keep` elements (the reduce passes append)
template <class T>
int ensure_keep(sa_ctx *c, DBuf &b, size_t count, size_t keep, T **out) {
    const size_t need = std::max<size_t>(count, 1) * sizeof(T);
    if (b.bytes < need) {
        void *p = nullptr;
        const size_t alloc = need + need / 4;
        hipError_t e = hipMalloc(&p, alloc);
        if (e != hipSuccess) return fail(c, SA_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        if (keep && b.p) HIPCHK(hipMemcpyAsync(p, b.p, keep * sizeof(T), hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (b.p && !b.borrowed) (void)hipFree(b.p);
        b.p = p;
        b.bytes = alloc;
        b.borrowed = false;
    }
    *out = (T *)b.p;
    return SA_OK;
}

}  // extern "C++"

int sa_dist_buckets(sa_ctx *c, void *recv_recs, const uint64_t *recv_counts, uint64_t *bound) {
    if (!c || !recv_counts) return SA_E_ARG;
    if (!c->dist) return fail(c, SA_E_STATE, "sa_dist_init first");
    c->dist_bkt = false;
    c->pbcum.clear();
    const int P = c->nranks;
    // seg[s] = first received record of source s; seg[P + 1 + s] = the global
    // occurrence index of source s's first k-mer (its records carry local ones)
    std::vector<uint64_t> seg(2 * (size_t)P + 1, 0);
    for (int s = 0; s < P; ++s) {
        seg[s + 1] = seg[s] + recv_counts[s];
        seg[P + 1 + s] = c->gocc[c->dstarts[s]];
    }
    const uint64_t n = seg[P];
    if (n && !recv_recs) return SA_E_ARG;
    (void)hipSetDevice(c->device);
    int rc = ensure_prepared(c);
    if (rc) return rc;
    const uint32_t N = (uint32_t)c->dlen.size();
    if (n >= 0xFFFFFFF0ull) return fail(c, SA_E_OVERFLOW, "more than 2^32 - 16 k-mers received on one rank");
    Counters *cnt;
    ENSURE(c->d_cnt, 1, &cnt);
    HIPCHK(hipMemsetAsync(cnt, 0, sizeof(Counters), c->stream));  // (the bucket and pair stages rely on it)
    // received records are in global occurrence order (sources in rank order,
    // each in occurrence order): local index i <-> i-th owned occurrence
    uint2 *rl; uint32_t *vals, *vals2; uint64_t *loff, *keys2, *dseg; uint8_t *stmp;
    ENSURE(c->d_seg, seg.size(), &dseg);
    HIPCHK(hipMemcpyAsync(dseg, seg.data(), seg.size() * 8, hipMemcpyHostToDevice, c->stream));
    // reads and loc ranks fit 4 bytes (e.g. 800k global reads of 500 bp: 20 + 9
    // bits): the occurrence table is packed, 12-byte records in the partition
    // sort, written straight into the sort's value buffer (else {read, loc rank}
    // pairs, 16-byte records)
    // ... or, when the global ids do not fit but every source's reads do, source-relative
    // (read - the source's first read, the source in the key's top bits: RecvGen::src_shift;
    // configs[3]'s 10M reads: 16-byte records through the sort otherwise -- the sort 31 ms per
    // shard at its real density, profiles/r06/big/c3real)
    static const bool fuse_env = !getenv("SA_RECV_FUSED") || atoi(getenv("SA_RECV_FUSED")) != 0;
    // The fused pass counts digits on the raw received keys but ranks the relabelled ones
    // (low word = local index, top bits the source when source-relative): the two agree only
    // while the first pass's digit lies between them, i.e. its shift 64 - log_ranks - PB >= 32
    // (PB up to 23: log_ranks <= 9)
    const bool fuse_ok = fuse_env && n > 0 && 64 - c->log_ranks - part_bits(n) >= 32;
    uint32_t max_src = 0;
    for (int s = 0; s < P; ++s) max_src = std::max(max_src, c->dstarts[s + 1] - c->dstarts[s]);
    const bool glob_fit = bits_for(N ? N - 1 : 0) + c->lb <= 32;
    // (SA_SRC_REL = 1 / 0: source-relative whenever it fits / never -- A/B and the GPU tests of the mode at
    // small sizes)
    static const int src_env = getenv("SA_SRC_REL") ? atoi(getenv("SA_SRC_REL")) : -1;
    const bool src_rel = (src_env == 1 || (src_env < 0 && !glob_fit)) && fuse_ok && c->log_ranks > 0 &&
                         64 - c->log_ranks - 8 * ((part_bits(n) + 7) / 8) >= 32 &&
                         bits_for(max_src ? max_src - 1 : 0) + c->lb <= 32;
    const bool packed = glob_fit || src_rel;
    c->dist_src_shift = src_rel ? 64 - c->log_ranks : 0;
    rl = nullptr;
    if (!packed) ENSURE(c->d_rl, n, &rl);
    ENSURE(c->d_loff, (size_t)N + 1, &loff);
    ENSURE(c->d_vals, n, &vals);
    uint32_t *pv = packed ? vals : nullptr;
    ENSURE(c->d_vals2, n, &vals2);
    ENSURE(c->d_keys2, n, &keys2);
    ENSURE(c->d_sorttmp, std::max(radix_sort_temp_bytes(n), buckets_temp_bytes(n)), &stmp);
    uint64_t *keys = (uint64_t *)recv_recs;
    // the read id and loc rank of every received occurrence, its record's low
    // word relabelled to its local index (record i of this rank), and the local
    // read offsets: with a packed occurrence table, inside the partition sort's
    // first pass (RecvGen: the received records are read once, not rewritten
    // first -- 8 serial shards of the bench shape, emit + sort per shard
    // profiles/r05/sharded; SA_RECV_FUSED=0: the separate pass, A/B runs)
    const bool fused = fuse_ok && packed;
    RecvGen RG{};
    if (fused) {
        RG.seg = dseg; RG.P = (uint32_t)P; RG.starts = (const uint32_t *)c->d_starts.p;
        RG.occ_off = (const uint64_t *)c->d_gocc.p; RG.npr = c->gnpr;
        RG.npr_magic = c->gnpr >= 2 ? ~0ull / c->gnpr + 1 : 0ull;
        RG.len = (const int32_t *)c->d_glen.p; RG.lbase = (const uint32_t *)c->d_lbase.p;
        RG.lrank = (const uint32_t *)c->d_lrank.p; RG.k = c->set.kmer_size; RG.lb = c->lb;
        RG.loff = loff; RG.n_reads = N;
        PartArgs sc{};  // (the uniform-length loc-rank identity, as the bucket build checks it)
        set_part_shortcuts(c, sc, c->gnpr);
        RG.lr_ident = sc.lr_ident;
        RG.src_shift = c->dist_src_shift;
    } else {
        StageScope st(c, SA_STAGE_EMIT);
        HIPCHK(launch_prepare_received(keys, n, dseg, (uint32_t)P, (const uint32_t *)c->d_starts.p,
                                       (const uint64_t *)c->d_gocc.p, c->gnpr,
                                       (const int32_t *)c->d_glen.p, (const uint32_t *)c->d_lbase.p,
                                       (const uint32_t *)c->d_lrank.p, c->set.kmer_size, packed ? nullptr : rl, pv,
                                       c->lb, loff, c->stream));
        HIPCHK(launch_local_offsets(packed ? nullptr : rl, pv, c->lb, n, N, loff, c->stream));
    }
    PartArgs PA{};
    unsigned long long big_buckets = 0;
    // phase 1: no readback between the bucket build and the bound kernel, which
    // exits at once when a partition still needs the global path (phase 2 below)
    rc = bucket_stage(c, keys, keys2, vals, vals2, n, loff, N, 0, packed ? nullptr : rl, nullptr, false, stmp, cnt,
                      PA, big_buckets, c->log_ranks, 1, pv, nullptr, fused ? &RG : nullptr, true);
    if (rc) return rc;
    PairIn PI{};
    PI.rec = PA.rec; PI.xrec = PA.xrec; PI.lst = PA.lst;
    // per-read upper bounds of the partials (the pass plan), per lead owner on the host
    uint64_t *pb; unsigned long long *pown;
    ENSURE(c->d_pbound, (size_t)N + 1 + ((size_t)N + 63) / 64, &pb);  // per read, then per 64 reads
    ENSURE(c->d_pbown, (size_t)P + 1, &pown);
    const uint32_t *dst = (const uint32_t *)c->d_starts.p;
    HIPCHK(launch_read_bound(loff, N, PI, dst, (uint32_t)P, pb, pown, c->stream, &cnt->big_n));
    Counters *hp;
    if (int rc_p = pinned_counters(c, &hp)) return rc_p;
    // (the owner bounds ride in the pinned counter copy's bound_own: one DMA, no
    // pageable staging)
    HIPCHK(hipMemcpyAsync(cnt->bound_own, pown, ((size_t)P + 1) * 8, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(hp, cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->pbown.assign(hp->bound_own, hp->bound_own + P + 1);
    const unsigned long long lds_buckets = shard_sum(hp->bkt_counts);
    if (hp->big_n) {  // partitions above 4,096 records (high-copy repeats): the global path, then the bounds
        rc = bucket_stage(c, keys, keys2, vals, vals2, n, loff, N, 0, packed ? nullptr : rl, nullptr, false, stmp,
                          cnt, PA, big_buckets, c->log_ranks, 2, pv);
        if (rc) return rc;
        PI.xrec = PA.xrec;
        HIPCHK(launch_read_bound(loff, N, PI, dst, (uint32_t)P, pb, pown, c->stream));
        HIPCHK(hipMemcpyAsync(hp->bound_own, pown, ((size_t)P + 1) * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c->pbown.assign(hp->bound_own, hp->bound_own + P + 1);
    }
    resolve_timing(c);
    c->dist_in = PI;
    c->dist_recv = n;
    c->dist_bkt = true;
    c->dist_npass = 1;
    c->stats.buckets = lds_buckets + big_buckets;
    c->stats.role_pairs = 0;
    c->stats.pairs = 0;
    c->stats.dispatched = 0;
    if (bound) *bound = c->pbown[P];
    return SA_OK;
}

int sa_dist_plan(sa_ctx *c, uint64_t budget, uint32_t *npass) {
    if (!c || !npass) return SA_E_ARG;
    if (!c->dist_bkt) return fail(c, SA_E_STATE, "sa_dist_buckets first");
    const int P = c->nranks;
    const uint64_t total = c->pbown[P];
    budget = std::max<uint64_t>(budget, 1);
    if (total <= budget) {
        c->dist_npass = *npass = 1;
        return SA_OK;
    }
    (void)hipSetDevice(c->device);
    if (int rc = ensure_pbcum(c)) return rc;
    uint64_t maxlen = 1;
    for (int r = 0; r < P; ++r) maxlen = std::max<uint64_t>(maxlen, c->dstarts[r + 1] - c->dstarts[r]);
    // the largest pass of an np-pass plan on this rank (every owner's range of the pass)
    auto worst = [&](uint64_t np) {
        uint64_t w = 0;
        for (uint64_t p = 0; p < np; ++p) {
            uint64_t t = 0;
            for (int r = 0; r < P; ++r) {
                uint32_t a, b;
                pass_range(c, r, (uint32_t)p, (uint32_t)np, a, b);
                t += bound_sum(c, a, b);
            }
            w = std::max(w, t);
        }
        return w;
    };
    uint64_t np = std::min<uint64_t>(maxlen, (total + budget - 1) / budget);
    while (np < maxlen && worst(np) > budget) np = std::min<uint64_t>(maxlen, np + std::max<uint64_t>(1, np / 8));
    if (np > 0xFFFFFFFull) return fail(c, SA_E_OVERFLOW, "lead-range pass plan: too many passes");
    c->dist_npass = *npass = (uint32_t)np;
    return SA_OK;
}

int sa_dist_count_pass(sa_ctx *c, uint32_t pass, uint32_t npass, uint64_t *counts) {
    if (!c || !counts || npass == 0 || pass >= npass) return SA_E_ARG;
    if (!c->dist_bkt) return fail(c, SA_E_STATE, "sa_dist_buckets first");
    (void)hipSetDevice(c->device);
    const int P = c->nranks;
    const uint32_t N = (uint32_t)c->dlen.size();
    const uint64_t n = c->dist_recv;
    Counters *cnt;
    ENSURE(c->d_cnt, 1, &cnt);
    const uint64_t *loff = (const uint64_t *)c->d_loff.p;
    const uint32_t *dst = (const uint32_t *)c->d_starts.p;
    // Every global read has ~1/P of its occurrences here (~60 of a 500 bp read
    // at P = 8): one wave per ~PMW_TARGET local occurrences (a few consecutive
    // reads), every distinct partial kept (count >= 1: the filter needs the
    // global sums), written straight into the regions of the rank owning its
    // lead -- the send buffers are then one copy of the regions, owner-major.
    // (round 4, 8 serial virtual shards of the bench shape: one wave per read
    // counted in 2.55 ms per step against 1.55 for multi-read items -- a read's
    // ~60 local occurrences do not pay for a wave's table setup; and partials
    // sorted by owner after the count cost an order stage of 0.3 ms more)
    // Items are sized to the partials they will hold when the last build of these reads
    // says how dense they are: ~96 expected partials per item, half the wave table's fill
    // limit (round 6: at configs[3]'s real density a local occurrence yields ~1.5 partials,
    // so 128-occurrence items overflowed the 192-partner table and went to the recount
    // tiers -- 37 ms of a shard's 72 ms of pair counting, profiles/r06/big/c3real; at the
    // bench shape, 0.33 per occurrence, the target stays 128)
    // ... and at most 256 occurrences (bench shape, 8 serial shards, same box, 2 rounds: pairs
    // 1.20-1.27 ms per shard at 128, 1.04 at 256, 1.05 at 384: fewer table set-ups and claims;
    // profiles/r06/ab/ab_pmw_cap.txt; SA_PMW_CAP for A/B).  The first build, density unknown,
    // keeps PMW_TARGET.
    static const uint32_t tcap = getenv("SA_PMW_CAP") ? (uint32_t)atoi(getenv("SA_PMW_CAP")) : 2 * PMW_TARGET;
    uint32_t target = PMW_TARGET;
    if (c->dist_rho_ok && n) {
        const double per_occ = c->dist_rho * (double)c->pbown[P] / (double)n;
        if (per_occ > 0.0) target = (uint32_t)std::min<double>(tcap, std::max(16.0, 96.0 / per_occ));
    }
    uint32_t n_multi = 0;
    uint32_t *istart, *iend = nullptr, *iown = nullptr;
    uint64_t own_max = 0;  // the largest owner's bound of this pass's partials
    if (npass == 1) {  // every read: items over all local occurrences, no readback
        n_multi = (uint32_t)((n + target - 1) / target) + 1;
        ENSURE(c->d_items, 2 * ((size_t)n_multi + 1), &istart);
        HIPCHK(launch_pc_items(loff, N, target, n_multi, istart, c->stream));
        iown = istart + n_multi + 1;
        for (int r = 0; r < P; ++r) own_max = std::max<uint64_t>(own_max, c->pbown[r]);
    } else {  // this pass's lead range of every owner
        std::vector<uint32_t> rg(2 * (size_t)P);
        const bool cum = !c->pbcum.empty();
        for (int r = 0; r < P; ++r) {
            pass_range(c, r, pass, npass, rg[2 * r], rg[2 * r + 1]);
            own_max = std::max<uint64_t>(own_max, cum ? bound_sum(c, rg[2 * r], rg[2 * r + 1]) : c->pbown[r]);
        }
        uint32_t *drg, *ioff;
        ENSURE(c->d_prange, rg.size(), &drg);
        ENSURE(c->d_pioff, (size_t)P + 1, &ioff);
        HIPCHK(hipMemcpyAsync(drg, rg.data(), rg.size() * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(launch_pass_items_count(loff, drg, (uint32_t)P, target, ioff, c->stream));
        HIPCHK(hipMemcpyAsync(&n_multi, ioff + P, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        ENSURE(c->d_pitems, 3 * ((size_t)n_multi + 1), &istart);
        iend = istart + n_multi + 1;
        iown = istart + 2 * ((size_t)n_multi + 1);
        HIPCHK(launch_pass_items_fill(loff, drg, (uint32_t)P, target, ioff, n_multi, istart, iend, c->stream));
    }
    if (P > 1) HIPCHK(launch_pc_item_owners(istart, n_multi, dst, (uint32_t)P, iown, c->stream, iend));
    // output room: each owner's NSHARD regions hold 5/4 of that owner's bound spread
    // evenly (the bound is the partner-list elements, >= the distinct partials) -- or,
    // once a build of these reads has run, 1.5x its partials / bound ratio; a region
    // that still fills is grown and the pass recounted (pair_stage)
    const uint64_t R = (uint64_t)NSHARD * (uint64_t)std::max(P, 1);
    const double fcap = c->dist_rho_ok ? std::min(1.25, 1.5 * c->dist_rho + 0.01) : 1.25;
    c->pair_cap = ((uint64_t)((double)own_max * fcap) / NSHARD + 1024) * R;
    EmitParams E = emit_params(c);
    E.occ_off = loff;  // occurrences of read a on this rank: [loff[a], loff[a+1])
    E.npr = 0;
    uint64_t np = 0, cap_s = 0;
    int rc = pair_stage(c, E, c->dist_in, false, true, nullptr, N, cnt, np, cap_s, istart, n_multi, nullptr, nullptr,
                        nullptr, nullptr, (uint32_t)P, dst, iown, false, iend);
    if (rc) return rc;
    Counters hc;
    HIPCHK(hipMemcpyAsync(&hc, cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    resolve_timing(c);
    // owner o's partials: its NSHARD regions (one rank: the plain NSHARD regions)
    const std::vector<unsigned long long> fill =
        P > 1 ? c->ocur : std::vector<unsigned long long>(hc.cursor, hc.cursor + NSHARD);
    c->part_off.assign(fill.size() + 1, 0);
    for (int o = 0; o < P; ++o) counts[o] = 0;
    uint64_t acc = 0;
    for (size_t r = 0; r < fill.size(); ++r) {
        const uint64_t f = std::min<unsigned long long>(fill[r], cap_s);
        c->part_off[r] = acc;
        acc += f;
        counts[r / NSHARD] += f;
    }
    c->part_off[fill.size()] = acc;
    c->part_np = acc;
    c->part_cap = cap_s;
    if (pass + 1 == npass) {  // (passes run from the last to the first)
        c->stats.role_pairs = 0;
        c->dist_parts_acc = 0;
    }
    c->stats.role_pairs += shard_sum(hc.role_pairs);
    c->dist_parts_acc += acc;
    if (pass == 0 && c->pbown[P] > 0) {  // the whole count ran: these reads' partials / bound
        c->dist_rho = (double)c->dist_parts_acc / (double)c->pbown[P];
        c->dist_rho_ok = true;
        if (getenv("SA_DEBUG_PHASES"))
            fprintf(stderr, "[sa rho] rank %d: %llu partials / %llu bound = %.4f\n", c->rank,
                    (unsigned long long)c->dist_parts_acc, (unsigned long long)c->pbown[P], c->dist_rho);
    }
    return SA_OK;
}

extern "C++" {
namespace sa {
// The first build of a read set does not know its partials / bound ratio (rho: the pass
// budget and the pair-count items are sized by it).  A probe counts the partials of the top
// 1/64 of every owner's leads -- counted, not kept -- and takes their ratio to the same
// leads' bound (round 6: configs[3]'s real read set on 8 virtual shards planned 23 passes
// at rho = 1 instead of ~10, and its 128-occurrence items overflowed into the recount tier:
// count 756 ms + reduce 236 ms in the first build against 316 + 161 once rho was known)
int dist_probe_rho(sa_ctx *c) {
    if (!c || !c->dist_bkt || c->dist_rho_ok) return SA_OK;
    const int P = c->nranks;
    if (c->pbown.size() != (size_t)P + 1 || c->pbown[P] == 0) return SA_OK;
    (void)hipSetDevice(c->device);
    if (int rc = ensure_pbcum(c)) return rc;
    constexpr uint32_t NP = 64;
    uint64_t b = 0;
    for (int r = 0; r < P; ++r) {
        uint32_t lo, hi;
        pass_range(c, r, NP - 1, NP, lo, hi);
        b += bound_sum(c, lo, hi);
    }
    if (b == 0) return SA_OK;
    std::vector<uint64_t> counts((size_t)P);
    const uint64_t rp = c->stats.role_pairs, acc = c->dist_parts_acc;
    int rc = sa_dist_count_pass(c, NP - 1, NP, counts.data());
    if (rc) return rc;
    c->stats.role_pairs = rp;  // (the probe's counts belong to no build)
    c->dist_parts_acc = acc;
    uint64_t parts = 0;
    for (uint64_t v : counts) parts += v;
    c->dist_rho = std::max(0.02, (double)parts / (double)b);
    c->dist_rho_ok = true;
    if (getenv("SA_DEBUG_PHASES"))
        fprintf(stderr, "[sa probe] rank %d: %llu partials / %llu bound = %.4f (whole bound %llu)\n", c->rank,
                (unsigned long long)parts, (unsigned long long)b, c->dist_rho, (unsigned long long)c->pbown[P]);
    return SA_OK;
}
}  // namespace sa
}  // extern "C++"

int sa_dist_count(sa_ctx *c, void *recv_recs, const uint64_t *recv_counts, uint64_t *counts) {
    if (!c || !counts || !recv_counts) return SA_E_ARG;
    int rc = sa_dist_buckets(c, recv_recs, recv_counts, nullptr);
    return rc ? rc : sa_dist_count_pass(c, 0, 1, counts);
}

int sa_dist_partials(sa_ctx *c, void *fst, void *snd, void *cnt_out) {
    if (!c) return SA_E_ARG;
    if (!c->dist) return fail(c, SA_E_STATE, "sa_dist_init first");
    if (c->part_np && (!fst || !snd || !cnt_out)) return SA_E_ARG;
    (void)hipSetDevice(c->device);
    // the owner regions, concatenated owner-major: the send buffers of exchange 2
    const uint32_t nreg = (uint32_t)c->part_off.size() - 1;
    uint64_t *doff;
    ENSURE(c->d_pq, c->part_off.size(), &doff);
    HIPCHK(hipMemcpyAsync(doff, c->part_off.data(), c->part_off.size() * 8, hipMemcpyHostToDevice, c->stream));
    const unsigned long long *dcur = nreg > NSHARD ? (const unsigned long long *)c->d_ocur.p : nullptr;
    Counters *cnt;
    ENSURE(c->d_cnt, 1, &cnt);
    if (!dcur) dcur = cnt->cursor;
    uint64_t max_fill = 0;
    for (uint32_t r = 0; r < nreg; ++r) max_fill = std::max<uint64_t>(max_fill, c->part_off[r + 1] - c->part_off[r]);
    HIPCHK(launch_copy_owner_regions((const uint32_t *)c->d_pf.p, (const uint32_t *)c->d_ps.p,
                                     (const uint32_t *)c->d_pc.p, c->part_cap, nreg, dcur, doff, (uint32_t *)fst,
                                     (uint32_t *)snd, (uint32_t *)cnt_out, max_fill, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return SA_OK;
}

int sa_dist_reduce_pass(sa_ctx *c, const void *fst, const void *snd, const void *cnt_in, uint64_t n, uint32_t pass,
                        uint32_t npass) {
    if (!c || (n && (!fst || !snd || !cnt_in)) || npass == 0 || pass >= npass) return SA_E_ARG;
    if (!c->dist) return fail(c, SA_E_STATE, "sa_dist_init first");
    (void)hipSetDevice(c->device);
    const uint32_t N = (uint32_t)c->dlen.size();
    const int idb = bits_for(N ? N - 1 : 0);
    Counters *cnt;
    ENSURE(c->d_cnt, 1, &cnt);
    // this rank's leads of the pass; passes run from the last (highest leads) to the
    // first, so each one's dispatch (lead descending) is appended after the previous
    uint32_t lbase, lend;
    pass_range(c, c->rank, pass, npass, lbase, lend);
    const uint32_t nl = lend - lbase;
    if (pass + 1 == npass) {
        c->disp_acc = 0;
        c->stats.pairs = 0;
        c->stats.dispatched = 0;
    }
    const uint64_t acc = c->disp_acc;
    c->built = c->aligned = false;
    c->lead.clear(); c->trail.clear(); c->count.clear();
    c->pfst.clear(); c->psnd.clear(); c->pcnt.clear();
    uint64_t *ok, *ok2; uint32_t *ov, *ov2, *sum, *keep, *pos; uint8_t *otmp, *scan;
    ENSURE(c->d_okeys, n, &ok);
    ENSURE(c->d_okeys2, n, &ok2);
    ENSURE(c->d_ovals, n, &ov);
    ENSURE(c->d_ovals2, n, &ov2);
    ENSURE(c->d_osort, radix_sort_temp_bytes(n), &otmp);
    ENSURE(c->d_psum, n, &sum);
    ENSURE(c->d_pkeep, n, &keep);
    ENSURE(c->d_ppos, n, &pos);
    ENSURE(c->d_scan, scan_temp_bytes(std::max<uint64_t>(n, nl)), &scan);
    HIPCHK(hipMemsetAsync(cnt->distinct, 0, sizeof(cnt->distinct), c->stream));
    HIPCHK(hipMemsetAsync(cnt->totals, 0, sizeof(cnt->totals), c->stream));
    HIPCHK(hipMemsetAsync(&cnt->overflow_n, 0, sizeof(cnt->overflow_n), c->stream));
    auto finish = [&](uint32_t nd, unsigned long long ndist) {
        // (the next pass's tier routing, from the tiers or the sort alike; SA_LR_ROUTE=0:
        // the m / ranks floor alone, A/B)
        static const bool route_on = !getenv("SA_LR_ROUTE") || atoi(getenv("SA_LR_ROUTE")) != 0;
        if (n && route_on) c->dist_route = (float)((double)ndist / (double)n);
        c->disp_acc = acc + nd;
        c->n_disp = c->disp_acc;
        c->stats.pairs += ndist;
        c->stats.dispatched = c->disp_acc;
        c->stats.id_mode = SA_IDS_WIDE;
        c->mode = SA_IDS_WIDE;
        c->built = pass == 0;  // (the first pass is the last to run)
        c->aligned = false;
        return (int)SA_OK;
    };
    // this rank's leads: per-lead segments of the received partials, summed and
    // filtered in LDS (a wave per lead up to 768 distinct partners, a block per lead
    // up to 12,288: dist.hip's four tiers), then one scan + one copy in lead-descending
    // order; a lead with more than 12,288 (high-copy repeats, k = 12) sends the pass to
    // the (lead, trail) radix sort below (SA_LR_FORCE_SORT=1 sends every pass there: tests)
    if (!(getenv("SA_LR_FORCE_SORT") && atoi(getenv("SA_LR_FORCE_SORT")) != 0)) {
        uint32_t *lr;
        uint2 *seg = (uint2 *)ok;
        ENSURE(c->d_lr, 5 * ((size_t)nl + 1), &lr);
        uint32_t *lcnt = lr, *loff = lr + ((size_t)nl + 1), *lcur = lr + 2 * ((size_t)nl + 1),
                 *kcnt = lr + 3 * ((size_t)nl + 1), *kex = lr + 4 * ((size_t)nl + 1);
        uint8_t *scan2 = scan;
        Counters *hp;
        if (int rc_ = pinned_counters(c, &hp)) return rc_;
        {
            StageScope st(c, SA_STAGE_ORDER);
            HIPCHK(launch_lead_reduce((const uint32_t *)fst, (const uint32_t *)snd, (const uint32_t *)cnt_in, n, lbase,
                                      nl, c->set.min_collisions, c->set.max_collisions, lcnt, loff, lcur, seg, kcnt,
                                      cnt->distinct, &cnt->overflow_n, (uint32_t)c->nranks, c->dist_route, scan2,
                                      &cnt->totals[1], c->stream));
            HIPCHK(exclusive_scan_u32(kcnt, kex, nl, &cnt->totals[0], scan2, c->stream));
        }
        HIPCHK(hipMemcpyAsync(hp, cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (nl && hp->overflow_n == 0) {
            const uint32_t nd = hp->totals[0];
            const unsigned long long ndist = shard_sum(hp->distinct);
            int32_t *dlead, *dtrail, *dcount;
            if (int r_ = ensure_keep(c, c->d_lead, acc + nd, acc, &dlead)) return r_;
            if (int r_ = ensure_keep(c, c->d_trail, acc + nd, acc, &dtrail)) return r_;
            if (int r_ = ensure_keep(c, c->d_count, acc + nd, acc, &dcount)) return r_;
            {
                StageScope st(c, SA_STAGE_ORDER);
                HIPCHK(launch_lead_copy(seg, loff, kcnt, kex, &cnt->totals[0], nl, lbase, dlead + acc, dtrail + acc,
                                        dcount + acc, c->stream));
            }
            HIPCHK(hipStreamSynchronize(c->stream));
            resolve_timing(c);
            return finish(nd, ndist);
        }
        HIPCHK(hipMemsetAsync(cnt->distinct, 0, sizeof(cnt->distinct), c->stream));
        HIPCHK(hipMemsetAsync(cnt->totals, 0, sizeof(cnt->totals), c->stream));
    }
    {
        StageScope st(c, SA_STAGE_ORDER);
        HIPCHK(launch_reduce_keys((const uint32_t *)fst, (const uint32_t *)snd, n, idb, ok, ov, c->stream));
        HIPCHK(radix_sort(&ok, &ov, &ok2, &ov2, n, 0, 2 * idb, otmp, c->stream));
        HIPCHK(launch_reduce_heads(ok, ov, n, (const uint32_t *)cnt_in, c->set.min_collisions, c->set.max_collisions,
                                   sum, keep, cnt->distinct, c->stream));
        if (n) HIPCHK(exclusive_scan_u32(keep, pos, n, &cnt->totals[0], scan, c->stream));
    }
    uint32_t nd = 0;
    HIPCHK(hipMemcpyAsync(&nd, &cnt->totals[0], 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    int32_t *dlead, *dtrail, *dcount;
    if (int r_ = ensure_keep(c, c->d_lead, acc + nd, acc, &dlead)) return r_;
    if (int r_ = ensure_keep(c, c->d_trail, acc + nd, acc, &dtrail)) return r_;
    if (int r_ = ensure_keep(c, c->d_count, acc + nd, acc, &dcount)) return r_;
    HIPCHK(launch_reduce_compact(ok, n, idb, sum, keep, pos, dlead + acc, dtrail + acc, dcount + acc, c->stream));
    Counters hc;
    HIPCHK(hipMemcpyAsync(&hc, cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    resolve_timing(c);
    return finish(nd, shard_sum(hc.distinct));
}

int sa_dist_reduce(sa_ctx *c, const void *fst, const void *snd, const void *cnt_in, uint64_t n) {
    return sa_dist_reduce_pass(c, fst, snd, cnt_in, n, 0, 1);
}

int sa_dist_codes(sa_ctx *c, void *codes, void *bad, uint64_t *nwords) {
    if (!c || !nwords) return SA_E_ARG;
    if (!c->dist) return fail(c, SA_E_STATE, "sa_dist_init first");
    (void)hipSetDevice(c->device);
    int rc = ensure_prepared(c);
    if (rc) return rc;
    const uint32_t nl = (uint32_t)(c->boff.size() - 1);
    const uint64_t nw = c->woff[nl];
    *nwords = nw;
    if (!codes && !bad) return SA_OK;
    DevReads R = dev_reads(c);
    HIPCHK(launch_pack_reads(R, c->stream));  // idempotent; the codes may not exist yet
    if (codes && nw) HIPCHK(hipMemcpyAsync(codes, c->d_codes.p, nw * 4, hipMemcpyDeviceToDevice, c->stream));
    if (bad && nl) HIPCHK(hipMemcpyAsync(bad, c->d_bad.p, (size_t)nl * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return SA_OK;
}

int sa_dist_set_reads(sa_ctx *c, const void *codes, const void *bad, uint64_t nwords) {
    if (!c) return SA_E_ARG;
    if (!c->dist) return fail(c, SA_E_STATE, "sa_dist_init first");
    (void)hipSetDevice(c->device);
    const uint32_t N = (uint32_t)c->dlen.size();
    std::vector<uint64_t> gw((size_t)N + 1, 0);
    for (uint32_t i = 0; i < N; ++i) gw[i + 1] = gw[i] + (uint64_t)((c->dlen[i] + 15) / 16);
    if (gw[N] != nwords) return fail(c, SA_E_ARG, "word count does not match the global read lengths");
    if ((nwords && !codes) || (N && !bad)) return SA_E_ARG;
    uint32_t *gcodes; uint64_t *gwoff; int32_t *glen, *gbad;
    ENSURE(c->d_gcodes, nwords + 2, &gcodes);  // pad: windows read past a read's last word
    ENSURE(c->d_gwoff, (size_t)N + 1, &gwoff);
    ENSURE(c->d_glen, (size_t)N + 1, &glen);
    ENSURE(c->d_gbad, (size_t)N + 1, &gbad);
    HIPCHK(hipMemsetAsync(gcodes + nwords, 0, 8, c->stream));
    // (a virtual shard's buffers may be the all-gathered copy itself, lent by multi.cpp)
    if (nwords && gcodes != codes)
        HIPCHK(hipMemcpyAsync(gcodes, codes, nwords * 4, hipMemcpyDeviceToDevice, c->stream));
    if (N && gbad != bad) HIPCHK(hipMemcpyAsync(gbad, bad, (size_t)N * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(gwoff, gw.data(), gw.size() * 8, hipMemcpyHostToDevice, c->stream));
    if (N) HIPCHK(hipMemcpyAsync(glen, c->dlen.data(), (size_t)N * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->dist_reads = true;
    return SA_OK;
}

int sa_load_hoxd(sa_settings *s, const char *path) {
    if (!s || !path) return SA_E_ARG;
    return read_hoxd(path, s->cost) == 0 ? SA_OK : SA_E_INPUT;
}

}  // extern "C"
