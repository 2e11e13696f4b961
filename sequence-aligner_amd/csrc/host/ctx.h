// ctx.h -- the library context (struct sa_ctx behind include/sa_overlap.h) and
// host helpers shared by api.cpp (one device) and multi.cpp (sharded contexts).
#pragma once
#include "../../../include/sa_overlap.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../sa_internal.h"

struct sa_multi;

namespace sa {

struct DBuf {
    void *p = nullptr;
    size_t bytes = 0;
    // lent by the sharded context's pool (SA_OPT_LEAN_MEMORY, virtual shards): never freed
    // by the child; a child that needs more allocates its own and the pool takes it back
    bool borrowed = false;
};

// device-resident counters, one memset per build; the hot ones are NSHARD-way
// sharded (see sa_internal.h) and summed here
struct Counters {
    unsigned long long cursor[NSHARD];
    unsigned long long role_pairs[NSHARD];
    unsigned long long role_pairs_dummy[NSHARD];
    unsigned long long distinct[NSHARD];
    unsigned long long cells[NSHARD];
    unsigned long long bkt_counts[2 * NSHARD];
    uint32_t overflow_n;
    int32_t err;
    uint32_t totals[4];
    uint32_t big_n;
    uint32_t mid_n;
    uint32_t mid2_n;
    uint32_t fb_n;   // (split tier) partitions whose halves do not fit 1,024 records
    uint32_t xrec_n;     // escape records written (big partitions)
    uint32_t rtotal;     // per-read pair mode: dispatched pairs (scan total)
    uint32_t shard_off[NSHARD + 2];
    unsigned long long bound_own[257];  // sharded: partial bound per lead owner + total (read back pinned)
};

inline unsigned long long shard_sum(const unsigned long long *v) {
    unsigned long long t = 0;
    for (int i = 0; i < NSHARD; ++i) t += v[i];
    return t;
}

}  // namespace sa

using sa::DBuf;

struct sa_ctx {
    // sharded context (sa_ctx_create_multi / sa_ctx_create_rank): its shards and
    // exchanges (multi.cpp); null for a plain single-device context
    sa_multi *multi = nullptr;
    uint64_t reads_gen = 0;  // bumped by every sa_add_reads (shards re-split on change)
    sa_settings set{};
    int device = 0;
    hipStream_t stream = nullptr;
    // second stream for work that overlaps the main chain (the read-order sort
    // beside the partition sort, the 2,048 / 4,096-record bucket tiers beside
    // the 1,024-record pass) and its fork / join events; created on first use
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_fork2 = nullptr, ev_join2 = nullptr;
    // pinned host copy of the device counters: each build's readbacks are one
    // DMA each (a pageable copy stages through a driver buffer)
    sa::Counters *hcnt = nullptr;
    std::string err;
    // reads (host)
    std::vector<char> bases;
    std::vector<uint64_t> boff{0};
    bool reads_dirty = true, uploaded = false;
    // derived (host)
    std::vector<int32_t> len;
    std::vector<uint64_t> woff, occ_off;
    std::vector<uint32_t> lbase, lrank;
    std::vector<uint8_t> tagtab;
    int lb = 1, m = 0, maxd = 0, maxL = 0, minL = 0;
    uint32_t uniform_npr = 0;
    uint64_t n_occ = 0, n_words = 0;
    uint32_t max_occ = 0;
    int32_t mode = SA_IDS_WIDE;
    // device buffers
    DBuf d_ascii, d_boff, d_woff, d_len, d_codes, d_bad, d_occ_off, d_lbase, d_lrank, d_tagtab;
    DBuf d_keys, d_vals, d_keys2, d_vals2, d_sorttmp;
    DBuf d_md, d_ed, d_bmdo, d_bedo, d_bstart, d_gbid, d_gmds, d_gede, d_ogid, d_bkttmp;
    DBuf d_mdidx, d_edidx, d_occidx, d_bnst, d_brank, d_bhash, d_bfirst;
    DBuf d_pstart, d_biglist, d_rec, d_srec, d_bnmd, d_ishead, d_bnst2;
    DBuf d_tmd, d_ted, d_tmdi, d_tedi, d_xrec;  // big-partition scratch lists, escape records
    DBuf d_tier, d_ovlrp;                       // pair-count recount tier items, overflow role pairs
    DBuf d_meta;                                // mixed lengths: {first occurrence, lrank base} per read
    int pos_bits = 0;                           // > 0: records carry read << pos_bits | pos
    uint64_t meta_gen = ~0ull;
    int meta_k = 0;
    uint32_t *bkt_rank_dev = nullptr;
    DBuf d_pf, d_ps, d_pc, d_pr, d_ovl, d_cnt;
    DBuf d_okeys, d_ovals, d_okeys2, d_ovals2, d_osort;
    DBuf d_lead, d_trail, d_count, d_aln, d_p1, d_p1tf, d_p1st, d_tb, d_ltb, d_lmax;
    DBuf d_rkey, d_rkey2, d_rord, d_rord2, d_rtmp;
    DBuf d_rreg, d_rcnt, d_rex;  // per-read pair regions, counts, their exclusive scan
    // per-read mode: the recounted reads' pairs sorted (lead, trail, count) and
    // each such read's segment start + 1 (0: the read's pairs are in its region)
    DBuf d_shl, d_sht, d_shc, d_rsh;
    uint64_t recounted = 0;      // last build: dispatched pairs of reads recounted by the tiers (per-read mode)
    uint32_t first_overflow = 0; // last build: reads whose first-pass table overflowed (recounted)
    bool used_per_read = false;  // last build used the per-read regions
    uint64_t pair_cap = 0;
    uint64_t n_disp = 0;
    // distributed mode (sa_dist_*): this rank's slice of a global read set
    bool dist = false, dist_reads = false;
    int rank = 0, nranks = 1, log_ranks = 0;
    int dist_src_shift = 0;                // this build's packed values are source-relative (RecvGen)
    float dist_route = 0.f;                // distinct partners per partial of the last reduced pass (tier routing)
    std::vector<uint32_t> dstarts;   // [nranks+1] first global read of each rank
    std::vector<int32_t> dlen;       // length of every global read
    std::vector<uint64_t> gocc;      // global occurrence offsets [N+1]
    uint32_t gnpr = 0;               // uniform k-mers per read over all reads (0: mixed)
    int32_t gmaxL = 0, gminL = 0;
    uint64_t part_np = 0;            // partial pairs after sa_dist_count
    // ... in owner-major regions of part_cap entries (d_pf / d_ps / d_pc; fill
    // in d_ocur / ocur, or the Counters cursors with one rank): region r's go
    // to part_off[r] of the send buffers
    unsigned long long part_cap = 0;
    std::vector<uint64_t> part_off;
    std::vector<unsigned long long> ocur;
    DBuf d_gocc, d_seg, d_rl, d_srl, d_srl2, d_loff, d_starts, d_bounds, d_gcodes, d_gwoff, d_glen, d_gbad, d_psum, d_pkeep, d_ppos;
    DBuf d_scan, d_bigtot, d_items, d_pq, d_ocur;
    DBuf d_lr;                       // owner-side reduce by lead: counts, offsets, cursors, kept, kept scan
    // lead-range passes (sa_dist_buckets -> sa_dist_plan -> per pass sa_dist_count_pass,
    // exchange 2, sa_dist_reduce_pass): the buckets are built once, then each pass counts
    // the partials of 1/npass of every owner's leads, so the partials held at once are
    // bounded by the pass (SURVEY.md 8(e) exchange 2 at configs[4]'s density)
    bool dist_bkt = false;                 // buckets of the received records are built
    sa::PairIn dist_in{};                  // their records and lists (device)
    uint64_t dist_recv = 0;                // records received
    std::vector<unsigned long long> pbown; // partial bound per lead owner [nranks], total last
    std::vector<uint64_t> pbcum;           // host prefix sums of the partial bounds (multi-pass plans),
    uint32_t pb_gran = 1;                  // per block of pb_gran reads (1 or 64)
    uint32_t dist_npass = 1;               // the last plan's pass count
    // partials / bound of the last build of these reads (1 until one ran): the bound
    // counts partner-list elements, ~20x the distinct partials at the bench shape
    // (overlapping reads share many k-mers), ~1.3-2x at configs[4]'s k = 12 -- the
    // pair regions and the pass plan are sized by bound x 1.5 rho
    double dist_rho = 1.0;
    bool dist_rho_ok = false;
    uint64_t dist_parts_acc = 0;           // partials of the passes run so far
    uint64_t disp_acc = 0;                 // dispatched pairs the reduce passes appended so far
    DBuf d_pbound, d_pbown, d_prange, d_pioff, d_pitems;
    DBuf d_trove;                          // strict ids: the device Trove layout's keys, order and scratch
    // k-mer table statistics (sa_kmer_histogram)
    DBuf d_hk0, d_hk1, d_hflag, d_hidx, d_hpos, d_htmp, d_hist, d_hovf, d_hsmall;
    std::vector<uint64_t> hsize, hcount;
    // options / state
    bool keep_pairs = false, timing = false;
    int align_kernel = 0;  // SA_OPT_ALIGN_KERNEL
    int first_pass = 0;         // SA_OPT_FIRST_PASS: 0 probe, 1 always, 2 skip (wide ids)
    uint32_t launch_slice = 0;  // SA_OPT_LAUNCH_SLICE (0: only when a grid would pass 2^31 work-items)
    int aligner = SA_ALIGNER_LINEAR;  // SA_OPT_ALIGNER (--linear-align / --quadratic-align)
    uint64_t local_batch_bytes = 16ull << 30;  // traceback-code budget of one quadratic launch
    bool built = false, aligned = false;
#ifdef SA_PB_STAMPS
    uint64_t *stamps_dev = nullptr;  // (timing probe builds, partition.hip PB_STAMP)
    uint32_t stamps_np = 0;
#endif
    bool host_valid = false;  // alns / ovl hold the last alignment's results (sa_align or first use)
    // results (host)
    std::vector<int32_t> lead, trail, count;
    std::vector<int32_t> pfst, psnd, pcnt;
    std::vector<sa_alignment> alns;
    std::string ovl;
    sa_stats stats{};
    // timing
    struct Pending { int stage; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> ev_pool;
    double stage_ms[SA_NUM_STAGES] = {0};
    uint64_t stage_n[SA_NUM_STAGES] = {0};
};

// sharded contexts (multi.cpp); api.cpp routes the public calls of a context
// with c->multi here.  single_build / single_align run the one-device path on
// the context itself (strict-id inputs of a multi context).
namespace sa {
bool multi_sharded(const sa_ctx *c);
bool multi_rank_mode(const sa_ctx *c);
int multi_rank(const sa_ctx *c);
void multi_destroy(sa_ctx *c);
int multi_build(sa_ctx *c, bool readback, int (*single_build)(sa_ctx *, bool));
int multi_dispatch(sa_ctx *c);
int multi_align(sa_ctx *c, bool readback, int (*single_align)(sa_ctx *, bool));
int multi_host_results(sa_ctx *c);
int multi_all_ok(sa_ctx *c, bool ok);
int multi_gather_ovl(sa_ctx *c, std::string &all);
int multi_set_option(sa_ctx *c, int option, int64_t value);
void multi_stage_times(const sa_ctx *c, double *ms, uint64_t *n);
void multi_reset_stage_times(sa_ctx *c);
// (api.cpp) the first build of a read set: its partials / bound ratio from a probe pass
int dist_probe_rho(sa_ctx *c);
int multi_sync(sa_ctx *c);
uint64_t multi_exchanged_bytes(const sa_ctx *c);
}  // namespace sa
