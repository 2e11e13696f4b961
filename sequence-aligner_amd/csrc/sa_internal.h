// sa_internal.h -- device-side data layout and kernel launchers of the
// MI355X hash-overlap stage.  Host orchestration lives in host/pipeline.cpp;
// kernels live in kernels/*.hip.  See DESIGN.md for the HBM layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sa {

// ---- packed reads --------------------------------------------------------
// Read r (0-based; reference id r+1) occupies words [woff[r], woff[r+1]) of
// `codes`; base p sits in word woff[r] + p/16 at bits 30-2*(p%16) (MSB first),
// 2-bit HOXD order A0 C1 G2 T3 (BioLibs.scala:144-149).  Non-ACGT -> 0 and
// `bad[r]` = first such position (else INT32_MAX).
struct DevReads {
    uint32_t n = 0;
    const uint8_t *ascii = nullptr;   // raw bases
    const uint64_t *boff = nullptr;   // [n+1] byte offsets
    const uint64_t *woff = nullptr;   // [n+1] word offsets (+1 pad word at the end)
    const int32_t *len = nullptr;     // [n]
    uint32_t *codes = nullptr;        // packed 2-bit words
    int32_t *bad = nullptr;           // [n]
};

// ---- k-mer emission parameters --------------------------------------------
struct EmitParams {
    int32_t k;                 // kmer size
    int32_t m;                 // min(16, k): hashed window (ObjectStore.scala:52)
    int32_t lb;                // locrank bits in the sort key
    const uint64_t *occ_off;   // [n+1] first occurrence index of each read
    uint32_t npr;              // > 0: every read has npr k-mers (occ_off[r] = r * npr)
    const uint32_t *lbase;     // [maxd+1] offset of denominator d = L-k in lrank
    const uint32_t *lrank;     // rank of float32 i/d among all distinct locs
    int32_t maxd;
    uint64_t *rkey;            // [n] per-read locality key (min k-mer mix; nullable)
    uint32_t *rord;            // [n] read ids (sort payload for rkey)
    int32_t pos_bits;          // > 0: the record's low word is read << pos_bits | pos (mixed lengths)
    // mixed lengths without pos_bits codes: per-occurrence {read, loc rank}
    // table (nullable), so the bucket build finds both with one load
    uint2 *occ_rl;
    // uniform lengths (KeyGen): the first radix pass's tile histogram, counted by the
    // pack kernel from the hashes it computes anyway (launch_pack_emit_hist; nullptr: off)
    uint32_t *hist;
    int hist_shift;            // the pass's digit: bits [hist_shift, hist_shift + 8) of the record
};

// bijective 32-bit mix of the seqHash: equal mix <=> equal hash, so a bucket
// stays contiguous after sorting, while partitions by the top bits are balanced
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x7feb352du;
    h ^= h >> 15; h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}

// 16 codes starting at base position p of a read whose first word is `w`
// (MSB-first window), used for hashing and diagonal compares.
__device__ __forceinline__ uint32_t window16(const uint32_t *w, int32_t p) {
    const uint32_t a = w[p >> 4];
    const int s = p & 15;
    if (s == 0) return a;
    const uint32_t b = w[(p >> 4) + 1];
    return (a << (2 * s)) | (b >> (32 - 2 * s));
}

// mix32(Kmer.seqHash) of the k-mer at position p (ObjectStore.scala:48-67: the
// first min(16, k) bases, h = (h << 2) ^ code); shift = 32 - 2 min(16, k)
__device__ __forceinline__ uint32_t kmer_mix(const uint32_t *w, int32_t p, int shift) {
    uint32_t x = window16(w, p);
    x = shift == 32 ? 0u : (x >> shift);
    // HOXD order (A0 C1 G2 T3) -> seqHash order (A0 C1 T2 G3): c ^ (c >> 1)
    x ^= (x >> 1) & 0x55555555u;
    return mix32(x);
}

// The k-mer records of uniform-length reads (read r's packed words at
// codes + r * nw, npr k-mers each), generated where a sort pass would load them:
// record i = mix32(seqHash) << 32 | i, exactly what pack_emit_kernel stores at
// keys[i] (radix_sort_gen)
struct KeyGen {
    const uint32_t *codes;
    uint32_t nw;               // packed words per read
    uint32_t npr;              // k-mers per read (>= 1)
    uint64_t npr_magic;        // floor((2^64 - 1) / npr) + 1 (npr >= 2)
    int shift;                 // 32 - 2 min(16, k)
    int hist_shift = -1;       // >= 0: the tile histogram of the pass at this shift is already
                               // in the sort's temp (launch_pack_emit_hist): no upsweep
};
__device__ __forceinline__ uint64_t gen_key(const KeyGen &g, uint64_t i) {
    const uint32_t r = g.npr == 1 ? (uint32_t)i : (uint32_t)__umul64hi((unsigned long long)i, g.npr_magic);
    const int32_t pos = (int32_t)((uint32_t)i - r * g.npr);
    return ((uint64_t)kmer_mix(g.codes + (uint64_t)r * g.nw, pos, g.shift) << 32) | (uint32_t)i;
}

// Inclusive add-scan over the 64 lanes of a wave in DPP moves (row_shr 1, 2, 4,
// 8 within each row of 16, then row_bcast 15 / 31 across rows): VALU only, where
// a __shfl_up ladder is six dependent ds_bpermute round trips through the LDS
// pipe.  Lanes whose DPP source is outside the row keep `old` = 0.
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15, rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31, rows 2, 3
    return v;
}

// The same scan with max (values >= 0): inclusive, and exclusive (wave_shr:1)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {  // lane l gets lane l - 1's value, lane 0 gets 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}

// Ballot multisplit: the mask of valid lanes whose digit d agrees with this
// lane's in bits [0, nbits) (nbits <= 8, wave-uniform).  Per bit: v_bfe_i32 for
// an all-ones / zero bit mask m, one ballot, and peer &= ~(ballot ^ m) as one
// v_bitop3_b32 per 32-bit half (truth table 0x90 over (peer, ballot, m)); the
// ternary `bit ? bb : ~bb` form compiled to 9 VALU per bit (compares, a select,
// two xors, two ands).
__device__ __forceinline__ uint64_t wave_peers(uint32_t d, bool valid, int nbits = 8) {
    const uint64_t v = __ballot(valid);
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        if (b >= nbits) break;  // uniform
        const uint32_t m = (uint32_t)((int32_t)(d << (31 - b)) >> 31);
        const uint64_t bb = __ballot(m != 0u);
        lo = __builtin_amdgcn_bitop3_b32(lo, (uint32_t)bb, m, 0x90);
        hi = __builtin_amdgcn_bitop3_b32(hi, (uint32_t)(bb >> 32), m, 0x90);
    }
    return ((uint64_t)hi << 32) | lo;
}

// ---- partner lists and per-occurrence records ------------------------------
// Every bucket owns one slice of the combined partner list `lst` (read index
// per entry), laid out around a split point c:
//     [ middle entries, loc DEScending | edge roles (st, en), loc AScending ]
//                                      ^ c
// so an edge k-mer's partners as fst -- the middle entries with loc < own --
// are [c - nE, c) and a middle k-mer's -- the edge roles with loc <= own -- are
// [c, c + nD) (addKmerPair's orientation, KmerTable.scala:65-71; the st/md/en
// split, :106-115).  The partition of sorted offset ps owns lst[3 ps, 3 ps + 3 n),
// so c < 3 n < 2^34 (n < 2^32 k-mers per device).
// One 8-byte record per occurrence g: x = c mod 2^32, y = nE | nD << 14 |
// (c >> 32) << 28 | me << 30 (me = number of edge tags, 0..2).  me == 3 marks an
// escape: y & 0x3FFFFFFF indexes the 16-byte xrec table, which holds the
// decoded form (counts above 16,382: high-copy repeats).
constexpr uint32_t REC_CNT_MAX = 0x3FFEu;
__device__ __forceinline__ uint2 encode_rec(uint64_t c, uint32_t nE, uint32_t nD, uint32_t me) {
    return make_uint2((uint32_t)c, nE | (nD << 14) | ((uint32_t)(c >> 32) << 28) | (me << 30));
}
// decoded: {c mod 2^32, nE | me << 30, c >> 32, nD}
__device__ __forceinline__ uint4 decoded_rec(uint64_t c, uint32_t nE, uint32_t nD, uint32_t me) {
    return make_uint4((uint32_t)c, nE | (me << 30), (uint32_t)(c >> 32), nD);
}
// Relaxed LDS load of a word other lanes may be updating (hash-table keys,
// flags): a volatile access through a generic pointer compiles to a FLAT load
// (vmcnt + lgkmcnt waits that also drain every outstanding global load); the
// relaxed atomic keeps the LDS address space -> one ds_read
template <typename T>
__device__ __forceinline__ T lds_relaxed(T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint4 decode_rec(uint2 r, const uint4 *xrec) {
    if ((r.y >> 30) == 3u) return xrec[r.y & 0x3FFFFFFFu];
    return decoded_rec(((uint64_t)((r.y >> 28) & 3u) << 32) | r.x, r.y & 0x3FFFu, (r.y >> 14) & 0x3FFFu, r.y >> 30);
}
// list index of a decoded record's off-th partner entry (off < nE: the middle
// entries [c - nE, c); then the edge roles [c, c + nD))
__device__ __forceinline__ uint64_t rec_entry(const uint4 &rc, uint32_t off) {
    return (((uint64_t)rc.z << 32) | rc.x) - (rc.y & 0x3FFFFFFFu) + off;
}


// bit 0 = st, bit 1 = md, bit 2 = en   (KmerTable.scala:106-115)
enum : uint8_t { TAG_ST = 1, TAG_MD = 2, TAG_EN = 4 };

// ---- bucket / list tables (after the (hash, locrank) sort) -----------------
struct Buckets {
    uint64_t n_occ = 0;
    uint32_t n_buckets = 0, n_groups = 0, n_md = 0, n_ed = 0;
    uint32_t *md_list = nullptr;     // read index of each middle occurrence, by (bucket, locrank, g)
    uint32_t *ed_list = nullptr;     // read index of each edge role (st, en)
    uint32_t *bkt_mdo = nullptr;     // [nb+1] first md entry of bucket
    uint32_t *bkt_edo = nullptr;     // [nb+1] first edge entry of bucket
    uint32_t *bkt_start = nullptr;   // [nb+1] first sorted position of bucket
    uint32_t *grp_bid = nullptr;     // [ng] bucket of group
    uint32_t *grp_mds = nullptr;     // [ng] md entries of the bucket before the group (locrank <)
    uint32_t *grp_ede = nullptr;     // [ng] edge entries of the bucket through the group (locrank <=)
    uint32_t *occ_gid = nullptr;     // [n_occ] group of occurrence g
    // strict-mode annotations (reference order replay)
    uint32_t *md_idx = nullptr;      // [n_md] index of the md entry in the bucket's (id,pos)-ordered md list
    uint32_t *ed_idx = nullptr;      // [n_ed] (phase<<31) | index in the st (phase 0) / en (phase 1) list
    uint32_t *occ_idx = nullptr;     // [3*n_occ] own st/md/en list index
    uint32_t *bkt_nst = nullptr;     // [nb] |st| of bucket
    uint32_t *bkt_rank = nullptr;    // [nb] KmerData iteration rank (host Trove replay)
};

// Inputs of the pair counter: the 8-byte record of every k-mer occurrence g
// (decode_rec -> {md_lo, nE | me << 30, ed_lo, nD}) and the combined list.
struct PairIn {
    const uint2 *rec;
    const uint4 *xrec;
    const uint32_t *lst;
    // strict mode
    const uint4 *srec;          // {bucket head position, own_e, own_m, 0}
    const uint32_t *lidx;       // per list entry: md -> index in the bucket's (id,pos)-ordered md list;
                                // edge -> (phase << 31) | index in its st (0) / en (1) list
    const uint32_t *bkt_nst, *bkt_nmd, *bkt_rank;  // indexed by bucket head position
};

struct PairParams {
    int32_t min_coll, max_coll;
    int32_t emit_all;      // 1: every distinct pair (PairData); 0: dispatched only
    int32_t strict;        // compute first-occurrence ranks
    int32_t split;         // partner residue classes (overflow fallback): partner % split == residue
    int32_t coded;         // read_list holds (read << 6 | residue) codes (recount tiers)
    uint32_t max_occ;      // max occurrences of one read (LDS sizing)
    uint32_t n_items;      // reads (x split) to process; blocks beyond it exit
    int32_t xcd_swizzle;   // 1: XCD-contiguous block -> item map (grid % 8 == 0)
    int32_t table;         // LDS hash slots per read: 256 (first pass) or 2048
    // non-null: every block exits at once when *abort != 0 -- the first pass is
    // launched before the host has read back whether any partition needs the
    // global bucket path (big_n); if one did, the pass is discarded and re-run
    const uint32_t *abort;
    int32_t per_read;      // 1: emit into PairOut::rreg / rcnt (first pass, wide ids, dispatched pairs only)
    uint32_t max_blocks;   // > 0: at most this many blocks per launch (item lists are sliced; tests)
    // > 0 (the 16,384 / 32,768-slot tiers): a one-chunk read whose distinct
    // partners, projected from the table's fill after at least 1 / (early >> 8)
    // of its role pairs, exceed (early & 255) / 8 x the fill limit stops there
    // and is handed to finer classes at once, the projection as its estimate
    int32_t early;
};

// A/B knob (environment SA_OCC_<NAME> = b > 0): the LDS a block allocates,
// padded so that at most b blocks fit one CU (MI355X: 160 KB of LDS per CU);
// `used` = the block's LDS without padding, returns the dynamic size to launch
// with (its own dynamic part `dyn` plus the pad)
inline size_t occ_lds(const char *env, size_t used, size_t dyn) {
    const char *v = getenv(env);
    const int b = v ? atoi(v) : 0;
    if (b <= 0) return dyn;
    const size_t cap = (160u * 1024u) / (size_t)b;
    return cap > used ? dyn + (cap - used) : dyn;
}

// Device-wide counters are sharded NSHARD ways (shard = blockIdx % NSHARD) and
// block-reduced first: same-address device atomics from every block serialise
// at one L2 channel (MI355X_MICROARCH.md, fan-in row).
constexpr int NSHARD = 64;

// Output of the pair counter: NSHARD regions of cap_s entries each; block b
// appends to region b % NSHARD.
struct PairOut {
    uint32_t *fst, *snd, *cnt;   // [NSHARD * cap_s]
    uint64_t *rank;              // [NSHARD * cap_s] (strict)
    unsigned long long *cursor;  // [NSHARD] entries written per region
    unsigned long long cap_s;
    unsigned long long *role_pairs;  // [NSHARD]
    unsigned long long *distinct;    // [NSHARD] distinct (a, partner) keys counted
    uint32_t *overflow_list;     // (read << 6 | residue) of the blocks whose LDS table overflowed
    uint32_t *overflow_rp;       // their role-pair totals (nullable)
    uint32_t *overflow_n;
    // per-read mode (PairParams::per_read): read a's kept pairs, trail
    // ascending, at rreg[a * PC_RREG ..] and their number at rcnt[a]; the
    // dispatch order (lead descending) is then one scan + one copy, no sort
    uint2 *rreg;                 // {trail, count}
    uint32_t *rcnt;
    // sharded path (owners > 1): the partials leave grouped by the rank owning
    // their lead -- region (owner * NSHARD + shard) of cap_s entries, cursor
    // [owners * NSHARD]; owner o holds the reads [owner_starts[o], owner_starts[o + 1])
    uint32_t owners;
    const uint32_t *owner_starts;
    const uint32_t *item_owner;  // multi-read items: owners of the item's first | last read << 16
    // multi-read items with their own ends (lead-range passes: the pass's read ranges leave
    // gaps, so item j is [item_start[j], item_end[j])); null: item_start[j + 1]
    const uint32_t *item_end;
};
constexpr uint32_t PC_RREG = 192;  // = the first pass's fill limit (256 slots at 3/4)
// fill limit of the recount tiers' tables (2,048 slots and up, bucketed
// probing), in eighths of the slots; the host sizes tiers and classes with it
#ifndef SA_TIER_FILL_EIGHTHS
#define SA_TIER_FILL_EIGHTHS 6
#endif
__host__ __device__ constexpr uint32_t pc_fill_max(uint32_t tab) {
    return tab >= 2048 ? tab / 8 * SA_TIER_FILL_EIGHTHS : tab * 3 / 4;
}

// Four alignment costs indexed by a 2-bit base code given as x8 = 8 * code.
// Cost8: one word of int8 bytes (HOXD70 and every matrix whose entries fit a
// byte after the common-divisor reduction); Cost16: two words of int16 halves
// (any other matrix up to |cost| <= 32,767) -- one extra select per lookup.
struct Cost8 {
    uint32_t p;
    __device__ __forceinline__ int32_t at(uint32_t x8) const { return __builtin_amdgcn_sbfe((int32_t)p, x8, 8); }
    __device__ __forceinline__ static Cost8 make(int32_t c0, int32_t c1, int32_t c2, int32_t c3) {
        return Cost8{(uint32_t)(c0 & 255) | ((uint32_t)(c1 & 255) << 8) | ((uint32_t)(c2 & 255) << 16) |
                     ((uint32_t)(c3 & 255) << 24)};
    }
};
struct Cost16 {
    uint32_t lo, hi;
    __device__ __forceinline__ int32_t at(uint32_t x8) const {
        return __builtin_amdgcn_sbfe((int32_t)((x8 & 16) ? hi : lo), (x8 & 8) << 1, 16);
    }
    __device__ __forceinline__ static Cost16 make(int32_t c0, int32_t c1, int32_t c2, int32_t c3) {
        return Cost16{(uint32_t)(c0 & 0xFFFF) | ((uint32_t)(c1 & 0xFFFF) << 16),
                      (uint32_t)(c2 & 0xFFFF) | ((uint32_t)(c3 & 0xFFFF) << 16)};
    }
};

struct AlignParams {
    int32_t k, gap_open, gap_extend, min_overlap;
    float one_minus_minid, min_identity, max_ignore;
    int32_t cost[16];
    int32_t cost_bits;           // 8: Cost8 packs, 16: Cost16 packs (host: after the common-divisor reduction)
    uint32_t rw;                 // traceback words per column (odd)
};

struct DevAlignment {            // mirrors sa_alignment
    int32_t lead, trail, start_i, start_j, end_i, end_j, correct, error, ahg, bhg, flags, reserved;
};

// ---- launchers (kernels/*.hip) ------------------------------------------
hipError_t launch_pack_reads(const DevReads &r, hipStream_t s);
// pack + emit in one pass (reads of <= 1,024 bases)
hipError_t launch_pack_emit(const DevReads &r, const EmitParams &p, uint64_t *keys, hipStream_t s);
// pack_emit without records (KeyGen) that also writes p.hist (the first key-only radix
// pass's tile histogram at p.hist_shift, tiles of radix_key_tile() records); n = records
uint32_t radix_key_tile();
hipError_t launch_pack_emit_hist(const DevReads &r, const EmitParams &p, uint64_t n, hipStream_t s);
hipError_t launch_kmer_emit(const DevReads &r, const EmitParams &p, uint64_t *keys, uint32_t *vals,
                            hipStream_t s);

// stable LSD radix sort of (key, val) on key bits [lo, hi); ping-pong buffers,
// result ends in (*keys, *vals) (pointers may be swapped).  tmp: sized by
// radix_sort_temp_bytes.
size_t radix_sort_temp_bytes(uint64_t n);
hipError_t radix_sort(uint64_t **keys, uint32_t **vals, uint64_t **keys_alt, uint32_t **vals_alt,
                      uint64_t n, int lo, int hi, void *tmp, hipStream_t s);
// the same with 64-bit values (16-byte records)
// radix_sort (key-only) of the n records KeyGen g describes: the first pass
// generates its keys instead of loading them (the records are never written
// unsorted); result in *keys
hipError_t radix_sort_gen(const KeyGen &g, uint64_t **keys, uint64_t **keys_alt, uint64_t n, int lo, int hi,
                          void *tmp, hipStream_t s);
hipError_t radix_sort_kv64(uint64_t **keys, uint64_t **vals, uint64_t **keys_alt, uint64_t **vals_alt, uint64_t n,
                           int lo, int hi, void *tmp, hipStream_t s);

// Received records of the sharded path (sa_dist_count): record i in receive
// order is mix << 32 | its occurrence index local to its source rank.  The
// first pass of radix_sort_recv decodes each as it loads -- the record's read
// and loc rank become its value (read << lb | loc rank), its low word becomes i
// -- and writes the local read offsets loff[a] (first i with read >= a, a in
// [0, n_reads]): the relabelling pass (prepare_received) folded into the sort
struct RecvGen {
    const uint64_t *seg;      // [2P + 1]: seg[s] first record of source s (seg[P] = n); seg[P + 1 + s]
                              // the global occurrence index of source s's first k-mer
    uint32_t P;
    const uint32_t *starts;   // [P + 1] first global read of each source
    const uint64_t *occ_off;  // global occurrence offsets (mixed lengths)
    uint32_t npr;             // uniform k-mers per read (0: mixed)
    unsigned long long npr_magic;
    const int32_t *len;
    const uint32_t *lbase, *lrank;
    int32_t k;
    int lb;
    uint64_t *loff;
    uint32_t n_reads;
    int lr_ident;             // uniform lengths whose loc rank is the position (no table lookup)
    // src_shift > 0: source-relative values -- (read - starts[s]) << lb | loc rank, and the
    // record's top log2 P key bits (its owner's, the same on every record of this rank)
    // replaced by the source s; PartArgs::src_shift undoes both (record_key).  For read sets
    // whose global ids do not fit 32 - lb bits but every source's do (configs[3]: 10M reads
    // of 486 k-mers, 24 + 9 bits; 1.25M per source, 21 + 9)
    int src_shift;
};
// (key, u32 value) radix sort of received records, values generated (RecvGen)
hipError_t radix_sort_recv(const RecvGen &g, uint64_t **keys, uint32_t **vals, uint64_t **keys_alt,
                           uint32_t **vals_alt, uint64_t n, int lo, int hi, void *tmp, hipStream_t s);

// GNU Trove 3.0.3 layout (csrc/host/trove.h semantics, rehash chain included) of m distinct
// keys inserted in index order, built on the device (trove_replay.hip): out_order[j] = the
// index of the key in the j-th slot of iteration order (slot cap - 1 down to 0).  tmp:
// trove_temp_bytes(m); the final capacity in *final_cap
size_t trove_temp_bytes(uint32_t m);
hipError_t trove_layout_device(const int32_t *keys, uint32_t m, uint32_t *out_order, void *tmp, hipStream_t s,
                               uint32_t *final_cap);
// KmerData's bucket iteration ranks (rank[head position] = its place in the Trove layout of
// the buckets' seqHash values in first-occurrence order; 0 elsewhere), the head count in
// *n_heads; tmp: kmerdata_temp_bytes(n)
size_t kmerdata_temp_bytes(uint64_t n);
hipError_t kmerdata_rank_device(const uint8_t *is_head, const uint32_t *bkt_first, uint64_t n, const DevReads &rd,
                                const uint64_t *occ_off, uint32_t n_reads, int m_hash, uint32_t *rank, void *tmp,
                                hipStream_t s, uint32_t *n_heads);
// the pairs (f, s, k) whose count k is in [min_c, max_c], compacted in order into fo / so /
// ko; their number in *total (device); flag / ex: n u32, stmp: scan_temp_bytes(n)
hipError_t launch_trove_keep(const int32_t *f, const int32_t *s, const int32_t *k, uint32_t n, int32_t min_c,
                             int32_t max_c, uint32_t *flag, uint32_t *ex, uint32_t *total, void *stmp, int32_t *fo,
                             int32_t *so, int32_t *ko, hipStream_t st);
hipError_t launch_trove_pair_keys(const int32_t *f, const int32_t *s, uint32_t n, int32_t *keys, hipStream_t st);
hipError_t launch_trove_gather3(const uint32_t *order, uint32_t n, const int32_t *f, const int32_t *s, const int32_t *k,
                                int32_t *fo, int32_t *so, int32_t *ko, hipStream_t st);

// exclusive scan of u32 (in place allowed), returns total in *total_dev
size_t scan_temp_bytes(uint64_t n);
hipError_t exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total_dev,
                              void *tmp, hipStream_t s);

// bucket/list build from sorted keys; totals written to totals_dev[4] =
// {buckets, groups, md, ed}
size_t buckets_temp_bytes(uint64_t n);
hipError_t build_buckets(const uint64_t *skeys, const uint32_t *svals, uint64_t n, int lb,
                         const uint8_t *tagtab, const uint64_t *occ_off, uint32_t n_reads,
                         uint32_t uniform_npr, const uint2 *rl, Buckets &b,
                         uint32_t *totals_dev, void *tmp, hipStream_t s);
hipError_t build_strict_index(const uint64_t *skeys, const uint32_t *svals, uint64_t n, int lb,
                              const uint8_t *tagtab, Buckets &b, hipStream_t s);

hipError_t launch_pair_count(const EmitParams &e, const PairIn &in, const PairParams &p, PairOut &o,
                             const uint32_t *read_list, uint32_t n_blocks, hipStream_t s);
// sharded path: one WAVE per range of reads with ~PMW_TARGET local occurrences
// (launch_pc_items builds item_start[n_items + 1] from the occurrence offsets)
#ifndef SA_PMW_TARGET
#define SA_PMW_TARGET 128
#endif
constexpr uint32_t PMW_TARGET = SA_PMW_TARGET;
hipError_t launch_pair_count_multi_wave(const EmitParams &e, const PairIn &in, const PairParams &p, PairOut &o,
                                        const uint32_t *item_start, uint32_t n_items, uint32_t n_reads, hipStream_t s);
hipError_t launch_pc_item_owners(const uint32_t *item_start, uint32_t n_items, const uint32_t *starts, uint32_t owners,
                                 uint32_t *item_owner, hipStream_t s, const uint32_t *item_end = nullptr);
// lead-range passes (sa_dist_count_pass): items over the reads of nr ranges rg[2r] ..
// rg[2r + 1] only (ioff: nr + 1 u32, the count kernel's exclusive item offsets, ioff[nr] =
// items), then their starts and ends
hipError_t launch_pass_items_count(const uint64_t *occ_off, const uint32_t *rg, uint32_t nr, uint32_t target,
                                   uint32_t *ioff, hipStream_t s);
hipError_t launch_pass_items_fill(const uint64_t *occ_off, const uint32_t *rg, uint32_t nr, uint32_t target,
                                  const uint32_t *ioff, uint32_t n_items, uint32_t *istart, uint32_t *iend,
                                  hipStream_t s);
// per-read upper bound of the partials each read leads on this rank (bound[n_reads]),
// summed per lead owner into own[0 .. owners) and in all into own[owners]
hipError_t launch_read_bound(const uint64_t *occ_off, uint32_t n_reads, const PairIn &in, const uint32_t *starts,
                             uint32_t owners, uint64_t *bound, unsigned long long *own, hipStream_t s,
                             const uint32_t *abort = nullptr);
hipError_t launch_pc_items(const uint64_t *occ_off, uint32_t n_reads, uint32_t target, uint32_t n_items,
                           uint32_t *item_start, hipStream_t s);

// ---- partition bucket build (partition.hip) ------------------------------
struct PartArgs {
    const uint64_t *sk;
    const uint32_t *sv;
    const uint32_t *start;       // [np+1]
    uint32_t np;
    int lb;
    int sort_bits;               // key bits below the partition id (sorted in LDS)
#ifdef SA_PB_STAMPS
    uint64_t *stamps;            // (timing probe builds: 8 words per partition of the main pass)
#endif
#ifdef SA_PB_PROBE_DUP
    uint2 *rec_dup;              // (bandwidth probe builds: every record stored a second time here)
#endif
    const uint8_t *tagtab;
    const uint64_t *occ_off;
    uint32_t n_reads, npr;
    uint64_t npr_magic;          // floor((2^64 - 1) / npr) + 1 (npr >= 2): read_of_g's division
    const uint2 *rl;             // {read, loc rank} by occurrence index (distributed mode, mixed lengths) or null
    const uint2 *srl;            // the same, sorted with the records (aligned with sk) or null
    // or packed into 4 bytes when read bits + lb <= 32 (12-byte records through
    // the partition sort instead of 16): read << lb | loc rank, by occurrence
    // index (pv) and sorted with the records (spv)
    const uint32_t *pv, *spv;
    // source-relative packed values (RecvGen::src_shift): the source s sits in the key's top
    // bits from src_shift on; the read is src_starts[s] + (value >> lb) and the key's top bits
    // are the owner's again (src_own: those bits of this rank's high key words)
    int32_t src_shift;
    uint32_t src_own;
    const uint32_t *src_starts;
    // sk holds 8-byte records (mix32 << 32 | occurrence index); the loc rank is
    // rl[g].y when given (distributed mode, mixed lengths), else re-derived from
    // the read's length and the position (lrank[lbase[L - k] + pos])
    const int32_t *len;
    const uint32_t *lbase, *lrank;
    int32_t k;
    // uniform lengths whose loc ranks are the positions themselves (no NaN loc):
    // lrank[lbase[npr - 1] + pos] == pos, so the rank needs no dependent gather
    int32_t lr_ident;
    // the tags as loc-rank intervals (tagtab is three runs in rank order: st a
    // prefix, md an interval, en an interval ending below the NaN rank):
    // tag = [lr < tg_st] st | [lr - tg_md0 < tg_mdn] md | [lr - tg_en0 < tg_enn] en;
    // tg_on = 0: look tagtab up instead
    int32_t tg_on;
    uint32_t tg_st, tg_md0, tg_mdn, tg_en0, tg_enn;
    // mixed read lengths, wide ids: records carry read << pos_bits | pos and
    // meta[read] = {first occurrence index, lrank offset of its length}
    int32_t pos_bits;
    const uint2 *meta;
    uint32_t *lst;               // combined partner list [3 n]
    uint2 *rec;                  // [n_occ] by g
    uint4 *xrec;                 // escape records (big partitions only)
    uint32_t *xrec_n;
    uint32_t *big_list, *big_n;  // partitions above 4,096 records (global path)
    uint32_t *mid_list, *mid_n;    // partitions above 1,024 records (2,048-record LDS pass)
    uint32_t *mid2_list, *mid2_n;  // partitions above 2,048 records (4,096-record LDS pass)
    // split tier (split = 1): the partitions of 1,025-2,048 records are built as two
    // halves by the next hash bit by 1,024-record blocks; the ones whose halves do
    // not fit go to the 2,048-record pass through fb_list
    uint32_t *fb_list, *fb_n;
    int32_t split;
    unsigned long long *counts;  // [2][NSHARD]: buckets, groups
    // strict
    uint32_t *lidx;              // parallel to lst
    uint4 *srec;                 // [n_occ] by g
    uint32_t *bkt_nst, *bkt_nmd, *bkt_first;  // at bucket head sorted positions
    uint8_t *is_head;            // [n] head flags
};
// the tag of loc rank lr (tagtab[lr], by intervals when tg_on)
__device__ __forceinline__ uint32_t part_tag(const PartArgs &A, uint32_t lr) {
    if (!A.tg_on) return A.tagtab[lr];
    return (lr < A.tg_st ? (uint32_t)TAG_ST : 0u) | (lr - A.tg_md0 < A.tg_mdn ? (uint32_t)TAG_MD : 0u) |
           (lr - A.tg_en0 < A.tg_enn ? (uint32_t)TAG_EN : 0u);
}
hipError_t launch_part_starts(const PartArgs &a, uint64_t n, int shift, hipStream_t s);
hipError_t launch_part_build(const PartArgs &a, bool strict, int cap, hipStream_t s);
// 8-byte records of one big partition -> (mix << lb | locrank, g) for the global scan path
hipError_t launch_convert_records(const uint64_t *rec8, uint32_t n, const PartArgs &a, uint64_t *okeys,
                                  uint32_t *ovals, uint32_t ps, hipStream_t s);
// big partition at sorted offset ps: its temporary (ascending, partition-
// relative) md / edge lists of the global scan moved into the combined layout
// (and the strict list indices with them), then the per-occurrence records
hipError_t launch_relayout_lists(const Buckets &b, uint32_t ps, uint32_t n, const uint32_t *totals_dev,
                                 const PartArgs &a, bool strict, hipStream_t s);
hipError_t launch_records_from_tables(const uint64_t *sk, const uint32_t *sv, uint32_t ps, uint32_t n, int lb,
                                      const uint8_t *tagtab, const Buckets &b, const PartArgs &a, int strict,
                                      hipStream_t s);

// compact the NSHARD output regions into sort keys (vals = region-space index)
hipError_t launch_make_order_keys(const uint32_t *fst, const uint32_t *snd, const uint64_t *rank,
                                  const unsigned long long *cursor, unsigned long long cap_s, int by_rank,
                                  int idbits, uint64_t *keys, uint32_t *vals, uint32_t *shard_off,
                                  hipStream_t s, const uint32_t *starts = nullptr, uint32_t P = 0);
// per-read mode: the dispatch list (lead descending, trail ascending) from the
// per-read regions; ex = exclusive scan of rcnt, total = its sum.  Reads the
// recount tiers handled take their pairs from the sorted shared list instead:
// rsh[read] = 1 + its segment's start in (sh_trail, sh_count) (0: region)
hipError_t launch_copy_read_regions(const uint2 *rreg, const uint32_t *rcnt, const uint32_t *ex,
                                    const uint32_t *total, uint32_t n_reads, const uint32_t *rsh,
                                    const int32_t *sh_trail, const int32_t *sh_count, int32_t *lead, int32_t *trail,
                                    int32_t *count, hipStream_t s);
// segments of a lead-descending (1-based) lead list: rsh[lead - 1] = 1 + start,
// rcnt[lead - 1] = length
hipError_t launch_mark_segments(const int32_t *lead, uint64_t n, uint32_t *rsh, uint32_t *rcnt, hipStream_t s);
hipError_t launch_gather_pairs(const uint32_t *perm, uint64_t n, const uint32_t *fst, const uint32_t *snd,
                               const uint32_t *cnt, int32_t *lead, int32_t *trail, int32_t *count,
                               hipStream_t s);

hipError_t launch_dovetail(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                           const AlignParams &p, int group_lanes, DevAlignment *out, int32_t *err,
                           unsigned long long *cells, hipStream_t s);
// one pair per lane, band held in LW = 16 / 24 / 32 registers (w <= LW - 1),
// |A| <= 30000 (dovetail_lane.hip); exact (LW 16 only): w == 15 for every
// pair.  dovetail_lane_width(wmax) = the LW for the widest band (0: none fits).
// Phase 1 writes p1 / rows2_key / order (identity); the host sorts
// (rows2_key, order) and phase 2 takes pairs in that order.
int dovetail_lane_width(int32_t wmax);
hipError_t launch_dovetail_p1(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                              const AlignParams &p, int lw, bool exact, int32_t *p1, uint64_t *rows2_key,
                              uint32_t *order, int32_t *err, unsigned long long *cells, hipStream_t s);
// phase 1 with two pairs per lane in packed 16-bit halves (band exactly 16
// cells, int8 costs, gap costs <= 0, every score < 2^16 - 256: the caller checks)
hipError_t launch_dovetail_p1x2(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                                const AlignParams &p, int32_t *p1, uint64_t *rows2_key, uint32_t *order, int32_t *err,
                                unsigned long long *cells, hipStream_t s);
// phase 1 (two pairs per lane) in nseg row segments of every 64-lane group, one ticketed
// one-wave workgroup per (segment, group): ticket_flags = 1 + dovetail_p1x2_groups(n) u32,
// state = dovetail_p1x2_state_words(n) u32 (unused when nseg == 1)
uint32_t dovetail_p1x2_groups(uint64_t n);
size_t dovetail_p1x2_state_words(uint64_t n);
hipError_t launch_dovetail_p1x2_seg(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                                    const AlignParams &p, int32_t *p1, uint64_t *rows2_key, uint32_t *order,
                                    int32_t *err, unsigned long long *cells, int32_t nseg, uint32_t *ticket_flags,
                                    uint32_t *state, hipStream_t s);
hipError_t launch_dovetail_p2(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                              const AlignParams &p, int lw, bool exact, const int32_t *p1, const uint32_t *order,
                              DevAlignment *out, int32_t *err, hipStream_t s);
// phase 2 with traceback codes in HBM: lanes t0 .. t0+nt of the order, nt
// rounded up to 64; tb = dovetail_tb_words(nt, longest lead, lw) u32 words
size_t dovetail_tb_words(uint64_t nt, int32_t max_len, int lw);
// two pairs per lane (packed 16-bit; lw 16 EXACT, int8 costs, gaps <= 0, scores and
// argmax rows within 16 bits): 8 rows of codes per pair per word
size_t dovetail_tbx2_words(uint64_t nt, int32_t max_len);
hipError_t launch_dovetail_p2tbx2(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                                  uint64_t t0, uint64_t nt, const AlignParams &p, const int32_t *p1,
                                  const uint32_t *order, DevAlignment *out, int32_t *err, uint32_t *tb,
                                  hipStream_t s);
hipError_t launch_dovetail_p2tb(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                                uint64_t t0, uint64_t nt, const AlignParams &p, int lw, bool exact, const int32_t *p1,
                                const uint32_t *order, DevAlignment *out, int32_t *err, uint32_t *tb,
                                hipStream_t s);

// full-matrix local alignment (`--quadratic-align`, local_align.hip): pairs
// p0 .. p0+np of the dispatch list; stripe S = columns per lane (4/8/16/32,
// trails <= 64*S bp), wpl = code words per lane for the longest lead
// (local_align_wpl), tb = np * 64 * wpl u32 words, lmax = np int4 scratch
int local_align_stripe(int32_t max_len);
uint32_t local_align_wpl(int stripe, int32_t max_len);
hipError_t launch_local_align(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t p0,
                              uint64_t np, const AlignParams &p, int stripe, uint32_t wpl, uint32_t *tb, int4 *lmax,
                              DevAlignment *out, int32_t *err, unsigned long long *cells, hipStream_t s);

// k-mer table statistics (kmer_hist.hip): records sorted on their top 32 bits
// -> distinct hashes (*nheads) and hist[s] = hashes with s occurrences for
// s < KMER_HIST_CAP, larger sizes appended to ovf[0 .. *novf).  flag / idx /
// pos: n u32 each; scan_tmp: scan_temp_bytes(n).
constexpr uint32_t KMER_HIST_CAP = 1u << 16;
hipError_t launch_kmer_hist(const uint64_t *sorted, uint64_t n, uint32_t *flag, uint32_t *idx, uint32_t *pos,
                            uint32_t *nheads, void *scan_tmp, unsigned long long *hist, unsigned long long *ovf,
                            uint32_t *novf, hipStream_t s);

// distributed (multi-GPU) glue, dist.hip
hipError_t launch_iota(uint32_t *v, uint64_t n, hipStream_t s);
// rl[i] = {read, loc rank}; or, with pv, pv[i] = read << lb | loc rank.  With
// loff, also the read offsets loff[a] whose boundary falls inside a wave;
// launch_local_offsets (same rl / pv, loff) then fills in the rest
hipError_t launch_prepare_received(uint64_t *recs, uint64_t n, const uint64_t *seg, uint32_t P,
                                   const uint32_t *starts, const uint64_t *occ_off, uint32_t npr, const int32_t *len,
                                   const uint32_t *lbase, const uint32_t *lrank, int32_t k, uint2 *rl,
                                   uint32_t *pv, int lb, uint64_t *loff, hipStream_t s);
hipError_t launch_local_offsets(const uint2 *rl, const uint32_t *pv, int lb, uint64_t n, uint32_t n_reads,
                                uint64_t *loff, hipStream_t s);
hipError_t launch_owner_bounds(const uint64_t *keys, uint64_t n, int shift, uint32_t P, uint64_t *bounds,
                               hipStream_t s);
// the owner regions of the partials (PairOut::owners), concatenated in region
// order (owner-major): region r's min(cursor[r], cap_s) entries to out + off[r]
hipError_t launch_copy_owner_regions(const uint32_t *fst, const uint32_t *snd, const uint32_t *cnt,
                                     unsigned long long cap_s, uint32_t n_regions, const unsigned long long *cursor,
                                     const uint64_t *off, uint32_t *of, uint32_t *os, uint32_t *oc,
                                     uint64_t max_fill, hipStream_t s);
hipError_t launch_reduce_keys(const uint32_t *fst, const uint32_t *snd, uint64_t n, int idb, uint64_t *keys,
                              uint32_t *vals, hipStream_t s);
hipError_t launch_reduce_heads(const uint64_t *skeys, const uint32_t *sidx, uint64_t n, const uint32_t *cnt,
                               int32_t min_c, int32_t max_c, uint32_t *sum, uint32_t *keep,
                               unsigned long long *distinct, hipStream_t s);
// owner-side reduce by lead: per-lead segments of the received partials, LDS
// aggregation per lead (kcnt = kept pairs, written trail-ascending over the
// segment start): one wave per lead (192 partners), then one wave per lead with
// 1,024 slots (768), the leads beyond one block each (3,072); *overflow set when a
// lead has more (the caller then sorts); lcnt / lcur: nl u32, loff: nl + 1 u32,
// seg: n uint2, ranks: the partials' senders (routing: a lead has at least
// m / ranks distinct partners), total_dev: n (the scan total)
hipError_t launch_lead_reduce(const uint32_t *fst, const uint32_t *snd, const uint32_t *cnt, uint64_t n, uint32_t base,
                              uint32_t nl, int32_t min_c, int32_t max_c, uint32_t *lcnt, uint32_t *loff, uint32_t *lcur,
                              uint2 *seg, uint32_t *kcnt, unsigned long long *distinct, uint32_t *overflow,
                              uint32_t ranks, float route, void *scan_tmp, uint32_t *total_dev, hipStream_t s);
// the lead-descending dispatch from the reduced segments (kex = exclusive scan
// of kcnt, total = its sum); ids 1-based, lead = base + l + 1
hipError_t launch_lead_copy(const uint2 *seg, const uint32_t *loff, const uint32_t *kcnt, const uint32_t *kex,
                            const uint32_t *total, uint32_t nl, uint32_t base, int32_t *lead, int32_t *trail,
                            int32_t *count, hipStream_t s);
hipError_t launch_reduce_compact(const uint64_t *skeys, uint64_t n, int idb, const uint32_t *sum, const uint32_t *keep,
                                 const uint32_t *pos, int32_t *lead, int32_t *trail, int32_t *count, hipStream_t s);

}  // namespace sa
