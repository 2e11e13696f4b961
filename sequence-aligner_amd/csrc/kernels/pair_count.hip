// pair_count.hip -- edge<->middle candidate-pair counting and collision filter.
//
// Device replacement of KmerTable.calcPairData / addKmerPair / calcDispatchData
// (KmerTable.scala:57-187).  Organised by the pair's FIRST read (the occurrence
// with the larger loc, KmerTable.scala:65-71): one workgroup per read `a`
// enumerates exactly the role pairs whose fst is `a` --
//   each edge (st/en) k-mer of a  x  middle k-mers of its bucket with loc <  own
//   each middle k-mer of a        x  edge roles of its bucket with loc <= own
// -- so every (st x md) / (en x md) pair of the reference is visited once, by
// the read that becomes `fst`, and all counts of key (a, b) land in ONE LDS hash
// table: no global atomics, no role-pair materialisation.  The [min, max]
// collision filter is applied on chip.  Strict mode also tracks each key's
// first-occurrence rank in calcPairData's traversal order, from which the host
// replays GNU Trove's PairData layout.
// Each k-mer's partner ranges arrive as one coalesced 8-byte record
// (partition.hip; decode_rec, sa_internal.h).  Work is load-balanced inside the workgroup over the prefix
// sum of per-k-mer partner counts; partner ids are gathered PC_BATCH at a time.
// Bound: gather latency / LDS atomics; HBM bytes are small.
#include "../sa_internal.h"

#include <type_traits>

namespace sa {

constexpr int PC_THREADS = 256;
// LDS hash slots per read: a read has ~20-60 distinct partners at 20x coverage,
// so the first pass runs a 256-slot table (small LDS -> 8 workgroups per CU);
// reads that fill it (repeats, random short-k collisions) are re-run with 2,048
// slots, then 16,384 (128 KB of LDS: one workgroup per CU; wide ids only), then
// split into partner-residue classes
constexpr int PC_TAB_SMALL = 256;
constexpr int PC_TAB_BIG = 2048;
constexpr int PC_TAB_HUGE = 16384;
// the packed form of the big tier (wide ids, partners < 2^24 - 1, max_coll <=
// 255): one word per slot, partner | count << 24, and a bitmap of the slots
// whose 8-bit count wrapped (count > 255: never inside [min, max]); 32,768
// slots (24,576 partners at 3/4 load) in the 16,384-slot tier's 128 KB, so
// configs[4]'s k = 12 reads (~24k partners at the 6.25M slice) need one pass
// where the two-word table needed two or three (one per partner-residue class)
constexpr int PC_TAB_HUGE2 = 32768;
constexpr int PC_CHUNK = 512;            // occurrences per pass over a read
constexpr int PC_BATCH = 8;              // partner loads in flight per thread
// the per-occurrence records are read once: non-temporal loads keep them from
// displacing the partner lists in L2
__device__ __forceinline__ uint2 load_rec_raw(const PairIn &in, uint64_t g) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 w = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(in.rec + g));
    return make_uint2(w.x, w.y);
}
__device__ __forceinline__ uint4 load_rec(const PairIn &in, uint64_t g) {
    return decode_rec(load_rec_raw(in, g), in.xrec);
}
constexpr uint32_t PC_EMPTY = 0xFFFFFFFFu;
constexpr int PC_PROBE_MAX = 256;

template <int TAB>
__device__ __forceinline__ uint32_t pc_hash(uint32_t p) {
    return (p * 0x9E3779B1u) >> (32 - __builtin_ctz((unsigned)TAB));
}

// the rank owning read a: largest o with starts[o] <= a (owners ranks, starts[owners] = reads)
__device__ __forceinline__ uint32_t owner_of(const uint32_t *starts, uint32_t owners, uint32_t a) {
    uint32_t lo = 0, hi = owners;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (starts[mid] <= a) lo = mid; else hi = mid;
    }
    return lo;
}

// Elements (role pairs) of a chunk are enumerated in windows of PC_WIN; eo[e]
// = 1 + the occurrence holding element w0 + e, filled by the thread owning the
// occurrence (its element range is in its registers: no scan, one barrier).
constexpr int PC_WIN = 2048;

// Per-table block shape.  The 16,384-slot tier holds 128 KB of table, so only
// one block fits a CU: it runs 1,024 threads (16 waves to hide the partner
// gathers, not 4), 1,024-occurrence chunks and 6,144-element windows (6
// partner loads in flight per thread: the packed tier's LDS holds 12 KB of
// window map beside its 128 KB table; 8 would pass the 160 KB; the two-word
// 16,384-slot table keeps 4); the smaller tables keep 256 threads.
#ifndef PC_HUGE_CHUNK
#define PC_HUGE_CHUNK 1024
#endif
#ifndef PC_HUGE_BATCH
#define PC_HUGE_BATCH 6  // (configs[4]'s k = 12 slice, pairs stage: 4 -> 5.79 s, 5 -> 5.57, 6 -> 5.51)
#endif
template <int TAB> struct PcShape {
    static constexpr int NT = TAB >= PC_TAB_HUGE ? 1024 : PC_THREADS;
    static constexpr bool PACKED = TAB >= PC_TAB_HUGE2;
    static constexpr int CHUNK = TAB >= PC_TAB_HUGE ? PC_HUGE_CHUNK : PC_CHUNK;
    // (the two-word 16,384-slot table fills 128 KB with keys and counts: 4 loads,
    // 4,096-element windows, or the block passes 160 KB of LDS)
    static constexpr int BATCH = TAB >= PC_TAB_HUGE2 ? PC_HUGE_BATCH : TAB >= PC_TAB_HUGE ? 4 : PC_BATCH;
    static constexpr int WIN = TAB >= PC_TAB_HUGE ? 1024 * BATCH : PC_WIN;
};

template <int TAB>
struct PcShared {
    static constexpr int NT = PcShape<TAB>::NT, CHUNK = PcShape<TAB>::CHUNK;
    static constexpr bool PACKED = PcShape<TAB>::PACKED;
    uint32_t key[TAB];         // packed: partner | count << 24
    uint32_t cnt[PACKED ? 1 : TAB];
    uint32_t sat[PACKED ? TAB / 32 : 1];  // packed: the slot's count wrapped past 255
    uint32_t pref[CHUNK + 1];
    // per-occurrence partner ranges (partition.hip): decoded, or (packed, to fit
    // the LDS) the raw 8-byte records, decoded where an element is read
    typename std::conditional<PACKED, uint2, uint4>::type rec[CHUNK];
    uint16_t eo[PcShape<TAB>::WIN];  // element -> occurrence (+1) of the current window
    uint32_t lds4[NT / 64];
    uint32_t emit4[2][NT / 64];  // emission: per-wave kept counts (double-buffered)
    uint32_t emit_base[2];
    uint32_t fill, overflow, out_base;
    uint32_t xfill;            // role-pair index (within the read) of the insert that filled the table
};
template <int TAB>
struct PcSharedStrict {
    unsigned long long rank[TAB];
    uint4 srec[PcShape<TAB>::CHUNK];  // {bucket head pos, own_e, own_m, 0}
};

template <int NT = PC_THREADS>
__device__ __forceinline__ uint32_t pc_block_excl_scan(uint32_t v, uint32_t *lds4, uint32_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_add(v);
    if (lane == 63) lds4[w] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) {
        const uint32_t x = lds4[i];
        if (i < w) off += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

__device__ __forceinline__ uint4 pc_rec(const uint4 &r, const PairIn &) { return r; }
__device__ __forceinline__ uint4 pc_rec(const uint2 &r, const PairIn &in) { return decode_rec(r, in.xrec); }

// Returns whether the insert created the key.  The table's fill is counted by
// the caller, one LDS atomic per wave and batch (pc_fill).
//
// The recount tiers (TAB >= 2,048) probe in 16-byte buckets of four slots: one
// LDS round trip reads a bucket, the insert takes its first empty slot.  A
// lane's probes are a chain of dependent LDS reads, and a wave waits for its
// longest chain: near 3/4 load, slot-by-slot linear probing made that tail
// tens of round trips per insert (configs[4]'s k = 12 reads, whose inserts
// mostly create keys, spent ~200 us per read in the 32,768-slot tier).  Keys
// only ever go EMPTY -> key, and always into the first empty slot of the probe
// order, so the filled slots are a prefix of it: a scan stops at the first
// match or empty slot, and a CAS that loses to another key re-reads the bucket.
template <int TAB>
__device__ __forceinline__ bool pc_key_is(uint32_t word, uint32_t partner) {
    if constexpr (PcShape<TAB>::PACKED) return (word & 0xFFFFFFu) == partner;  // (EMPTY's low bits are not an id)
    else return word == partner;
}

template <bool STRICT, int TAB>
__device__ __forceinline__ void pc_hit(PcShared<TAB> &S, PcSharedStrict<TAB> &X, uint32_t slot, uint32_t w,
                                       unsigned long long rank) {
    if constexpr (PcShape<TAB>::PACKED) {  // count << 24, wrap -> the slot's saturation bit
        const uint32_t prev = atomicAdd(&S.key[slot], w << 24);
        if ((prev >> 24) + w > 255u) atomicOr(&S.sat[slot >> 5], 1u << (slot & 31));
    } else {
        atomicAdd(&S.cnt[slot], w);
        if constexpr (STRICT) atomicMin(&X.rank[slot], rank);
    }
}

template <bool STRICT, int TAB>
__device__ __forceinline__ bool pc_insert(PcShared<TAB> &S, PcSharedStrict<TAB> &X, uint32_t partner, uint32_t w,
                                          unsigned long long rank) {
    if constexpr (TAB >= PC_TAB_BIG) {
        const uint32_t fresh = PcShape<TAB>::PACKED ? partner | (w << 24) : partner;
        uint32_t b = pc_hash<TAB>(partner) & ~3u;
        // bounded: a retry means another key took a slot of this bucket (<= 4 per
        // bucket), and a run of PC_PROBE_MAX / 4 buckets only happens in a table
        // that is (nearly) full -- then recounted by a finer class
        for (int it = 0; it < PC_PROBE_MAX; ++it) {
            if ((it & 7) == 7 && lds_relaxed(&S.overflow)) return false;
            // the bucket as two relaxed 8-byte loads (ds_read_b64: half the LDS
            // instructions of four word loads; each word is read atomically)
            const uint64_t k01 = lds_relaxed(reinterpret_cast<uint64_t *>(&S.key[b]));
            const uint64_t k23 = lds_relaxed(reinterpret_cast<uint64_t *>(&S.key[b + 2]));
            const uint32_t k[4] = {(uint32_t)k01, (uint32_t)(k01 >> 32), (uint32_t)k23, (uint32_t)(k23 >> 32)};
            int at = 4;
            bool hit = false;
#pragma unroll
            for (int i = 3; i >= 0; --i) {  // the first match or empty slot
                if (pc_key_is<TAB>(k[i], partner)) { at = i; hit = true; }
                else if (k[i] == PC_EMPTY) { at = i; hit = false; }
            }
            if (at == 4) {  // bucket full of other keys: the next one
                b = (b + 4) & (TAB - 1);
                continue;
            }
            if (hit) {
                pc_hit<STRICT, TAB>(S, X, b + at, w, rank);
                return false;
            }
            const uint32_t old = atomicCAS(&S.key[b + at], PC_EMPTY, fresh);
            if (old == PC_EMPTY) {
                if constexpr (!PcShape<TAB>::PACKED) pc_hit<STRICT, TAB>(S, X, b + at, w, rank);
                return true;
            }
            if (pc_key_is<TAB>(old, partner)) {
                pc_hit<STRICT, TAB>(S, X, b + at, w, rank);
                return false;
            }
            // another key took the slot: read the bucket again
        }
        S.overflow = 1;
        return false;
    } else {
        uint32_t slot = pc_hash<TAB>(partner);
        // probe runs are bounded: at <= 3/4 load they average < 9 slots, and a
        // run of TAB / 4 only happens in a table that is (nearly) full -- it is
        // then recounted by a bigger tier, so every insert stays O(TAB / 4)
        constexpr int PMAX = TAB / 4 < PC_PROBE_MAX ? TAB / 4 : PC_PROBE_MAX;
        for (int probe = 0; probe < PMAX; ++probe) {
            // a slot's key goes EMPTY -> partner once and never changes again, so a
            // plain LDS read that sees a key is final: hits (>99% of inserts at 20x --
            // a read meets each partner in ~100 shared k-mers) take one atomic, not
            // two, and the CAS only runs on a slot that still reads EMPTY
            uint32_t old = lds_relaxed(&S.key[slot]);
            if (old == PC_EMPTY) old = atomicCAS(&S.key[slot], PC_EMPTY, partner);
            if (old == PC_EMPTY || old == partner) {
                pc_hit<STRICT, TAB>(S, X, slot, w, rank);
                return old == PC_EMPTY;
            }
            slot = (slot + 1) & (TAB - 1);
        }
        S.overflow = 1;
        return false;
    }
}

// the wave's new keys of one batch into the fill count: past 3/4 of the table
// the block is recounted by the next tier (xfill: the batch's first element,
// the role-pair index where the table was found full)
template <int TAB>
__device__ __forceinline__ void pc_fill(PcShared<TAB> &S, uint32_t newk, uint32_t eidx) {
    constexpr uint32_t FILL_MAX = pc_fill_max(TAB);
    const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_add(newk), 63);
    if ((threadIdx.x & 63) == 0 && wtot) {
        const uint32_t old = atomicAdd(&S.fill, wtot);
        if (old + wtot > FILL_MAX) {
            S.overflow = 1;
            atomicMin(&S.xfill, eidx);
        }
    }
}

template <bool STRICT, int TAB>
__global__ __launch_bounds__(PcShape<TAB>::NT) void pair_count_kernel(EmitParams e, PairIn in, PairParams p, PairOut o,
                                                                const uint32_t *read_list) {
    extern __shared__ __align__(16) uint8_t smem[];
    PcShared<TAB> &S = *reinterpret_cast<PcShared<TAB> *>(smem);
    PcSharedStrict<TAB> &X =
        *reinterpret_cast<PcSharedStrict<TAB> *>(smem + ((sizeof(PcShared<TAB>) + 15) & ~size_t(15)));
    constexpr int NT = PcShape<TAB>::NT, CHUNK = PcShape<TAB>::CHUNK, WIN = PcShape<TAB>::WIN,
                  BATCH = PcShape<TAB>::BATCH;
    const int tid = threadIdx.x;
    const uint32_t split = (uint32_t)p.split;
    uint32_t bid = blockIdx.x;
    if (p.xcd_swizzle) {
        // blocks are dealt round-robin over the 8 XCDs: give each XCD a contiguous
        // run of the (locality-sorted) read list so overlapping reads share its L2
        bid = (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    }
    if (bid >= p.n_items) return;  // whole block: before any barrier
    if (p.abort && *p.abort) return;
    // recount tiers take codes (read << 6 | residue class); the first pass reads
    uint32_t a, residue;
    if (p.coded) {
        const uint32_t code = read_list[bid];
        a = code >> 6;
        residue = code & 63u;
    } else {
        a = read_list ? read_list[bid] : bid;
        residue = 0;
    }

    for (int i = tid; i < TAB; i += NT) {
        S.key[i] = PC_EMPTY;
        if constexpr (!PcShape<TAB>::PACKED) S.cnt[i] = 0;
        if constexpr (STRICT) X.rank[i] = ~0ull;
    }
    if constexpr (PcShape<TAB>::PACKED)
        for (int i = tid; i < TAB / 32; i += NT) S.sat[i] = 0;
    if (tid == 0) { S.fill = 0; S.overflow = 0; S.xfill = 0xFFFFFFFFu; }

    // (uniform lengths: no dependent offset load before the record loads)
    const uint64_t g0 = e.npr ? (uint64_t)a * e.npr : e.occ_off[a];
    const uint32_t nocc = e.npr ? e.npr : (uint32_t)(e.occ_off[a + 1] - g0);
    unsigned long long role_pairs = 0;
    unsigned long long x_over = ~0ull;  // role pairs enumerated when the table filled
    unsigned long long early_est = 0;   // early stop: the projected distinct partners
    // (the table initialisation is ordered before any insert by the chunk scan's barriers)

    for (uint32_t c0 = 0; c0 < nocc; c0 += CHUNK) {
        const uint32_t cn = min((uint32_t)CHUNK, nocc - c0);
        // --- per-occurrence partner ranges: one 8-byte record each
        constexpr int PER = CHUNK / NT;
        uint32_t mytot[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t oi = tid * PER + j;  // thread-contiguous
            uint32_t tot = 0;
            if (oi < cn) {
                uint4 rc;
                if constexpr (PcShape<TAB>::PACKED) {
                    const uint2 raw = load_rec_raw(in, g0 + c0 + oi);
                    S.rec[oi] = raw;
                    rc = decode_rec(raw, in.xrec);
                } else {
                    rc = load_rec(in, g0 + c0 + oi);
                    S.rec[oi] = rc;
                }
                tot = (rc.y & 0x3FFFFFFFu) + rc.w;
                if constexpr (STRICT) X.srec[oi] = in.srec[g0 + c0 + oi];
            }
            mytot[j] = tot;
        }
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) s += mytot[j];
        uint32_t total;
        uint32_t ex = pc_block_excl_scan<NT>(s, S.lds4, &total);
        uint32_t myex[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t oi = tid * PER + j;
            if (oi <= cn) S.pref[oi] = ex;
            myex[j] = ex;
            ex += mytot[j];
        }
        if (tid == NT - 1 && cn == CHUNK) S.pref[CHUNK] = total;
        role_pairs += total;

        // --- lane-interleaved enumeration: consecutive lanes take consecutive
        //     elements, so a wave's partner loads walk one occurrence's list range
        //     (a few cache lines per instruction, not 64)
        for (uint32_t w0 = 0; w0 < total; w0 += WIN) {
            __syncthreads();  // pref / rec written; the previous window's eo consumed
            // an overflowed table is recounted by the next tier: skip the rest of
            // the enumeration (the chunk totals -- role pairs -- are still summed)
            if (S.overflow) {
                if (x_over == ~0ull) x_over = role_pairs - total + w0;
                break;
            }
            // Big tiers: a read that will not fit is found early.  Partners are met
            // no later than they recur, so fill(x) / x over the first x of the read's
            // role pairs is at least distinct / total -- the projection over-reads,
            // and a read only stops when it is past the fill limit by the margin.
            // (One-chunk reads: total is the read's; S.fill is final for the windows
            // before this barrier and the same for every thread.)
            if constexpr (TAB >= PC_TAB_HUGE) {
                if (p.early && nocc <= (uint32_t)CHUNK && w0 >= total / (uint32_t)(p.early >> 8) && w0 > 0) {
                    const unsigned long long proj = (unsigned long long)S.fill * total / w0;
                    if (proj * 8 > (unsigned long long)pc_fill_max(TAB) * (unsigned)(p.early & 255)) {
                        early_est = proj;
                        x_over = w0;
                        if (tid == 0) S.overflow = 1;  // (read again only after the chunk's barrier)
                        break;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < PER; ++j) {  // this thread's occurrences' elements inside the window
                const uint32_t e0 = max(myex[j], w0), e1 = min(myex[j] + mytot[j], w0 + (uint32_t)WIN);
                const uint16_t v = (uint16_t)(tid * PER + j + 1);
                for (uint32_t el = e0; el < e1; ++el) S.eo[el - w0] = v;
            }
            __syncthreads();
            const uint32_t wn = min((uint32_t)WIN, total - w0);
            for (uint32_t e0 = 0; e0 < wn; e0 += NT * BATCH) {
                uint32_t part[BATCH], wv[BATCH];
                unsigned long long rk[BATCH];
#pragma unroll
                for (int bb = 0; bb < BATCH; ++bb) {
                    part[bb] = a;  // "same read" = skip
                    wv[bb] = 0;
                    rk[bb] = 0;
                    const uint32_t el = e0 + bb * NT + tid;
                    if (el < wn) {
                        const uint32_t oi = (uint32_t)S.eo[el] - 1u;
                        const uint32_t off = w0 + el - S.pref[oi];
                        const uint4 rc = pc_rec(S.rec[oi], in);
                        const uint32_t nE = rc.y & 0x3FFFFFFFu;
                        const uint64_t q = rec_entry(rc, off);
                        part[bb] = in.lst[q];
                        if (off < nE) {
                            wv[bb] = rc.y >> 30;
                            if constexpr (STRICT) {
                                const uint4 sr = X.srec[oi];
                                const uint32_t hb = sr.x;
                                const uint32_t nmd = in.bkt_nmd[hb], nst = in.bkt_nst[hb];
                                const unsigned long long within =
                                    (unsigned long long)(sr.y >> 31) * nst * nmd +
                                    (unsigned long long)(sr.y & 0x7FFFFFFFu) * nmd + in.lidx[q];
                                rk[bb] = ((unsigned long long)in.bkt_rank[hb] << 37) | within;
                            }
                        } else {
                            wv[bb] = 1;
                            if constexpr (STRICT) {
                                const uint4 sr = X.srec[oi];
                                const uint32_t hb = sr.x;
                                const uint32_t nmd = in.bkt_nmd[hb], nst = in.bkt_nst[hb];
                                const uint32_t pe = in.lidx[q];
                                const unsigned long long within =
                                    (unsigned long long)(pe >> 31) * nst * nmd +
                                    (unsigned long long)(pe & 0x7FFFFFFFu) * nmd + sr.z;
                                rk[bb] = ((unsigned long long)in.bkt_rank[hb] << 37) | within;
                            }
                        }
                    }
                }
                // (round 4: issuing a batch's first bucket reads and CASes together
                // measured slower on configs[4]'s k = 12 slice, 7.1 -> 8.6 s of pair
                // counting: the per-insert loop stays)
                uint32_t newk = 0;
#pragma unroll
                for (int bb = 0; bb < BATCH; ++bb) {
                    const uint32_t partner = part[bb];
                    if (partner == a) continue;                 // same read (KmerTable.scala:61-63)
                    if (split > 1 && (partner % split) != residue) continue;
                    newk += pc_insert<STRICT, TAB>(S, X, partner, wv[bb], rk[bb]) ? 1u : 0u;
                }
                pc_fill<TAB>(S, newk, (uint32_t)min(role_pairs - total + w0 + e0, 0xFFFFFFFEull));
                if (S.overflow) break;
            }
        }
        __syncthreads();
    }

    if (nocc == 0) __syncthreads();  // (no chunk barriers ordered the table initialisation)
    const uint32_t shard = blockIdx.x % NSHARD;
    if (tid == 0 && role_pairs) atomicAdd(&o.role_pairs[shard], role_pairs);  // recount tiers: a dummy counter
    if (tid == 0 && !S.overflow) atomicAdd(&o.distinct[shard], (unsigned long long)S.fill);
    if (S.overflow) {  // recounted by the next tier: this read's class only
        if (tid == 0) {
            if (p.per_read) o.rcnt[a] = 0;  // (the recount tiers emit its pairs into the shared regions)
            const uint32_t at = atomicAdd(o.overflow_n, 1u);
            o.overflow_list[at] = (a << 6) | residue;
            // its distinct partners, extrapolated from the fill rate (FILL_MAX
            // partners in the first xfill role pairs -- the index of the insert
            // that filled the table; else the window where it was seen full):
            // the host picks the tier
            if (o.overflow_rp) {
                const unsigned long long x = S.xfill != 0xFFFFFFFFu ? (unsigned long long)S.xfill + 1
                                             : x_over == ~0ull || x_over == 0 ? role_pairs : x_over;
                const unsigned long long est =
                    early_est ? early_est : (unsigned long long)pc_fill_max(TAB) * role_pairs / (x ? x : 1);
                o.overflow_rp[at] = est > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)est;
            }
        }
        return;
    }
    if (p.per_read) {
        // --- per-read region (TAB = 256: one slot per thread): compact the
        //     kept keys in LDS, rank each by its trail among them (<= 192,
        //     distinct), store at its rank -- the region is trail-ascending
        if constexpr (TAB == NT) {
            const uint32_t kk = S.key[tid], kc = S.cnt[tid];
            const bool keep = kk != PC_EMPTY && (int32_t)kc >= p.min_coll && (int32_t)kc <= p.max_coll;
            uint32_t m;
            const uint32_t ex = pc_block_excl_scan<NT>(keep ? 1u : 0u, S.lds4, &m);
            uint32_t *ck = reinterpret_cast<uint32_t *>(S.rec);  // enumeration state is dead
            if (keep) ck[ex] = kk;
            __syncthreads();
            if (keep) {
                uint32_t r = 0;
                for (uint32_t i = 0; i < m; ++i) r += ck[i] < kk ? 1u : 0u;
                o.rreg[(uint64_t)a * PC_RREG + r] = make_uint2(kk, kc);
            }
            if (tid == 0) o.rcnt[a] = m;
        }
        return;
    }
    // --- emit (a, partner, count[, rank]), 32 slots per thread at a time:
    //     wave scans, one claim per block, two barriers per chunk
    constexpr int PER = TAB / NT;
    constexpr int CH = PER < 32 ? PER : 32;
    // (sharded: the regions of the rank owning read a)
    const uint32_t rslot = o.owners > 1 ? owner_of(o.owner_starts, o.owners, a) * NSHARD + shard : shard;
    const unsigned long long region = (unsigned long long)rslot * o.cap_s;
    const int lane = tid & 63, wvi = tid >> 6;
    for (int c0 = 0; c0 < PER; c0 += CH) {
        uint32_t keep = 0;
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const uint32_t sl = tid * PER + c0 + j;
            if constexpr (PcShape<TAB>::PACKED) {  // (no emit_all: the host keeps max_coll <= 255)
                const uint32_t kw = S.key[sl], c = kw >> 24;
                if (kw != PC_EMPTY && !((S.sat[sl >> 5] >> (sl & 31)) & 1u) && (int32_t)c >= p.min_coll &&
                    (int32_t)c <= p.max_coll)
                    keep |= 1u << j;
            } else {
                const uint32_t c = S.cnt[sl];
                if (S.key[sl] != PC_EMPTY && (p.emit_all || ((int32_t)c >= p.min_coll && (int32_t)c <= p.max_coll)))
                    keep |= 1u << j;
            }
        }
        const int buf = (c0 / CH) & 1;  // slow readers of the previous chunk's counts are not overwritten
        const uint32_t mine = __popc(keep);
        const uint32_t inc = wave_incl_add(mine);
        if (lane == 63) S.emit4[buf][wvi] = inc;
        __syncthreads();
        uint32_t total = 0, ex = inc - mine;
#pragma unroll
        for (int q = 0; q < NT / 64; ++q) {
            const uint32_t v = S.emit4[buf][q];
            total += v;
            if (q < wvi) ex += v;
        }
        if (total == 0) continue;  // uniform: every thread sees the same total
        if (tid == 0) S.emit_base[buf] = (uint32_t)atomicAdd(&o.cursor[rslot], (unsigned long long)total);
        __syncthreads();
        const unsigned long long base = (unsigned long long)S.emit_base[buf] + ex;
        uint32_t k = 0;
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            if (!(keep & (1u << j))) continue;
            const uint32_t sl = tid * PER + c0 + j;
            const unsigned long long lat = base + k++;
            const unsigned long long at = region + lat;
            if (lat < o.cap_s) {
                o.fst[at] = a;
                if constexpr (PcShape<TAB>::PACKED) {
                    o.snd[at] = S.key[sl] & 0xFFFFFFu;
                    o.cnt[at] = S.key[sl] >> 24;
                } else {
                    o.snd[at] = S.key[sl];
                    o.cnt[at] = S.cnt[sl];
                }
                if constexpr (STRICT) o.rank[at] = X.rank[sl];
            }
        }
    }
}

template <int TAB>
static size_t pc_lds_bytes(bool strict) {
    static_assert(sizeof(PcShared<TAB>) <= 160 * 1024, "a pair-count block must fit the CU's 160 KB of LDS");
    size_t s = (sizeof(PcShared<TAB>) + 15) & ~size_t(15);
    if (strict) s += sizeof(PcSharedStrict<TAB>);
    return s;
}

size_t pair_count_lds_bytes(bool strict) { return pc_lds_bytes<PC_TAB_BIG>(strict); }

template <bool STRICT, int TAB>
static hipError_t pc_launch(const EmitParams &e, const PairIn &in, const PairParams &p, PairOut &o,
                            const uint32_t *read_list, uint32_t n_blocks, hipStream_t s) {
    const size_t lds = pc_lds_bytes<TAB>(STRICT);
    (void)hipFuncSetAttribute((const void *)pair_count_kernel<STRICT, TAB>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    // a dispatch's grid is counted in work-items with 32 bits: 6.25M reads at
    // 1,024 threads (configs[4]'s slice in the 16,384-slot tier) would wrap it.
    // Larger item lists go in slices of the list (the XCD-contiguous swizzle
    // is a schedule only, so the slices drop it)
    constexpr uint32_t NT = PcShape<TAB>::NT;
    uint32_t max_blocks = (0x80000000u / NT) & ~7u;
    if (p.max_blocks && p.max_blocks < max_blocks) max_blocks = p.max_blocks;
    if (n_blocks <= max_blocks) {
        hipLaunchKernelGGL((pair_count_kernel<STRICT, TAB>), dim3(n_blocks), dim3(NT), lds, s, e, in, p, o, read_list);
        return hipGetLastError();
    }
    if (!read_list) return hipErrorInvalidValue;  // (every large launch walks an item list)
    for (uint32_t b0 = 0; b0 < n_blocks && b0 < p.n_items; b0 += max_blocks) {
        PairParams q = p;
        q.xcd_swizzle = 0;
        q.n_items = min(p.n_items - b0, max_blocks);
        hipLaunchKernelGGL((pair_count_kernel<STRICT, TAB>), dim3(q.n_items), dim3(NT), lds, s, e, in, q, o,
                           read_list + b0);
        const hipError_t er = hipGetLastError();
        if (er != hipSuccess) return er;
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------
// First pass, one WAVE per read (wide ids, per-read regions -- the bench path).
// The one-read workgroup above spends about half its time in per-read framework:
// ~10 block barriers per read and 8 reads in flight per CU (4 waves each at the
// 32-wave limit).  Here a 256-thread block carries four reads, one per wave, and
// every synchronisation is within the wave (LDS operations of a wave complete in
// order, so a wave barrier -- a compiler fence -- is all the eo / pref / rec
// hand-offs need): 28 reads in flight per CU (5.6 KB of LDS per read), no block
// barrier.  Enumeration is the same lane-interleaved walk over 512-element
// windows of 128-occurrence chunks, the same table (256 slots, 192 at the fill
// limit), overflow accounting and per-read region as pair_count_kernel<false, 256>.
// ---------------------------------------------------------------------------
constexpr int PW_WAVES = 4;
#ifndef PW_CHUNK_OCC
#define PW_CHUNK_OCC 64
#endif
#ifndef PW_BATCH_EL
#define PW_BATCH_EL 8
#endif
#ifndef PW_MIN_WAVES
#define PW_MIN_WAVES 8                     // per SIMD: <= 64 VGPRs, the 32-wave CU limit
#endif
constexpr int PW_CHUNK = PW_CHUNK_OCC;     // occurrences per chunk
constexpr int PW_OCC = PW_CHUNK / 64;      // ... per lane
constexpr int PW_BATCH = PW_BATCH_EL;      // partner gathers in flight per lane
constexpr int PW_WIN = 64 * PW_BATCH;      // elements per window (one batch per lane)

struct PwShared {  // one per wave
    uint32_t key[PC_TAB_SMALL];
    uint32_t cnt[PC_TAB_SMALL];
    uint4 rec[PW_CHUNK];   // {list entry of element 0 (u64), edge-role end, edge weight} per occurrence
    uint16_t eo[PW_WIN];
    uint32_t fill, overflow, xfill, pad;
};
static_assert(PW_BATCH % 8 == 0, "each lane owns PW_BATCH contiguous u16 entries of eo, in 16-byte words");

__device__ __forceinline__ void pw_insert_probe(PwShared &S, uint32_t partner, uint32_t w, uint32_t eidx,
                                                uint32_t slot) {
    constexpr uint32_t FILL_MAX = PC_TAB_SMALL * 3 / 4;
    for (int probe = 0; probe < PC_TAB_SMALL / 4; ++probe) {  // bounded as in pc_insert
        uint32_t old = lds_relaxed(&S.key[slot]);  // a set key is final (pc_insert)
        if (old == PC_EMPTY) old = atomicCAS(&S.key[slot], PC_EMPTY, partner);
        if (old == PC_EMPTY || old == partner) {
            if (old == PC_EMPTY && atomicAdd(&S.fill, 1u) >= FILL_MAX) {
                S.overflow = 1;
                atomicMin(&S.xfill, eidx);
            }
            atomicAdd(&S.cnt[slot], w);
            return;
        }
        slot = (slot + 1) & (PC_TAB_SMALL - 1);
    }
    S.overflow = 1;
}
// a read meets each partner in ~100 shared k-mers, so nearly every insert finds
// its key in the home slot: that case is one read + one add, outside the probe
// loop (whose exec-mask bookkeeping is ~30 scalar instructions per insert)
__device__ __forceinline__ void pw_insert(PwShared &S, uint32_t partner, uint32_t w, uint32_t eidx) {
    const uint32_t h = pc_hash<PC_TAB_SMALL>(partner);
    if (lds_relaxed(&S.key[h]) == partner) {
        atomicAdd(&S.cnt[h], w);
        return;
    }
    pw_insert_probe(S, partner, w, eidx, h);
}

__global__ __launch_bounds__(PW_WAVES * 64, PW_MIN_WAVES) void pair_count_wave_kernel(EmitParams e, PairIn in, PairParams p,
                                                                         PairOut o, const uint32_t *read_list,
                                                                         uint32_t n_blocks) {
    __shared__ PwShared SH[PW_WAVES];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    PwShared &S = SH[wv];
    uint32_t bid = blockIdx.x;
    if (p.xcd_swizzle) bid = (blockIdx.x & 7u) * (n_blocks >> 3) + (blockIdx.x >> 3);  // as pair_count_kernel
    const uint32_t item = bid * PW_WAVES + wv;
    if (item >= p.n_items) return;  // whole wave: nothing below synchronises beyond it
    if (p.abort && *p.abort) return;
    const uint32_t a = read_list ? read_list[item] : item;

    for (int i = lane; i < PC_TAB_SMALL; i += 64) {
        S.key[i] = PC_EMPTY;
        S.cnt[i] = 0;
    }
    if (lane == 0) { S.fill = 0; S.overflow = 0; S.xfill = 0xFFFFFFFFu; }
    const uint64_t g0 = e.npr ? (uint64_t)a * e.npr : e.occ_off[a];
    const uint32_t nocc = e.npr ? e.npr : (uint32_t)(e.occ_off[a + 1] - g0);
    unsigned long long role_pairs = 0;
    unsigned long long x_over = ~0ull;
    bool over = false;
    __builtin_amdgcn_wave_barrier();

    // a chunk's records are loaded at the end of the one before (issuing them
    // behind the chunk's first partner gathers instead measured slower: 0.594
    // vs 0.578 ms per bench step, the live registers cost the gathers' batch)
    uint2 nxt[PW_OCC];
#pragma unroll
    for (int j = 0; j < PW_OCC; ++j) {
        const uint32_t oi = lane * PW_OCC + j;
        nxt[j] = oi < nocc ? load_rec_raw(in, g0 + oi) : make_uint2(0, 0);
    }
    for (uint32_t c0 = 0; c0 < nocc && !over; c0 += PW_CHUNK) {
        const uint32_t cn = min((uint32_t)PW_CHUNK, nocc - c0);
        uint32_t mytot[PW_OCC];
        uint4 rcj[PW_OCC];
#pragma unroll
        for (int j = 0; j < PW_OCC; ++j) {
            const uint32_t oi = lane * PW_OCC + j;  // lane-contiguous
            uint32_t tot = 0;
            rcj[j] = make_uint4(0, 0, 0, 0);
            if (oi < cn) {
                rcj[j] = decode_rec(nxt[j], in.xrec);
                tot = (rcj[j].y & 0x3FFFFFFFu) + rcj[j].w;
            }
            mytot[j] = tot;
        }
        uint32_t sum = 0;
#pragma unroll
        for (int j = 0; j < PW_OCC; ++j) sum += mytot[j];
        const uint32_t inc = wave_incl_add(sum);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        uint32_t myex[PW_OCC];
        myex[0] = inc - sum;
#pragma unroll
        for (int j = 1; j < PW_OCC; ++j) myex[j] = myex[j - 1] + mytot[j - 1];
        // per occurrence, what an element ew of the chunk needs: its list entry is
        // adj + ew (adj = c - nE - first element), it is an edge-role pair (weight
        // me) while ew < first element + nE, else a middle one (weight 1)
#pragma unroll
        for (int j = 0; j < PW_OCC; ++j)
            if (lane * PW_OCC + j < cn) {
                const uint32_t nE = rcj[j].y & 0x3FFFFFFFu;
                const uint64_t adj = (((uint64_t)rcj[j].z << 32) | rcj[j].x) - nE - myex[j];
                S.rec[lane * PW_OCC + j] = make_uint4((uint32_t)adj, (uint32_t)(adj >> 32), myex[j] + nE, rcj[j].y >> 30);
            }
        const unsigned long long rp0 = role_pairs;  // role pairs before this chunk
        role_pairs += total;
        uint32_t carry = 0;  // occurrence (+1) owning the window's first element
        for (uint32_t w0 = 0; w0 < total; w0 += PW_WIN) {
            __builtin_amdgcn_wave_barrier();  // pref / rec written; the previous window's eo read
            if (lds_relaxed(&S.overflow)) {   // recounted by the next tier: totals only
                if (x_over == ~0ull) x_over = rp0 + w0;
                over = true;
                break;
            }
            // element -> occurrence map of the window without a per-element loop:
            // zero it, mark the first element of every non-empty occurrence that
            // starts inside (positions are distinct), then a max-scan -- over the
            // lane's PW_BATCH contiguous entries in registers, then across lanes
            // (DPP), seeded with the occurrence running into the window
            uint4 *eo4 = reinterpret_cast<uint4 *>(S.eo);
#pragma unroll
            for (int q = 0; q < PW_BATCH / 8; ++q) eo4[lane * (PW_BATCH / 8) + q] = make_uint4(0, 0, 0, 0);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = 0; j < PW_OCC; ++j)
                if (mytot[j] && myex[j] >= w0 && myex[j] < w0 + (uint32_t)PW_WIN)
                    S.eo[myex[j] - w0] = (uint16_t)(lane * PW_OCC + j + 1);
            __builtin_amdgcn_wave_barrier();
            {
                uint32_t v[PW_BATCH];
#pragma unroll
                for (int q = 0; q < PW_BATCH / 8; ++q) {
                    const uint4 x = eo4[lane * (PW_BATCH / 8) + q];
                    const uint32_t w4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        v[8 * q + 2 * t] = w4[t] & 0xFFFFu;
                        v[8 * q + 2 * t + 1] = w4[t] >> 16;
                    }
                }
                uint32_t run = 0;
#pragma unroll
                for (int i = 0; i < PW_BATCH; ++i) { run = max(run, v[i]); v[i] = run; }
                const uint32_t incl = wave_incl_max(run);
                const uint32_t into = max(carry, wave_shr1(incl));  // owner entering this lane's entries
#pragma unroll
                for (int q = 0; q < PW_BATCH / 8; ++q) {
                    uint32_t w4[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        w4[t] = max(v[8 * q + 2 * t], into) | (max(v[8 * q + 2 * t + 1], into) << 16);
                    eo4[lane * (PW_BATCH / 8) + q] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
                }
                carry = max(carry, (uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
            }
            __builtin_amdgcn_wave_barrier();
            const uint32_t wn = min((uint32_t)PW_WIN, total - w0);
            uint32_t part[PW_BATCH], wt[PW_BATCH];
#pragma unroll
            for (int bb = 0; bb < PW_BATCH; ++bb) {
                part[bb] = a;  // "same read" = skip
                wt[bb] = 0;
                const uint32_t el = bb * 64 + lane;
                if (el < wn) {
                    const uint32_t ew = w0 + el;
                    const uint4 r = S.rec[(uint32_t)S.eo[el] - 1u];
                    part[bb] = in.lst[(((uint64_t)r.y << 32) | r.x) + ew];
                    wt[bb] = ew < r.z ? r.w : 1u;
                }
            }
#pragma unroll
            for (int bb = 0; bb < PW_BATCH; ++bb) {
                if (part[bb] == a) continue;  // same read (KmerTable.scala:61-63)
                pw_insert(S, part[bb], wt[bb], (uint32_t)min(rp0 + w0 + bb * 64 + lane, 0xFFFFFFFEull));
            }
        }
        if (!over)
#pragma unroll
            for (int j = 0; j < PW_OCC; ++j) {
                const uint32_t oi = lane * PW_OCC + j;
                if (c0 + PW_CHUNK + oi < nocc) nxt[j] = load_rec_raw(in, g0 + c0 + PW_CHUNK + oi);
            }
        // the rest of the read's chunks still count their role pairs after an overflow
        if (over)
            for (uint32_t c1 = c0 + PW_CHUNK; c1 < nocc; c1 += PW_CHUNK) {
                const uint32_t cn1 = min((uint32_t)PW_CHUNK, nocc - c1);
                uint32_t t = 0;
#pragma unroll
                for (int j = 0; j < PW_OCC; ++j) {
                    const uint32_t oi = lane * PW_OCC + j;
                    if (oi < cn1) {
                        const uint4 rc = load_rec(in, g0 + c1 + oi);
                        t += (rc.y & 0x3FFFFFFFu) + rc.w;
                    }
                }
                role_pairs += (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_add(t), 63);
            }
        __builtin_amdgcn_wave_barrier();
    }
    const bool overflow = lds_relaxed(&S.overflow) != 0;
    const uint32_t shard = item % NSHARD;
    if (lane == 0 && role_pairs) atomicAdd(&o.role_pairs[shard], role_pairs);
    if (lane == 0 && !overflow) atomicAdd(&o.distinct[shard], (unsigned long long)lds_relaxed(&S.fill));
    if (overflow) {  // recounted by the next tier (pair_count_kernel, 2,048 / 16,384 slots)
        if (lane == 0) {
            o.rcnt[a] = 0;
            const uint32_t at = atomicAdd(o.overflow_n, 1u);
            o.overflow_list[at] = a << 6;
            if (o.overflow_rp) {  // distinct partners extrapolated from the fill point (pair_count_kernel)
                const uint32_t xf = lds_relaxed(&S.xfill);
                const unsigned long long x = xf != 0xFFFFFFFFu ? (unsigned long long)xf + 1
                                             : x_over == ~0ull || x_over == 0 ? role_pairs : x_over;
                const unsigned long long est = (unsigned long long)(PC_TAB_SMALL * 3 / 4) * role_pairs / (x ? x : 1);
                o.overflow_rp[at] = est > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)est;
            }
        }
        return;
    }
    // ---- per-read region: the kept keys compacted, each ranked by its trail
    uint32_t kk[4], kc[4], keep = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        kk[j] = S.key[lane * 4 + j];
        kc[j] = S.cnt[lane * 4 + j];
        if (kk[j] != PC_EMPTY && (int32_t)kc[j] >= p.min_coll && (int32_t)kc[j] <= p.max_coll) keep |= 1u << j;
    }
    const uint32_t mine = __popc(keep);
    const uint32_t kin = wave_incl_add(mine);
    const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)kin, 63);
    uint32_t *ck = reinterpret_cast<uint32_t *>(S.rec);  // enumeration state is dead (m <= 192 words)
    uint32_t at = kin - mine;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (keep & (1u << j)) ck[at++] = kk[j];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (!(keep & (1u << j))) continue;
        uint32_t r = 0;
        for (uint32_t i = 0; i < m; ++i) r += ck[i] < kk[j] ? 1u : 0u;
        o.rreg[(uint64_t)a * PC_RREG + r] = make_uint2(kk[j], kc[j]);
    }
    if (lane == 0) o.rcnt[a] = m;
}

hipError_t launch_pair_count(const EmitParams &e, const PairIn &in, const PairParams &p, PairOut &o,
                             const uint32_t *read_list, uint32_t n_blocks, hipStream_t s) {
    if (n_blocks == 0) return hipSuccess;
    // the wide-id first pass with per-read regions: one wave per read
    if (!p.strict && p.table == PC_TAB_SMALL && p.per_read && !p.coded && p.split <= 1) {
        const uint32_t nb = (p.n_items + PW_WAVES - 1) / PW_WAVES;
        const uint32_t grid = p.xcd_swizzle ? (nb + 7) & ~7u : nb;
        if (!p.max_blocks || grid <= p.max_blocks) {
            static const size_t pw_dyn = occ_lds("SA_OCC_PW", sizeof(PwShared) * PW_WAVES, 0);  // (A/B)
            if (pw_dyn)
                (void)hipFuncSetAttribute((const void *)pair_count_wave_kernel,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)pw_dyn);
            hipLaunchKernelGGL(pair_count_wave_kernel, dim3(grid), dim3(PW_WAVES * 64), pw_dyn, s, e, in, p, o, read_list,
                               grid);
            return hipGetLastError();
        }
    }
    if (p.strict) {
        if (p.table == PC_TAB_SMALL) return pc_launch<true, PC_TAB_SMALL>(e, in, p, o, read_list, n_blocks, s);
        if (p.table == PC_TAB_BIG) return pc_launch<true, PC_TAB_BIG>(e, in, p, o, read_list, n_blocks, s);
        return hipErrorInvalidValue;  // strict ids stop at 2,048 slots (then split)
    }
    if (p.table == PC_TAB_SMALL) return pc_launch<false, PC_TAB_SMALL>(e, in, p, o, read_list, n_blocks, s);
    if (p.table == PC_TAB_BIG) return pc_launch<false, PC_TAB_BIG>(e, in, p, o, read_list, n_blocks, s);
    if (p.table == PC_TAB_HUGE) return pc_launch<false, PC_TAB_HUGE>(e, in, p, o, read_list, n_blocks, s);
    if (p.table == PC_TAB_HUGE2) {
        // (the host routes here only with partners < 2^24 - 1, max_coll <= 255, no emit_all)
        if (p.emit_all || p.max_coll > 255) return hipErrorInvalidValue;
        return pc_launch<false, PC_TAB_HUGE2>(e, in, p, o, read_list, n_blocks, s);
    }
    return hipErrorInvalidValue;
}

// Multi-read items (sharded hash stage): keys are (read, partner) in 64 bits
constexpr unsigned long long PCM_EMPTY = ~0ull;

__device__ __forceinline__ uint32_t pcm_hash(unsigned long long k) {
    const uint32_t x = ((uint32_t)k * 0x9E3779B1u) ^ ((uint32_t)(k >> 32) * 0x85EBCA77u);
    return x >> (32 - 10);
}

// ---------------------------------------------------------------------------
// Multi-read items, one WAVE each (sharded hash stage, round 4).  A 256-thread
// block form ran ~16 block barriers per 512-occurrence item; here a 256-thread
// block carries four items of ~PMW_TARGET local occurrences (a few reads), one
// per wave, with the single-device wave kernel's hand-offs (wave barriers,
// marker + max-scan element map, per-occurrence list bases) and a wave-private
// 256-slot table keyed by (read, partner).  Every distinct partial is kept
// (count >= 1: the filter needs the global sums).  Output claims are made once
// per BLOCK: the four waves' kept counts are scanned at one block barrier and
// one device atomic claims the block's range (a claim per item made the wave
// form slower than the blocks in round 3).  With several ranks (PairOut::owners)
// the claim is per block AND owner of the lead, into that owner's regions, so
// the partials leave grouped by destination rank with no sort (a block's reads
// are consecutive, so nearly every block has one owner).  An item whose table
// fills appends its reads to the overflow list for the recount tiers.
// ---------------------------------------------------------------------------
constexpr int PMW_WAVES = 4;
constexpr int PMW_TAB = 256;
#ifndef SA_PMW_CHUNK  // (A/B builds)
#define SA_PMW_CHUNK 64
#endif
#ifndef SA_PMW_MIN_WAVES  // (8 waves per SIMD: <= 64 VGPRs, with the 32-bit keys' 18.5 KB of LDS per
#define SA_PMW_MIN_WAVES 8  // block -- 8 serial shards, pairs 1.261 -> 1.230 ms, ab_pmw_k32.txt)
#endif
// occurrences per chunk, 1 per lane (2 per lane: 21.6 -> 26.7 KB of LDS per block, 7 -> 5 waves
// per SIMD; 8 serial shards of the bench shape, pairs 1.350 -> 1.325 ms with 1 per lane,
// profiles/r05/sharded/ab_pmw_chunk.txt)
constexpr int PMW_CHUNK = SA_PMW_CHUNK;
constexpr int PMW_OCC = PMW_CHUNK / 64;
#ifndef SA_PMW_BATCH
#define SA_PMW_BATCH 8
#endif
constexpr int PMW_BATCH = SA_PMW_BATCH;     // partner gathers in flight per lane
constexpr int PMW_WIN = 64 * PMW_BATCH;     // elements per window
static_assert(PMW_BATCH % 8 == 0, "the window's element offsets move as uint4 pairs: 8 per lane step");
constexpr uint32_t PMW_FILL_MAX = PMW_TAB * 3 / 4;

#ifndef SA_PMW_RB_MAX
#define SA_PMW_RB_MAX 64  // (A/B builds: 0 = the owning read by a search in global memory)
#endif
constexpr int PMW_RB_MAX = SA_PMW_RB_MAX > 0 ? SA_PMW_RB_MAX : 1;
// Table keys: (read, partner) as read << 32 | partner, or -- when every global read id fits 26
// bits -- as (read - the item's first read) << 26 | partner in 32 bits (items of <= 64 reads;
// a wider item goes to the recount tiers): half the key LDS and 32-bit LDS atomics
constexpr int PMW_K32_PBITS = 26;
template <typename K> struct PmwKey;
template <> struct PmwKey<unsigned long long> {
    static constexpr unsigned long long EMPTY = ~0ull;
    __device__ static unsigned long long make(uint32_t r, uint32_t ra, uint32_t part) {
        (void)ra;
        return ((unsigned long long)r << 32) | part;
    }
    __device__ static uint32_t lead(unsigned long long k, uint32_t ra) { (void)ra; return (uint32_t)(k >> 32); }
    __device__ static uint32_t part(unsigned long long k) { return (uint32_t)k; }
    __device__ static uint32_t slot(unsigned long long k) {
        const uint32_t x = ((uint32_t)k * 0x9E3779B1u) ^ ((uint32_t)(k >> 32) * 0x85EBCA77u);
        return x >> (32 - 8);
    }
};
template <> struct PmwKey<uint32_t> {
    static constexpr uint32_t EMPTY = 0xFFFFFFFFu;  // (never a key: partners < 2^26 - 1)
    __device__ static uint32_t make(uint32_t r, uint32_t ra, uint32_t part) { return ((r - ra) << PMW_K32_PBITS) | part; }
    __device__ static uint32_t lead(uint32_t k, uint32_t ra) { return ra + (k >> PMW_K32_PBITS); }
    __device__ static uint32_t part(uint32_t k) { return k & ((1u << PMW_K32_PBITS) - 1u); }
    __device__ static uint32_t slot(uint32_t k) { return (k * 0x9E3779B1u) >> (32 - 8); }
};

template <typename K>
struct PmwShared {  // one per wave
    K key[PMW_TAB];
    uint32_t cnt[PMW_TAB];
    uint4 rec[PMW_CHUNK];     // {list entry of element 0 (u64), edge-role end, edge weight}
    uint32_t aid[PMW_CHUNK];  // read of each occurrence of the chunk
    uint16_t eo[PMW_WIN];
    uint32_t rbo[PMW_RB_MAX];  // the item's read starts relative to its first occurrence
    uint32_t fill, overflow, kept, pad;
};

#ifndef PMW_FASTPATH
#define PMW_FASTPATH 0  // (8 serial shards: pairs 1.455-1.468 ms without, 1.481-1.501 with)
#endif
template <typename K>
__device__ __forceinline__ void pmw_insert(PmwShared<K> &S, K key, uint32_t w) {
    constexpr K EMPTY = PmwKey<K>::EMPTY;
    uint32_t slot = PmwKey<K>::slot(key);
    if (PMW_FASTPATH && lds_relaxed(&S.key[slot]) == key) {  // the home-slot hit: no probe loop
        atomicAdd(&S.cnt[slot], w);
        return;
    }
    for (int probe = 0; probe < PMW_TAB / 4; ++probe) {
        K old = lds_relaxed(&S.key[slot]);  // final once set
        if (old == EMPTY) old = atomicCAS(&S.key[slot], EMPTY, key);
        if (old == EMPTY || old == key) {
            if (old == EMPTY && atomicAdd(&S.fill, 1u) >= PMW_FILL_MAX) S.overflow = 1;
            atomicAdd(&S.cnt[slot], w);
            return;
        }
        slot = (slot + 1) & (PMW_TAB - 1);
    }
    S.overflow = 1;
}

template <typename K>
__global__ __launch_bounds__(PMW_WAVES * 64, SA_PMW_MIN_WAVES) void pair_count_multi_wave_kernel(EmitParams e, PairIn in, PairParams p,
                                                                                PairOut o,
                                                                                const uint32_t *item_start) {
    using KK = PmwKey<K>;
    __shared__ PmwShared<K> SH[PMW_WAVES];
    __shared__ uint32_t wkept[PMW_WAVES], wlast[PMW_WAVES], blk_base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    PmwShared<K> &S = SH[wv];
    // big partitions still to build (bucket_stage phase 1): the whole block exits before
    // its first barrier -- the flag was set before this launch, every thread reads the same
    if (p.abort && *p.abort) return;
    const uint32_t item = blockIdx.x * PMW_WAVES + wv;
    // (no early return below: every wave reaches the block's output claim)
    const bool live = item < p.n_items;
    // (lead-range passes: the pass's items carry their own ends -- its ranges leave gaps)
    const uint32_t ra = live ? item_start[item] : 0u,
                   rb = live ? (o.item_end ? o.item_end[item] : item_start[item + 1]) : 0u;
    const uint32_t own2 = live && o.owners > 1 ? o.item_owner[item] : 0u;  // (lo | hi << 16, pc_item_owners)
    for (int i = lane; i < PMW_TAB; i += 64) {
        S.key[i] = KK::EMPTY;
        S.cnt[i] = 0;
    }
    // (32-bit keys hold the read as an offset of 6 bits: a wider item is recounted by the tiers)
    const bool too_wide = sizeof(K) == 4 && rb - ra > 64u;
    if (lane == 0) { S.fill = 0; S.overflow = too_wide ? 1u : 0u; }
    const uint64_t g0 = ra < rb ? e.occ_off[ra] : 0ull;
    const uint32_t nocc = ra < rb ? (uint32_t)(e.occ_off[rb] - g0) : 0u;
    unsigned long long role_pairs = 0;
    bool over = false;
    // the item's read boundaries staged in LDS (one coalesced load): each occurrence finds its
    // read there, not by dependent loads of occ_off
    const bool rb_lds = SA_PMW_RB_MAX > 0 && rb - ra + 1 <= (uint32_t)PMW_RB_MAX;  // (wave-uniform)
    if (rb_lds && (uint32_t)lane <= rb - ra) S.rbo[lane] = (uint32_t)(e.occ_off[ra + lane] - g0);
    __builtin_amdgcn_wave_barrier();
    for (uint32_t c0 = 0; c0 < nocc; c0 += PMW_CHUNK) {
        const uint32_t cn = min((uint32_t)PMW_CHUNK, nocc - c0);
        uint32_t mytot[PMW_OCC];
        uint4 rcj[PMW_OCC];
        uint32_t own[PMW_OCC];
#pragma unroll
        for (int j = 0; j < PMW_OCC; ++j) {
            const uint32_t oi = lane * PMW_OCC + j;  // lane-contiguous
            rcj[j] = make_uint4(0, 0, 0, 0);
            mytot[j] = 0;
            own[j] = ra;
            if (oi < cn) {
                const uint64_t g = g0 + c0 + oi;
                rcj[j] = load_rec(in, g);
                mytot[j] = (rcj[j].y & 0x3FFFFFFFu) + rcj[j].w;
                // owning read: largest r with occ_off[r] <= g (in LDS, or a few cached
                // loads; the item's boundaries broadcast from registers measured slower)
                uint32_t lo = ra, hi = rb;
                if (rb_lds) {
                    const uint32_t rel = c0 + oi;
                    uint32_t l = 0, h = rb - ra;
                    while (h - l > 1) {
                        const uint32_t mid = (l + h) >> 1;
                        if (S.rbo[mid] <= rel) l = mid; else h = mid;
                    }
                    lo = ra + l;
                } else {
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (e.occ_off[mid] <= g) lo = mid; else hi = mid;
                    }
                }
                own[j] = lo;
            }
        }
        uint32_t sum = 0;
#pragma unroll
        for (int j = 0; j < PMW_OCC; ++j) sum += mytot[j];
        const uint32_t inc = wave_incl_add(sum);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        uint32_t myex[PMW_OCC];
        myex[0] = inc - sum;
#pragma unroll
        for (int j = 1; j < PMW_OCC; ++j) myex[j] = myex[j - 1] + mytot[j - 1];
        if (!over) {
#pragma unroll
            for (int j = 0; j < PMW_OCC; ++j)
                if (lane * PMW_OCC + j < cn) {
                    const uint32_t nE = rcj[j].y & 0x3FFFFFFFu;
                    const uint64_t adj = (((uint64_t)rcj[j].z << 32) | rcj[j].x) - nE - myex[j];
                    S.rec[lane * PMW_OCC + j] = make_uint4((uint32_t)adj, (uint32_t)(adj >> 32), myex[j] + nE,
                                                           rcj[j].y >> 30);
                    S.aid[lane * PMW_OCC + j] = own[j];
                }
        }
        role_pairs += total;
        uint32_t carry = 0;
        for (uint32_t w0 = 0; w0 < total && !over; w0 += PMW_WIN) {
            __builtin_amdgcn_wave_barrier();
            if (lds_relaxed(&S.overflow)) {
                over = true;
                break;
            }
            uint4 *eo4 = reinterpret_cast<uint4 *>(S.eo);
#pragma unroll
            for (int q = 0; q < PMW_BATCH / 8; ++q) eo4[lane * (PMW_BATCH / 8) + q] = make_uint4(0, 0, 0, 0);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = 0; j < PMW_OCC; ++j)
                if (mytot[j] && myex[j] >= w0 && myex[j] < w0 + (uint32_t)PMW_WIN)
                    S.eo[myex[j] - w0] = (uint16_t)(lane * PMW_OCC + j + 1);
            __builtin_amdgcn_wave_barrier();
            {
                uint32_t v[PMW_BATCH];
#pragma unroll
                for (int q = 0; q < PMW_BATCH / 8; ++q) {
                    const uint4 x = eo4[lane * (PMW_BATCH / 8) + q];
                    const uint32_t w4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        v[8 * q + 2 * t] = w4[t] & 0xFFFFu;
                        v[8 * q + 2 * t + 1] = w4[t] >> 16;
                    }
                }
                uint32_t run = 0;
#pragma unroll
                for (int i = 0; i < PMW_BATCH; ++i) { run = max(run, v[i]); v[i] = run; }
                const uint32_t incl = wave_incl_max(run);
                const uint32_t into = max(carry, wave_shr1(incl));
#pragma unroll
                for (int q = 0; q < PMW_BATCH / 8; ++q) {
                    uint32_t w4[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        w4[t] = max(v[8 * q + 2 * t], into) | (max(v[8 * q + 2 * t + 1], into) << 16);
                    eo4[lane * (PMW_BATCH / 8) + q] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
                }
                carry = max(carry, (uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
            }
            __builtin_amdgcn_wave_barrier();
            const uint32_t wn = min((uint32_t)PMW_WIN, total - w0);
            uint32_t part[PMW_BATCH], wt[PMW_BATCH], ow[PMW_BATCH];
#pragma unroll
            for (int bb = 0; bb < PMW_BATCH; ++bb) {
                wt[bb] = 0;
                part[bb] = 0;
                ow[bb] = 0;
                const uint32_t el = bb * 64 + lane;
                if (el < wn) {
                    const uint32_t ew = w0 + el;
                    const uint32_t oc = (uint32_t)S.eo[el] - 1u;
                    const uint4 r = S.rec[oc];
                    ow[bb] = S.aid[oc];
                    part[bb] = in.lst[(((uint64_t)r.y << 32) | r.x) + ew];
                    wt[bb] = ew < r.z ? r.w : 1u;
                }
            }
#pragma unroll
            for (int bb = 0; bb < PMW_BATCH; ++bb) {
                if (wt[bb] == 0 || part[bb] == ow[bb]) continue;  // same read (KmerTable.scala:61-63)
                pmw_insert<K>(S, KK::make(ow[bb], ra, part[bb]), wt[bb]);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    over = over || lds_relaxed(&S.overflow) != 0;
    const uint32_t shard = blockIdx.x % NSHARD;
    if (live && lane == 0 && role_pairs) atomicAdd(&o.role_pairs[shard], role_pairs);
    if (live && over && lane == 0) {  // recount these reads one per block (pair_count_kernel tiers)
        const uint32_t at = atomicAdd(o.overflow_n, rb - ra);
        for (uint32_t r = ra; r < rb; ++r) o.overflow_list[at + (r - ra)] = r << 6;
    }
    // kept keys of this wave (none when it overflowed), then one claim per block
    // and owner: the block's reads [first, last] span the owners [o_lo, o_hi]
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < PMW_TAB / 64; ++j) {
        const uint32_t sl = lane * (PMW_TAB / 64) + j;
        if (live && !over && S.key[sl] != KK::EMPTY) keep |= 1u << j;
    }
    if (live && !over && lane == 0) atomicAdd(&o.distinct[shard], (unsigned long long)lds_relaxed(&S.fill));
    uint32_t o_lo = 0, o_hi = 0;
    if (o.owners > 1) {
        if (lane == 0) {
            wkept[wv] = live && ra < rb ? (own2 & 0xFFFFu) : 0xFFFFFFFFu;
            wlast[wv] = live && ra < rb ? (own2 >> 16) : 0u;
        }
        __syncthreads();
        o_lo = 0xFFFFFFFFu;
#pragma unroll
        for (int q = 0; q < PMW_WAVES; ++q) {
            o_lo = min(o_lo, wkept[q]);
            o_hi = max(o_hi, wlast[q]);
        }
        if (o_lo == 0xFFFFFFFFu) o_lo = o_hi = 0;  // (no reads in the block: nothing kept)
        __syncthreads();  // wkept is reused for the counts below
    }
    for (uint32_t ow = o_lo; ow <= o_hi; ++ow) {
        uint32_t km = keep;
        if (o_lo != o_hi && km) {  // a block across an owner boundary (rare): this owner's keys
#pragma unroll
            for (int j = 0; j < PMW_TAB / 64; ++j) {
                const uint32_t sl = lane * (PMW_TAB / 64) + j;
                if (((km >> j) & 1u) && owner_of(o.owner_starts, o.owners, KK::lead(S.key[sl], ra)) != ow)
                    km &= ~(1u << j);
            }
        }
        const uint32_t mine = __popc(km);
        const uint32_t winc = wave_incl_add(mine);
        if (lane == 63) wkept[wv] = winc;
        __syncthreads();
        uint32_t btot = 0, wex = 0;
#pragma unroll
        for (int q = 0; q < PMW_WAVES; ++q) {
            const uint32_t x = wkept[q];
            if (q < wv) wex += x;
            btot += x;
        }
        const uint32_t rslot = ow * NSHARD + shard;
        if (threadIdx.x == 0) blk_base = btot ? (uint32_t)atomicAdd(&o.cursor[rslot], (unsigned long long)btot) : 0u;
        __syncthreads();
        if (mine) {
            const unsigned long long region = (unsigned long long)rslot * o.cap_s;
            unsigned long long lat = (unsigned long long)blk_base + wex + (winc - mine);
#pragma unroll
            for (int j = 0; j < PMW_TAB / 64; ++j) {
                if (!(km & (1u << j))) continue;
                const uint32_t sl = lane * (PMW_TAB / 64) + j;
                if (lat < o.cap_s) {
                    const unsigned long long at = region + lat;
                    o.fst[at] = KK::lead(S.key[sl], ra);
                    o.snd[at] = KK::part(S.key[sl]);
                    o.cnt[at] = S.cnt[sl];
                }
                ++lat;
            }
        }
    }
}

#ifndef SA_PMW_K32
#define SA_PMW_K32 1  // (A/B builds: 0 = 64-bit keys always)
#endif
hipError_t launch_pair_count_multi_wave(const EmitParams &e, const PairIn &in, const PairParams &p, PairOut &o,
                                        const uint32_t *item_start, uint32_t n_items, uint32_t n_reads,
                                        hipStream_t s) {
    if (n_items == 0) return hipSuccess;
    PairParams q = p;
    q.n_items = n_items;
    const dim3 grid((n_items + PMW_WAVES - 1) / PMW_WAVES), block(PMW_WAVES * 64);
    if (SA_PMW_K32 && n_reads < (1u << PMW_K32_PBITS) - 1u)  // every partner id fits 26 bits
        hipLaunchKernelGGL(pair_count_multi_wave_kernel<uint32_t>, grid, block, 0, s, e, in, q, o, item_start);
    else
        hipLaunchKernelGGL(pair_count_multi_wave_kernel<unsigned long long>, grid, block, 0, s, e, in, q, o,
                           item_start);
    return hipGetLastError();
}


// item j = reads [first read with occ_off >= j * target, same for j + 1)
__global__ void pc_items_kernel(const uint64_t *occ_off, uint32_t n_reads, uint32_t target, uint32_t n_items,
                                uint32_t *item_start) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n_items) return;
    if (j == n_items) { item_start[j] = n_reads; return; }
    const uint64_t t = (uint64_t)j * target;
    uint32_t lo = 0, hi = n_reads;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (occ_off[mid] < t) lo = mid + 1; else hi = mid;
    }
    item_start[j] = lo;
}

// owners of item j's first and last read, lo | hi << 16 (sharded emission: no
// search on the pair counter's critical path)
__global__ void pc_item_owners_kernel(const uint32_t *item_start, const uint32_t *item_end, uint32_t n_items,
                                      const uint32_t *starts, uint32_t owners, uint32_t *item_owner) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_items) return;
    const uint32_t ra = item_start[j], rb = item_end ? item_end[j] : item_start[j + 1];
    item_owner[j] = ra < rb ? owner_of(starts, owners, ra) | (owner_of(starts, owners, rb - 1) << 16) : 0xFFFFu;
}

hipError_t launch_pc_item_owners(const uint32_t *item_start, uint32_t n_items, const uint32_t *starts, uint32_t owners,
                                 uint32_t *item_owner, hipStream_t s, const uint32_t *item_end) {
    if (!n_items) return hipSuccess;
    // owners travel as lo | hi << 16 (the multi-wave kernel decodes & 0xFFFF, >> 16);
    // sa_dist_init caps nranks at 256, this keeps the packing honest on its own
    if (owners == 0 || owners > 0xFFFFu) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pc_item_owners_kernel, dim3((n_items + 255) / 256), dim3(256), 0, s, item_start, item_end,
                       n_items, starts, owners, item_owner);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Lead-range passes of the sharded count (sa_dist_count_pass).  A pass counts the
// partials of the leads in nr read ranges rg[2r] .. rg[2r + 1] (one range per lead
// owner), so the partials held at once are bounded by the pass, not by the read set.
// Its items are the ranges' reads cut every `target` local occurrences exactly as
// pc_items_kernel cuts all reads; range r's items are [ioff[r], ioff[r + 1]).
// ---------------------------------------------------------------------------
__global__ void pass_items_count_kernel(const uint64_t *occ_off, const uint32_t *rg, uint32_t nr, uint32_t target,
                                        uint32_t *ioff) {
    if (threadIdx.x || blockIdx.x) return;  // nr <= 256 ranges: one serial scan
    uint32_t acc = 0;
    for (uint32_t r = 0; r < nr; ++r) {
        ioff[r] = acc;
        const uint64_t n = occ_off[rg[2 * r + 1]] - occ_off[rg[2 * r]];
        acc += (uint32_t)((n + target - 1) / target);
    }
    ioff[nr] = acc;
}

// first read x in [a, b] with occ_off[x] >= v (occ_off[b] >= v)
__device__ __forceinline__ uint32_t occ_lower_bound(const uint64_t *occ_off, uint32_t a, uint32_t b, uint64_t v) {
    while (a < b) {
        const uint32_t mid = a + ((b - a) >> 1);
        if (occ_off[mid] < v) a = mid + 1; else b = mid;
    }
    return a;
}

__global__ void pass_items_fill_kernel(const uint64_t *occ_off, const uint32_t *rg, uint32_t nr, uint32_t target,
                                       const uint32_t *ioff, uint32_t n_items, uint32_t *istart, uint32_t *iend) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_items) return;
    uint32_t lo = 0, hi = nr;  // the range holding item j: largest r with ioff[r] <= j
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ioff[mid] <= j) lo = mid; else hi = mid;
    }
    const uint32_t t = j - ioff[lo], ni = ioff[lo + 1] - ioff[lo];
    const uint32_t a = rg[2 * lo], b = rg[2 * lo + 1];
    const uint64_t base = occ_off[a];
    istart[j] = t == 0 ? a : occ_lower_bound(occ_off, a, b, base + (uint64_t)t * target);
    iend[j] = t + 1 == ni ? b : occ_lower_bound(occ_off, a, b, base + (uint64_t)(t + 1) * target);
}

hipError_t launch_pass_items_count(const uint64_t *occ_off, const uint32_t *rg, uint32_t nr, uint32_t target,
                                   uint32_t *ioff, hipStream_t s) {
    if (nr == 0 || nr > 256) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pass_items_count_kernel, dim3(1), dim3(64), 0, s, occ_off, rg, nr, target, ioff);
    return hipGetLastError();
}

hipError_t launch_pass_items_fill(const uint64_t *occ_off, const uint32_t *rg, uint32_t nr, uint32_t target,
                                  const uint32_t *ioff, uint32_t n_items, uint32_t *istart, uint32_t *iend,
                                  hipStream_t s) {
    if (!n_items) return hipSuccess;
    hipLaunchKernelGGL(pass_items_fill_kernel, dim3((n_items + 255) / 256), dim3(256), 0, s, occ_off, rg, nr, target,
                       ioff, n_items, istart, iend);
    return hipGetLastError();
}

// Upper bound of the partials each read can lead on this rank: its local occurrences'
// partner-list elements (every element is at most one distinct (lead, partner) key,
// KmerTable.scala:57-80), bound[a].  Sums per lead owner into own[o] (o < owners) and the
// total into own[owners]: the host plans the lead-range passes from them.  One wave per 64
// consecutive reads walks their occurrences coalesced (a thread per read striding through
// its own records touched 64 lines per load: +0.7 ms per shard at the bench shape), finds
// each occurrence's read among the 65 staged starts and sums in LDS.
// abort (nullable): big partitions still to build (bucket_stage phase 1) -- their records
// are not written yet, so every block exits at once and the host runs this again later
constexpr int RB_WAVES = 4;
__global__ __launch_bounds__(RB_WAVES * 64) void read_bound_kernel(const uint64_t *occ_off, uint32_t n_reads, PairIn in,
                                                                   const uint32_t *starts, uint32_t owners,
                                                                   uint64_t *bound, unsigned long long *own,
                                                                   const uint32_t *abort) {
    if (abort && *abort) return;
    __shared__ uint32_t rbo[RB_WAVES][65];
    __shared__ unsigned long long acc[RB_WAVES][64];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t a0 = (blockIdx.x * RB_WAVES + wv) * 64u;
    if (a0 >= n_reads) return;  // (wave-uniform; no block barrier below)
    const uint32_t nr = min(64u, n_reads - a0);
    const uint64_t g0 = occ_off[a0], g1 = occ_off[a0 + nr];
    if (lane <= nr) rbo[wv][lane] = (uint32_t)(occ_off[a0 + lane] - g0);
    acc[wv][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    for (uint64_t g = g0 + lane; g < g1; g += 64) {
        const uint4 r = load_rec(in, g);
        const uint32_t rel = (uint32_t)(g - g0);
        uint32_t lo = 0, hi = nr;  // largest read index l with rbo[l] <= rel
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (rbo[wv][mid] <= rel) lo = mid; else hi = mid;
        }
        atomicAdd(&acc[wv][lo], (unsigned long long)((r.y & 0x3FFFFFFFu) + r.w));
    }
    __builtin_amdgcn_wave_barrier();
    const uint64_t s = lane < nr ? acc[wv][lane] : 0ull;
    unsigned long long t = s;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
    // per read, and per block of 64 reads after them (bound[n_reads + 1 + a0 / 64]): a plan
    // over many reads reads back the blocks' (8 B per 64 reads)
    if (lane < nr) bound[a0 + lane] = s;
    if (lane == 0) bound[n_reads + 1 + (a0 >> 6)] = t;
    // one atomic per wave and owner: a wave's reads are consecutive, so nearly always
    // one owner (the first and last read agree)
    const uint32_t ow0 = owner_of(starts, owners, a0), ow1 = owner_of(starts, owners, a0 + nr - 1);
    if (ow0 == ow1) {
        if (lane == 0) {
            atomicAdd(&own[ow0], t);
            atomicAdd(&own[owners], t);
        }
    } else if (lane < nr && s) {
        atomicAdd(&own[owner_of(starts, owners, a0 + lane)], (unsigned long long)s);
        atomicAdd(&own[owners], (unsigned long long)s);
    }
}

hipError_t launch_read_bound(const uint64_t *occ_off, uint32_t n_reads, const PairIn &in, const uint32_t *starts,
                             uint32_t owners, uint64_t *bound, unsigned long long *own, hipStream_t s,
                             const uint32_t *abort) {
    if (owners == 0 || owners > 256) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(own, 0, ((size_t)owners + 1) * sizeof(unsigned long long), s);
    if (e != hipSuccess || !n_reads) return e;
    hipLaunchKernelGGL(read_bound_kernel, dim3((n_reads + RB_WAVES * 64 - 1) / (RB_WAVES * 64)), dim3(RB_WAVES * 64), 0,
                       s, occ_off, n_reads, in, starts, owners, bound, own, abort);
    return hipGetLastError();
}

hipError_t launch_pc_items(const uint64_t *occ_off, uint32_t n_reads, uint32_t target, uint32_t n_items,
                           uint32_t *item_start, hipStream_t s) {
    hipLaunchKernelGGL(pc_items_kernel, dim3((n_items + 1 + 255) / 256), dim3(256), 0, s, occ_off, n_reads, target,
                       n_items, item_start);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// output ordering helpers
// ---------------------------------------------------------------------------
// exclusive prefix of the NSHARD region counts (one tiny block)
__global__ void shard_offsets_kernel(const unsigned long long *cursor, unsigned long long cap_s, uint32_t *off) {
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int i = 0; i < NSHARD; ++i) {
            off[i] = acc;
            acc += (uint32_t)min(cursor[i], cap_s);
        }
        off[NSHARD] = acc;
    }
}

__global__ void make_order_keys_kernel(const uint32_t *fst, const uint32_t *snd, const uint64_t *rank,
                                       const unsigned long long *cursor, unsigned long long cap_s, int by_rank,
                                       int idbits, uint64_t *keys, uint32_t *vals, const uint32_t *off,
                                       const uint32_t *starts, uint32_t P) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // region-space index
    const uint32_t shard = (uint32_t)(i / cap_s);
    if (shard >= NSHARD) return;
    const uint64_t j = i - (uint64_t)shard * cap_s;
    if (j >= cursor[shard]) return;
    const uint32_t pos = off[shard] + (uint32_t)j;
    // wide: lead descending then trail ascending; strict: first-occurrence rank
    const uint64_t top = (1ull << idbits) - 1;
    // by_rank 0: lead descending, trail ascending (wide canonical order);
    // 1: first-occurrence rank (strict); 3: the rank owning the lead (distributed
    // send side: starts[P + 1], largest o with starts[o] <= lead)
    uint64_t key;
    if (by_rank == 3) {
        uint32_t lo = 0, hi = P;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (starts[mid] <= fst[i]) lo = mid; else hi = mid;
        }
        key = lo;
    } else {
        key = by_rank == 1 ? rank[i] : (((top - fst[i]) << idbits) | snd[i]);
    }
    keys[pos] = key;
    vals[pos] = (uint32_t)i;
}

hipError_t launch_make_order_keys(const uint32_t *fst, const uint32_t *snd, const uint64_t *rank,
                                  const unsigned long long *cursor, unsigned long long cap_s, int by_rank,
                                  int idbits, uint64_t *keys, uint32_t *vals, uint32_t *shard_off,
                                  hipStream_t s, const uint32_t *starts, uint32_t P) {
    hipLaunchKernelGGL(shard_offsets_kernel, dim3(1), dim3(64), 0, s, cursor, cap_s, shard_off);
    const uint64_t tot = (uint64_t)NSHARD * cap_s;
    hipLaunchKernelGGL(make_order_keys_kernel, dim3((uint32_t)((tot + 255) / 256)), dim3(256), 0, s, fst, snd, rank,
                       cursor, cap_s, by_rank, idbits, keys, vals, (const uint32_t *)shard_off, starts, P);
    return hipGetLastError();
}

__global__ void gather_pairs_kernel(const uint32_t *perm, uint64_t n, const uint32_t *fst, const uint32_t *snd,
                                    const uint32_t *cnt, int32_t *lead, int32_t *trail, int32_t *count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = perm[i];
    lead[i] = (int32_t)fst[j] + 1;  // reference ids are 1-based
    trail[i] = (int32_t)snd[j] + 1;
    count[i] = (int32_t)cnt[j];
}

// one wave per read: its region's entries to their place in the lead-descending
// dispatch list, offset = (sum of the counts of reads above it) = total - ex - cnt;
// a read the recount tiers handled (rsh[a] != 0) copies its segment of the
// sorted shared list instead
__global__ void copy_read_regions_kernel(const uint2 *rreg, const uint32_t *rcnt, const uint32_t *ex,
                                         const uint32_t *total, uint32_t n_reads, const uint32_t *rsh,
                                         const int32_t *sh_trail, const int32_t *sh_count, int32_t *lead,
                                         int32_t *trail, int32_t *count) {
    const uint32_t a = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (a >= n_reads) return;
    const uint32_t m = rcnt[a];
    const uint32_t off = *total - ex[a] - m;
    const uint32_t h = rsh ? rsh[a] : 0u;
    if (h) {
        for (uint32_t j = threadIdx.x & 63u; j < m; j += 64) {
            lead[off + j] = (int32_t)a + 1;
            trail[off + j] = sh_trail[h - 1 + j];  // (already 1-based)
            count[off + j] = sh_count[h - 1 + j];
        }
        return;
    }
    for (uint32_t j = threadIdx.x & 63u; j < m; j += 64) {
        const uint2 v = rreg[(uint64_t)a * PC_RREG + j];
        lead[off + j] = (int32_t)a + 1;  // reference ids are 1-based
        trail[off + j] = (int32_t)v.x + 1;
        count[off + j] = (int32_t)v.y;
    }
}

hipError_t launch_copy_read_regions(const uint2 *rreg, const uint32_t *rcnt, const uint32_t *ex,
                                    const uint32_t *total, uint32_t n_reads, const uint32_t *rsh,
                                    const int32_t *sh_trail, const int32_t *sh_count, int32_t *lead, int32_t *trail,
                                    int32_t *count, hipStream_t s) {
    if (!n_reads) return hipSuccess;
    hipLaunchKernelGGL(copy_read_regions_kernel, dim3((n_reads + 3) / 4), dim3(256), 0, s, rreg, rcnt, ex, total,
                       n_reads, rsh, sh_trail, sh_count, lead, trail, count);
    return hipGetLastError();
}

// segment heads first (rsh = 1 + start), then the tails read them (rcnt = length)
__global__ void mark_heads_kernel(const int32_t *lead, uint64_t n, uint32_t *rsh) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i == 0 || lead[i - 1] != lead[i]) rsh[lead[i] - 1] = (uint32_t)i + 1u;
}
__global__ void mark_tails_kernel(const int32_t *lead, uint64_t n, const uint32_t *rsh, uint32_t *rcnt) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i + 1 == n || lead[i + 1] != lead[i]) rcnt[lead[i] - 1] = (uint32_t)i + 2u - rsh[lead[i] - 1];
}

hipError_t launch_mark_segments(const int32_t *lead, uint64_t n, uint32_t *rsh, uint32_t *rcnt, hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 grid((uint32_t)((n + 255) / 256));
    hipLaunchKernelGGL(mark_heads_kernel, grid, dim3(256), 0, s, lead, n, rsh);
    hipLaunchKernelGGL(mark_tails_kernel, grid, dim3(256), 0, s, lead, n, (const uint32_t *)rsh, rcnt);
    return hipGetLastError();
}

hipError_t launch_gather_pairs(const uint32_t *perm, uint64_t n, const uint32_t *fst, const uint32_t *snd,
                               const uint32_t *cnt, int32_t *lead, int32_t *trail, int32_t *count, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(gather_pairs_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, perm, n, fst, snd,
                       cnt, lead, trail, count);
    return hipGetLastError();
}

}  // namespace sa
