// partition.hip -- bucket build by hash partition, finished in LDS (gfx950).
//
// After two stable radix passes on the top P bits of mix(seqHash) the k-mer
// records form 2^P partitions, each holding whole buckets (a bucket = one
// distinct hash = one KmerData entry, KmerTable.scala:41-53) in (read, pos)
// order.  One 256-thread workgroup per partition then, entirely in LDS:
//   1. bitonic-sorts its records by (key = mix << lb | locrank, g),
//   2. finds bucket heads (new hash) and group heads (new hash or loc),
//   3. scans middle flags / edge-role counts, last bucket/group head, next group head,
//   4. writes each bucket's slice of the combined partner list (read index per
//      entry) into the partition's slice lst[3 ps, 3 ps + 3 n) (no global scan
//      needed), middle entries loc-descending before the split point c, edge
//      roles loc-ascending after it (sa_internal.h), and one 8-byte record per
//      k-mer, scattered to its occurrence index g: {c, nE | nD << 15 | me << 30}
//      edge role partners  = md entries of the bucket with loc <  own: [c - nE, c)
//      middle role partners = edge entries of the bucket with loc <= own: [c, c + nD)
//      (addKmerPair's orientation rule, KmerTable.scala:65-71: fst = larger loc, tie -> middle)
//      The scattered store is what this kernel spends most of its time on (a
//      random 16-byte store over 778 MB costs 1.57 ms at the bench shape, an
//      8-byte one over 389 MB 0.89 ms: tools/scatter_probe.hip), hence 8 bytes.
// Strict mode also writes the (read,pos)-order list indices calcPairData's
// traversal order is built from, per-bucket |st|, |md| and first occurrence.
// Partitions larger than the LDS capacity take the global scan path
// (buckets.hip) and records_from_tables_kernel below.  Bound: HBM / LDS.
#include "../sa_internal.h"

namespace sa {

// read of occurrence g.  Uniform lengths: floor(g / npr) as the high word of
// g * M, M = floor((2^64 - 1) / npr) + 1 (PartArgs::npr_magic, host-side): M =
// 2^64 / npr + e with 0 <= e < 1, so g * M / 2^64 = g / npr + (< 2^-32), which
// never reaches the next integer for g, npr < 2^32 -- a few multiplies instead
// of the ~35-instruction integer-division expansion, twice per record
__device__ __forceinline__ uint32_t read_of_g(uint32_t g, const uint64_t *occ_off, uint32_t n_reads, uint32_t npr,
                                              uint64_t npr_magic) {
    if (npr) return npr == 1 ? g : (uint32_t)__umul64hi((unsigned long long)g, (unsigned long long)npr_magic);
    uint32_t lo = 0, hi = n_reads;  // largest r with occ_off[r] <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (occ_off[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

// the sorted 8-byte records are read once: non-temporal loads keep them out of
// L2, which is left to merge the scattered record stores
__device__ __forceinline__ uint64_t load_sk(const uint64_t *p) { return __builtin_nontemporal_load(p); }

// sort key (mix << lb | loc rank) and occurrence code of an 8-byte record: the
// occurrence index g, or (pos_bits > 0: mixed read lengths) read << pos_bits |
// pos, whose read meta {first occurrence, loc-rank base} gives g and the loc
// rank with one load (instead of a search over the occurrence offsets); with
// an occurrence table, the record's {read, loc rank} entry rlp gives the loc
// rank and the read (rr, else untouched)
__device__ __forceinline__ unsigned long long record_key(uint64_t rec, const PartArgs &A, uint32_t &code,
                                                         uint32_t &rr, const uint2 *rlp, const uint32_t *pvp) {
    code = (uint32_t)rec;
    const uint32_t g = code;
    uint32_t lr;
    if (A.pos_bits) {
        const uint32_t pos = code & ((1u << A.pos_bits) - 1u);
        lr = A.lrank[A.meta[code >> A.pos_bits].y + pos];
    } else if (pvp) {  // packed read << lb | loc rank
        const uint32_t v = *pvp;
        lr = v & ((1u << A.lb) - 1u);
        rr = v >> A.lb;
        if (A.src_shift) {  // source-relative: the source from the key's top bits, then the owner's bits back
            const uint32_t s = (uint32_t)(rec >> A.src_shift);
            rr += A.src_starts[s];
            const uint64_t low = (1ull << A.src_shift) - 1ull;
            rec = (rec & low) | ((uint64_t)A.src_own << 32);
        }
    } else if (rlp) {
        const uint2 v = *rlp;
        lr = v.y;
        rr = v.x;
    } else {
        const uint32_t r = read_of_g(g, A.occ_off, A.n_reads, A.npr, A.npr_magic);
        const uint32_t pos = A.npr ? g - r * A.npr : g - (uint32_t)A.occ_off[r];
        if (A.lr_ident) {
            lr = pos;
        } else {
            const int32_t d = A.npr ? (int32_t)A.npr - 1 : A.len[r] - A.k;
            lr = A.lrank[A.lbase[d] + pos];
        }
    }
    return ((rec >> 32) << A.lb) | lr;
}

// ---------------------------------------------------------------------------
// the LDS partition builder
// ---------------------------------------------------------------------------
// A tier of CAP records runs CAP / 4 threads (4 items each): the 1,024-record
// tier 4 waves, the 2,048-record tier 8, the 4,096-record tier 16.  A block's
// latency is set by its chain of LDS passes and barriers, nearly the same for
// any CAP at 4 items per thread, so bigger partitions spread that chain over
// more records.
constexpr uint32_t SPLIT_MAX = 2048;  // partitions the split tier takes (grid 2 SPLIT_MAX)
template <int CAP> struct PbShape {
    static constexpr int NT = CAP / 4, WAVES = NT / 64, IT = 4;
};

template <int CAP>
struct PartShared {
    static constexpr int WAVES = PbShape<CAP>::WAVES;
    unsigned long long key[CAP];
    uint32_t g[CAP];                 // occurrence code of load slot i
    uint16_t oi[CAP];                // load slot of sorted item s (moves with the key)
    // the sort's digit counts are dead once the partition is sorted and the
    // per-item counts are only written after it: one region, and 16-bit counts
    // (<= 2 * CAP), so the 1,024-record block fits 18.5 KB -> 8 blocks per CU
    union {
        struct {
            uint32_t cnt[WAVES][256];  // LDS radix sort: per-wave digit counts
            uint16_t ofs[WAVES][256];  // each wave's scatter base per digit
        };
        struct {
            uint16_t mdx[CAP + 2];     // exclusive md count (partition-local)
            uint16_t edx[CAP + 2];     // exclusive edge-role count
            uint4 agg[WAVES];          // per-wave inclusive aggregates of the combined block scan
            uint2 aggu[WAVES];
        };
    };
};
// (with an occurrence table, a u32 read per load slot follows in dynamic LDS)
static_assert(sizeof(PartShared<1024>) <= 20480, "1,024-record block must fit 8 per CU");

// Stable LSD radix sort of the partition's (key, load slot) in LDS over key bits
// [0, bits): wave w owns elements [w*CAP/4, (w+1)*CAP/4) (slices of 64), ranks
// come from a 64-lane ballot multisplit + wave-private counts, elements are held
// in registers across the scatter.  Every wave derives its own scatter bases
// from all waves' counts (lane l: digits 4l..4l+3), so a pass has two block
// barriers (counts complete; scatter complete).
template <int CAP, class SH>
__device__ __forceinline__ void lds_radix_sort(SH &S, uint32_t n, int bits) {
    constexpr int WAVES = PbShape<CAP>::WAVES;
    constexpr int SUB = CAP / WAVES, SL = SUB / 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int shift = 0; shift < bits; shift += 8) {
        // digit width of this pass: the last one ranks only the bits that are
        // left (25-bit keys: 8 + 8 + 8 + 1 ballots, not 32)
        const int nbits = bits - shift < 8 ? bits - shift : 8;
        const uint32_t dmask = (1u << nbits) - 1u;
        reinterpret_cast<uint4 *>(S.cnt[w])[lane] = make_uint4(0, 0, 0, 0);
        // per element: the key, and its load slot | rank among equal digits << 16
        // in one register (ranks < 2 CAP); the digit is recomputed from the key
        unsigned long long k[SL];
        uint32_t gr[SL];
#pragma unroll
        for (int j = 0; j < SL; ++j) {
            const uint32_t i = w * SUB + j * 64 + lane;
            k[j] = i < n ? S.key[i] : 0ull;
            gr[j] = i < n ? S.oi[i] : 0u;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < SL; ++j) {
            const uint32_t i = w * SUB + j * 64 + lane;
            const bool valid = i < n;
            const uint32_t d = (uint32_t)(k[j] >> shift) & dmask;
            const uint64_t peer = wave_peers(d, valid, nbits);
            const uint32_t before = valid ? S.cnt[w][d] : 0u;
            gr[j] |= (before + __popcll(peer & lt_mask)) << 16;
            __builtin_amdgcn_wave_barrier();
            if (valid && (peer & lt_mask) == 0) S.cnt[w][d] = before + __popcll(peer);
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();  // counts complete; every element is in registers
        {
            uint32_t tot[4] = {0, 0, 0, 0}, mine[4] = {0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < WAVES; ++q) {
                const uint4 c = reinterpret_cast<const uint4 *>(S.cnt[q])[lane];
                tot[0] += c.x; tot[1] += c.y; tot[2] += c.z; tot[3] += c.w;
                if (q < w) { mine[0] += c.x; mine[1] += c.y; mine[2] += c.z; mine[3] += c.w; }
            }
            const uint32_t lsum = tot[0] + tot[1] + tot[2] + tot[3];
            uint32_t acc = wave_incl_add(lsum) - lsum;  // digits below 4 * lane, all waves
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                S.ofs[w][4 * lane + i] = (uint16_t)(acc + mine[i]);
                acc += tot[i];
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < SL; ++j) {
            const uint32_t i = w * SUB + j * 64 + lane;
            if (i < n) {
                const uint32_t pos = S.ofs[w][(uint32_t)(k[j] >> shift) & dmask] + (gr[j] >> 16);
                S.key[pos] = k[j];
                S.oi[pos] = (uint16_t)gr[j];
            }
        }
        __syncthreads();  // scatter complete; the counts may be cleared
    }
}

// One partition p in one block.  Partitions above CAP records are handed on:
// the 1,024-record kernel lists them for the 2,048-record pass (mid_list), that
// pass lists its overflow for the 4,096-record pass (mid2_list), and that one
// lists the partitions above 4,096 for the global path (big_list).
// a partition's bounds and its records, loaded into registers (all of a
// thread's loads issued before any is used)
template <int CAP>
struct PartLoad {
    uint32_t ps, n;
    uint64_t recs[PbShape<CAP>::IT];
};
template <int CAP>
__device__ __forceinline__ void part_load(const PartArgs &A, const uint32_t p, PartLoad<CAP> &L) {
    constexpr int IT = PbShape<CAP>::IT, NT = PbShape<CAP>::NT;
    L.ps = A.start[p];
    L.n = A.start[p + 1] - L.ps;
    if (L.n == 0 || L.n > (uint32_t)CAP) return;
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint32_t i = threadIdx.x + j * NT;
        L.recs[j] = load_sk(A.sk + L.ps + (i < L.n ? i : L.n - 1));
    }
}

// timing probe builds (make OUT=build_stamps EXTRA=-DSA_PB_STAMPS=1): thread 0
// of each main-pass block records wall_clock64() at its phase boundaries
#ifdef SA_PB_STAMPS
#define PB_STAMP(A, p, i)                                                              \
    do {                                                                               \
        if (CAP == 1024 && threadIdx.x == 0 && (A).stamps) (A).stamps[8 * (uint64_t)(p) + (i)] = wall_clock64(); \
    } while (0)
#else
#define PB_STAMP(A, p, i) do { } while (0)
#endif

template <int CAP, bool STRICT>
__device__ __forceinline__ void part_build_one(const PartArgs &A, const uint32_t p, PartShared<CAP> &S,
                                               uint32_t *Sr, const PartLoad<CAP> &L) {
    constexpr int IT = PbShape<CAP>::IT, NT = PbShape<CAP>::NT;
    const int tid = threadIdx.x;
    const uint32_t ps = L.ps;
    const uint32_t n = L.n;
    if (n == 0) return;
    if (n > (uint32_t)CAP) {  // (the bounds kernel listed the partitions above 1,024)
        if (tid == 0) {
            if (CAP >= 4096) A.big_list[atomicAdd(A.big_n, 1u)] = p;
            else if (CAP >= 2048) A.mid2_list[atomicAdd(A.mid2_n, 1u)] = p;
        }
        return;
    }
    // ---- load, then stable LDS radix sort on the key bits below the partition id
    //      (all of a thread's record loads are issued before any is used, so a
    //      block waits one HBM latency here, not one per record)
    {
        const uint64_t *recs = L.recs;
        // (keys of the clamped slots too: their loc-rank gathers issue together)
        unsigned long long kk[IT];
        uint32_t gg[IT], rr[IT];
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t i = tid + j * NT, ic = i < n ? i : n - 1;
            rr[j] = 0;
            const uint2 *rlp = A.srl ? A.srl + ps + ic : (A.rl ? A.rl + (uint32_t)recs[j] : nullptr);
            const uint32_t *pvp = A.spv ? A.spv + ps + ic : (A.pv ? A.pv + (uint32_t)recs[j] : nullptr);
            kk[j] = record_key(recs[j], A, gg[j], rr[j], rlp, pvp);
        }
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t i = tid + j * NT;
            if (i < n) {
                S.key[i] = kk[j];
                S.g[i] = gg[j];
                S.oi[i] = (uint16_t)i;
                if (Sr) Sr[i] = rr[j];
            }
        }
    }
    __syncthreads();
    PB_STAMP(A, p, 1);
    lds_radix_sort<CAP>(S, n, A.sort_bits);
    PB_STAMP(A, p, 2);
    // ---- per-thread contiguous items: flags and local aggregates -----------
    const int lb = A.lb;
    const unsigned long long lbm = (1ull << lb) - 1;
    const uint32_t b0 = tid * IT;
    uint32_t md_c = 0, ed_c = 0, last_bh = 0, last_gh = 0, first_gh = 0xFFFFFFFFu, first_bh = 0xFFFFFFFFu;
    uint32_t n_bh = 0, n_gh = 0;
    uint32_t tagp = 0;          // item j's tag bits at 4 j (one register for the IT tags)
    uint32_t fbh = 0, fgh = 0;  // bit j: item b0 + j heads a bucket / a loc group (kept for the outputs)
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint32_t s = b0 + j;
        if (s < n) {
            const unsigned long long k = S.key[s];
            const uint32_t t = part_tag(A, (uint32_t)(k & lbm));
            tagp |= t << (4 * j);
            const bool bh = s == 0 || (S.key[s - 1] >> lb) != (k >> lb);
            const bool gh = s == 0 || S.key[s - 1] != k;
            fbh |= bh ? 1u << j : 0u;
            fgh |= gh ? 1u << j : 0u;
            md_c += (t & TAG_MD) ? 1u : 0u;
            ed_c += ((t & TAG_ST) ? 1u : 0u) + ((t & TAG_EN) ? 1u : 0u);
            if (bh) { last_bh = s; ++n_bh; if (first_bh == 0xFFFFFFFFu) first_bh = s; }
            if (gh) { last_gh = s; ++n_gh; if (first_gh == 0xFFFFFFFFu) first_gh = s; }
        }
    }
    // one combined block scan (one barrier): exclusive sums of (md | edge << 16)
    // and (bucket heads | group heads << 16) as DPP add-scans; the exclusive
    // prefix max of the last bucket / group head and the exclusive suffix min
    // of the first group / bucket head are each one lane's value -- the nearest
    // lane below / above holding a head (head positions grow with the lane) --
    // found by ballot and fetched with one bpermute (element 0 is always a
    // head; counts < 2^16)
    uint32_t sme = md_c | (ed_c << 16), shd = n_bh | (n_gh << 16);
    const uint32_t sme0 = sme;
    const int lane = tid & 63, wv = tid >> 6;
    sme = wave_incl_add(sme);
    shd = wave_incl_add(shd);
    const uint64_t bb = __ballot(n_bh != 0), bg = __ballot(n_gh != 0);
    const uint64_t below = (1ull << lane) - 1ull, above = ~below << 1;  // lanes < lane, lanes > lane
    // (63 - clz / ctz of an empty mask select an out-of-wave lane: masked below)
    const int lbb = 63 - __clzll(bb & below), lbg = 63 - __clzll(bg & below);
    const int lab = __ffsll((long long)(bb & above)) - 1, lag = __ffsll((long long)(bg & above)) - 1;
    uint32_t xbh = (uint32_t)__shfl((int)last_bh, lbb & 63, 64), xgh = (uint32_t)__shfl((int)last_gh, lbg & 63, 64);
    uint32_t xubh = (uint32_t)__shfl((int)first_bh, lab & 63, 64), xugh = (uint32_t)__shfl((int)first_gh, lag & 63, 64);
    if (!(bb & below)) xbh = 0;
    if (!(bg & below)) xgh = 0;
    if (!(bb & above)) xubh = 0xFFFFFFFFu;
    if (!(bg & above)) xugh = 0xFFFFFFFFu;
    // wave aggregates: the highest / lowest lane holding a head
    const uint32_t mbh = bb ? (uint32_t)__builtin_amdgcn_readlane((int)last_bh, 63 - __clzll(bb)) : 0u;
    const uint32_t mgh = bg ? (uint32_t)__builtin_amdgcn_readlane((int)last_gh, 63 - __clzll(bg)) : 0u;
    const uint32_t ubh = bb ? (uint32_t)__builtin_amdgcn_readlane((int)first_bh, __ffsll((long long)bb) - 1) : 0xFFFFFFFFu;
    const uint32_t ugh = bg ? (uint32_t)__builtin_amdgcn_readlane((int)first_gh, __ffsll((long long)bg) - 1) : 0xFFFFFFFFu;
    if (lane == 63) S.agg[wv] = make_uint4(sme, shd, mbh, mgh);
    if (lane == 0) S.aggu[wv] = make_uint2(ugh, ubh);
    sme -= sme0;
    __syncthreads();
    uint32_t blk_heads = 0;
#pragma unroll
    for (int q = 0; q < PbShape<CAP>::WAVES; ++q) {
        const uint4 a = S.agg[q];
        const uint2 u = S.aggu[q];
        blk_heads += a.y;
        if (q < wv) { sme += a.x; xbh = max(xbh, a.z); xgh = max(xgh, a.w); }
        if (q > wv) { xugh = min(xugh, u.x); xubh = min(xubh, u.y); }
    }
    const uint32_t md_ex = sme & 0xFFFFu, ed_ex = sme >> 16;
    const uint32_t bh_in = xbh, gh_in = xgh;
    const uint32_t gh_next = min(xugh, n), bh_next = min(xubh, n);
    // per-item exclusive counts into LDS
    {
        uint32_t m = md_ex, e = ed_ex;
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t s = b0 + j;
            if (s <= n) { S.mdx[s] = m; S.edx[s] = e; }
            const uint32_t t = (tagp >> (4 * j)) & 15u;
            m += (t & TAG_MD) ? 1u : 0u;
            e += ((t & TAG_ST) ? 1u : 0u) + ((t & TAG_EN) ? 1u : 0u);
        }
        if (b0 + IT == (uint32_t)CAP && n == (uint32_t)CAP) { S.mdx[CAP] = m; S.edx[CAP] = e; }
    }
    __syncthreads();
    PB_STAMP(A, p, 3);
    // next group head and next bucket head of item j: the thread's next head
    // bit above j (fgh / fbh), else gh_next / bh_next -- recomputed where used,
    // not held in 2 IT registers
    auto next_head = [&](uint32_t f, int j, uint32_t nxt) -> uint32_t {
        const uint32_t above = f >> (j + 1);
        return above ? b0 + (uint32_t)j + 1u + (uint32_t)__builtin_ctz(above) : nxt;
    };
    // ---- outputs --------------------------------------------------------
    // The partition's list slice [3 ps, 3 ps + ltot) is assembled in LDS (the
    // key array is free once the heads are found; 2 CAP words hold any default
    // tag layout, <= 2 entries per record) and leaves as coalesced non-temporal
    // stores: the ~230 MB of lists then stay out of the 256 MB MALL, which is
    // left to merge the records' scattered 8-byte stores (389 MB at the bench).
    // Same box (profiles/r04/ab/ab_lst_staged_nt.txt): bucket build 1.32 ->
    // 1.20 ms; staged with plain stores 1.32 (SA_LST_STAGE A/B: 0 direct
    // scattered stores, 1 staged, 2 staged + non-temporal)
#ifndef SA_LST_STAGE
#define SA_LST_STAGE 2
#endif
    uint32_t *stg = reinterpret_cast<uint32_t *>(S.key);
    const uint32_t ltot = S.mdx[n] + S.edx[n];
    const bool staged = SA_LST_STAGE && !STRICT && ltot <= 2u * (uint32_t)CAP;
    const uint64_t lbase = 3ull * ps;
    uint32_t bh = bh_in, gh = gh_in;
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint32_t s = b0 + j;
        if (s >= n) break;
        const bool isb = (fbh >> j) & 1u, isg = (fgh >> j) & 1u;
        if (isb) bh = s;
        if (isg) gh = s;
        const uint32_t t = (tagp >> (4 * j)) & 15u;
        const uint32_t slot = S.oi[s];
        const uint32_t code = S.g[slot];
        uint32_t r, g;
        if (A.pos_bits) {  // read << pos_bits | pos (record_key)
            r = code >> A.pos_bits;
            g = A.meta[r].x + (code & ((1u << A.pos_bits) - 1u));
        } else {
            g = code;
            r = Sr ? Sr[slot] : read_of_g(g, A.occ_off, A.n_reads, A.npr, A.npr_magic);
        }
        const uint32_t st = (t & TAG_ST) ? 1u : 0u, en = (t & TAG_EN) ? 1u : 0u, md = (t & TAG_MD) ? 1u : 0u;
        // split point of the bucket [bh, nextb): its md entries end at c
        const uint64_t c = 3ull * ps + S.mdx[next_head(fbh, j, bh_next)] + S.edx[bh];
        const uint64_t mpos = c - 1u - (S.mdx[s] - S.mdx[bh]), epos = c + (S.edx[s] - S.edx[bh]);
        if (staged) {
            if (md) stg[mpos - lbase] = r;
            if (st) stg[epos - lbase] = r;
            if (en) stg[epos + st - lbase] = r;
        } else {
            if (md) A.lst[mpos] = r;
            if (st) A.lst[epos] = r;
            if (en) A.lst[epos + st] = r;
        }
        const uint32_t me = st + en;
        const uint32_t nE = me ? (S.mdx[gh] - S.mdx[bh]) : 0u;        // <= CAP: no escape here
        const uint32_t nD = md ? (S.edx[next_head(fgh, j, gh_next)] - S.edx[bh]) : 0u;  // <= 2 CAP
        A.rec[g] = encode_rec(c, nE, nD, me);
#ifdef SA_PB_PROBE_DUP
        if (A.rec_dup) A.rec_dup[g] = encode_rec(c, nE, nD, me);  // (probe: twice the scattered stores)
#endif
        if constexpr (STRICT) {
            // bucket extent [bh, be)
            const unsigned long long k = S.key[s];
            uint32_t be = s + 1;
            while (be < n && (S.key[be] >> lb) == (k >> lb)) ++be;
            uint32_t nst = 0, nmd = 0, nen = 0, st_tot = 0, md_tot = 0, gmin = 0xFFFFFFFFu;
            for (uint32_t q = bh; q < be; ++q) {
                const uint32_t tq = A.tagtab[S.key[q] & lbm];
                const uint32_t gq = S.g[S.oi[q]];
                st_tot += (tq & TAG_ST) ? 1u : 0u;
                md_tot += (tq & TAG_MD) ? 1u : 0u;
                gmin = min(gmin, gq);
                if (gq < g) {
                    nst += (tq & TAG_ST) ? 1u : 0u;
                    nmd += (tq & TAG_MD) ? 1u : 0u;
                    nen += (tq & TAG_EN) ? 1u : 0u;
                }
            }
            if (md) A.lidx[mpos] = nmd;
            if (st) A.lidx[epos] = nst;
            if (en) A.lidx[epos + st] = (1u << 31) | nen;
            A.srec[g] = make_uint4(ps + bh, st ? nst : ((1u << 31) | nen), nmd, 0u);
            if (isb) {
                A.bkt_nst[ps + s] = st_tot;
                A.bkt_nmd[ps + s] = md_tot;
                A.bkt_first[ps + s] = gmin;
                A.is_head[ps + s] = 1;
            }
        }
    }
    if (staged) {
        __syncthreads();
        for (uint32_t i = tid; i < ltot; i += NT) {
            if (SA_LST_STAGE == 2) __builtin_nontemporal_store(stg[i], A.lst + lbase + i);
            else A.lst[lbase + i] = stg[i];
        }
    }
    PB_STAMP(A, p, 4);
#ifdef SA_PB_STAMPS
    if (CAP == 1024 && tid == 0 && A.stamps) A.stamps[8 * (uint64_t)p + 5] = (uint64_t)__smid() | ((uint64_t)n << 32);
#endif
    // bucket / group counts for statistics (block totals of the combined scan), sharded
    if (tid == 0) {
        atomicAdd(&A.counts[p % NSHARD], (unsigned long long)(blk_heads & 0xFFFFu));
        atomicAdd(&A.counts[NSHARD + p % NSHARD], (unsigned long long)(blk_heads >> 16));
    }
}

// CAP 1,024: one block per partition.  CAP 2,048 / 4,096: a fixed grid walks
// the list the previous pass handed on (~1% of partitions at 20x coverage) -- no
// block is spent reading the bounds of a partition already built while holding
// 44 / 84 KB of LDS, and a partition of ~1,100 records is sorted over 2,048
// slots, not 4,096 (the tail of the stage is one such block's latency).
template <int CAP, bool STRICT, bool MAIN>
__global__ __launch_bounds__(PbShape<CAP>::NT) void part_build_kernel(PartArgs A) {
    extern __shared__ __align__(16) uint8_t smem_raw[];
    PartShared<CAP> &S = *reinterpret_cast<PartShared<CAP> *>(smem_raw);
    uint32_t *Sr = A.rl || A.pv ? reinterpret_cast<uint32_t *>(smem_raw + sizeof(PartShared<CAP>)) : nullptr;
    if constexpr (MAIN) {
        // the main pass: one block per partition (two per block, the second's
        // records loading while the first is built, measured no faster: 1.32 ms
        // either way, profiles/r04/ab/ab_tier_order_pair_build.txt)
        PartLoad<CAP> L;
        PB_STAMP(A, blockIdx.x, 0);
        part_load<CAP>(A, blockIdx.x, L);
        part_build_one<CAP, STRICT>(A, blockIdx.x, S, Sr, L);
    } else {
        // (split tier: the partitions it handed on, then the mid-list entries past its grid)
        const bool fb = CAP < 4096 && A.split;
        const uint32_t *list = CAP >= 4096 ? A.mid2_list : (fb ? A.fb_list : A.mid_list);
        const uint32_t m0 = *(CAP >= 4096 ? A.mid2_n : (fb ? A.fb_n : A.mid_n));
        const uint32_t mid = fb ? *A.mid_n : 0u, extra = mid > SPLIT_MAX ? mid - SPLIT_MAX : 0u;
        for (uint32_t i = blockIdx.x; i < m0 + extra; i += gridDim.x) {
            __syncthreads();  // LDS of the previous partition fully consumed
            const uint32_t p = i < m0 ? list[i] : A.mid_list[SPLIT_MAX + (i - m0)];
            PartLoad<CAP> L;
            part_load<CAP>(A, p, L);
            part_build_one<CAP, STRICT>(A, p, S, Sr, L);
        }
    }
}

// The split tier (PartArgs::split): a partition of 1,025-2,048 records is built
// as two halves -- the next hash bit below the partition id, so every bucket
// stays whole in one half -- by two 1,024-record blocks, each loading the whole
// partition and keeping its half in load order (one block scan).  Half h's list
// slice starts at 3 (ps + h n0).  These blocks have the main pass's shape and
// interleave with it; the 2,048-record blocks they replace (8 waves, 37 KB of
// LDS, ~650 partitions at the bench shape) were starved beside the main pass and
// then crowded its last ~200 us (profiles/r04/pb_stamps.txt).  Partitions whose
// halves do not fit 1,024 records go to the 2,048-record pass (fb_list), those
// above 2,048 to the 4,096-record pass.
#ifndef SA_SPLIT_MIN_WAVES
#define SA_SPLIT_MIN_WAVES 6  // per SIMD: <= 80 VGPRs, near the main pass's 7
#endif
__global__ __launch_bounds__(PbShape<1024>::NT, SA_SPLIT_MIN_WAVES) void part_split_kernel(PartArgs A) {
    constexpr int CAP = 1024, NT = PbShape<CAP>::NT, IT = PbShape<CAP>::IT, R = 2 * CAP / NT;
    extern __shared__ __align__(16) uint8_t smem_raw[];
    PartShared<CAP> &S = *reinterpret_cast<PartShared<CAP> *>(smem_raw);
    uint32_t *Sr = A.rl || A.pv ? reinterpret_cast<uint32_t *>(smem_raw + sizeof(PartShared<CAP>)) : nullptr;
    __shared__ uint32_t wtot[NT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t m = min(*A.mid_n, SPLIT_MAX);  // (the 2,048-record pass takes the rest)
    const int hbit = 31 + A.sort_bits - A.lb;  // the record bit under the partition id
    const uint32_t item = blockIdx.x;  // one half per block (no loop: a loop around the
    if (item < 2 * m) {                // build keeps the arguments live, ~120 VGPRs)
        const uint32_t p = A.mid_list[item >> 1], h = item & 1u;
        const uint32_t ps = A.start[p], n = A.start[p + 1] - ps;
        if (n > 2u * CAP) {  // the 4,096-record pass (or the global path)
            if (h == 0 && tid == 0) A.mid2_list[atomicAdd(A.mid2_n, 1u)] = p;
            return;
        }
        // records tid * R .. tid * R + R - 1: counted, then read again (L2) to stage
        uint32_t c0 = 0, ch = 0;
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint32_t i = tid * R + j;
            const uint64_t r = i < n ? A.sk[ps + i] : 0ull;
            const uint32_t b = (uint32_t)(r >> hbit) & 1u;
            c0 += (i < n && b == 0) ? 1u : 0u;
            ch += (i < n && b == h) ? 1u : 0u;
        }
        const uint32_t v = c0 | (ch << 16);  // (counts <= 2,048)
        const uint32_t inc = wave_incl_add(v);
        if (lane == 63) wtot[wv] = inc;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int q = 0; q < NT / 64; ++q) {
            const uint32_t x = wtot[q];
            if (q < wv) pre += x;
            tot += x;
        }
        const uint32_t n0 = tot & 0xFFFFu, nh = h ? n - n0 : n0;
        if (n0 > (uint32_t)CAP || n - n0 > (uint32_t)CAP) {  // a half too large: the 2,048-record pass
            if (h == 0 && tid == 0) A.fb_list[atomicAdd(A.fb_n, 1u)] = p;
            return;
        }
        // the half in load order, staged in the key array, then in part_load's layout
        uint32_t pos = (pre + inc - v) >> 16;
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint32_t i = tid * R + j;
            const uint64_t r = i < n ? A.sk[ps + i] : 0ull;
            if (i < n && ((uint32_t)(r >> hbit) & 1u) == h) S.key[pos++] = r;
        }
        __syncthreads();
        PartLoad<CAP> L;
        L.ps = ps + (h ? n0 : 0u);
        L.n = nh;
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t i = tid + j * NT;
            L.recs[j] = S.key[i < nh ? i : (nh ? nh - 1 : 0u)];
        }
        __syncthreads();  // staging read before part_build_one reuses the key array
        part_build_one<CAP, false>(A, p, S, Sr, L);
    }
}

template <int CAP>
static size_t part_lds() { return sizeof(PartShared<CAP>); }

// ---------------------------------------------------------------------------
// big partitions (global scan path, buckets.hip): the scan wrote ascending,
// partition-relative md / edge lists (bucket b's md entries at bkt_mdo[b] ..,
// edge entries at bkt_edo[b] ..); move them into the combined layout, bucket b's
// split point being c_b = 3 ps + bkt_mdo[b + 1] + bkt_edo[b]
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bucket_of_entry(const uint32_t *off, uint32_t nb, uint32_t e) {
    uint32_t lo = 0, hi = nb;  // last b with off[b] <= e
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= e) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ void relayout_lists_kernel(Buckets b, uint32_t ps, const uint32_t *totals, uint32_t *lst, uint32_t *lidx) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nb = totals[0], n_md = totals[2], n_ed = totals[3];
    if (e < n_md) {
        const uint32_t bk = bucket_of_entry(b.bkt_mdo, nb, e);
        const uint64_t q = 3ull * ps + b.bkt_mdo[bk + 1] + b.bkt_edo[bk] - 1u - (e - b.bkt_mdo[bk]);
        lst[q] = b.md_list[e];
        if (lidx) lidx[q] = b.md_idx[e];
    }
    if (e < n_ed) {
        const uint32_t bk = bucket_of_entry(b.bkt_edo, nb, e);
        const uint64_t q = 3ull * ps + b.bkt_mdo[bk + 1] + e;  // = c_b + (e - bkt_edo[bk])
        lst[q] = b.ed_list[e];
        if (lidx) lidx[q] = b.ed_idx[e];
    }
}

hipError_t launch_relayout_lists(const Buckets &b, uint32_t ps, uint32_t n, const uint32_t *totals_dev,
                                 const PartArgs &a, bool strict, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t m = 2 * n;  // edge entries <= 2 n
    hipLaunchKernelGGL(relayout_lists_kernel, dim3((m + 255) / 256), dim3(256), 0, s, b, ps, totals_dev, a.lst,
                       strict ? a.lidx : nullptr);
    return hipGetLastError();
}

__global__ void records_from_tables_kernel(const uint64_t *sk, const uint32_t *sv, uint32_t ps, uint32_t n, int lb,
                                           const uint8_t *tagtab, Buckets b, PartArgs A, int strict) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const uint64_t lbm = (1ull << lb) - 1;
    const uint32_t g = sv[ps + s];
    const uint32_t t = tagtab[sk[ps + s] & lbm];
    const uint32_t gid = b.occ_gid[g];
    const uint32_t bid = b.grp_bid[gid];
    const uint32_t st = (t & TAG_ST) ? 1u : 0u, en = (t & TAG_EN) ? 1u : 0u, md = (t & TAG_MD) ? 1u : 0u;
    const uint32_t me = st + en;
    const uint32_t mdo = b.bkt_mdo[bid], edo = b.bkt_edo[bid];
    const uint64_t c = 3ull * ps + b.bkt_mdo[bid + 1] + edo;
    const uint32_t nE = me ? (b.grp_mds[gid] - mdo) : 0u;
    const uint32_t nD = md ? (b.grp_ede[gid] - edo) : 0u;
    if (nE <= REC_CNT_MAX && nD <= REC_CNT_MAX) {
        A.rec[g] = encode_rec(c, nE, nD, me);
    } else {  // a high-copy repeat: the counts do not fit 14 bits
        const uint32_t xi = atomicAdd(A.xrec_n, 1u);
        A.xrec[xi] = decoded_rec(c, nE, nD, me);
        A.rec[g] = make_uint2((uint32_t)c, (3u << 30) | xi);
    }
    if (strict) {
        const uint32_t s0 = b.bkt_start[bid];
        A.srec[g] = make_uint4(ps + s0, st ? b.occ_idx[3ull * g] : ((1u << 31) | b.occ_idx[3ull * g + 2]),
                               b.occ_idx[3ull * g + 1], 0u);
        if (s == s0) {
            const uint32_t s1 = b.bkt_start[bid + 1];
            uint32_t gmin = 0xFFFFFFFFu;
            for (uint32_t q = s0; q < s1; ++q) gmin = min(gmin, sv[ps + q]);
            A.bkt_nst[ps + s] = b.bkt_nst[bid];
            A.bkt_nmd[ps + s] = b.bkt_mdo[bid + 1] - mdo;
            A.bkt_first[ps + s] = gmin;
            A.is_head[ps + s] = 1;
        }
    }
}

// ---------------------------------------------------------------------------
// partition starts: start[p] = first sorted index whose partition id is >= p
// (p = 0 .. np; an empty partition gets the next one's start).  One binary
// search per partition over the sorted records -- log2(n) cached loads each
// instead of a pass over all n records plus a serial suffix-min fill.  (Bits
// above the partition id -- the owner rank's in distributed mode -- are the
// same for every key and masked off.)  Thread p also finds start[p + 1] (the
// two searches interleaved) and lists the partitions above 1,024 records, so
// the 2,048 / 4,096-record tiers need not wait for the 1,024-record pass: they
// run beside it on a second stream.
__global__ void part_bounds_kernel(const uint64_t *sk, uint64_t n, int shift, uint32_t mask, uint32_t np,
                                   uint32_t *start, uint32_t *mid_list, uint32_t *mid_n) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p > np) return;
    const bool two = p < np;
    uint64_t lo = 0, hi = n, lo1 = 0, hi1 = two ? n : 0;
    while (lo < hi || lo1 < hi1) {
        if (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (((uint32_t)(sk[mid] >> shift) & mask) < p) lo = mid + 1; else hi = mid;
        }
        if (lo1 < hi1) {
            const uint64_t mid = (lo1 + hi1) >> 1;
            if (((uint32_t)(sk[mid] >> shift) & mask) < p + 1) lo1 = mid + 1; else hi1 = mid;
        }
    }
    start[p] = (uint32_t)lo;
    if (two && lo1 - lo > 1024) mid_list[atomicAdd(mid_n, 1u)] = p;
}

hipError_t launch_part_starts(const PartArgs &a, uint64_t n, int shift, hipStream_t s) {
    // partitions above the main pass's 1,024 records are listed for the 2,048 tier
    hipLaunchKernelGGL(part_bounds_kernel, dim3((a.np + 1 + 255) / 256), dim3(256), 0, s, a.sk, n, shift, a.np - 1,
                       a.np, const_cast<uint32_t *>(a.start), a.mid_list, a.mid_n);
    return hipGetLastError();
}

// one tier of the bucket build: CAP 1,024 over every partition, 2,048 / 4,096
// over the lists the bounds kernel / the 2,048 tier made
// Main-pass blocks per CU, set by their LDS (MI355X: 160 KB per CU).  Fewer
// resident blocks than the registers allow measured faster: the 1,024-record
// blocks share the CUs with the split / 2,048-record tiers on the side stream,
// and their scattered record stores contend in the MALL.  Same box, 3 pairs,
// bench shape (profiles/r05/ab/ab_pb_blocks_per_cu.txt): 7 (the register limit)
// 1.183-1.189 ms, 6 1.177-1.187, 5 1.136-1.143, 4 1.309-1.310
#ifndef SA_PB_BLOCKS_PER_CU
#define SA_PB_BLOCKS_PER_CU 5
#endif
constexpr size_t PB_CU_LDS = 160 * 1024;
inline size_t pb_main_lds(size_t need) {
    const size_t cap = SA_PB_BLOCKS_PER_CU > 0 ? PB_CU_LDS / SA_PB_BLOCKS_PER_CU : 0;
    return cap > need ? cap : need;
}

hipError_t launch_part_build(const PartArgs &a, bool strict, int cap, hipStream_t s) {
    if (!a.np) return hipSuccess;
#define PB_LAUNCH(CAPV, GRID, ST, MAINV)                                                                   \
    do {                                                                                                 \
        size_t lds = part_lds<CAPV>() + (a.rl || a.pv ? 4 * (size_t)(CAPV) : 0);                       \
        if (MAINV) lds = pb_main_lds(lds);                                                               \
        (void)hipFuncSetAttribute((const void *)part_build_kernel<CAPV, ST, MAINV>,                      \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                 \
        hipLaunchKernelGGL((part_build_kernel<CAPV, ST, MAINV>), dim3(GRID), dim3(PbShape<CAPV>::NT), lds, s, a); \
    } while (0)
    const uint32_t mid_grid = a.np < 1024u ? a.np : 1024u;
    if (cap == 1) {  // the split tier (non-strict, records without sorted values)
        const size_t lds0 = part_lds<1024>() + (a.rl || a.pv ? 4 * (size_t)1024 : 0);
        const size_t lds = occ_lds("SA_OCC_SPLIT", lds0, lds0);  // (A/B)
        (void)hipFuncSetAttribute((const void *)part_split_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL(part_split_kernel, dim3(2 * (a.np < SPLIT_MAX ? a.np : SPLIT_MAX)), dim3(PbShape<1024>::NT),
                           lds, s, a);
    } else if (cap == 1024) {
        if (strict) PB_LAUNCH(1024, a.np, true, true); else PB_LAUNCH(1024, a.np, false, true);
    } else if (cap == 2048) {
        if (strict) PB_LAUNCH(2048, mid_grid, true, false); else PB_LAUNCH(2048, mid_grid, false, false);
    } else {
        if (strict) PB_LAUNCH(4096, mid_grid, true, false); else PB_LAUNCH(4096, mid_grid, false, false);
    }
#undef PB_LAUNCH
    return hipGetLastError();
}

// (rec8 = the sorted records from position ps on.  With sorted packed values -- the sharded
// path, A.spv -- record i's value is spv[ps + i], as in the LDS tiers: the unsorted table A.pv
// shares its buffer with the sort and holds sorted values by now.  ovals may alias spv's
// range: each thread reads its value before it writes)
__global__ void convert_records_kernel(const uint64_t *rec8, uint32_t n, PartArgs A, uint64_t *okeys,
                                       uint32_t *ovals, uint32_t ps) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t code, r;
    okeys[i] = record_key(rec8[i], A, code, r, A.rl ? A.rl + (uint32_t)rec8[i] : nullptr,
                          A.spv ? A.spv + ps + i : (A.pv ? A.pv + (uint32_t)rec8[i] : nullptr));
    // the global scan path indexes by occurrence: decode a (read, pos) code
    ovals[i] = A.pos_bits ? A.meta[code >> A.pos_bits].x + (code & ((1u << A.pos_bits) - 1u)) : code;
}

hipError_t launch_convert_records(const uint64_t *rec8, uint32_t n, const PartArgs &a, uint64_t *okeys,
                                  uint32_t *ovals, uint32_t ps, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(convert_records_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rec8, n, a, okeys, ovals, ps);
    return hipGetLastError();
}

hipError_t launch_records_from_tables(const uint64_t *sk, const uint32_t *sv, uint32_t ps, uint32_t n, int lb,
                                      const uint8_t *tagtab, const Buckets &b, const PartArgs &a, int strict,
                                      hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(records_from_tables_kernel, dim3((n + 255) / 256), dim3(256), 0, s, sk, sv, ps, n, lb, tagtab, b,
                       a, strict);
    return hipGetLastError();
}

}  // namespace sa
