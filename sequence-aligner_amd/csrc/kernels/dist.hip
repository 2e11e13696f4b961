// dist.hip -- device helpers of the sharded (multi-GPU) hash stage, SURVEY.md 8(e).
//
// Rank r holds reads [starts[r], starts[r+1]) (global, 0-based).  k-mer
// records travel to the rank owning their hash range (exchange 1); each owner
// builds its buckets and counts partial (lead, trail) pairs for every read
// (KmerTable.calcPairData restricted to its buckets); the partials travel to
// the rank owning the lead (exchange 2), which sums them and applies the
// [min, max] collision filter (calcDispatchData).  The helpers here are the
// small glue kernels around those exchanges; the heavy kernels are shared
// with the single-GPU path.  Bound: HBM (integer streaming / binary search).
#include "../sa_internal.h"

namespace sa {

namespace {

constexpr int DT = 256;

inline dim3 grid_for(uint64_t n) {
    uint64_t b = (n + DT - 1) / DT;
    return dim3((uint32_t)(b ? b : 1));
}

__global__ void iota_kernel(uint32_t *v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * DT + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

// received 8-byte records (mix << 32 | occurrence index local to the source
// rank): seg[s] = first record from source s (s < P, seg[P] = n), seg[P+1+s] =
// the global occurrence index of source s's first k-mer, starts[s] its first
// read.  rl[i] = {read of the occurrence, its loc rank (lrank[lbase[L - k] +
// pos])}; the low word becomes i
__global__ void prepare_received_kernel(uint64_t *recs, uint64_t n, const uint64_t *__restrict__ seg, uint32_t P,
                                        const uint32_t *__restrict__ starts, const uint64_t *occ_off, uint32_t npr,
                                        const int32_t *len, const uint32_t *__restrict__ lbase,
                                        const uint32_t *lrank, int32_t k, uint2 *rl, uint32_t *pv, int lb,
                                        unsigned long long npr_magic, uint64_t *loff) {
    const uint64_t i = (uint64_t)blockIdx.x * DT + threadIdx.x;
    if (i >= n) return;
    // the source whose segment holds i: searched once per wave on its first
    // record (wave-uniform: scalar loads, no dependent vector round trips),
    // then stepped forward by the few lanes past a segment boundary
    const uint64_t i0 = (uint64_t)blockIdx.x * DT + (threadIdx.x & ~63u);
    uint32_t s = 0, hi = P;
    while (hi - s > 1) {
        const uint32_t mid = (s + hi) >> 1;
        if (seg[mid] <= i0) s = mid; else hi = mid;
    }
    s = (uint32_t)__builtin_amdgcn_readfirstlane((int)s);
    while (s + 1 < P && seg[s + 1] <= i) ++s;
    const uint64_t rec = recs[i];
    const uint32_t local = (uint32_t)rec;
    uint32_t r, pos;
    if (npr) {
        // local / npr as the high word of local * magic (magic = floor((2^64 - 1) /
        // npr) + 1: exact for local, npr < 2^32; partition.hip read_of_g)
        const uint32_t q = npr == 1 ? local : (uint32_t)__umul64hi((unsigned long long)local, npr_magic);
        r = starts[s] + q;
        pos = local - q * npr;
    } else {
        const uint64_t g = seg[P + 1 + s] + local;
        uint32_t lo = starts[s], up = starts[s + 1];  // largest r with occ_off[r] <= g
        while (up - lo > 1) {
            const uint32_t mid = (lo + up) >> 1;
            if (occ_off[mid] <= g) lo = mid; else up = mid;
        }
        r = lo;
        pos = (uint32_t)(g - occ_off[r]);
    }
    // local_offsets fused in: loff[a] = first i with read(i) >= a.  Record i
    // opens the reads (read(i - 1), read(i)], read(i - 1) from the lane before;
    // the first lane of each wave and the end are left to local_offsets_fix
    const uint32_t prev = __shfl_up((int)r, 1, 64);
    const uint32_t lr = lrank[(npr ? lbase[npr - 1] : lbase[len[r] - k]) + pos];
    if (pv) pv[i] = (r << lb) | lr;
    else rl[i] = make_uint2(r, lr);
    recs[i] = (rec & 0xFFFFFFFF00000000ull) | (uint32_t)i;
    if (loff && (threadIdx.x & 63) != 0)
        for (uint32_t a = prev + 1; a <= r; ++a) loff[a] = i;
}

// the read boundaries prepare_received leaves: at each wave's first record
// (and record 0) and past the last record (reads after it: loff = n)
__global__ void local_offsets_fix_kernel(const uint2 *rl, const uint32_t *pv, int lb, uint64_t n, uint32_t n_reads,
                                         uint64_t *loff) {
    const uint64_t w = (uint64_t)blockIdx.x * DT + threadIdx.x;
    const uint64_t i = w * 64;
    if (i > n) return;
    auto read_of = [&](uint64_t j) { return pv ? pv[j] >> lb : rl[j].x; };
    const uint32_t prev = i == 0 ? 0u : read_of(i - 1) + 1u;  // first read not yet started
    const uint32_t cur = i == n ? n_reads + 1u : read_of(i) + 1u;
    for (uint32_t a = prev; a < cur; ++a) loff[a] = i;
    if (i < n && i + 64 > n)  // n not a multiple of 64: the reads after the last record
        for (uint32_t a = read_of(n - 1) + 1u; a <= n_reads; ++a) loff[a] = n;
}

// loff[a] = first i with rl[i].x >= a, for a in [0, n_reads] (reads ascending):
// the local occurrences of read a are [loff[a], loff[a+1]).  One pass over the
// records: record i starts the reads (rl[i-1].x, rl[i].x] (usually one), the
// last record closes the reads after it
__global__ void local_offsets_kernel(const uint2 *rl, const uint32_t *pv, int lb, uint64_t n, uint32_t n_reads,
                                     uint64_t *loff) {
    const uint64_t i = (uint64_t)blockIdx.x * DT + threadIdx.x;
    if (i > n) return;
    auto read_of = [&](uint64_t j) { return pv ? pv[j] >> lb : rl[j].x; };
    const uint32_t prev = i == 0 ? 0u : read_of(i - 1) + 1u;  // first read not yet started
    const uint32_t cur = i == n ? n_reads + 1u : read_of(i) + 1u;
    for (uint32_t a = prev; a < cur; ++a) loff[a] = i;
}

// bounds[o] = first i with (keys[i] >> shift) >= o, o in [0, P]
__global__ void owner_bounds_kernel(const uint64_t *keys, uint64_t n, int shift, uint32_t P, uint64_t *bounds) {
    const uint32_t o = threadIdx.x;
    if (o > P) return;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((keys[mid] >> shift) < o) lo = mid + 1; else hi = mid;
    }
    bounds[o] = lo;
}

// received partials -> keys in the wide canonical order (lead desc, trail asc)
__global__ void reduce_keys_kernel(const uint32_t *fst, const uint32_t *snd, uint64_t n, int idb, uint64_t *keys,
                                   uint32_t *vals) {
    const uint64_t i = (uint64_t)blockIdx.x * DT + threadIdx.x;
    if (i >= n) return;
    const uint64_t top = (1ull << idb) - 1;
    keys[i] = ((top - fst[i]) << idb) | snd[i];
    vals[i] = (uint32_t)i;
}

// segment heads of the sorted partials: sum their counts (every (lead, trail)
// arrives at most once per source rank) and apply the [min, max] filter
__global__ void reduce_heads_kernel(const uint64_t *skeys, const uint32_t *sidx, uint64_t n, const uint32_t *cnt,
                                    int32_t min_c, int32_t max_c, uint32_t *sum, uint32_t *keep,
                                    unsigned long long *distinct) {
    const uint64_t i = (uint64_t)blockIdx.x * DT + threadIdx.x;
    uint32_t head = 0;
    if (i < n) {
        const uint64_t k = skeys[i];
        head = (i == 0 || skeys[i - 1] != k) ? 1u : 0u;
        uint32_t s = 0, kp = 0;
        if (head) {
            for (uint64_t j = i; j < n && skeys[j] == k; ++j) s += cnt[sidx[j]];
            kp = ((int32_t)s >= min_c && (int32_t)s <= max_c) ? 1u : 0u;
        }
        sum[i] = s;
        keep[i] = kp;
    }
    // distinct pairs: block-reduced, one sharded atomic per block
    __shared__ uint32_t nh;
    if (threadIdx.x == 0) nh = 0;
    __syncthreads();
    if (head) atomicAdd(&nh, 1u);
    __syncthreads();
    if (threadIdx.x == 0 && nh) atomicAdd(&distinct[blockIdx.x % NSHARD], (unsigned long long)nh);
}

__global__ void reduce_compact_kernel(const uint64_t *skeys, uint64_t n, int idb, const uint32_t *sum,
                                      const uint32_t *keep, const uint32_t *pos, int32_t *lead, int32_t *trail,
                                      int32_t *count) {
    const uint64_t i = (uint64_t)blockIdx.x * DT + threadIdx.x;
    if (i >= n || !keep[i]) return;
    const uint64_t top = (1ull << idb) - 1;
    const uint64_t k = skeys[i];
    const uint32_t p = pos[i];
    lead[p] = (int32_t)(top - (k >> idb)) + 1;  // 1-based ids downstream
    trail[p] = (int32_t)(k & top) + 1;
    count[p] = (int32_t)sum[i];
}

// ---- owner-side reduce by lead (replaces the (lead, trail) radix sort) ----
// received partials (fst = global lead, snd, cnt) -> per-lead segments ->
// per-lead LDS aggregation (sum, [min, max] filter, trail-ascending rank) ->
// lead-descending copy.  A lead with more than 192 distinct partners sets
// *overflow and the caller falls back to the sort.
// Partials arrive clustered by the sender's pair-count blocks (a few leads
// each, interleaved), so per-partial global atomics on the lead counters
// serialise on the same addresses.  A tile of LT partials is first counted in
// an LDS table keyed by lead (LT_SLOTS slots, linear probing); each distinct
// lead then takes one global atomic for the whole tile (a lead whose probe
// run fails falls back to its own global atomic).  PLACE = false: counts
// only (lcnt); true: every partial gets its position in its lead's segment
// (loff + tile base + its rank among the tile's partials of that lead).
constexpr int LT_THREADS = 256, LT_PER = 8, LT = LT_THREADS * LT_PER, LT_SLOTS = 1024;

template <bool PLACE>
__global__ __launch_bounds__(LT_THREADS) void lead_tile_kernel(const uint32_t *fst, const uint32_t *snd,
                                                               const uint32_t *cnt, uint64_t n, uint32_t base,
                                                               uint32_t *lcnt, const uint32_t *loff, uint32_t *lcur,
                                                               uint2 *seg) {
    __shared__ uint32_t key[LT_SLOTS], num[LT_SLOTS];
    for (int j = threadIdx.x; j < LT_SLOTS; j += LT_THREADS) { key[j] = 0xFFFFFFFFu; num[j] = 0; }
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * LT;
    uint32_t l[LT_PER], slot[LT_PER], rk[LT_PER];
#pragma unroll
    for (int j = 0; j < LT_PER; ++j) {
        const uint64_t i = t0 + (uint64_t)j * LT_THREADS + threadIdx.x;
        l[j] = i < n ? fst[i] - base : 0xFFFFFFFFu;
        slot[j] = 0xFFFFFFFFu;
        if (l[j] == 0xFFFFFFFFu) continue;
        uint32_t h = (l[j] * 0x9E3779B1u) >> 22;  // 10 bits: LT_SLOTS
        for (int probe = 0; probe < 32; ++probe) {
            uint32_t old = lds_relaxed(&key[h]);
            if (old == 0xFFFFFFFFu) old = atomicCAS(&key[h], 0xFFFFFFFFu, l[j]);
            if (old == 0xFFFFFFFFu || old == l[j]) {
                slot[j] = h;
                rk[j] = atomicAdd(&num[h], 1u);
                break;
            }
            h = (h + 1) & (LT_SLOTS - 1);
        }
    }
    __syncthreads();
    // one global atomic per distinct lead of the tile
    for (int j = threadIdx.x; j < LT_SLOTS; j += LT_THREADS) {
        const uint32_t k = key[j];
        if (k == 0xFFFFFFFFu) continue;
        if (PLACE) num[j] = atomicAdd(&lcur[k], num[j]);  // the tile's base within the lead's segment
        else atomicAdd(&lcnt[k], num[j]);
    }
    if (!PLACE) {
#pragma unroll
        for (int j = 0; j < LT_PER; ++j)
            if (l[j] != 0xFFFFFFFFu && slot[j] == 0xFFFFFFFFu) atomicAdd(&lcnt[l[j]], 1u);
        return;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < LT_PER; ++j) {
        if (l[j] == 0xFFFFFFFFu) continue;
        const uint64_t i = t0 + (uint64_t)j * LT_THREADS + threadIdx.x;
        const uint32_t at = slot[j] != 0xFFFFFFFFu ? num[slot[j]] + rk[j] : atomicAdd(&lcur[l[j]], 1u);
        seg[loff[l[j]] + at] = make_uint2(snd[i], cnt[i]);
    }
}

constexpr int LR_SLOTS = 256, LR_FILL = 192;
constexpr uint32_t LR_EMPTY = 0xFFFFFFFFu;
// the second tier: one wave per listed lead, a 1,024-slot table (768 partners).  A lead
// with more than 2 x 192 partials goes to it without trying the first table (round 6:
// at configs[3]'s real density a lead meets ~510 distinct partners in ~740 partials, so
// every lead overflowed the 192-partner table -- after hashing all its partials -- and
// the block-per-lead pass took them one block each on a fixed 256-block grid: 3.8 ms per
// shard and pass, profiles/r06/big/c3real)
constexpr int LRM_SLOTS = 1024, LRM_FILL = 768;
constexpr uint32_t LR_ROUTE = 2 * LR_FILL, LRM_CHUNK = 16;

// One wave sums lead l's partials into a wave-private SLOTS-slot table (trail -> count
// sum), then compacts the kept entries, ranks them by trail and writes them back over the
// start of the lead's own segment; kcnt[l] = kept (KmerTable.calcDispatchData's filter,
// :155-187).  More than FILL distinct partners (or a failed probe run): kcnt[l] = 0 and
// the lead is listed for the next tier.  Returns the distinct partners counted.
template <int SLOTS, int FILL, bool CHECK>
__device__ __forceinline__ uint32_t lead_wave(uint2 *seg, const uint32_t *loff, uint32_t l, uint32_t *key,
                                              uint32_t *val, uint2 *kept, int lane, int32_t min_c, int32_t max_c,
                                              uint32_t *kcnt, uint32_t next_mark) {
    constexpr int LOG = SLOTS == 256 ? 8 : SLOTS == 1024 ? 10 : 12;
    static_assert((1 << LOG) == SLOTS, "table size");
    constexpr int PER = SLOTS / 64;
    __builtin_amdgcn_wave_barrier();  // (the wave's previous lead is done with the table)
    for (int j = lane; j < SLOTS; j += 64) { key[j] = LR_EMPTY; val[j] = 0; }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    const uint32_t s0 = loff[l], m = loff[l + 1] - s0;
    bool ovf = false;
    // CHECK: stop once the wave has inserted more than FILL keys -- the lead cannot fit
    // (round 6: at configs[4]-shape k = 12 the 1,024-slot tier hashed every partial of
    // ~5,000-partial leads into a full table, 64-probe runs each -- 9.3 ms per shard and
    // pass, the largest kernel of the build -- before handing them on).  Checked once per
    // 8 x 64 partials, and only while the routing has no ratio to go by (the first pass of
    // a context): the check cost the tiers 5-9 % at configs[3]'s real density, where the
    // ratio keeps such leads out of them
    uint32_t fresh = 0;
    const uint32_t blk = CHECK ? 8 * 64 : m;
    for (uint32_t b0 = 0; b0 < m; b0 += blk) {
        const uint32_t b1 = m - b0 > blk ? b0 + blk : m;
        for (uint32_t j = b0 + (uint32_t)lane; j < b1; j += 64) {
            const uint2 v = seg[s0 + j];
            uint32_t h = (v.x * 0x9E3779B1u) >> (32 - LOG);
            int probe = 0;
            for (; probe < 64; ++probe) {
                uint32_t old = lds_relaxed(&key[h]);
                if (old == LR_EMPTY) old = atomicCAS(&key[h], LR_EMPTY, v.x);
                if (old == LR_EMPTY || old == v.x) {
                    if (CHECK) fresh += old == LR_EMPTY ? 1u : 0u;
                    atomicAdd(&val[h], v.y);
                    break;
                }
                h = (h + 1) & (SLOTS - 1);
            }
            if (probe == 64) ovf = true;
        }
        if (CHECK && (__any(ovf) || (uint32_t)__shfl((int)wave_incl_add(fresh), 63, 64) > (uint32_t)FILL)) {
            ovf = true;
            break;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    // this lane's PER slots: distinct keys, kept ones compacted by wave prefix
    uint32_t nd = 0, kp = 0;
    // (the lane's slots into registers first: kept may alias the table)
    uint32_t kk[PER], kc[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        kk[q] = key[lane * PER + q];
        kc[q] = val[lane * PER + q];
        if (kk[q] != LR_EMPTY) {
            ++nd;
            if ((int32_t)kc[q] >= min_c && (int32_t)kc[q] <= max_c) kp |= 1u << q;
        }
    }
    const uint32_t tot_nd = (uint32_t)__shfl((int)wave_incl_add(nd), 63, 64);
    if (tot_nd > (uint32_t)FILL || __any(ovf)) {
        if (lane == 0) kcnt[l] = next_mark;
        return 0;
    }
    const uint32_t mine = __popc(kp);
    const uint32_t ex = wave_incl_add(mine) - mine;
    const uint32_t k = (uint32_t)__shfl((int)(ex + mine), 63, 64);
    uint32_t at = ex;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
#pragma unroll
    for (int q = 0; q < PER; ++q)
        if (kp & (1u << q)) kept[at++] = make_uint2(kk[q], kc[q]);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    for (uint32_t j = lane; j < k; j += 64) {
        const uint2 e = kept[j];
        uint32_t r = 0;
        for (uint32_t q = 0; q < k; ++q) r += kept[q].x < e.x ? 1u : 0u;
        seg[s0 + r] = e;  // (the segment's partials are all consumed)
    }
    if (lane == 0) kcnt[l] = k;
    __builtin_amdgcn_wave_barrier();  // (kept / key are reused by the wave's next lead)
    return tot_nd;
}

// The tiers' marks in kcnt: a lead the first table cannot take is marked KC_MID (the
// 1,024-slot wave tier), KC_BIG (the 4,096-slot block tier) or KC_HUGE (the 16,384-slot
// block tier) -- a mark, not a list: at configs[3]'s real density nearly every lead
// leaves the first tier, and one list cursor took ~89k same-address atomics per shard and
// pass (0.9 ms).  Leads are routed by their partial count m: a lead has at least m / ranks
// distinct partners (a partner meets it on at most every rank once), and about m x route
// (the last pass's distinct partners per partial), so a lead whose estimate passes a
// tier's FILL skips it, and one past 12,288 sends the whole reduce to the sort at once
// (*overflow).  Only the m / ranks floor is a proof; a wrong estimate costs time.
constexpr uint32_t KC_MID = 0xFFFFFFFFu, KC_BIG = 0xFFFFFFFEu, KC_HUGE = 0xFFFFFFFDu;
constexpr int LRB_SLOTS = 4096, LRB_FILL = 3072;
// the fourth tier (round 6): configs[4]-shape k = 12 leads meet ~4,000-8,000 distinct
// partners, past the 4,096-slot table, and every pass went to the sort
constexpr int LRH_SLOTS = 16384, LRH_FILL = 12288, LRH_THREADS = 1024;
// leads per chunk of the block tiers: a pass holds ~10^4-10^5 leads, and 256-lead chunks
// left most CUs without one
constexpr uint32_t LRB_CHUNK = 64;
// kept entries past which a block tier sorts them (bitonic) instead of counting ranks
constexpr int LRB_BITONIC = 512;
__device__ __forceinline__ void set_overflow(uint32_t *overflow) {
    if (__hip_atomic_load(overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) atomicOr(overflow, 1u);
}

// one wave per lead; distinct pairs counted once per block
__global__ __launch_bounds__(256) void lead_reduce_kernel(uint2 *seg, const uint32_t *loff, uint32_t nl, int32_t min_c,
                                                          int32_t max_c, uint32_t *kcnt,
                                                          unsigned long long *distinct, uint32_t ranks,
                                                          float route, uint32_t *overflow) {
    __shared__ uint32_t key[4][LR_SLOTS], val[4][LR_SLOTS];
    __shared__ uint2 kept[4][LR_FILL];
    __shared__ uint32_t nd_blk;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t l = blockIdx.x * 4 + w;
    if (threadIdx.x == 0) nd_blk = 0;
    __syncthreads();
    if (l < nl) {
        uint32_t nd = 0;
        const uint64_t m = loff[l + 1] - loff[l];
        // est: the lead's expected distinct partners -- the m / ranks floor, or m x the
        // last pass's distinct-per-partial ratio (x 0.85 for the spread between leads).  A
        // lead routed past a tier it would have fit costs time, never results
        const uint64_t lo = m / ranks, ex = (uint64_t)((float)m * route * 0.85f);
        const uint64_t est = lo > ex ? lo : ex;
        if (m > (uint64_t)ranks * LRH_FILL || est > (uint64_t)LRH_FILL) {
            // (an estimate past the last tier sends the pass to the sort now: the tiers
            // would hash the lead twice before failing on it)
            if (lane == 0) { kcnt[l] = 0; set_overflow(overflow); }
        } else if (est > (uint64_t)LRB_FILL) {
            if (lane == 0) kcnt[l] = KC_HUGE;
        } else if (est > (uint64_t)LRM_FILL) {
            if (lane == 0) kcnt[l] = KC_BIG;
        } else if (m > LR_ROUTE) {
            if (lane == 0) kcnt[l] = KC_MID;
        } else {
            nd = lead_wave<LR_SLOTS, LR_FILL, false>(seg, loff, l, key[w], val[w], kept[w], lane, min_c, max_c, kcnt, KC_MID);
        }
        if (lane == 0 && nd) atomicAdd(&nd_blk, nd);  // (a marked lead is counted by its tier)
    }
    __syncthreads();
    if (threadIdx.x == 0 && nd_blk) atomicAdd(&distinct[blockIdx.x % NSHARD], (unsigned long long)nd_blk);
}

// the second tier: one-wave blocks (8 KB of LDS each: 20 per CU) striding over the leads
// LRM_CHUNK at a time -- one coalesced load of their kcnt, a ballot of the marked ones
template <bool CHECK>
__global__ __launch_bounds__(64) void lead_reduce_mid_kernel(uint2 *seg, const uint32_t *loff, uint32_t nl,
                                                             int32_t min_c, int32_t max_c, uint32_t *kcnt,
                                                             unsigned long long *distinct, const uint32_t *overflow) {
    // 8 KB: the kept entries (<= 768 x 8 B) alias the table once it is read into registers,
    // so 20 one-wave blocks fit a CU (with a separate kept array, 14 KB: 11)
    __shared__ uint32_t tab[2 * LRM_SLOTS];
    uint32_t *key = tab, *val = tab + LRM_SLOTS;
    uint2 *kept = reinterpret_cast<uint2 *>(tab);
    const int lane = threadIdx.x;
    unsigned long long nd = 0;
    // chunks of LRM_CHUNK leads: enough blocks to fill the CUs (one 64-lead chunk per block
    // left ~5 waves per CU, each walking 64 dense leads in a row)
    for (uint32_t c0 = blockIdx.x * LRM_CHUNK; c0 < nl; c0 += gridDim.x * LRM_CHUNK) {
        if (__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
            break;  // (the sort takes over; wave-uniform)
        const uint32_t l0 = c0 + (uint32_t)lane;
        unsigned long long todo = __ballot(lane < (int)LRM_CHUNK && l0 < nl && kcnt[l0] == KC_MID);
        while (todo) {
            const int b = __builtin_ctzll(todo);
            todo &= todo - 1;
            nd += lead_wave<LRM_SLOTS, LRM_FILL, CHECK>(seg, loff, c0 + (uint32_t)b, key, val, kept, lane, min_c, max_c,
                                                 kcnt, KC_BIG);
        }
    }
    if (lane == 0 && nd) atomicAdd(&distinct[blockIdx.x % NSHARD], nd);
}

// The block tiers: blocks of NT threads striding over the leads LRB_CHUNK at a time, each
// lead marked MARK summed by the whole block in a SLOTS-slot table (FILL partners) and
// filtered as above, the kept entries ranked by trail over the block.  Past FILL partners
// (or a failed probe run) the block stops hashing the lead at once and marks it NEXT, or
// with NEXT == 0 sets *overflow, which sends the caller to the sort.  The kept entries
// alias the table (read into registers first): 16,384 slots are 128 KB, one block per CU.
template <int SLOTS, int FILL, int NT>
__device__ __forceinline__ void lead_block_tier(uint2 *seg, const uint32_t *loff, uint32_t nl, int32_t min_c,
                                                int32_t max_c, uint32_t *kcnt, unsigned long long *distinct,
                                                uint32_t *overflow, uint32_t mark, uint32_t next, uint32_t *tab) {
    constexpr int LOG = SLOTS == 4096 ? 12 : 14;
    static_assert((1 << LOG) == SLOTS, "table size");
    constexpr int PER = SLOTS / NT;
    constexpr int MAXP = 256;
    __shared__ uint32_t fill, bad, nk, stop;
    __shared__ unsigned long long todo_s;
    uint32_t *key = tab, *val = tab + SLOTS;
    uint2 *kept = reinterpret_cast<uint2 *>(tab);
    for (uint32_t c0 = blockIdx.x * LRB_CHUNK; c0 < nl; c0 += gridDim.x * LRB_CHUNK) {
        __syncthreads();  // (todo_s of the previous chunk consumed)
        if (threadIdx.x < 64) {
            const uint32_t l0 = c0 + threadIdx.x;
            const unsigned long long b = __ballot(l0 < nl && kcnt[l0] == mark);
            if (threadIdx.x == 0) todo_s = b;
        }
        __syncthreads();
        unsigned long long todo = todo_s;
        while (todo) {
            const uint32_t l = c0 + (uint32_t)__builtin_ctzll(todo);
            todo &= todo - 1;
            __syncthreads();  // the previous lead's LDS consumed
            for (int j = threadIdx.x; j < SLOTS; j += NT) { key[j] = LR_EMPTY; val[j] = 0; }
            if (threadIdx.x == 0) {
                fill = 0; bad = 0; nk = 0;
                stop = __hip_atomic_load(overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            if (stop) return;  // (block-uniform: the sort takes over, this block's work would be redone)
            const uint32_t s0 = loff[l], m = loff[l + 1] - s0;
            for (uint32_t j = threadIdx.x; j < m; j += NT) {
                if (lds_relaxed(&bad)) break;  // (the lead cannot fit: stop hashing it)
                const uint2 v = seg[s0 + j];
                uint32_t h = (v.x * 0x9E3779B1u) >> (32 - LOG);
                int probe = 0;
                for (; probe < MAXP; ++probe) {
                    uint32_t old = lds_relaxed(&key[h]);
                    if (old == LR_EMPTY) old = atomicCAS(&key[h], LR_EMPTY, v.x);
                    if (old == LR_EMPTY || old == v.x) {
                        if (old == LR_EMPTY && atomicAdd(&fill, 1u) >= (uint32_t)FILL) bad = 1;
                        atomicAdd(&val[h], v.y);
                        break;
                    }
                    h = (h + 1) & (SLOTS - 1);
                }
                if (probe == MAXP) bad = 1;
            }
            __syncthreads();
            if (bad) {
                if (threadIdx.x == 0) {
                    if (next) kcnt[l] = next;
                    else set_overflow(overflow);
                }
                continue;
            }
            uint32_t kk[PER], kc[PER];
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                kk[q] = key[q * NT + threadIdx.x];
                kc[q] = val[q * NT + threadIdx.x];
            }
            __syncthreads();  // (the table is read: kept overwrites it)
#pragma unroll
            for (int q = 0; q < PER; ++q)
                if (kk[q] != LR_EMPTY && (int32_t)kc[q] >= min_c && (int32_t)kc[q] <= max_c)
                    kept[atomicAdd(&nk, 1u)] = make_uint2(kk[q], kc[q]);
            __syncthreads();
            const uint32_t k = nk;
            if (k > (uint32_t)LRB_BITONIC) {
                // many kept (high-copy repeats): a bitonic sort by trail over the next power
                // of two (<= SLOTS entries of 8 B: the table's own bytes), pads last -- the
                // rank count below is k^2 / NT reads each (6,000 kept: 11.6 -> 2.3 ms per
                // 16,384-slot launch, profiles/r06/tiers/paths_*)
                uint32_t P = 64;
                while (P < k) P <<= 1;
                for (uint32_t j = k + threadIdx.x; j < P; j += NT) kept[j] = make_uint2(LR_EMPTY, 0u);
                __syncthreads();
                for (uint32_t size = 2; size <= P; size <<= 1)
                    for (uint32_t stride = size >> 1; stride; stride >>= 1) {
                        for (uint32_t t = threadIdx.x; t < P / 2; t += NT) {
                            const uint32_t i = 2 * t - (t & (stride - 1)), i2 = i + stride;
                            const uint2 a = kept[i], b = kept[i2];
                            if ((a.x > b.x) == ((i & size) == 0)) { kept[i] = b; kept[i2] = a; }
                        }
                        __syncthreads();
                    }
                for (uint32_t j = threadIdx.x; j < k; j += NT) seg[s0 + j] = kept[j];
            } else {
                for (uint32_t j = threadIdx.x; j < k; j += NT) {
                    const uint2 e = kept[j];
                    uint32_t r = 0;
                    for (uint32_t q = 0; q < k; ++q) r += kept[q].x < e.x ? 1u : 0u;
                    seg[s0 + r] = e;  // (every partial of the segment was read before the barrier)
                }
            }
            if (threadIdx.x == 0) {
                kcnt[l] = k;
                atomicAdd(&distinct[blockIdx.x % NSHARD], (unsigned long long)fill);
            }
        }
    }
}

// the third tier: 4,096 slots (3,072 partners) per 256-thread block, 32 KB: 5 per CU
__global__ __launch_bounds__(256) void lead_reduce_big_kernel(uint2 *seg, const uint32_t *loff, uint32_t nl,
                                                              int32_t min_c, int32_t max_c, uint32_t *kcnt,
                                                              unsigned long long *distinct, uint32_t *overflow) {
    __shared__ uint32_t tab[2 * LRB_SLOTS];
    lead_block_tier<LRB_SLOTS, LRB_FILL, 256>(seg, loff, nl, min_c, max_c, kcnt, distinct, overflow, KC_BIG, KC_HUGE,
                                              tab);
}

// the fourth tier: 16,384 slots (12,288 partners) per 1,024-thread block, 128 KB of
// dynamic LDS: one per CU
__global__ __launch_bounds__(LRH_THREADS) void lead_reduce_huge_kernel(uint2 *seg, const uint32_t *loff, uint32_t nl,
                                                                       int32_t min_c, int32_t max_c, uint32_t *kcnt,
                                                                       unsigned long long *distinct,
                                                                       uint32_t *overflow) {
    extern __shared__ __align__(16) uint32_t htab[];
    lead_block_tier<LRH_SLOTS, LRH_FILL, LRH_THREADS>(seg, loff, nl, min_c, max_c, kcnt, distinct, overflow, KC_HUGE,
                                                      0u, htab);
}

// lead-descending dispatch: lead l's kept entries go to total - kex[l] - kcnt[l]
__global__ void lead_copy_kernel(const uint2 *seg, const uint32_t *loff, const uint32_t *kcnt, const uint32_t *kex,
                                 const uint32_t *total, uint32_t nl, uint32_t base, int32_t *lead, int32_t *trail,
                                 int32_t *count) {
    const uint32_t l = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (l >= nl) return;
    const uint32_t m = kcnt[l], off = *total - kex[l] - m, s0 = loff[l];
    for (uint32_t j = threadIdx.x & 63u; j < m; j += 64) {
        const uint2 e = seg[s0 + j];
        lead[off + j] = (int32_t)(base + l) + 1;  // 1-based ids downstream
        trail[off + j] = (int32_t)e.x + 1;
        count[off + j] = (int32_t)e.y;
    }
}

}  // namespace

hipError_t launch_lead_reduce(const uint32_t *fst, const uint32_t *snd, const uint32_t *cnt, uint64_t n, uint32_t base,
                              uint32_t nl, int32_t min_c, int32_t max_c, uint32_t *lcnt, uint32_t *loff, uint32_t *lcur,
                              uint2 *seg, uint32_t *kcnt, unsigned long long *distinct, uint32_t *overflow,
                              uint32_t ranks, float route, void *scan_tmp, uint32_t *total_dev, hipStream_t s) {
    if (!nl) return hipSuccess;
    hipError_t e;
    if ((e = hipMemsetAsync(lcnt, 0, (size_t)nl * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(lcur, 0, (size_t)nl * 4, s)) != hipSuccess) return e;
    const dim3 tiles((uint32_t)((n + LT - 1) / LT));
    if (n) hipLaunchKernelGGL(lead_tile_kernel<false>, tiles, dim3(LT_THREADS), 0, s, fst, snd, cnt, n, base, lcnt,
                              (const uint32_t *)nullptr, lcur, (uint2 *)nullptr);
    if ((e = exclusive_scan_u32(lcnt, loff, nl, total_dev, scan_tmp, s)) != hipSuccess) return e;
    // loff[nl] = n (the scan leaves nl entries)
    if ((e = hipMemcpyAsync(loff + nl, total_dev, 4, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
    if (n) hipLaunchKernelGGL(lead_tile_kernel<true>, tiles, dim3(LT_THREADS), 0, s, fst, snd, cnt, n, base, lcnt,
                              (const uint32_t *)loff, lcur, seg);
    hipLaunchKernelGGL(lead_reduce_kernel, dim3((nl + 3) / 4), dim3(256), 0, s, seg, loff, nl, min_c, max_c, kcnt,
                       distinct, ranks, route, overflow);
    const uint32_t cm = (nl + LRM_CHUNK - 1) / LRM_CHUNK;
    const dim3 gm(cm < 256u * 20u ? cm : 256u * 20u);
    if (route > 0.f)
        hipLaunchKernelGGL(lead_reduce_mid_kernel<false>, gm, dim3(64), 0, s, seg, loff, nl, min_c, max_c, kcnt,
                           distinct, (const uint32_t *)overflow);
    else
        hipLaunchKernelGGL(lead_reduce_mid_kernel<true>, gm, dim3(64), 0, s, seg, loff, nl, min_c, max_c, kcnt, distinct,
                           (const uint32_t *)overflow);
    const uint32_t cb = (nl + LRB_CHUNK - 1) / LRB_CHUNK;
    hipLaunchKernelGGL(lead_reduce_big_kernel, dim3(cb < 256u * 5u ? cb : 256u * 5u), dim3(256), 0, s, seg, loff, nl,
                       min_c, max_c, kcnt, distinct, overflow);
    constexpr size_t hlds = 2u * LRH_SLOTS * 4u;
    (void)hipFuncSetAttribute((const void *)lead_reduce_huge_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)hlds);
    hipLaunchKernelGGL(lead_reduce_huge_kernel, dim3(cb < 256u ? cb : 256u), dim3(LRH_THREADS), hlds, s, seg, loff,
                       nl, min_c, max_c, kcnt, distinct, overflow);
    return hipGetLastError();
}

hipError_t launch_lead_copy(const uint2 *seg, const uint32_t *loff, const uint32_t *kcnt, const uint32_t *kex,
                            const uint32_t *total, uint32_t nl, uint32_t base, int32_t *lead, int32_t *trail,
                            int32_t *count, hipStream_t s) {
    if (!nl) return hipSuccess;
    hipLaunchKernelGGL(lead_copy_kernel, dim3((nl + 3) / 4), dim3(256), 0, s, seg, loff, kcnt, kex, total, nl, base,
                       lead, trail, count);
    return hipGetLastError();
}

hipError_t launch_iota(uint32_t *v, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(iota_kernel, grid_for(n), dim3(DT), 0, s, v, n);
    return hipGetLastError();
}

hipError_t launch_prepare_received(uint64_t *recs, uint64_t n, const uint64_t *seg, uint32_t P,
                                   const uint32_t *starts, const uint64_t *occ_off, uint32_t npr, const int32_t *len,
                                   const uint32_t *lbase, const uint32_t *lrank, int32_t k, uint2 *rl,
                                   uint32_t *pv, int lb, uint64_t *loff, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(prepare_received_kernel, grid_for(n), dim3(DT), 0, s, recs, n, seg, P, starts, occ_off, npr,
                       len, lbase, lrank, k, rl, pv, lb, npr >= 2 ? ~0ull / npr + 1 : 0ull, loff);
    return hipGetLastError();
}

hipError_t launch_local_offsets(const uint2 *rl, const uint32_t *pv, int lb, uint64_t n, uint32_t n_reads,
                                uint64_t *loff, hipStream_t s) {
    if (!n) {
        hipLaunchKernelGGL(local_offsets_kernel, grid_for(n + 1), dim3(DT), 0, s, rl, pv, lb, n, n_reads, loff);
        return hipGetLastError();
    }
    // (prepare_received wrote the boundaries inside each wave)
    hipLaunchKernelGGL(local_offsets_fix_kernel, grid_for(n / 64 + 1), dim3(DT), 0, s, rl, pv, lb, n, n_reads, loff);
    return hipGetLastError();
}

hipError_t launch_owner_bounds(const uint64_t *keys, uint64_t n, int shift, uint32_t P, uint64_t *bounds,
                               hipStream_t s) {
    hipLaunchKernelGGL(owner_bounds_kernel, dim3(1), dim3(((P + 1 + 63) / 64) * 64), 0, s, keys, n, shift, P,
                       bounds);
    return hipGetLastError();
}

// the owner regions concatenated: block (x, r) copies entries [x CC, (x + 1) CC)
// of region r (a grid of chunks, not one block per region: the regions hold
// ~20k partials each at the bench shape, too few blocks to fill the chip)
constexpr uint32_t CC = 4 * DT;
__global__ void copy_owner_regions_kernel(const uint32_t *fst, const uint32_t *snd, const uint32_t *cnt,
                                          unsigned long long cap_s, const unsigned long long *cursor,
                                          const uint64_t *off, uint32_t *of, uint32_t *os, uint32_t *oc) {
    const uint32_t r = blockIdx.y;
    const unsigned long long m = min(cursor[r], cap_s), src = (unsigned long long)r * cap_s;
    const uint64_t dst = off[r];
    const unsigned long long j0 = (unsigned long long)blockIdx.x * CC;
#pragma unroll
    for (uint32_t q = 0; q < CC / DT; ++q) {
        const unsigned long long j = j0 + q * DT + threadIdx.x;
        if (j < m) {
            of[dst + j] = fst[src + j];
            os[dst + j] = snd[src + j];
            oc[dst + j] = cnt[src + j];
        }
    }
}

hipError_t launch_copy_owner_regions(const uint32_t *fst, const uint32_t *snd, const uint32_t *cnt,
                                     unsigned long long cap_s, uint32_t n_regions, const unsigned long long *cursor,
                                     const uint64_t *off, uint32_t *of, uint32_t *os, uint32_t *oc,
                                     uint64_t max_fill, hipStream_t s) {
    if (!n_regions || !max_fill) return hipSuccess;
    const dim3 grid((uint32_t)((max_fill + CC - 1) / CC), n_regions);
    hipLaunchKernelGGL(copy_owner_regions_kernel, grid, dim3(DT), 0, s, fst, snd, cnt, cap_s, cursor, off, of, os, oc);
    return hipGetLastError();
}

hipError_t launch_reduce_keys(const uint32_t *fst, const uint32_t *snd, uint64_t n, int idb, uint64_t *keys,
                              uint32_t *vals, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(reduce_keys_kernel, grid_for(n), dim3(DT), 0, s, fst, snd, n, idb, keys, vals);
    return hipGetLastError();
}

hipError_t launch_reduce_heads(const uint64_t *skeys, const uint32_t *sidx, uint64_t n, const uint32_t *cnt,
                               int32_t min_c, int32_t max_c, uint32_t *sum, uint32_t *keep,
                               unsigned long long *distinct, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(reduce_heads_kernel, grid_for(n), dim3(DT), 0, s, skeys, sidx, n, cnt, min_c, max_c, sum, keep,
                       distinct);
    return hipGetLastError();
}

hipError_t launch_reduce_compact(const uint64_t *skeys, uint64_t n, int idb, const uint32_t *sum, const uint32_t *keep,
                                 const uint32_t *pos, int32_t *lead, int32_t *trail, int32_t *count, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(reduce_compact_kernel, grid_for(n), dim3(DT), 0, s, skeys, n, idb, sum, keep, pos, lead, trail,
                       count);
    return hipGetLastError();
}

}  // namespace sa
