// sort_scan.hip -- hand-written device primitives for gfx950:
//   * exclusive prefix scan of u32 (reduce-then-scan, 3 launches)
//   * stable LSD radix sort of (u64 key, u32 value) over a key bit range,
//     8-bit digits, per-wave 64-lane ballot multisplit for stable local ranks.
// These group k-mer records by hash (the device replacement of KmerData,
// KmerTable.scala:26-53) and order candidate pairs.  Bound: HBM.
#include "../sa_internal.h"

namespace sa {

constexpr int SC_THREADS = 256;
constexpr int SC_ITEMS = 8;
constexpr int SC_TILE = SC_THREADS * SC_ITEMS;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
    (void)lane;
    return wave_incl_add(v);
}

// Block-wide exclusive scan of one value per thread (256 threads); returns the
// exclusive prefix, *total = block sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *lds4, uint32_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v, lane);
    if (lane == 63) lds4[w] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < SC_THREADS / 64; ++i) {
        const uint32_t x = lds4[i];
        if (i < w) off += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

__global__ __launch_bounds__(SC_THREADS) void scan_reduce_kernel(const uint32_t *in, uint64_t n,
                                                                 uint32_t *partial) {
    __shared__ uint32_t lds4[4];
    const uint64_t base = (uint64_t)blockIdx.x * SC_TILE;
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        const uint64_t i = base + (uint64_t)j * SC_THREADS + threadIdx.x;
        if (i < n) s += in[i];
    }
    uint32_t tot;
    block_excl_scan(s, lds4, &tot);
    if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

// single block: exclusive scan of partial[0..m) in place, total -> *total
__global__ __launch_bounds__(SC_THREADS) void scan_partials_kernel(uint32_t *partial, uint32_t m,
                                                                   uint32_t *total) {
    __shared__ uint32_t lds4[4];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < m; base += SC_THREADS) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < m ? partial[i] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan(v, lds4, &tot);
        if (i < m) partial[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

__global__ __launch_bounds__(SC_THREADS) void scan_down_kernel(const uint32_t *in, uint32_t *out,
                                                               uint64_t n, const uint32_t *partial) {
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t tile[SC_TILE];
    const uint64_t base = (uint64_t)blockIdx.x * SC_TILE;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {  // coalesced load into LDS
        const uint64_t i = base + (uint64_t)j * SC_THREADS + threadIdx.x;
        tile[j * SC_THREADS + threadIdx.x] = i < n ? in[i] : 0;
    }
    __syncthreads();
    uint32_t v[SC_ITEMS], s = 0;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {  // thread-contiguous items
        v[j] = tile[threadIdx.x * SC_ITEMS + j];
        s += v[j];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan(s, lds4, &tot) + partial[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        tile[threadIdx.x * SC_ITEMS + j] = ex;
        ex += v[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        const uint64_t i = base + (uint64_t)j * SC_THREADS + threadIdx.x;
        if (i < n) out[i] = tile[j * SC_THREADS + threadIdx.x];
    }
}

size_t scan_temp_bytes(uint64_t n) {
    const uint64_t nb = (n + SC_TILE - 1) / SC_TILE;
    return (nb + 64) * sizeof(uint32_t);
}

hipError_t exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total_dev,
                              void *tmp, hipStream_t s) {
    if (n == 0) {
        if (total_dev) return hipMemsetAsync(total_dev, 0, sizeof(uint32_t), s);
        return hipSuccess;
    }
    const uint64_t nb = (n + SC_TILE - 1) / SC_TILE;
    uint32_t *partial = (uint32_t *)tmp;
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((uint32_t)nb), dim3(SC_THREADS), 0, s, in, n, partial);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(SC_THREADS), 0, s, partial, (uint32_t)nb, total_dev);
    hipLaunchKernelGGL(scan_down_kernel, dim3((uint32_t)nb), dim3(SC_THREADS), 0, s, in, out, n,
                       (const uint32_t *)partial);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// radix sort
// ---------------------------------------------------------------------------
constexpr int RS_THREADS = 256;
// keys per thread of a radix tile: 32 (8,192-key tiles) for key-only sorts --
// the k-mer partition sort: digit runs of ~32 keys leave as longer coalesced
// stores (same-box A/B at the bench shape, sort 0.58 -> 0.55 ms; 2,048-key
// tiles 0.69 ms), 16 where values ride along (their LDS staging at 8,192 keys
// would leave one workgroup per CU)
constexpr int RS_ITEMS_KEYS = 32;
#ifndef SA_RS_ITEMS_VALS  // (A/B builds)
#define SA_RS_ITEMS_VALS 32
#endif
// 12-byte records, 8,192-key tiles (8 serial shards of the bench shape: the records' sort
// 1.32 -> 1.20 ms per shard against 4,096; values staged in the key slots after the keys
// went out, two workgroups per CU: 1.35 -> 1.16 ms)
constexpr int RS_ITEMS_VALS = SA_RS_ITEMS_VALS;
constexpr int RS_ITEMS_KV = 16;    // 16-byte records: 4,096-key tiles of 4 waves
template <int ITEMS> struct RsTile {
    static constexpr int TILE = RS_THREADS * ITEMS;
};

// Tile histograms, BLOCK-major: hist[tile * 256 + digit] (one coalesced 1 KB
// row per tile; the digit-major layout made every tile write 256 scattered
// words and the downsweep read them back scattered).  All 16 keys of a thread
// are loaded before the first count, and each wave counts into its own 256
// bins (less same-address contention in the LDS atomics).
// (an 8,192-key tile is counted by 512 threads, 16 keys each: the same work per
// thread as the 4,096-key tiles' upsweep; 256 threads x 32 keys ran 68 us per
// pass at the bench shape against ~35)
template <int RS_ITEMS>
struct RsUp {
    static constexpr int THREADS = RS_ITEMS > 16 ? RS_THREADS * (RS_ITEMS / 16) : RS_THREADS;
    static constexpr int ITEMS = RS_ITEMS > 16 ? 16 : RS_ITEMS;
};
template <int RS_ITEMS, bool GEN = false>
__global__ __launch_bounds__(RsUp<RS_ITEMS>::THREADS) void rs_upsweep_kernel(const uint64_t *keys, uint64_t n,
                                                                            int shift, uint32_t *hist,
                                                                            uint32_t nblocks, KeyGen kg) {
    (void)nblocks;
    constexpr int RS_TILE = RsTile<RS_ITEMS>::TILE, NT = RsUp<RS_ITEMS>::THREADS, IT = RsUp<RS_ITEMS>::ITEMS;
    constexpr int NW = NT / 64;
    __shared__ uint32_t cnt[NW][256];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < NW * 256; i += NT) (&cnt[0][0])[i] = 0;
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    unsigned long long k[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint64_t i = base + (uint64_t)j * NT + tid;
        if constexpr (GEN) k[j] = i < n ? gen_key(kg, i) : 0ull;
        else k[j] = i < n ? __builtin_nontemporal_load(keys + i) : 0ull;  // read once per pass
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint64_t i = base + (uint64_t)j * NT + tid;
        if (i < n) atomicAdd(&cnt[w][(uint32_t)(k[j] >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid < 256) {
        uint32_t s = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) s += cnt[q][tid];
        hist[(uint64_t)blockIdx.x * 256 + tid] = s;
    }
}

// Global scatter offsets from the block-major tile histograms, in place:
// hist[b*256 + d] <- sum_{d' < d} total[d'] + sum_{b' < b} hist[b'*256 + d].
// Three launches over chunks of RS_CHUNK tiles, every access a coalesced row:
// column sums per chunk, a per-digit scan over the chunk sums (+ digit totals),
// then each chunk's column scan.
constexpr int RS_CHUNK = 32;

__global__ __launch_bounds__(256) void rs_colsum_kernel(const uint32_t *hist, uint32_t nb, uint32_t *csum) {
    const uint32_t d = threadIdx.x, c = blockIdx.x;
    uint32_t v[RS_CHUNK];
#pragma unroll
    for (int r = 0; r < RS_CHUNK; ++r) {
        const uint32_t b = c * RS_CHUNK + r;
        v[r] = b < nb ? hist[(uint64_t)b * 256 + d] : 0u;
    }
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < RS_CHUNK; ++r) s += v[r];
    csum[(uint64_t)c * 256 + d] = s;
}

// one block per digit: exclusive scan of that digit's chunk sums, total -> tot[d]
__global__ __launch_bounds__(SC_THREADS) void rs_chunkscan_kernel(uint32_t *csum, uint32_t nc, uint32_t *tot) {
    __shared__ uint32_t lds4[4];
    const uint32_t d = blockIdx.x;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < nc; c0 += SC_THREADS) {
        const uint32_t c = c0 + threadIdx.x;
        const uint32_t v = c < nc ? csum[(uint64_t)c * 256 + d] : 0u;
        uint32_t t;
        const uint32_t ex = block_excl_scan(v, lds4, &t);
        if (c < nc) csum[(uint64_t)c * 256 + d] = carry + ex;
        carry += t;
    }
    if (threadIdx.x == 0) tot[d] = carry;
}

__global__ __launch_bounds__(256) void rs_colscan_kernel(uint32_t *hist, uint32_t nb, const uint32_t *csum,
                                                         const uint32_t *tot) {
    __shared__ uint32_t lds4[4];
    const uint32_t d = threadIdx.x, c = blockIdx.x;
    uint32_t t;
    uint32_t acc = block_excl_scan(tot[d], lds4, &t) + csum[(uint64_t)c * 256 + d];
    uint32_t v[RS_CHUNK];
#pragma unroll
    for (int r = 0; r < RS_CHUNK; ++r) {
        const uint32_t b = c * RS_CHUNK + r;
        v[r] = b < nb ? hist[(uint64_t)b * 256 + d] : 0u;
    }
#pragma unroll
    for (int r = 0; r < RS_CHUNK; ++r) {
        const uint32_t b = c * RS_CHUNK + r;
        if (b < nb) hist[(uint64_t)b * 256 + d] = acc;
        acc += v[r];
    }
}

static hipError_t rs_offsets(uint32_t *hist, uint64_t nb, void *tmp, hipStream_t s) {
    const uint32_t nc = (uint32_t)((nb + RS_CHUNK - 1) / RS_CHUNK);
    uint32_t *csum = (uint32_t *)tmp, *tot = csum + (uint64_t)nc * 256;
    hipLaunchKernelGGL(rs_colsum_kernel, dim3(nc), dim3(256), 0, s, (const uint32_t *)hist, (uint32_t)nb, csum);
    hipLaunchKernelGGL(rs_chunkscan_kernel, dim3(256), dim3(SC_THREADS), 0, s, csum, nc, tot);
    hipLaunchKernelGGL(rs_colscan_kernel, dim3(nc), dim3(256), 0, s, hist, (uint32_t)nb, (const uint32_t *)csum,
                       (const uint32_t *)tot);
    return hipGetLastError();
}

// the scatter's input keys are read once: non-temporal loads leave L2 to merge
// the digit-run stores
__device__ __forceinline__ unsigned long long rs_load_key(const uint64_t *p) { return __builtin_nontemporal_load(p); }

// Stable scatter.  Wave w owns the contiguous sub-tile [base + w*1024, +1024),
// read as 16 coalesced slices of 64; each element's rank among equal digits of
// its wave comes from a 64-lane ballot multisplit (8 ballots -> peer mask) plus
// a wave-private running count in LDS, so the only barriers are per tile.  The
// tile is then staged in LDS in digit order and written out in digit-contiguous
// runs (coalesced), at hist[digit][block] + run offset.
constexpr int RS_WAVES = RS_THREADS / 64;

// An 8,192-key tile runs 512 threads (8 waves of 1,024 keys, 16 per lane: the
// per-wave work and registers of the 4,096-key tiles, twice the waves to hide
// the loads); a 4,096-key tile 256 threads.
template <int RS_ITEMS>
struct RsDown {
    static constexpr int TILE = RsTile<RS_ITEMS>::TILE;
    static constexpr int WAVES = TILE / 1024, THREADS = WAVES * 64, SUB = 1024, SLICES = SUB / 64;
};

// (with values the key slots take the staged values after the keys went out: the
// tile keeps a key-only footprint -- 2 workgroups per CU at 8,192 keys, not 1)
template <bool VALS, int RS_TILE, int WAVES>
struct RsShared {
    unsigned long long key[RS_TILE];
    uint32_t cnt[WAVES][256];      // per-wave digit counts
    uint32_t lofs[256];            // tile-local start of each digit run
    uint32_t gofs[256];            // global start of each digit run
    uint32_t wsum[4];              // the digit scan's wave sums
};

// (wave_peers: sa_internal.h)

// The sources' table (seg[0 .. 2P], starts[0 .. P]) staged in LDS once per block when
// P <= RS_RECV_PMAX: the per-slice and per-lane source searches then cost LDS reads, not
// chains of dependent global loads (the pass ran 3x a plain 12-byte pass on them).
constexpr uint32_t RS_RECV_PMAX = 64;
struct RecvTab {
    const uint64_t *seg;
    const uint32_t *starts;
};

// a received record's read and loc rank (RecvGen; source s holds record i;
// st0 = starts[s0] of the slice's source s0, loaded once per slice)
__device__ __forceinline__ void recv_decode(const RecvGen &g, const RecvTab &t, uint32_t s, uint32_t s0, uint32_t st0,
                                            uint64_t rec, uint32_t &r, uint32_t &lr) {
    const uint32_t local = (uint32_t)rec;
    uint32_t pos;
    if (g.npr) {
        // local / npr as the high word of local * magic (exact for local, npr < 2^32)
        const uint32_t q = g.npr == 1 ? local : (uint32_t)__umul64hi((unsigned long long)local, g.npr_magic);
        r = (s == s0 ? st0 : t.starts[s]) + q;
        pos = local - q * g.npr;
        if (g.lr_ident) {
            lr = pos;
            return;
        }
    } else {
        const uint64_t go = t.seg[g.P + 1 + s] + local;
        uint32_t lo = t.starts[s], up = t.starts[s + 1];  // largest r with occ_off[r] <= go
        while (up - lo > 1) {
            const uint32_t mid = (lo + up) >> 1;
            if (g.occ_off[mid] <= go) lo = mid; else up = mid;
        }
        r = lo;
        pos = (uint32_t)(go - g.occ_off[r]);
    }
    lr = g.lrank[(g.npr ? g.lbase[g.npr - 1] : g.lbase[g.len[r] - g.k]) + pos];
}
// the source of record i: the last s with seg[s] <= i, from a lower bound s0
__device__ __forceinline__ uint32_t recv_source(const RecvGen &g, const RecvTab &t, uint32_t s0, uint64_t i) {
    while (s0 + 1 < g.P && t.seg[s0 + 1] <= i) ++s0;
    return s0;
}

// VALS = false: key-only sort (records that carry their payload in the key).
// RECV: the values are generated from the keys (RecvGen, first pass only)
// (launch bounds: 4 waves per SIMD -- two 8-wave workgroups of an 8,192-key tile per CU,
// as its LDS allows -- so <= 128 VGPRs)
template <bool VALS, int RS_ITEMS, bool GEN = false, bool RECV = false>
__global__ __launch_bounds__(RsDown<RS_ITEMS>::THREADS, 4) void rs_downsweep_kernel(const uint64_t *kin,
                                                                                 const uint32_t *vin, uint64_t *kout,
                                                                                 uint32_t *vout, uint64_t n, int shift,
                                                                                 const uint32_t *hist,
                                                                                 uint32_t nblocks, KeyGen kg,
                                                                                 int nt_out, RecvGen rg) {
    using D = RsDown<RS_ITEMS>;
    constexpr int RS_TILE = D::TILE, RS_SUB = D::SUB, RS_SLICES = D::SLICES, WAVES = D::WAVES, NT = D::THREADS;
    extern __shared__ __align__(16) uint8_t rs_smem[];
    RsShared<VALS, RS_TILE, WAVES> &S = *reinterpret_cast<RsShared<VALS, RS_TILE, WAVES> *>(rs_smem);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    for (int q = lane; q < 256; q += 64) S.cnt[w][q] = 0;
    // no barrier needed: each wave only touches its own counters until the block barrier
    unsigned long long k[RS_SLICES];
    uint32_t v[RS_SLICES], rk[RS_SLICES];
    const uint64_t sub = base + (uint64_t)w * RS_SUB;
#pragma unroll
    for (int j = 0; j < RS_SLICES; ++j) {
        const uint64_t i = sub + (uint64_t)j * 64 + lane;
        if constexpr (GEN) k[j] = i < n ? gen_key(kg, i) : ~0ull;
        else k[j] = i < n ? rs_load_key(kin + i) : ~0ull;
        if constexpr (!RECV) v[j] = (VALS && i < n) ? vin[i] : 0u;
    }
    if constexpr (RECV) {
        __shared__ uint64_t tseg[2 * RS_RECV_PMAX + 1];
        __shared__ uint32_t tstarts[RS_RECV_PMAX + 1];
        RecvTab tab{rg.seg, rg.starts};
        if (rg.P <= RS_RECV_PMAX) {  // (uniform)
            for (uint32_t q = tid; q <= 2 * rg.P; q += NT) tseg[q] = rg.seg[q];
            for (uint32_t q = tid; q <= rg.P; q += NT) tstarts[q] = rg.starts[q];
            __syncthreads();
            tab = RecvTab{tseg, tstarts};
        }
        // decode: the sub-tile's first source by a wave-uniform search, then
        // stepped forward per slice and per lane past segment boundaries
        uint32_t s = 0, hi = rg.P;
        while (hi - s > 1) {
            const uint32_t mid = (s + hi) >> 1;
            if (tab.seg[mid] <= sub) s = mid; else hi = mid;
        }
        s = (uint32_t)__builtin_amdgcn_readfirstlane((int)s);
        // read of the element before the sub-tile (loff boundaries at its start)
        uint32_t rprev = 0xFFFFFFFFu;  // "read -1" before record 0
        if (sub > 0 && sub <= n) {
            const uint64_t ip = sub - 1;
            uint32_t sp = s;
            while (sp > 0 && tab.seg[sp] > ip) --sp;
            uint32_t lrp;
            recv_decode(rg, tab, sp, sp, tab.starts[sp], rs_load_key(kin + ip), rprev, lrp);
        }
#pragma unroll
        for (int j = 0; j < RS_SLICES; ++j) {
            const uint64_t i = sub + (uint64_t)j * 64 + lane;
            const bool valid = i < n;
            s = (uint32_t)__builtin_amdgcn_readfirstlane((int)recv_source(rg, tab, s, sub + (uint64_t)j * 64));
            const uint32_t st0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)tab.starts[s]);
            uint32_t r = 0, lr = 0, sl = s;
            if (valid) {
                sl = recv_source(rg, tab, s, i);
                recv_decode(rg, tab, sl, s, st0, k[j], r, lr);
            }
            if (rg.src_shift) {  // source-relative value, the source in the key's top bits
                v[j] = ((r - (valid ? tab.starts[sl] : 0u)) << rg.lb) | lr;
                if (valid)
                    k[j] = (k[j] & (((1ull << rg.src_shift) - 1ull) & 0xFFFFFFFF00000000ull)) |
                           ((uint64_t)sl << rg.src_shift) | (uint32_t)i;
            } else {
                v[j] = (r << rg.lb) | lr;
                if (valid) k[j] = (k[j] & 0xFFFFFFFF00000000ull) | (uint32_t)i;
            }
            // loff[a] = i for the reads (read(i - 1), read(i)] (read(-1) = -1)
            uint32_t prev = (uint32_t)__shfl_up((int)r, 1, 64);
            if (lane == 0) prev = rprev;
            rprev = (uint32_t)__builtin_amdgcn_readlane((int)r, 63);
            if (valid) {
                for (uint32_t a = prev + 1u; a <= r; ++a) rg.loff[a] = i;
                if (i + 1 == n)  // the reads after the last record
                    for (uint32_t a = r + 1u; a <= rg.n_reads; ++a) rg.loff[a] = n;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < RS_SLICES; ++j) {
        const uint64_t i = sub + (uint64_t)j * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (uint32_t)(k[j] >> shift) & 255u;
        const uint64_t peer = wave_peers(d, valid);
        const uint32_t before = valid ? S.cnt[w][d] : 0u;
        rk[j] = before + __popcll(peer & lt_mask);
        __builtin_amdgcn_wave_barrier();
        if (valid && (peer & lt_mask) == 0) S.cnt[w][d] = before + __popcll(peer);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // digit tid (threads 0-255): tile total, tile-local run start (exclusive scan
    // over digits), global start
    uint32_t tot = 0, inc = 0;
    if (tid < 256) {
#pragma unroll
        for (int q = 0; q < WAVES; ++q) tot += S.cnt[q][tid];
        inc = wave_incl_add(tot);  // block exclusive scan of tot over the 256 digits
        if (lane == 63) S.wsum[w] = inc;
    }
    __syncthreads();
    if (tid < 256) {
        uint32_t pre = 0;
        for (int q = 0; q < w; ++q) pre += S.wsum[q];
        const uint32_t lo = pre + inc - tot;
        S.lofs[tid] = lo;
        S.gofs[tid] = hist[(uint64_t)blockIdx.x * 256 + tid];
        // per-wave bases inside the tile, in place of the counts
        uint32_t acc = lo;
#pragma unroll
        for (int q = 0; q < WAVES; ++q) {
            const uint32_t c = S.cnt[q][tid];
            S.cnt[q][tid] = acc;
            acc += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RS_SLICES; ++j) {
        const uint64_t i = sub + (uint64_t)j * 64 + lane;
        if (i < n) {
            const uint32_t d = (uint32_t)(k[j] >> shift) & 255u;
            rk[j] += S.cnt[w][d];  // the element's slot in the staged tile
            S.key[rk[j]] = k[j];
        }
    }
    __syncthreads();
    const uint32_t nt = (uint32_t)min((uint64_t)RS_TILE, n - base);
    if constexpr (!VALS) {
        for (uint32_t i = tid; i < nt; i += NT) {
            const unsigned long long kk = S.key[i];
            const uint32_t d = (uint32_t)(kk >> shift) & 255u;
            const uint32_t pos = S.gofs[d] + (i - S.lofs[d]);
            if (nt_out) __builtin_nontemporal_store(kk, kout + pos);
            else kout[pos] = kk;
        }
    } else {
        // keys out, each thread keeping its slots' output positions; then the values
        // take the slots and follow to the same positions
        constexpr int PER = RS_TILE / NT;
        uint32_t gp[PER];
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            const uint32_t i = tid + m * NT;
            gp[m] = 0;
            if (i < nt) {
                const unsigned long long kk = S.key[i];
                const uint32_t d = (uint32_t)(kk >> shift) & 255u;
                gp[m] = S.gofs[d] + (i - S.lofs[d]);
                if (nt_out) __builtin_nontemporal_store(kk, kout + gp[m]);
                else kout[gp[m]] = kk;
            }
        }
        __syncthreads();
        uint32_t *sv = reinterpret_cast<uint32_t *>(S.key);
#pragma unroll
        for (int j = 0; j < RS_SLICES; ++j)
            if (sub + (uint64_t)j * 64 + lane < n) sv[rk[j]] = v[j];
        __syncthreads();
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            const uint32_t i = tid + m * NT;
            if (i < nt) vout[gp[m]] = sv[i];
        }
    }
}

// 16-byte records (u64 key, u64 value): the tile is staged through LDS twice --
// keys (with their digits), then the values in the same slots -- so the LDS
// footprint stays that of a key-only tile (3 workgroups per CU, not 2)
constexpr int RS_TILE_KV = RsTile<RS_ITEMS_KV>::TILE;
struct RsSharedKV {
    unsigned long long buf[RS_TILE_KV];  // staged keys, then staged values
    uint8_t dig[RS_TILE_KV];
    uint32_t cnt[RS_WAVES][256];
    uint32_t lofs[256];
    uint32_t gofs[256];
};

__global__ __launch_bounds__(RS_THREADS) void rs_downsweep_kv64_kernel(const uint64_t *kin, const uint64_t *vin,
                                                                       uint64_t *kout, uint64_t *vout, uint64_t n,
                                                                       int shift, const uint32_t *hist,
                                                                       uint32_t nblocks) {
    constexpr int RS_TILE = RS_TILE_KV, RS_SUB = RS_TILE / RS_WAVES, RS_SLICES = RS_SUB / 64;
    extern __shared__ __align__(16) uint8_t rs_smem[];
    RsSharedKV &S = *reinterpret_cast<RsSharedKV *>(rs_smem);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    for (int q = lane; q < 256; q += 64) S.cnt[w][q] = 0;
    unsigned long long k[RS_SLICES], v[RS_SLICES];
    uint32_t rk[RS_SLICES];
    const uint64_t sub = base + (uint64_t)w * RS_SUB;
#pragma unroll
    for (int j = 0; j < RS_SLICES; ++j) {
        const uint64_t i = sub + (uint64_t)j * 64 + lane;
        k[j] = i < n ? rs_load_key(kin + i) : ~0ull;
        v[j] = i < n ? rs_load_key(vin + i) : 0ull;
    }
#pragma unroll
    for (int j = 0; j < RS_SLICES; ++j) {
        const uint64_t i = sub + (uint64_t)j * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (uint32_t)(k[j] >> shift) & 255u;
        const uint64_t peer = wave_peers(d, valid);
        const uint32_t before = valid ? S.cnt[w][d] : 0u;
        rk[j] = before + __popcll(peer & lt_mask);
        __builtin_amdgcn_wave_barrier();
        if (valid && (peer & lt_mask) == 0) S.cnt[w][d] = before + __popcll(peer);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {
        uint32_t tot = 0;
#pragma unroll
        for (int q = 0; q < RS_WAVES; ++q) tot += S.cnt[q][tid];
        const uint32_t inc = wave_incl_add(tot);
        if (lane == 63) S.lofs[w] = inc;
        __syncthreads();
        uint32_t pre = 0;
        for (int q = 0; q < w; ++q) pre += S.lofs[q];
        __syncthreads();
        const uint32_t lo = pre + inc - tot;
        S.lofs[tid] = lo;
        S.gofs[tid] = hist[(uint64_t)blockIdx.x * 256 + tid];
        uint32_t acc = lo;
#pragma unroll
        for (int q = 0; q < RS_WAVES; ++q) {
            const uint32_t c = S.cnt[q][tid];
            S.cnt[q][tid] = acc;
            acc += c;
        }
    }
    __syncthreads();
    uint32_t pos[RS_SLICES];
#pragma unroll
    for (int j = 0; j < RS_SLICES; ++j) {
        const uint64_t i = sub + (uint64_t)j * 64 + lane;
        pos[j] = 0;
        if (i < n) {
            const uint32_t d = (uint32_t)(k[j] >> shift) & 255u;
            pos[j] = S.cnt[w][d] + rk[j];
            S.buf[pos[j]] = k[j];
            S.dig[pos[j]] = (uint8_t)d;
        }
    }
    __syncthreads();
    const uint32_t nt = (uint32_t)min((uint64_t)RS_TILE, n - base);
    for (uint32_t i = tid; i < nt; i += RS_THREADS) {
        const uint32_t d = S.dig[i];
        kout[S.gofs[d] + (i - S.lofs[d])] = S.buf[i];
    }
    __syncthreads();  // staged keys written out: the slots take the values
#pragma unroll
    for (int j = 0; j < RS_SLICES; ++j) {
        const uint64_t i = sub + (uint64_t)j * 64 + lane;
        if (i < n) S.buf[pos[j]] = v[j];
    }
    __syncthreads();
    for (uint32_t i = tid; i < nt; i += RS_THREADS) {
        const uint32_t d = S.dig[i];
        vout[S.gofs[d] + (i - S.lofs[d])] = S.buf[i];
    }
}

size_t radix_sort_temp_bytes(uint64_t n) {  // (the smallest tile: the most tiles)
    constexpr int RS_TILE = RsTile<RS_ITEMS_KV>::TILE;
    const uint64_t nb = (n + RS_TILE - 1) / RS_TILE;
    const uint64_t nc = (nb + RS_CHUNK - 1) / RS_CHUNK;
    const uint64_t hist = 256 * (nb ? nb : 1);
    return (hist + 256 * (nc + 1)) * sizeof(uint32_t) + 256;
}

// one key-only pass at RS_ITEMS keys per lane-slot of a tile
uint32_t radix_key_tile() { return RsTile<RS_ITEMS_KEYS>::TILE; }

// (counted = true: hist already holds this pass's tile counts -- launch_pack_emit_hist)
template <int RS_ITEMS, bool GEN = false>
static hipError_t rs_pass_keys(const uint64_t *kin, uint64_t *kout, uint64_t n, int shift, uint32_t *hist,
                               void *stmp, hipStream_t s, const KeyGen &kg = KeyGen{}, bool nt_out = false,
                               bool counted = false) {
    using SK = RsShared<false, RsTile<RS_ITEMS>::TILE, RsDown<RS_ITEMS>::WAVES>;
    static const size_t sk_lds = occ_lds("SA_OCC_RS", sizeof(SK), sizeof(SK));  // (A/B)
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)rs_downsweep_kernel<false, RS_ITEMS, GEN>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sk_lds);
        attr_set = true;
    }
    const uint64_t nb = (n + RsTile<RS_ITEMS>::TILE - 1) / RsTile<RS_ITEMS>::TILE;
    if (!counted)
        hipLaunchKernelGGL((rs_upsweep_kernel<RS_ITEMS, GEN>), dim3((uint32_t)nb), dim3(RsUp<RS_ITEMS>::THREADS), 0,
                           s, kin, n, shift, hist, (uint32_t)nb, kg);
    hipError_t e = rs_offsets(hist, nb, stmp, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((rs_downsweep_kernel<false, RS_ITEMS, GEN>), dim3((uint32_t)nb),
                       dim3(RsDown<RS_ITEMS>::THREADS), sk_lds, s, kin, nullptr, kout, nullptr, n, shift,
                       (const uint32_t *)hist, (uint32_t)nb, kg, nt_out ? 1 : 0, RecvGen{});
    return hipGetLastError();
}

// key-only passes past 2^27 keys (1 GB per pass: configs[3]'s per-GPU slice)
// take 16,384-key tiles on 16 waves -- runs of ~64 keys per digit, for an
// output far beyond the MALL: slice sort 12.0 -> 10.5 ms; at the bench shape
// (48.6M keys) they measured slower than 8,192 (0.53 vs 0.50 ms)
constexpr uint64_t RS_BIG_TILE_KEYS = 1ull << 27;

// 12-byte (key, u32 value) passes at ITEMS keys per lane-slot of a tile: 8,192-key tiles, and
// 16,384 past 2^27 records (as the key-only passes: runs of ~64 keys per digit for an output far
// beyond the MALL)
template <int ITEMS>
static hipError_t rs_sort_vals(uint64_t **keys, uint32_t **vals, uint64_t **keys_alt, uint32_t **vals_alt,
                               uint64_t n, int lo, int hi, void *tmp, hipStream_t s) {
    constexpr int TV = RsTile<ITEMS>::TILE;
    using SV = RsShared<true, TV, RsDown<ITEMS>::WAVES>;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)rs_downsweep_kernel<true, ITEMS>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(SV));
        attr_set = true;
    }
    uint32_t *hist = (uint32_t *)tmp;
    const uint64_t nb = (n + TV - 1) / TV;
    void *stmp = (void *)(hist + 256 * nb);
    for (int shift = lo; shift < hi; shift += 8) {
        hipLaunchKernelGGL((rs_upsweep_kernel<ITEMS>), dim3((uint32_t)nb), dim3(RsUp<ITEMS>::THREADS), 0, s, *keys, n,
                           shift, hist, (uint32_t)nb, KeyGen{});
        hipError_t e = rs_offsets(hist, nb, stmp, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((rs_downsweep_kernel<true, ITEMS>), dim3((uint32_t)nb), dim3(RsDown<ITEMS>::THREADS),
                           sizeof(SV), s, *keys, *vals, *keys_alt, *vals_alt, n, shift, (const uint32_t *)hist,
                           (uint32_t)nb, KeyGen{}, 0, RecvGen{});
        uint32_t *tv = *vals; *vals = *vals_alt; *vals_alt = tv;
        uint64_t *tk = *keys; *keys = *keys_alt; *keys_alt = tk;
    }
    return hipGetLastError();
}

hipError_t radix_sort(uint64_t **keys, uint32_t **vals, uint64_t **keys_alt, uint32_t **vals_alt,
                      uint64_t n, int lo, int hi, void *tmp, hipStream_t s) {
    if (n <= 1 || hi <= lo) return hipSuccess;
    const bool with_vals = vals != nullptr && *vals != nullptr;
    uint32_t *hist = (uint32_t *)tmp;
    if (!with_vals) {
        void *stmp = (void *)(hist + 256 * ((n + RsTile<RS_ITEMS_KEYS>::TILE - 1) / RsTile<RS_ITEMS_KEYS>::TILE));
        for (int shift = lo; shift < hi; shift += 8) {
            const hipError_t e = n >= RS_BIG_TILE_KEYS
                                     ? rs_pass_keys<2 * RS_ITEMS_KEYS>(*keys, *keys_alt, n, shift, hist, stmp, s)
                                     : rs_pass_keys<RS_ITEMS_KEYS>(*keys, *keys_alt, n, shift, hist, stmp, s);
            if (e != hipSuccess) return e;
            uint64_t *tk = *keys; *keys = *keys_alt; *keys_alt = tk;
        }
        return hipGetLastError();
    }
    return n >= RS_BIG_TILE_KEYS ? rs_sort_vals<2 * RS_ITEMS_VALS>(keys, vals, keys_alt, vals_alt, n, lo, hi, tmp, s)
                                 : rs_sort_vals<RS_ITEMS_VALS>(keys, vals, keys_alt, vals_alt, n, lo, hi, tmp, s);
}

template <int ITEMS>
static hipError_t rs_recv_pass(const RecvGen &g, uint64_t **keys, uint32_t **vals, uint64_t **keys_alt,
                               uint32_t **vals_alt, uint64_t n, int lo, void *tmp, hipStream_t s) {
    constexpr int TV = RsTile<ITEMS>::TILE;
    using SV = RsShared<true, TV, RsDown<ITEMS>::WAVES>;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)rs_downsweep_kernel<true, ITEMS, false, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(SV));
        attr_set = true;
    }
    const uint64_t nb = (n + TV - 1) / TV;
    uint32_t *hist = (uint32_t *)tmp;
    void *stmp = (void *)(hist + 256 * nb);
    // raw received records in, relabelled keys + generated values out
    hipLaunchKernelGGL((rs_upsweep_kernel<ITEMS>), dim3((uint32_t)nb), dim3(RsUp<ITEMS>::THREADS), 0, s, *keys, n, lo,
                       hist, (uint32_t)nb, KeyGen{});
    hipError_t e = rs_offsets(hist, nb, stmp, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((rs_downsweep_kernel<true, ITEMS, false, true>), dim3((uint32_t)nb), dim3(RsDown<ITEMS>::THREADS),
                       sizeof(SV), s, *keys, (const uint32_t *)nullptr, *keys_alt, *vals_alt, n, lo,
                       (const uint32_t *)hist, (uint32_t)nb, KeyGen{}, 0, g);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    { uint32_t *tv = *vals; *vals = *vals_alt; *vals_alt = tv; }
    { uint64_t *tk = *keys; *keys = *keys_alt; *keys_alt = tk; }
    return hipSuccess;
}

hipError_t radix_sort_recv(const RecvGen &g, uint64_t **keys, uint32_t **vals, uint64_t **keys_alt,
                           uint32_t **vals_alt, uint64_t n, int lo, int hi, void *tmp, hipStream_t s) {
    if (n == 0 || hi <= lo) return hipErrorInvalidValue;  // (the caller relabels without a sort)
    // first pass: the received records decoded and relabelled (RecvGen); then as radix_sort
    const hipError_t e = n >= RS_BIG_TILE_KEYS
                             ? rs_recv_pass<2 * RS_ITEMS_VALS>(g, keys, vals, keys_alt, vals_alt, n, lo, tmp, s)
                             : rs_recv_pass<RS_ITEMS_VALS>(g, keys, vals, keys_alt, vals_alt, n, lo, tmp, s);
    if (e != hipSuccess) return e;
    return lo + 8 < hi ? radix_sort(keys, vals, keys_alt, vals_alt, n, lo + 8, hi, tmp, s) : hipSuccess;
}

__global__ void gen_keys_kernel(KeyGen g, uint64_t n, uint64_t *keys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[i] = gen_key(g, i);
}

hipError_t radix_sort_gen(const KeyGen &g, uint64_t **keys, uint64_t **keys_alt, uint64_t n, int lo, int hi,
                          void *tmp, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n <= 1 || hi <= lo) {  // nothing to sort: the records as emitted
        hipLaunchKernelGGL(gen_keys_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, g, n, *keys);
        return hipGetLastError();
    }
    uint32_t *hist = (uint32_t *)tmp;
    void *stmp = (void *)(hist + 256 * ((n + RsTile<RS_ITEMS_KEYS>::TILE - 1) / RsTile<RS_ITEMS_KEYS>::TILE));
    // the last pass writes with non-temporal stores: the bucket build that reads
    // the sorted records next keeps the MALL for its scattered record stores
    // (same box, 4 pairs: hash step 2.503 -> 2.494 ms; SA_SORT_NT=0 for A/B)
    static const bool nt_env = !getenv("SA_SORT_NT") || atoi(getenv("SA_SORT_NT"));
    // first pass: generated keys -> *keys; the rest as radix_sort
    const bool nt0 = nt_env && lo + 8 >= hi;
    hipError_t e = n >= RS_BIG_TILE_KEYS
                       ? rs_pass_keys<2 * RS_ITEMS_KEYS, true>(nullptr, *keys, n, lo, hist, stmp, s, g, nt0)
                       : rs_pass_keys<RS_ITEMS_KEYS, true>(nullptr, *keys, n, lo, hist, stmp, s, g, nt0,
                                                           g.hist_shift == lo);
    if (e != hipSuccess) return e;
    for (int shift = lo + 8; shift < hi; shift += 8) {
        const bool nt = nt_env && shift + 8 >= hi;
        e = n >= RS_BIG_TILE_KEYS ? rs_pass_keys<2 * RS_ITEMS_KEYS>(*keys, *keys_alt, n, shift, hist, stmp, s, KeyGen{}, nt)
                                  : rs_pass_keys<RS_ITEMS_KEYS>(*keys, *keys_alt, n, shift, hist, stmp, s, KeyGen{}, nt);
        if (e != hipSuccess) return e;
        uint64_t *tk = *keys; *keys = *keys_alt; *keys_alt = tk;
    }
    return hipGetLastError();
}

// (key u64, value u64) pairs: 16-byte records (the sharded bucket build's
// {slot | read, loc rank}); same passes as radix_sort
hipError_t radix_sort_kv64(uint64_t **keys, uint64_t **vals, uint64_t **keys_alt, uint64_t **vals_alt, uint64_t n,
                           int lo, int hi, void *tmp, hipStream_t s) {
    if (n <= 1 || hi <= lo) return hipSuccess;
    const uint64_t nb = (n + RS_TILE_KV - 1) / RS_TILE_KV;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)rs_downsweep_kv64_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)sizeof(RsSharedKV));
        attr_set = true;
    }
    uint32_t *hist = (uint32_t *)tmp;
    void *stmp = (void *)(hist + 256 * nb);
    for (int shift = lo; shift < hi; shift += 8) {
        hipLaunchKernelGGL((rs_upsweep_kernel<RS_ITEMS_KV>), dim3((uint32_t)nb), dim3(RsUp<RS_ITEMS_KV>::THREADS), 0,
                           s, *keys, n, shift, hist, (uint32_t)nb, KeyGen{});
        hipError_t e = rs_offsets(hist, nb, stmp, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(rs_downsweep_kv64_kernel, dim3((uint32_t)nb), dim3(RS_THREADS), sizeof(RsSharedKV), s,
                           *keys, *vals, *keys_alt, *vals_alt, n, shift, (const uint32_t *)hist, (uint32_t)nb);
        uint64_t *tv = *vals; *vals = *vals_alt; *vals_alt = tv;
        uint64_t *tk = *keys; *keys = *keys_alt; *keys_alt = tk;
    }
    return hipGetLastError();
}

}  // namespace sa
