// buckets.hip -- bucket/list build over the (hash, locrank, g)-sorted k-mer records.
//
// Device replacement of KmerData's per-hash ArrayBuffers and calcPairData's
// st/md/en split (KmerTable.scala:41-53, :97-115).  One multi-channel scan over
// the sorted records yields, per record, its bucket (distinct hash), its group
// (distinct hash+loc), and its slot in the middle list / edge list; the down
// pass writes those lists (read index per entry) plus the per-group partner
// ranges that make the pair counter's work a prefix of each list:
//   edge role  -> middle entries of the bucket with loc <  own   (fst = edge)
//   middle role-> edge entries of the bucket with loc <= own     (fst = middle; tie -> middle)
// which is addKmerPair's orientation rule (KmerTable.scala:65-71).
// Bound: HBM (scan + scatter).
#include "../sa_internal.h"

namespace sa {

constexpr int BK_THREADS = 256;
constexpr int BK_ITEMS = 8;
constexpr int BK_TILE = BK_THREADS * BK_ITEMS;

struct U4 { uint32_t x, y, z, w; };
__device__ __forceinline__ U4 add4(U4 a, U4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }

struct Flags { uint32_t bhead, ghead, md, ed, st, en; };

__device__ __forceinline__ Flags flags_at(const uint64_t *sk, uint64_t s, uint64_t n, int lb,
                                          const uint8_t *tagtab) {
    const uint64_t k = sk[s];
    Flags f;
    if (s == 0) { f.bhead = 1; f.ghead = 1; }
    else {
        const uint64_t p = sk[s - 1];
        f.bhead = (p >> lb) != (k >> lb);
        f.ghead = p != k;
    }
    const uint32_t t = tagtab[k & ((1ull << lb) - 1)];
    f.st = (t & TAG_ST) ? 1u : 0u;
    f.en = (t & TAG_EN) ? 1u : 0u;
    f.md = (t & TAG_MD) ? 1u : 0u;
    f.ed = f.st + f.en;
    return f;
}

__device__ __forceinline__ U4 wave_incl_scan4(U4 v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        U4 t;
        t.x = __shfl_up(v.x, off, 64); t.y = __shfl_up(v.y, off, 64);
        t.z = __shfl_up(v.z, off, 64); t.w = __shfl_up(v.w, off, 64);
        if (lane >= off) v = add4(v, t);
    }
    return v;
}

__device__ __forceinline__ U4 block_excl_scan4(U4 v, U4 *lds4, U4 *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const U4 inc = wave_incl_scan4(v, lane);
    if (lane == 63) lds4[w] = inc;
    __syncthreads();
    U4 off = {0, 0, 0, 0}, tot = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < BK_THREADS / 64; ++i) {
        const U4 x = lds4[i];
        if (i < w) off = add4(off, x);
        tot = add4(tot, x);
    }
    __syncthreads();
    *total = tot;
    return {off.x + inc.x - v.x, off.y + inc.y - v.y, off.z + inc.z - v.z, off.w + inc.w - v.w};
}

__global__ __launch_bounds__(BK_THREADS) void bk_reduce_kernel(const uint64_t *sk, uint64_t n, int lb,
                                                               const uint8_t *tagtab, U4 *partial) {
    __shared__ U4 lds4[4];
    const uint64_t base = (uint64_t)blockIdx.x * BK_TILE + (uint64_t)threadIdx.x * BK_ITEMS;
    U4 s = {0, 0, 0, 0};
    for (int j = 0; j < BK_ITEMS; ++j) {
        const uint64_t i = base + j;
        if (i < n) {
            const Flags f = flags_at(sk, i, n, lb, tagtab);
            s = add4(s, U4{f.bhead, f.ghead, f.md, f.ed});
        }
    }
    U4 tot;
    block_excl_scan4(s, lds4, &tot);
    if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ __launch_bounds__(BK_THREADS) void bk_partials_kernel(U4 *partial, uint32_t m, uint32_t *totals) {
    __shared__ U4 lds4[4];
    U4 carry = {0, 0, 0, 0};
    for (uint32_t base = 0; base < m; base += BK_THREADS) {
        const uint32_t i = base + threadIdx.x;
        const U4 v = i < m ? partial[i] : U4{0, 0, 0, 0};
        U4 tot;
        const U4 ex = block_excl_scan4(v, lds4, &tot);
        if (i < m) partial[i] = add4(carry, ex);
        carry = add4(carry, tot);
    }
    if (threadIdx.x == 0) {
        totals[0] = carry.x; totals[1] = carry.y; totals[2] = carry.z; totals[3] = carry.w;
    }
}

__device__ __forceinline__ uint32_t read_of(uint32_t g, const uint64_t *occ_off, uint32_t n_reads,
                                            uint32_t npr, const uint2 *rl) {
    if (rl) return rl[g].x;  // occurrence table (distributed mode, mixed lengths)
    if (npr) return g / npr;
    uint32_t lo = 0, hi = n_reads;  // largest r with occ_off[r] <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (occ_off[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(BK_THREADS) void bk_down_kernel(const uint64_t *sk, const uint32_t *sv, uint64_t n,
                                                             int lb, const uint8_t *tagtab,
                                                             const uint64_t *occ_off, uint32_t n_reads,
                                                             uint32_t npr, const uint2 *rl, const U4 *partial,
                                                             Buckets b) {
    __shared__ U4 lds4[4];
    const uint64_t base = (uint64_t)blockIdx.x * BK_TILE + (uint64_t)threadIdx.x * BK_ITEMS;
    Flags f[BK_ITEMS];
    U4 s = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < BK_ITEMS; ++j) {
        const uint64_t i = base + j;
        if (i < n) {
            f[j] = flags_at(sk, i, n, lb, tagtab);
            s = add4(s, U4{f[j].bhead, f[j].ghead, f[j].md, f[j].ed});
        } else {
            f[j] = Flags{0, 0, 0, 0, 0, 0};
        }
    }
    U4 tot;
    U4 ex = add4(block_excl_scan4(s, lds4, &tot), partial[blockIdx.x]);
#pragma unroll
    for (int j = 0; j < BK_ITEMS; ++j) {
        const uint64_t i = base + j;
        if (i >= n) break;
        const Flags &F = f[j];
        const uint32_t bid = ex.x + F.bhead - 1;
        const uint32_t gid = ex.y + F.ghead - 1;
        const uint32_t g = sv[i];
        const uint32_t r = read_of(g, occ_off, n_reads, npr, rl);
        if (F.md) b.md_list[ex.z] = r;
        if (F.st) b.ed_list[ex.w] = r;
        if (F.en) b.ed_list[ex.w + F.st] = r;
        if (F.bhead) { b.bkt_mdo[bid] = ex.z; b.bkt_edo[bid] = ex.w; b.bkt_start[bid] = (uint32_t)i; }
        if (F.ghead) { b.grp_mds[gid] = ex.z; b.grp_bid[gid] = bid; }
        const bool gend = (i + 1 == n) || (sk[i + 1] != sk[i]);
        if (gend) b.grp_ede[gid] = ex.w + F.ed;
        b.occ_gid[g] = gid;
        if (i + 1 == n) {  // sentinels
            b.bkt_mdo[bid + 1] = ex.z + F.md;
            b.bkt_edo[bid + 1] = ex.w + F.ed;
            b.bkt_start[bid + 1] = (uint32_t)n;
        }
        ex = add4(ex, U4{F.bhead, F.ghead, F.md, F.ed});
    }
}

size_t buckets_temp_bytes(uint64_t n) {
    const uint64_t nb = (n + BK_TILE - 1) / BK_TILE;
    return (nb + 16) * sizeof(U4);
}

hipError_t build_buckets(const uint64_t *skeys, const uint32_t *svals, uint64_t n, int lb,
                         const uint8_t *tagtab, const uint64_t *occ_off, uint32_t n_reads,
                         uint32_t uniform_npr, const uint2 *rl, Buckets &b,
                         uint32_t *totals_dev, void *tmp, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(totals_dev, 0, 4 * sizeof(uint32_t), s);
    const uint64_t nb = (n + BK_TILE - 1) / BK_TILE;
    U4 *partial = (U4 *)tmp;
    hipLaunchKernelGGL(bk_reduce_kernel, dim3((uint32_t)nb), dim3(BK_THREADS), 0, s, skeys, n, lb, tagtab, partial);
    hipLaunchKernelGGL(bk_partials_kernel, dim3(1), dim3(BK_THREADS), 0, s, partial, (uint32_t)nb, totals_dev);
    hipLaunchKernelGGL(bk_down_kernel, dim3((uint32_t)nb), dim3(BK_THREADS), 0, s, skeys, svals, n, lb, tagtab,
                       occ_off, n_reads, uniform_npr, rl, (const U4 *)partial, b);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Strict mode: (id,pos)-order indices inside each bucket's st / md / en lists,
// which calcPairData's traversal order is made of (KmerTable.scala:97-128).
// One thread per sorted record; O(bucket size) each (strict mode is < 32k reads).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void strict_index_kernel(const uint64_t *sk, const uint32_t *sv, uint64_t n,
                                                           int lb, const uint8_t *tagtab, Buckets b) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const uint64_t lbm = (1ull << lb) - 1;
    const uint32_t g = sv[s];
    const uint32_t bid = b.grp_bid[b.occ_gid[g]];
    const uint32_t s0 = b.bkt_start[bid], s1 = b.bkt_start[bid + 1];
    const uint32_t t = tagtab[sk[s] & lbm];
    uint32_t nst = 0, nmd = 0, nen = 0;       // same-tag records with smaller g
    uint32_t md_before = 0, ed_before = 0;    // list slots taken before s (sorted order)
    uint32_t st_total = 0;
    for (uint32_t q = s0; q < s1; ++q) {
        const uint32_t tq = tagtab[sk[q] & lbm];
        const uint32_t gq = sv[q];
        st_total += (tq & TAG_ST) ? 1u : 0u;
        if (gq < g) {
            nst += (tq & TAG_ST) ? 1u : 0u;
            nmd += (tq & TAG_MD) ? 1u : 0u;
            nen += (tq & TAG_EN) ? 1u : 0u;
        }
        if (q < s) {
            md_before += (tq & TAG_MD) ? 1u : 0u;
            ed_before += ((tq & TAG_ST) ? 1u : 0u) + ((tq & TAG_EN) ? 1u : 0u);
        }
    }
    b.occ_idx[3ull * g + 0] = nst;
    b.occ_idx[3ull * g + 1] = nmd;
    b.occ_idx[3ull * g + 2] = nen;
    if (t & TAG_MD) b.md_idx[b.bkt_mdo[bid] + md_before] = nmd;
    uint32_t e = b.bkt_edo[bid] + ed_before;
    if (t & TAG_ST) b.ed_idx[e++] = nst;                  // phase 0
    if (t & TAG_EN) b.ed_idx[e] = (1u << 31) | nen;       // phase 1
    if (s == s0) b.bkt_nst[bid] = st_total;
}

hipError_t build_strict_index(const uint64_t *skeys, const uint32_t *svals, uint64_t n, int lb,
                              const uint8_t *tagtab, Buckets &b, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(strict_index_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, skeys, svals, n,
                       lb, tagtab, b);
    return hipGetLastError();
}

// Strict mode: per bucket its hash and first occurrence (min g) -> host replays
// KmerData's insertion order (KmerTable.scala:45-50).
__global__ void bucket_first_kernel(const uint64_t *sk, const uint32_t *sv, Buckets b, int lb, uint32_t *hash_out,
                                    uint32_t *first_out) {
    const uint32_t bid = blockIdx.x * blockDim.x + threadIdx.x;
    if (bid >= b.n_buckets) return;
    const uint32_t s0 = b.bkt_start[bid], s1 = b.bkt_start[bid + 1];
    uint32_t g = 0xFFFFFFFFu;
    for (uint32_t q = s0; q < s1; ++q) g = min(g, sv[q]);
    hash_out[bid] = (uint32_t)(sk[s0] >> lb);
    first_out[bid] = g;
}

hipError_t launch_bucket_first(const uint64_t *skeys, const uint32_t *svals, const Buckets &b, int lb,
                               uint32_t *hash_out, uint32_t *first_out, hipStream_t s) {
    if (!b.n_buckets) return hipSuccess;
    hipLaunchKernelGGL(bucket_first_kernel, dim3((b.n_buckets + 255) / 256), dim3(256), 0, s, skeys, svals, b, lb,
                       hash_out, first_out);
    return hipGetLastError();
}

}  // namespace sa
