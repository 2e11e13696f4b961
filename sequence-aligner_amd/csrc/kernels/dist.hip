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
__global__ void prepare_received_kernel(uint64_t *recs, uint64_t n, const uint64_t *seg, uint32_t P,
                                        const uint32_t *starts, const uint64_t *occ_off, uint32_t npr,
                                        const int32_t *len, const uint32_t *lbase, const uint32_t *lrank, int32_t k,
                                        uint2 *rl) {
    const uint64_t i = (uint64_t)blockIdx.x * DT + threadIdx.x;
    if (i >= n) return;
    uint32_t s = 0, hi = P;  // the source whose segment holds i
    while (hi - s > 1) {
        const uint32_t mid = (s + hi) >> 1;
        if (seg[mid] <= i) s = mid; else hi = mid;
    }
    const uint64_t rec = recs[i];
    const uint32_t local = (uint32_t)rec;
    uint32_t r, pos;
    if (npr) {
        r = starts[s] + local / npr;
        pos = local % npr;
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
    rl[i] = make_uint2(r, lrank[lbase[(npr ? (int32_t)npr + k - 1 : len[r]) - k] + pos]);
    recs[i] = (rec & 0xFFFFFFFF00000000ull) | (uint32_t)i;
}

// loff[a] = first i with rl[i].x >= a, for a in [0, n_reads] (reads ascending):
// the local occurrences of read a are [loff[a], loff[a+1]).  One pass over the
// records: record i starts the reads (rl[i-1].x, rl[i].x] (usually one), the
// last record closes the reads after it
__global__ void local_offsets_kernel(const uint2 *rl, uint64_t n, uint32_t n_reads, uint64_t *loff) {
    const uint64_t i = (uint64_t)blockIdx.x * DT + threadIdx.x;
    if (i > n) return;
    const uint32_t prev = i == 0 ? 0u : rl[i - 1].x + 1u;  // first read not yet started
    const uint32_t cur = i == n ? n_reads + 1u : rl[i].x + 1u;
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

__global__ void gather_partials_kernel(const uint32_t *perm, uint64_t n, const uint32_t *fst, const uint32_t *snd,
                                       const uint32_t *cnt, uint32_t *of, uint32_t *os, uint32_t *oc) {
    const uint64_t i = (uint64_t)blockIdx.x * DT + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = perm[i];
    of[i] = fst[j];
    os[i] = snd[j];
    oc[i] = cnt[j];
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

}  // namespace

hipError_t launch_iota(uint32_t *v, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(iota_kernel, grid_for(n), dim3(DT), 0, s, v, n);
    return hipGetLastError();
}

hipError_t launch_prepare_received(uint64_t *recs, uint64_t n, const uint64_t *seg, uint32_t P,
                                   const uint32_t *starts, const uint64_t *occ_off, uint32_t npr, const int32_t *len,
                                   const uint32_t *lbase, const uint32_t *lrank, int32_t k, uint2 *rl,
                                   hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(prepare_received_kernel, grid_for(n), dim3(DT), 0, s, recs, n, seg, P, starts, occ_off, npr,
                       len, lbase, lrank, k, rl);
    return hipGetLastError();
}

hipError_t launch_local_offsets(const uint2 *rl, uint64_t n, uint32_t n_reads, uint64_t *loff, hipStream_t s) {
    hipLaunchKernelGGL(local_offsets_kernel, grid_for(n + 1), dim3(DT), 0, s, rl, n, n_reads, loff);
    return hipGetLastError();
}

hipError_t launch_owner_bounds(const uint64_t *keys, uint64_t n, int shift, uint32_t P, uint64_t *bounds,
                               hipStream_t s) {
    hipLaunchKernelGGL(owner_bounds_kernel, dim3(1), dim3(((P + 1 + 63) / 64) * 64), 0, s, keys, n, shift, P,
                       bounds);
    return hipGetLastError();
}

hipError_t launch_gather_partials(const uint32_t *perm, uint64_t n, const uint32_t *fst, const uint32_t *snd,
                                  const uint32_t *cnt, uint32_t *of, uint32_t *os, uint32_t *oc, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(gather_partials_kernel, grid_for(n), dim3(DT), 0, s, perm, n, fst, snd, cnt, of, os, oc);
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
