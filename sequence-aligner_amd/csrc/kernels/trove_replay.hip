// trove_replay.hip -- GNU Trove 3.0.3 slot layout of a key sequence, on the device.
//
// The strict-id output order is the iteration order of the reference's Trove maps
// (KmerTable.scala:26-37; semantics in csrc/host/trove.h): keys inserted one after
// another into an open-addressing table (slot = hash % cap, double-hashing step
// 1 + hash % (cap - 2), downwards), the table rehashed into next_prime(2 cap) --
// old slots reinserted from high to low -- whenever its size passes cap / 2, and
// iterated from slot cap - 1 down to 0.  The host replay (trove.h) is one insert
// after another at DRAM latency: ~170 ms of configs[0]'s 0.2 s end to end.
//
// Here each table of the rehash chain is built in parallel by deterministic
// reservations with eviction chains: a key's priority p is its place in the table's
// insertion order; a thread carries a key to its next probe slot and claims it with
// atomicMin(owner[slot], p).  An empty slot ends the chain; an earlier key there sends
// the carried key on to its next probe slot; a later key there is evicted -- the
// thread now carries it on from that slot.  Slot owners only ever decrease, so every
// slot a key has passed holds an earlier key for good, and when every chain has ended
// each key sits at the first slot of its probe sequence not held by an earlier key --
// exactly where sequential insertion in priority order puts it (insertions only,
// distinct keys).  One launch per table, no rounds; ~1 claim per key at load <= 1/2.
// The rehash chain stays sequential: a table's insertion order starts with the
// previous table's keys in descending slot order, so each table waits for the
// previous one; the sizes of every table are known up front.  (A CPU emulation with
// shuffled thread orders reproduced trove.h's layout for 0 .. 200,000 random keys.)
#include <algorithm>
#include <vector>

#include "../sa_internal.h"
#include "../host/trove.h"

namespace sa {
namespace {

constexpr uint32_t TR_EMPTY = 0xFFFFFFFFu;
constexpr int TR_T = 256;

__global__ void tr_fill_kernel(uint32_t *owner, uint32_t cap) {
    const uint32_t i = blockIdx.x * TR_T + threadIdx.x;
    if (i < cap) owner[i] = TR_EMPTY;
}

// the insertion order of a table: n_re keys carried over (already in ord), then the
// arrivals [a0, a0 + na) of the key sequence
__global__ void tr_append_kernel(uint32_t *ord, uint32_t n_re, uint32_t a0, uint32_t na) {
    const uint32_t j = blockIdx.x * TR_T + threadIdx.x;
    if (j < na) ord[n_re + j] = a0 + j;
}

// every key's chain: carried from its home slot until a slot is empty
__global__ void tr_chain_kernel(const int32_t *keys, const uint32_t *ord, uint32_t n, uint32_t cap, uint32_t *owner) {
    const uint32_t p0 = blockIdx.x * TR_T + threadIdx.x;
    if (p0 >= n) return;
    uint32_t cur = p0;
    uint32_t h = (uint32_t)(keys[ord[cur]] & 0x7fffffff);
    uint32_t t = h % cap;
    for (;;) {
        const uint32_t old = atomicMin(&owner[t], cur);
        if (old == TR_EMPTY) break;
        if (old > cur) {  // a later key evicted: it goes on from this slot
            cur = old;
            h = (uint32_t)(keys[ord[cur]] & 0x7fffffff);
        }
        const uint32_t step = 1u + h % (cap - 2u);
        t = t >= step ? t - step : t + cap - step;
    }
}

// slots in iteration order (cap - 1 down to 0): occupancy flags, then the keys' indices
__global__ void tr_flags_kernel(const uint32_t *owner, uint32_t cap, uint32_t *flag) {
    const uint32_t j = blockIdx.x * TR_T + threadIdx.x;
    if (j < cap) flag[j] = owner[cap - 1 - j] != TR_EMPTY ? 1u : 0u;
}
__global__ void tr_gather_kernel(const uint32_t *owner, uint32_t cap, const uint32_t *flag, const uint32_t *ex,
                                 const uint32_t *ord, uint32_t *out) {
    const uint32_t j = blockIdx.x * TR_T + threadIdx.x;
    if (j < cap && flag[j]) out[ex[j]] = ord[owner[cap - 1 - j]];
}

inline dim3 tr_grid(uint64_t n) { return dim3((uint32_t)((n + TR_T - 1) / TR_T)); }

}  // namespace

// the table sizes of inserting m keys into a fresh map (trove.h: reset, insert, rehash)
static void trove_levels(uint32_t m, std::vector<uint32_t> &cap, std::vector<uint32_t> &n_re,
                         std::vector<uint32_t> &a0, std::vector<uint32_t> &na) {
    const float f = 10.0f / 0.5f;
    int32_t c0 = (int32_t)f;
    if (f - (float)c0 > 0.0f) ++c0;
    int32_t c = TroveLayout::next_prime(c0);
    uint32_t size = 0, arrived = 0;
    for (;;) {
        const int32_t lf = (int32_t)((float)c * 0.5f);
        const uint32_t maxs = (uint32_t)(c - 1 < lf ? c - 1 : lf);
        const uint32_t take = std::min<uint32_t>(m - arrived, maxs + 1 - size);
        cap.push_back((uint32_t)c);
        n_re.push_back(size);
        a0.push_back(arrived);
        na.push_back(take);
        arrived += take;
        size += take;
        if (size <= maxs) break;  // every key in; no rehash pending
        c = TroveLayout::next_prime(c << 1);  // the insert that passed maxSize rehashes at once
    }
}

size_t trove_temp_bytes(uint32_t m) {
    std::vector<uint32_t> cap, n_re, a0, na;
    trove_levels(m, cap, n_re, a0, na);
    const uint64_t cmax = cap.back(), nmax = m;
    // owner, flag, ex (cap each), ord x 2 (n each), the scan total, scan scratch
    return (3 * cmax + 2 * nmax + 64) * 4 + scan_temp_bytes(cmax) + 256;
}

hipError_t trove_layout_device(const int32_t *keys, uint32_t m, uint32_t *out_order, void *tmp, hipStream_t s,
                               uint32_t *final_cap) {
    if (m == 0) {
        if (final_cap) *final_cap = 0;
        return hipSuccess;
    }
    std::vector<uint32_t> cap, n_re, a0, na;
    trove_levels(m, cap, n_re, a0, na);
    const uint64_t cmax = cap.back();
    uint32_t *owner = (uint32_t *)tmp, *flag = owner + cmax, *ex = flag + cmax;
    uint32_t *ordA = ex + cmax, *ordB = ordA + m, *total = ordB + m;
    void *stmp = (void *)(total + 64);
    uint32_t *ord = ordA, *next = ordB;
    hipError_t e;
    for (size_t l = 0; l < cap.size(); ++l) {
        const uint32_t C = cap[l], n = n_re[l] + na[l];
        if (na[l]) hipLaunchKernelGGL(tr_append_kernel, tr_grid(na[l]), dim3(TR_T), 0, s, ord, n_re[l], a0[l], na[l]);
        hipLaunchKernelGGL(tr_fill_kernel, tr_grid(C), dim3(TR_T), 0, s, owner, C);
        hipLaunchKernelGGL(tr_chain_kernel, tr_grid(n), dim3(TR_T), 0, s, keys, ord, n, C, owner);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        // the table's keys in iteration order: the next table's first keys, or the output
        uint32_t *dst = l + 1 < cap.size() ? next : out_order;
        hipLaunchKernelGGL(tr_flags_kernel, tr_grid(C), dim3(TR_T), 0, s, owner, C, flag);
        if ((e = exclusive_scan_u32(flag, ex, C, total, stmp, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(tr_gather_kernel, tr_grid(C), dim3(TR_T), 0, s, owner, C, flag, ex, ord, dst);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        std::swap(ord, next);
    }
    if (final_cap) *final_cap = cap.back();
    return hipSuccess;
}

}  // namespace sa

namespace sa {
namespace {
// PairData's keys, (fst << 16) ^ snd (KmerTable.scala:57-80), of the distinct pairs in
// first-occurrence order
__global__ void tr_pair_keys_kernel(const int32_t *f, const int32_t *s, uint32_t n, int32_t *keys) {
    const uint32_t i = blockIdx.x * TR_T + threadIdx.x;
    if (i < n) keys[i] = (int32_t)(((uint32_t)f[i] << 16) ^ (uint32_t)s[i]);
}
// the pairs permuted into iteration order (the host then reads them front to back)
__global__ void tr_gather3_kernel(const uint32_t *order, uint32_t n, const int32_t *f, const int32_t *s,
                                  const int32_t *k, int32_t *fo, int32_t *so, int32_t *ko) {
    const uint32_t j = blockIdx.x * TR_T + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = order[j];
    fo[j] = f[i];
    so[j] = s[i];
    ko[j] = k[i];
}
}  // namespace

hipError_t launch_trove_pair_keys(const int32_t *f, const int32_t *s, uint32_t n, int32_t *keys, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(tr_pair_keys_kernel, tr_grid(n), dim3(TR_T), 0, st, f, s, n, keys);
    return hipGetLastError();
}

hipError_t launch_trove_gather3(const uint32_t *order, uint32_t n, const int32_t *f, const int32_t *s, const int32_t *k,
                                int32_t *fo, int32_t *so, int32_t *ko, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(tr_gather3_kernel, tr_grid(n), dim3(TR_T), 0, st, order, n, f, s, k, fo, so, ko);
    return hipGetLastError();
}

}  // namespace sa

// ---------------------------------------------------------------------------
// KmerData (KmerTable.scala:45-50): the buckets' iteration rank, from the Trove layout
// of their seqHash values inserted in first-occurrence order.  A bucket is named by
// the sorted position of its head record (is_head / bkt_first from the bucket build).
// ---------------------------------------------------------------------------
namespace sa {
namespace {
__global__ void kd_by_g_kernel(const uint8_t *head, const uint32_t *first, uint64_t n, uint32_t *by_g) {
    const uint64_t i = (uint64_t)blockIdx.x * TR_T + threadIdx.x;
    if (i < n && head[i]) by_g[first[i]] = (uint32_t)i + 1u;
}
__global__ void kd_flags_kernel(const uint32_t *by_g, uint64_t n, uint32_t *flag) {
    const uint64_t g = (uint64_t)blockIdx.x * TR_T + threadIdx.x;
    if (g < n) flag[g] = by_g[g] != 0 ? 1u : 0u;
}
// the heads in first-occurrence order: their positions and the seqHash of their k-mer
// (ObjectStore.scala:48-67: the first min(16, k) bases, h = (h << 2) ^ code, A0 C1 T2 G3 --
// the packed HOXD codes A0 C1 G2 T3 mapped by c ^ (c >> 1))
__global__ void kd_keys_kernel(const uint32_t *by_g, const uint32_t *flag, const uint32_t *ex, uint64_t n,
                               DevReads rd, const uint64_t *occ_off, uint32_t n_reads, int shift, uint32_t *hpos,
                               int32_t *keys) {
    const uint64_t g = (uint64_t)blockIdx.x * TR_T + threadIdx.x;
    if (g >= n || !flag[g]) return;
    uint32_t lo = 0, hi = n_reads;  // the read of occurrence g: the largest r with occ_off[r] <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (occ_off[mid] <= g) lo = mid; else hi = mid;
    }
    const int32_t pos = (int32_t)(g - occ_off[lo]);
    uint32_t x = window16(rd.codes + rd.woff[lo], pos);
    x = shift == 32 ? 0u : (x >> shift);
    x ^= (x >> 1) & 0x55555555u;
    const uint32_t j = ex[g];
    hpos[j] = by_g[g] - 1u;
    keys[j] = (int32_t)x;
}
__global__ void kd_rank_kernel(const uint32_t *order, uint32_t m, const uint32_t *hpos, uint32_t *rank) {
    const uint32_t j = blockIdx.x * TR_T + threadIdx.x;
    if (j < m) rank[hpos[order[j]]] = j;
}
}  // namespace

size_t kmerdata_temp_bytes(uint64_t n) {
    // by_g, flag, ex, hpos, keys, order (n each), the head count, the layout's scratch
    return (6 * n + 64) * 4 + std::max<size_t>(scan_temp_bytes(n), trove_temp_bytes((uint32_t)n)) + 256;
}

hipError_t kmerdata_rank_device(const uint8_t *is_head, const uint32_t *bkt_first, uint64_t n, const DevReads &rd,
                                const uint64_t *occ_off, uint32_t n_reads, int m_hash, uint32_t *rank, void *tmp,
                                hipStream_t s, uint32_t *n_heads) {
    *n_heads = 0;
    hipError_t e;
    if ((e = hipMemsetAsync(rank, 0, n * 4, s)) != hipSuccess || n == 0) return e;
    uint32_t *by_g = (uint32_t *)tmp, *flag = by_g + n, *ex = flag + n, *hpos = ex + n;
    int32_t *keys = (int32_t *)(hpos + n);
    uint32_t *order = (uint32_t *)(keys + n), *total = order + n;
    void *stmp = (void *)(total + 64);
    if ((e = hipMemsetAsync(by_g, 0, n * 4, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(kd_by_g_kernel, tr_grid(n), dim3(TR_T), 0, s, is_head, bkt_first, n, by_g);
    hipLaunchKernelGGL(kd_flags_kernel, tr_grid(n), dim3(TR_T), 0, s, by_g, n, flag);
    if ((e = exclusive_scan_u32(flag, ex, n, total, stmp, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(kd_keys_kernel, tr_grid(n), dim3(TR_T), 0, s, by_g, flag, ex, n, rd, occ_off, n_reads,
                       32 - 2 * m_hash, hpos, keys);
    uint32_t m = 0;
    if ((e = hipMemcpyAsync(&m, total, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    *n_heads = m;
    uint32_t cap = 0;
    if ((e = trove_layout_device(keys, m, order, stmp, s, &cap)) != hipSuccess) return e;
    if (m) hipLaunchKernelGGL(kd_rank_kernel, tr_grid(m), dim3(TR_T), 0, s, order, m, hpos, rank);
    return hipGetLastError();
}
}  // namespace sa

// the pairs of PairData's iteration order whose count passes [min_c, max_c]
// (calcDispatchData's filter, KmerTable.scala:155-187), compacted in that order
namespace sa {
namespace {
__global__ void tr_keep_kernel(const int32_t *k, uint32_t n, int32_t min_c, int32_t max_c, uint32_t *flag) {
    const uint32_t j = blockIdx.x * TR_T + threadIdx.x;
    if (j < n) flag[j] = (k[j] >= min_c && k[j] <= max_c) ? 1u : 0u;
}
__global__ void tr_compact3_kernel(const uint32_t *flag, const uint32_t *ex, uint32_t n, const int32_t *f,
                                   const int32_t *s, const int32_t *k, int32_t *fo, int32_t *so, int32_t *ko) {
    const uint32_t j = blockIdx.x * TR_T + threadIdx.x;
    if (j >= n || !flag[j]) return;
    const uint32_t q = ex[j];
    fo[q] = f[j];
    so[q] = s[j];
    ko[q] = k[j];
}
}  // namespace

hipError_t launch_trove_keep(const int32_t *f, const int32_t *s, const int32_t *k, uint32_t n, int32_t min_c,
                             int32_t max_c, uint32_t *flag, uint32_t *ex, uint32_t *total, void *stmp, int32_t *fo,
                             int32_t *so, int32_t *ko, hipStream_t st) {
    if (!n) return hipMemsetAsync(total, 0, 4, st);
    hipLaunchKernelGGL(tr_keep_kernel, tr_grid(n), dim3(TR_T), 0, st, k, n, min_c, max_c, flag);
    hipError_t e = exclusive_scan_u32(flag, ex, n, total, stmp, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(tr_compact3_kernel, tr_grid(n), dim3(TR_T), 0, st, flag, ex, n, f, s, k, fo, so, ko);
    return hipGetLastError();
}
}  // namespace sa
