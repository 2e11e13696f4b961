// scatter_probe.hip -- memory-system probe behind the bucket-build design
// (DESIGN.md 4.4): cost of N random 8/16-byte stores as a function of the target
// array size (does the 256 MB Infinity Cache merge partial-line writes when the
// scatter window fits it?), of a windowed scatter (targets grouped into windows),
// and of N random 4-byte loads (L2 request rate).  Standalone; not part of the
// library.  Build: hipcc -O3 --offload-arch=gfx950 -o scatter_probe scatter_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// targets: idx[i] = permutation-like random slot in [0, slots) (precomputed)
__global__ void make_idx(uint32_t *idx, uint64_t n, uint64_t slots, uint32_t window_slots) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (window_slots) {
        // item i goes to window w = i / (n / nwin), random slot inside that window
        const uint64_t nwin = (slots + window_slots - 1) / window_slots;
        const uint64_t per = (n + nwin - 1) / nwin;
        const uint64_t w = i / per;
        // the last window may be partial: stay inside [0, slots)
        idx[i] = (uint32_t)((w * window_slots + hash32((uint32_t)i * 2654435761u) % window_slots) % slots);
    } else {
        idx[i] = (uint32_t)(((uint64_t)hash32((uint32_t)i) * slots) >> 32);
    }
}

template <int B>
struct Rec { uint32_t v[B / 4]; };

template <int B>
__global__ void scatter(const uint32_t *idx, uint64_t n, Rec<B> *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Rec<B> r;
#pragma unroll
    for (int j = 0; j < B / 4; ++j) r.v[j] = (uint32_t)i + j;
    out[idx[i]] = r;
}

__global__ void scatter_nt8(const uint32_t *idx, uint64_t n, uint64_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    __builtin_nontemporal_store((uint64_t)i * 3u, out + idx[i]);
}
__global__ void scatter4(const uint32_t *idx, uint64_t n, uint32_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[idx[i]] = (uint32_t)i;
}

// per-block cursor claims: lane b < nbins of every block adds 16 to cursor
// (b, block % nshard) and keeps the old value (the staged-scatter design's
// atomics: one claim per bin and partition)
__global__ void claim_kernel(unsigned long long *cur, uint32_t nbins, uint32_t nshard, uint32_t *sink) {
    const uint32_t b = threadIdx.x;
    if (b < nbins) {
        const unsigned long long old = atomicAdd(&cur[(uint64_t)b * nshard + blockIdx.x % nshard], 16ull);
        if (old == 0xFFFFFFFFFFull) sink[0] = (uint32_t)old;
    }
}

// Staged scatter (the round-3 bucket-build design): block b owns items
// [b*ipb, (b+1)*ipb) (one partition), bins them by g >> wshift in LDS, claims
// one run per bin from cursor (bin, b % ns), writes {g, value} there (region
// capacity cap; overflow -> direct store); then stage_scatter walks the
// regions bin-major so the stores in flight land in about one bin's span.
__global__ void stage_kernel(const uint32_t *idx, uint64_t n, uint32_t ipb, int wshift, uint32_t nbins, uint32_t ns,
                             uint64_t cap, unsigned long long *cur, uint32_t *sg, uint64_t *sv, uint64_t *out) {
    __shared__ uint32_t cnt[256];
    __shared__ uint64_t base[256];
    const uint64_t b0 = (uint64_t)blockIdx.x * ipb;
    if (threadIdx.x < nbins) cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t gv[4], bn[4], rk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = b0 + threadIdx.x + j * 256;
        bn[j] = 0xFFFFFFFFu;
        if (threadIdx.x + j * 256 < ipb && i < n) {
            gv[j] = idx[i];
            bn[j] = gv[j] >> wshift;
            rk[j] = atomicAdd(&cnt[bn[j]], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < nbins && cnt[threadIdx.x])
        base[threadIdx.x] = atomicAdd(&cur[(uint64_t)threadIdx.x * ns + blockIdx.x % ns], (unsigned long long)cnt[threadIdx.x]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (bn[j] == 0xFFFFFFFFu) continue;
        const uint64_t pos = base[bn[j]] + rk[j];
        const uint64_t v = (uint64_t)gv[j] * 3u;
        if (pos < cap) {
            const uint64_t at = ((uint64_t)bn[j] * ns + blockIdx.x % ns) * cap + pos;
            sg[at] = gv[j];
            sv[at] = v;
        } else {
            out[gv[j]] = v;
        }
    }
}
__global__ void stage_scatter(const unsigned long long *cur, uint32_t nregions, uint64_t cap, const uint32_t *sg,
                              const uint64_t *sv, uint64_t *out) {
    const uint64_t chunks = (cap + 1023) / 1024;
    const uint64_t r = blockIdx.x / chunks, c = blockIdx.x % chunks;
    if (r >= nregions) return;
    const uint64_t m = min((uint64_t)cur[r], cap);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t q = c * 1024 + j * 256 + threadIdx.x;
        if (q < m) out[sg[r * cap + q]] = sv[r * cap + q];
    }
}

template <int B>
__global__ void stream_write(uint64_t n, Rec<B> *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Rec<B> r;
#pragma unroll
    for (int j = 0; j < B / 4; ++j) r.v[j] = (uint32_t)i + j;
    out[i] = r;
}

__global__ void gather(const uint32_t *idx, uint64_t n, const uint32_t *src, uint32_t *sink) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = src[idx[i]];
    if (v == 0xDEADBEEFu) sink[0] = v;
}

static float time_it(void (*fn)(void *), void *arg, int reps) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    fn(arg);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) fn(arg);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

struct Args { const uint32_t *idx; uint64_t n; void *out; const uint32_t *src; uint32_t *sink; };
static Args g;
static dim3 grid_of(uint64_t n) { return dim3((uint32_t)((n + 255) / 256)); }
static void run_s8(void *) { hipLaunchKernelGGL(scatter<8>, grid_of(g.n), dim3(256), 0, 0, g.idx, g.n, (Rec<8> *)g.out); }
static void run_s16(void *) { hipLaunchKernelGGL(scatter<16>, grid_of(g.n), dim3(256), 0, 0, g.idx, g.n, (Rec<16> *)g.out); }
static void run_w8(void *) { hipLaunchKernelGGL(stream_write<8>, grid_of(g.n), dim3(256), 0, 0, g.n, (Rec<8> *)g.out); }
static void run_w16(void *) { hipLaunchKernelGGL(stream_write<16>, grid_of(g.n), dim3(256), 0, 0, g.n, (Rec<16> *)g.out); }
static void run_nt8(void *) { hipLaunchKernelGGL(scatter_nt8, grid_of(g.n), dim3(256), 0, 0, g.idx, g.n, (uint64_t *)g.out); }
static void run_s4(void *) { hipLaunchKernelGGL(scatter4, grid_of(g.n), dim3(256), 0, 0, g.idx, g.n, (uint32_t *)g.out); }
static void run_g4(void *) { hipLaunchKernelGGL(gather, grid_of(g.n), dim3(256), 0, 0, g.idx, g.n, g.src, g.sink); }

// Hash-indexed bucket directory probe: item i gathers dir[h(i) & mask]
// (its bucket's head, one random 4-byte load from a 2^T-entry table) and, with dep = 1,
// then a second load that depends on it (the first entry of that bucket's list, random in
// a list of the same size): the minimum a directory costs the pair counter per occurrence
// in place of the bucket build's scattered 8-byte record store.  Items are generated in
// the kernel (no index array), so the bytes moved are the gathers' alone.
__global__ void dir_gather(uint64_t n, const uint32_t *dir, uint32_t mask, int dep, uint32_t *sink) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t v = dir[hash32((uint32_t)i ^ (uint32_t)(i >> 32) * 0x9E3779B1u) & mask];
    if (dep) v = dir[(v * 2654435761u) & mask];
    if (v == 0xDEADBEEFu) sink[0] = v;
}

int main(int argc, char **argv) {
    // argv[1] = "big N": only the 8-byte scatter section at N items (round 3:
    // does the per-store cost grow with the target array -- TLB reach -- at
    // configs[3]'s per-GPU slice, N = 607.5M, 4.86 GB?)
    // argv[1] = "stage N IPB WSHIFT NSHARD": direct vs staged scatter of N random
    // targets (a permutation-like map into N 8-byte slots)
    if (argc > 5 && argv[1][0] == 's' && argv[1][1] == 't') {
        const uint64_t n = strtoull(argv[2], nullptr, 10);
        const uint32_t ipb = (uint32_t)strtoul(argv[3], nullptr, 10);
        const int wshift = atoi(argv[4]);
        const uint32_t ns = (uint32_t)strtoul(argv[5], nullptr, 10);
        const uint32_t nbins = (uint32_t)((n + (1ull << wshift) - 1) >> wshift);
        const uint64_t per = ((1ull << wshift) + ns - 1) / ns;
        const uint64_t cap = per + per / 50 + 1024;
        uint32_t *idx, *sg;
        uint64_t *out, *sv;
        unsigned long long *cur;
        CHK(hipMalloc(&idx, n * 4));
        CHK(hipMalloc(&out, n * 8));
        CHK(hipMalloc(&sg, (size_t)nbins * ns * cap * 4));
        CHK(hipMalloc(&sv, (size_t)nbins * ns * cap * 8));
        CHK(hipMalloc(&cur, (size_t)nbins * ns * 8));
        hipLaunchKernelGGL(make_idx, grid_of(n), dim3(256), 0, 0, idx, n, n, 0u);
        g.idx = idx; g.n = n; g.out = out;
        const float d = time_it(run_s8, 0, 3);
        hipEvent_t a, b, c;
        CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b)); CHK(hipEventCreate(&c));
        const uint32_t nblk = (uint32_t)((n + ipb - 1) / ipb);
        const uint32_t nreg = nbins * ns;
        const uint32_t sgrid = (uint32_t)(nreg * ((cap + 1023) / 1024));
        float t1 = 0, t2 = 0;
        for (int rep = 0; rep < 4; ++rep) {
            CHK(hipMemset(cur, 0, (size_t)nreg * 8));
            CHK(hipEventRecord(a));
            hipLaunchKernelGGL(stage_kernel, dim3(nblk), dim3(256), 0, 0, idx, n, ipb, wshift, nbins, ns, cap, cur, sg, sv,
                               out);
            CHK(hipEventRecord(b));
            hipLaunchKernelGGL(stage_scatter, dim3(sgrid), dim3(256), 0, 0, cur, nreg, cap, sg, sv, out);
            CHK(hipEventRecord(c));
            CHK(hipEventSynchronize(c));
            float x, y;
            CHK(hipEventElapsedTime(&x, a, b));
            CHK(hipEventElapsedTime(&y, b, c));
            if (rep) { t1 += x; t2 += y; }
        }
        printf("n=%llu direct %.3f ms | staged (ipb %u, bins %u x %u shards, %.0f MB each): stage %.3f + scatter %.3f = %.3f ms\n",
               (unsigned long long)n, d, ipb, nbins, ns, 8.0 * (1ull << wshift) / 1e6, t1 / 3, t2 / 3, (t1 + t2) / 3);
        return 0;
    }
    // argv[1] = "dir N T": N directory gathers from a 2^T-entry (4 * 2^T bytes) table,
    // one load and two dependent loads per item
    if (argc > 3 && argv[1][0] == 'd') {
        const uint64_t n = strtoull(argv[2], nullptr, 10);
        const int T = atoi(argv[3]);
        uint32_t *dir, *sink;
        CHK(hipMalloc(&dir, (4ull << T)));
        CHK(hipMalloc(&sink, 64));
        hipLaunchKernelGGL(make_idx, grid_of(1ull << T), dim3(256), 0, 0, dir, 1ull << T, 1ull << T, 0u);
        for (int dep = 0; dep < 2; ++dep) {
            hipEvent_t a, b;
            CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
            hipLaunchKernelGGL(dir_gather, grid_of(n), dim3(256), 0, 0, n, dir, (uint32_t)((1ull << T) - 1), dep, sink);
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(a));
            for (int r = 0; r < 3; ++r)
                hipLaunchKernelGGL(dir_gather, grid_of(n), dim3(256), 0, 0, n, dir, (uint32_t)((1ull << T) - 1), dep, sink);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, a, b));
            ms /= 3;
            printf("dir n=%llu table 2^%d (%.0f MB): %d load(s) per item %.3f ms (%.3f ms per 48.6M, %.1f G items/s)\n",
                   (unsigned long long)n, T, 4.0 * (1ull << T) / 1e6, dep + 1, ms, ms * 48.6e6 / n, n / (ms * 1e-3) / 1e9);
        }
        CHK(hipFree(dir)); CHK(hipFree(sink));
        return 0;
    }
    // argv[1] = "atom NBLOCKS NBINS NSHARD"
    if (argc > 4 && argv[1][0] == 'a') {
        const uint32_t nb = (uint32_t)strtoul(argv[2], nullptr, 10), nbins = (uint32_t)strtoul(argv[3], nullptr, 10),
                       ns = (uint32_t)strtoul(argv[4], nullptr, 10);
        unsigned long long *cur;
        uint32_t *sink;
        CHK(hipMalloc(&cur, (size_t)nbins * ns * 8));
        CHK(hipMalloc(&sink, 64));
        CHK(hipMemset(cur, 0, (size_t)nbins * ns * 8));
        hipEvent_t a, b;
        CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
        hipLaunchKernelGGL(claim_kernel, dim3(nb), dim3(256), 0, 0, cur, nbins, ns, sink);
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(a));
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(claim_kernel, dim3(nb), dim3(256), 0, 0, cur, nbins, ns, sink);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        printf("claims: %u blocks x %u bins over %u shards: %.3f ms\n", nb, nbins, ns, ms / 3);
        return 0;
    }
    // argv[1] = "span N SPAN_MB ALLOC_MB": N random 8-byte stores into the first
    // SPAN_MB of an ALLOC_MB array (does the cost follow the items, the span
    // they land in, or the allocation?)
    if (argc > 4 && argv[1][0] == 's') {
        const uint64_t n = strtoull(argv[2], nullptr, 10);
        const uint64_t span = strtoull(argv[3], nullptr, 10) * 1000000ull / 8;
        const uint64_t alloc = strtoull(argv[4], nullptr, 10) * 1000000ull;
        uint32_t *idx, *sink;
        void *out;
        CHK(hipMalloc(&idx, n * 4));
        CHK(hipMalloc(&out, alloc));
        CHK(hipMalloc(&sink, 64));
        CHK(hipMemset(out, 0, alloc));
        g.idx = idx; g.n = n; g.out = out; g.sink = sink; g.src = (const uint32_t *)out;
        hipLaunchKernelGGL(make_idx, grid_of(n), dim3(256), 0, 0, idx, n, span, 0u);
        const float s = time_it(run_s8, 0, 3);
        printf("n=%llu span %.0f MB alloc %.0f MB: %.3f ms (%.3f ms per 48.6M)\n", (unsigned long long)n,
               8.0 * span / 1e6, alloc / 1e6, s, s * 48.6e6 / n);
        const float s2 = time_it(run_nt8, 0, 3);
        printf("   non-temporal 8B: %.3f ms (%.3f ms per 48.6M)\n", s2, s2 * 48.6e6 / n);
        // the same slots as 4-byte words (a 4-byte record array of the same count: half the span)
        const float s3 = time_it(run_s4, 0, 3);
        printf("   4B words over %.0f MB: %.3f ms (%.3f ms per 48.6M)\n", 4.0 * span / 1e6, s3, s3 * 48.6e6 / n);
        CHK(hipFree(idx)); CHK(hipFree(out)); CHK(hipFree(sink));
        return 0;
    }
    if (argc > 2 && argv[1][0] == 'b') {
        const uint64_t n = strtoull(argv[2], nullptr, 10);
        uint32_t *idx, *sink;
        void *out;
        CHK(hipMalloc(&idx, n * 4));
        CHK(hipMalloc(&out, 8 * n));
        CHK(hipMalloc(&sink, 64));
        CHK(hipMemset(out, 0, 8 * n));
        g.idx = idx; g.n = n; g.out = out; g.sink = sink; g.src = (const uint32_t *)out;
        const float w = time_it(run_w8, 0, 3);
        printf("n=%llu coalesced write 8B: %.3f ms (%.2f ns/item x1000)\n", (unsigned long long)n, w, w * 1e3 / (n / 1e6));
        hipLaunchKernelGGL(make_idx, grid_of(n), dim3(256), 0, 0, idx, n, n, 0u);
        const float s = time_it(run_s8, 0, 3);
        printf("scatter 8B over %.0f MB: %.3f ms (%.3f ms per 48.6M)\n", 8.0 * n / 1e6, s, s * 48.6e6 / n);
        for (uint64_t win_mb : {2ull, 32ull, 256ull, 1024ull}) {
            const uint32_t ws = (uint32_t)(win_mb * 1000000ull / 8);
            if (ws >= n) continue;
            hipLaunchKernelGGL(make_idx, grid_of(n), dim3(256), 0, 0, idx, n, n, ws);
            const float t = time_it(run_s8, 0, 3);
            printf("  windowed %4llu MB: %.3f ms (%.3f ms per 48.6M)\n", (unsigned long long)win_mb, t, t * 48.6e6 / n);
        }
        CHK(hipFree(idx)); CHK(hipFree(out)); CHK(hipFree(sink));
        return 0;
    }
    const uint64_t n = 48600000ull;  // k-mer occurrences at the bench shape
    uint32_t *idx, *sink;
    void *out;
    const size_t max_bytes = 16 * n;  // 778 MB
    CHK(hipMalloc(&idx, n * 4));
    CHK(hipMalloc(&out, max_bytes));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(out, 0, max_bytes));
    g.idx = idx; g.n = n; g.out = out; g.sink = sink; g.src = (const uint32_t *)out;
    printf("coalesced write: 8B %.3f ms, 16B %.3f ms\n", time_it(run_w8, 0, 5), time_it(run_w16, 0, 5));
    // full-range random scatter (the round-1 record store) and windowed variants
    for (int B : {16}) {
        const uint64_t slots = n;  // one slot per item, target array = B * n
        hipLaunchKernelGGL(make_idx, grid_of(n), dim3(256), 0, 0, idx, n, slots, 0u);
        const float full = time_it(B == 8 ? run_s8 : run_s16, 0, 5);
        printf("scatter %dB over %.0f MB: %.3f ms\n", B, B * (double)slots / 1e6, full);
        for (uint64_t win_mb : {2ull, 32ull, 128ull}) {
            const uint32_t ws = (uint32_t)(win_mb * 1000000ull / B);
            if (ws >= slots) continue;
            hipLaunchKernelGGL(make_idx, grid_of(n), dim3(256), 0, 0, idx, n, slots, ws);
            printf("  windowed %3llu MB: %.3f ms\n", (unsigned long long)win_mb,
                   time_it(B == 8 ? run_s8 : run_s16, 0, 5));
        }
    }
    // random 4-byte gathers over working sets of various sizes
    for (uint64_t ws_mb : {4ull, 16ull, 64ull, 200ull, 700ull}) {
        const uint64_t slots = ws_mb * 1000000ull / 4;
        hipLaunchKernelGGL(make_idx, grid_of(n), dim3(256), 0, 0, idx, n, slots, 0u);
        const float t = time_it(run_g4, 0, 5);
        printf("gather 4B, %3llu MB working set: %.3f ms (%.1f G loads/s)\n", (unsigned long long)ws_mb, t,
               n / (t * 1e-3) / 1e9);
    }
    CHK(hipFree(idx)); CHK(hipFree(out)); CHK(hipFree(sink));
    return 0;
}
