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
static void run_g4(void *) { hipLaunchKernelGGL(gather, grid_of(g.n), dim3(256), 0, 0, g.idx, g.n, g.src, g.sink); }

int main(int argc, char **argv) {
    // argv[1] = "big N": only the 8-byte scatter section at N items (round 3:
    // does the per-store cost grow with the target array -- TLB reach -- at
    // configs[3]'s per-GPU slice, N = 607.5M, 4.86 GB?)
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
