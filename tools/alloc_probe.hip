// alloc_probe.hip -- does the cost of the bucket build's random 8-byte record
// scatter depend on where its 389 MB array lands?  Allocates K arrays one after
// another (all kept; default or contiguous flag) and times, for each, 48.6M
// random 8-byte stores (the bench shape), 5 repetitions.  Standalone; not part
// of the library.  Build: hipcc -O3 --offload-arch=gfx950 -o alloc_probe alloc_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__global__ void scatter8(uint64_t *out, uint32_t n, uint32_t salt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = hash32(i ^ salt) % n;
    out[t] = ((uint64_t)i << 32) | t;
}

int main(int argc, char **argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 6;
    const unsigned flags = argc > 2 ? (unsigned)atoi(argv[2]) : 0u;
    const uint32_t n = 48600000u;
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    for (int k = 0; k < K; ++k) {
        uint64_t *out;
        if (flags) CHK(hipExtMallocWithFlags((void **)&out, (size_t)n * 8, flags));
        else CHK(hipMalloc(&out, (size_t)n * 8));
        CHK(hipMemset(out, 0, (size_t)n * 8));
        scatter8<<<(n + 255) / 256, 256>>>(out, n, 12345u);  // warm (page tables)
        CHK(hipDeviceSynchronize());
        float best = 1e9f, sum = 0.f;
        for (int r = 0; r < 5; ++r) {
            CHK(hipEventRecord(a));
            scatter8<<<(n + 255) / 256, 256>>>(out, n, 777u * (r + 1));
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf("array %d at %p flags %u: random 8-B scatter best %.3f ms mean %.3f ms\n", k, (void *)out, flags, best,
               sum / 5);
        fflush(stdout);
    }
    return 0;
}
