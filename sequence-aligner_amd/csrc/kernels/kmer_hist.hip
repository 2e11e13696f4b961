// kmer_hist.hip -- k-mer table statistics for the diagnostic modes (gfx950).
//
// KmerTable.uniqueKmers / kmerCollisionHistogram (KmerTable.scala:189-221),
// printed by `--test-kmer-cover` (Project4.scala:299-320): the number of
// distinct k-mer hashes (KmerData.size) and, for every bucket size s, how many
// hashes have exactly s occurrences.  Input: the 8-byte k-mer records
// (mix32(seqHash) << 32 | g) fully sorted on their top 32 bits, so every bucket
// is one run.  One thread per record marks run heads; a scan numbers them; the
// head positions give the run lengths, which land in a size-indexed histogram
// (sizes >= KMER_HIST_CAP go to an overflow list the host folds in).  Bound:
// HBM (a few bytes per record), integer only.
#include "../sa_internal.h"

namespace sa {

__global__ void hist_heads_kernel(const uint64_t *sk, uint64_t n, uint32_t *flag) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    flag[s] = (s == 0 || (sk[s] >> 32) != (sk[s - 1] >> 32)) ? 1u : 0u;
}

__global__ void hist_positions_kernel(const uint32_t *flag, const uint32_t *idx, uint64_t n, uint32_t *pos) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    if (flag[s]) pos[idx[s]] = (uint32_t)s;
}

__global__ void hist_count_kernel(const uint32_t *pos, const uint32_t *nheads, uint64_t n,
                                  unsigned long long *hist, unsigned long long *ovf, uint32_t *novf) {
    const uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nh = *nheads;
    if (h >= nh) return;
    const uint64_t end = h + 1 < nh ? (uint64_t)pos[h + 1] : n;
    const uint64_t size = end - pos[h];
    if (size < KMER_HIST_CAP) atomicAdd(&hist[size], 1ull);
    else ovf[atomicAdd(novf, 1u)] = size;
}

hipError_t launch_kmer_hist(const uint64_t *sorted, uint64_t n, uint32_t *flag, uint32_t *idx, uint32_t *pos,
                            uint32_t *nheads, void *scan_tmp, unsigned long long *hist, unsigned long long *ovf,
                            uint32_t *novf, hipStream_t s) {
    hipError_t e = hipMemsetAsync(hist, 0, KMER_HIST_CAP * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(novf, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(nheads, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    const dim3 g((uint32_t)((n + 255) / 256));
    hipLaunchKernelGGL(hist_heads_kernel, g, dim3(256), 0, s, sorted, n, flag);
    if ((e = exclusive_scan_u32(flag, idx, n, nheads, scan_tmp, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(hist_positions_kernel, g, dim3(256), 0, s, flag, idx, n, pos);
    // one thread per head: at most n heads
    hipLaunchKernelGGL(hist_count_kernel, g, dim3(256), 0, s, pos, nheads, n, hist, ovf, novf);
    return hipGetLastError();
}

}  // namespace sa
