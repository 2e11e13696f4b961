// pack_emit.hip -- 2-bit read packing and per-read k-mer emission (gfx950).
//
// Replaces BioLibs.generateKmerSet (BioLibs.scala:54-61) + Kmer.seqHash
// (ObjectStore.scala:48-67).  One wavefront per read; lanes walk positions, so
// every k-mer record write is a coalesced 8-byte (key) + 4-byte (payload) store.
// Bound: HBM (integer byte work; no MFMA).
#include "../sa_internal.h"

namespace sa {

// 2-bit code of each byte of x (A0 C1 G2 T3 after folding to lower case) and a
// mask of the bytes that are not ACGT.  'a' 0x61, 'c' 0x63, 'g' 0x67, 't' 0x74.
__device__ __forceinline__ uint32_t codes4(uint32_t x, uint32_t &badm) {
    uint32_t code = 0;
    badm = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t ch = ((x >> (8 * b)) & 0xFFu) | 0x20u;
        const uint32_t c = ch == 'c' ? 1u : ch == 'g' ? 2u : ch == 't' ? 3u : 0u;
        const bool ok = c != 0u || ch == 'a';
        code |= c << (2 * b);
        badm |= ok ? 0u : (1u << b);
    }
    return code;  // byte b -> bits [2b, 2b+2)
}

// One wave per read, lane = one 16-base word.  A lane reads its 16 bytes as
// five aligned dwords (the ASCII buffer is padded) and funnel-shifts them into
// place: one coalesced kilobyte per wave-instruction instead of 16 byte loads.
__global__ __launch_bounds__(256) void pack_reads_kernel(DevReads r) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t rd = wave; rd < r.n; rd += nwaves) {
        const uint64_t b0 = r.boff[rd];
        const int32_t L = (int32_t)(r.boff[rd + 1] - b0);
        const uint64_t w0 = r.woff[rd];
        const int32_t nw = (L + 15) >> 4;
        int32_t first_bad = INT32_MAX;
        for (int32_t q = lane; q < nw; q += 64) {
            const int32_t p0 = q << 4;
            const uint64_t a = b0 + (uint64_t)p0;
            const uint32_t *wp = reinterpret_cast<const uint32_t *>(r.ascii + (a & ~3ull));
            const uint32_t sh = (uint32_t)(a & 3u);
            uint32_t d[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) d[j] = wp[j];
            const int32_t valid = min(16, L - p0);  // bytes of this word inside the read
            uint32_t word = 0, badm = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t x = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);  // bytes 4j .. 4j+3
                uint32_t bm;
                const uint32_t c = codes4(x, bm);
                // MSB-first: base t of the word at bits 30 - 2t
#pragma unroll
                for (int b = 0; b < 4; ++b) word |= ((c >> (2 * b)) & 3u) << (30 - 2 * (4 * j + b));
                badm |= bm << (4 * j);
            }
            const uint32_t vmask = valid >= 16 ? 0xFFFFu : ((1u << valid) - 1u);
            word &= valid >= 16 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (2 * valid));
            badm &= vmask;
            if (badm) first_bad = min(first_bad, p0 + (int32_t)__builtin_ctz(badm));
            r.codes[w0 + q] = word;
        }
        // wave-wide min of first_bad
        for (int off = 32; off > 0; off >>= 1) {
            const int32_t o = __shfl_xor(first_bad, off, 64);
            first_bad = o < first_bad ? o : first_bad;
        }
        if (lane == 0) r.bad[rd] = first_bad;
    }
}

// One wave per read, lane = position.  record = mix32(seqHash) << 32 | g.
__global__ __launch_bounds__(256) void kmer_emit_kernel(DevReads r, EmitParams e, uint64_t *keys,
                                                        uint32_t *vals) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const int shift = 32 - 2 * e.m;
    for (uint32_t rd = wave; rd < r.n; rd += nwaves) {
        const int32_t L = r.len[rd];
        const int32_t nk = L - e.k + 1;
        if (nk <= 0) {
            if (e.rkey && lane == 0) { e.rkey[rd] = 0xFFFFFFFFu; e.rord[rd] = rd; }
            continue;
        }
        const uint32_t *w = r.codes + r.woff[rd];
        const uint64_t g0 = e.occ_off[rd];
        const uint32_t *lr = e.occ_rl ? e.lrank + e.lbase[nk - 1] : nullptr;
        uint32_t kmin = 0xFFFFFFFFu;
        for (int32_t i = lane; i < nk; i += 64) {
            const uint32_t h = kmer_mix(w, i, shift);
            kmin = min(kmin, h);
            // 8-byte record: mixed hash | occurrence index, or read << pos_bits |
            // pos for mixed lengths (the loc rank is re-derived where it is
            // needed, partition.hip)
            const uint32_t occ = e.pos_bits ? (rd << e.pos_bits) | (uint32_t)i : (uint32_t)(g0 + i);
            keys[g0 + i] = ((uint64_t)h << 32) | (uint64_t)occ;
            if (e.occ_rl) e.occ_rl[g0 + i] = make_uint2(rd, lr[i]);
        }
        if (e.rkey) {
            // locality key: reads sharing their minimum k-mer overlap, so sorting
            // by it puts overlapping reads next to each other (pair_count order)
            for (int off = 32; off > 0; off >>= 1) kmin = min(kmin, (uint32_t)__shfl_xor(kmin, off, 64));
            if (lane == 0) { e.rkey[rd] = kmin; e.rord[rd] = rd; }
        }
    }
}

// Packing and emission in one pass for reads of <= 1,024 bases (<= 64 words)
// (keys == nullptr: packing, bad positions and locality keys only -- the
// partition sort then generates the records itself, radix_sort_gen):
// lane q packs word q as pack_reads_kernel does, keeps it in a register, and
// the k-mer windows are assembled from the wave's words with two lane shuffles
// -- no second launch, no reload of the packed words.  Records, locality keys
// and occurrence tables are exactly kmer_emit_kernel's.
__global__ __launch_bounds__(256) void pack_emit_kernel(DevReads r, EmitParams e, uint64_t *keys) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const int shift = 32 - 2 * e.m;
    for (uint32_t rd = wave; rd < r.n; rd += nwaves) {
        const uint64_t b0 = r.boff[rd];
        const int32_t L = (int32_t)(r.boff[rd + 1] - b0);
        const int32_t nw = (L + 15) >> 4;  // <= 64 (host-checked)
        int32_t first_bad = INT32_MAX;
        uint32_t word = 0;
        if ((int32_t)lane < nw) {
            const int32_t p0 = (int32_t)lane << 4;
            const uint64_t a = b0 + (uint64_t)p0;
            const uint32_t *wp = reinterpret_cast<const uint32_t *>(r.ascii + (a & ~3ull));
            const uint32_t sh = (uint32_t)(a & 3u);
            uint32_t d[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) d[j] = wp[j];
            const int32_t valid = min(16, L - p0);
            uint32_t badm = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t x = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
                uint32_t bm;
                const uint32_t c = codes4(x, bm);
#pragma unroll
                for (int b = 0; b < 4; ++b) word |= ((c >> (2 * b)) & 3u) << (30 - 2 * (4 * j + b));
                badm |= bm << (4 * j);
            }
            const uint32_t vmask = valid >= 16 ? 0xFFFFu : ((1u << valid) - 1u);
            word &= valid >= 16 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (2 * valid));
            badm &= vmask;
            if (badm) first_bad = p0 + (int32_t)__builtin_ctz(badm);
            r.codes[r.woff[rd] + lane] = word;
        }
        for (int off = 32; off > 0; off >>= 1) {
            const int32_t o = __shfl_xor(first_bad, off, 64);
            first_bad = o < first_bad ? o : first_bad;
        }
        if (lane == 0) r.bad[rd] = first_bad;
        // ---- emission (kmer_emit_kernel's records)
        const int32_t nk = L - e.k + 1;
        if (nk <= 0) {
            if (e.rkey && lane == 0) { e.rkey[rd] = 0xFFFFFFFFu; e.rord[rd] = rd; }
            continue;
        }
        const uint64_t g0 = e.npr ? (uint64_t)rd * e.npr : e.occ_off[rd];
        const uint32_t *lr = e.occ_rl ? e.lrank + e.lbase[nk - 1] : nullptr;
        uint32_t kmin = 0xFFFFFFFFu;
        for (int32_t i0 = 0; i0 < nk; i0 += 64) {  // wave-uniform trip count: every lane
            // takes part in the shuffles (a bpermute from an inactive lane reads nothing)
            const int32_t i = i0 + (int32_t)lane;
            // window16 from the wave's words: word i >> 4 and the next one (a
            // lane past the read's words only feeds bits the hash shifts out)
            const int q = (i >> 4) & 63, s2 = i & 15;
            const uint32_t wa = (uint32_t)__shfl((int)word, q, 64), wb = (uint32_t)__shfl((int)word, (q + 1) & 63, 64);
            if (i >= nk) continue;
            uint32_t x = s2 == 0 ? wa : ((wa << (2 * s2)) | (wb >> (32 - 2 * s2)));
            x = shift == 32 ? 0u : (x >> shift);
            x ^= (x >> 1) & 0x55555555u;
            const uint32_t h = mix32(x);
            kmin = min(kmin, h);
            const uint32_t occ = e.pos_bits ? (rd << e.pos_bits) | (uint32_t)i : (uint32_t)(g0 + i);
            if (keys) keys[g0 + i] = ((uint64_t)h << 32) | (uint64_t)occ;
            if (e.occ_rl) e.occ_rl[g0 + i] = make_uint2(rd, lr[i]);
        }
        if (e.rkey) {
            for (int off = 32; off > 0; off >>= 1) kmin = min(kmin, (uint32_t)__shfl_xor(kmin, off, 64));
            if (lane == 0) { e.rkey[rd] = kmin; e.rord[rd] = rd; }
        }
    }
}

// pack_emit_kernel's work for generated records (keys == nullptr) plus the first radix
// pass's tile histogram (radix_sort_gen's upsweep, which would generate every record once
// more): a block owns the records of TPB consecutive key-only tiles.  It packs every read
// overlapping them, writes words, bad position and locality key only for the reads whose
// first k-mer is its own (each read has exactly one such block), and counts its own k-mers'
// digits in LDS: hist[t * 256 + d], no global atomics.  Uniform lengths (npr k-mers per read).
// (NW waves per block, TPB tiles per block; same box at the bench shape, emit ms: one tile
// over 4 waves 0.122, over 8 waves 0.124, over 16 waves 0.135, 4 tiles over 4 waves 0.146 --
// profiles/r05/ab/ab_hist_in_pack.txt)
template <int T, int TPB, int NW>
__global__ __launch_bounds__(NW * 64) void pack_emit_hist_kernel(DevReads r, EmitParams e, uint64_t n) {
    __shared__ uint32_t cnt[TPB][256];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (uint32_t q = tid; q < TPB * 256; q += NW * 64) (&cnt[0][0])[q] = 0;
    __syncthreads();
    const int shift = 32 - 2 * e.m;
    const int dsh = e.hist_shift - 32;  // the digit in the hash word (hist_shift >= 32)
    const uint64_t t0 = (uint64_t)blockIdx.x * TPB * T, t1 = min(t0 + (uint64_t)TPB * T, n);
    const uint32_t npr = e.npr;
    const uint32_t r0 = (uint32_t)(t0 / npr), r1 = (uint32_t)((t1 - 1) / npr);
    for (uint32_t rd = r0 + w; rd <= r1; rd += NW) {
        const uint64_t b0 = r.boff[rd];
        const int32_t L = (int32_t)(r.boff[rd + 1] - b0);
        const int32_t nw = (L + 15) >> 4;  // <= 64 (host-checked)
        const uint64_t g0 = (uint64_t)rd * npr;
        const bool own = g0 >= t0;  // the read's first k-mer is in this tile
        int32_t first_bad = INT32_MAX;
        uint32_t word = 0;
        if ((int32_t)lane < nw) {
            const int32_t p0 = (int32_t)lane << 4;
            const uint64_t a = b0 + (uint64_t)p0;
            const uint32_t *wp = reinterpret_cast<const uint32_t *>(r.ascii + (a & ~3ull));
            const uint32_t sh = (uint32_t)(a & 3u);
            uint32_t d[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) d[j] = wp[j];
            const int32_t valid = min(16, L - p0);
            uint32_t badm = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t x = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
                uint32_t bm;
                const uint32_t c = codes4(x, bm);
#pragma unroll
                for (int b = 0; b < 4; ++b) word |= ((c >> (2 * b)) & 3u) << (30 - 2 * (4 * j + b));
                badm |= bm << (4 * j);
            }
            const uint32_t vmask = valid >= 16 ? 0xFFFFu : ((1u << valid) - 1u);
            word &= valid >= 16 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (2 * valid));
            badm &= vmask;
            if (badm) first_bad = p0 + (int32_t)__builtin_ctz(badm);
            if (own) r.codes[r.woff[rd] + lane] = word;
        }
        if (own) {
            for (int off = 32; off > 0; off >>= 1) {
                const int32_t o = __shfl_xor(first_bad, off, 64);
                first_bad = o < first_bad ? o : first_bad;
            }
            if (lane == 0) r.bad[rd] = first_bad;
        }
        // own reads: every k-mer (locality key); the others: only this tile's k-mers
        const int32_t nk = (int32_t)npr;
        const int32_t lo_i = own ? 0 : (int32_t)(t0 - g0);
        const int32_t hi_i = (int32_t)min<uint64_t>((uint64_t)nk, own ? (uint64_t)nk : t1 - g0);
        uint32_t kmin = 0xFFFFFFFFu;
        for (int32_t i0 = lo_i & ~63; i0 < hi_i; i0 += 64) {  // wave-uniform trip count (shuffles)
            const int32_t i = i0 + (int32_t)lane;
            const int q = (i >> 4) & 63, s2 = i & 15;
            const uint32_t wa = (uint32_t)__shfl((int)word, q, 64), wb = (uint32_t)__shfl((int)word, (q + 1) & 63, 64);
            if (i < lo_i || i >= hi_i) continue;
            uint32_t x = s2 == 0 ? wa : ((wa << (2 * s2)) | (wb >> (32 - 2 * s2)));
            x = shift == 32 ? 0u : (x >> shift);
            x ^= (x >> 1) & 0x55555555u;
            const uint32_t h = mix32(x);
            kmin = min(kmin, h);
            const uint64_t g = g0 + (uint64_t)i;
            if (g >= t0 && g < t1) atomicAdd(&cnt[(uint32_t)((g - t0) / T)][(h >> dsh) & 255u], 1u);
        }
        if (own && e.rkey) {
            for (int off = 32; off > 0; off >>= 1) kmin = min(kmin, (uint32_t)__shfl_xor(kmin, off, 64));
            if (lane == 0) { e.rkey[rd] = kmin; e.rord[rd] = rd; }
        }
    }
    __syncthreads();
    const uint64_t tiles = (n + T - 1) / T;
    for (uint32_t q = tid >> 8; q < TPB; q += NW / 4) {  // (NW a multiple of 4: 256 threads per row)
        const uint64_t t = (uint64_t)blockIdx.x * TPB + q;
        if (t < tiles) e.hist[t * 256 + (tid & 255)] = cnt[q][tid & 255];
    }
}

static uint32_t grid_for_waves(uint64_t waves) {
    uint64_t blocks = (waves + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    return (uint32_t)(blocks ? blocks : 1);
}

hipError_t launch_pack_reads(const DevReads &r, hipStream_t s) {
    if (r.n == 0) return hipSuccess;
    hipLaunchKernelGGL(pack_reads_kernel, dim3(grid_for_waves(r.n)), dim3(256), 0, s, r);
    return hipGetLastError();
}

hipError_t launch_kmer_emit(const DevReads &r, const EmitParams &p, uint64_t *keys, uint32_t *vals,
                            hipStream_t s) {
    if (r.n == 0) return hipSuccess;
    hipLaunchKernelGGL(kmer_emit_kernel, dim3(grid_for_waves(r.n)), dim3(256), 0, s, r, p, keys, vals);
    return hipGetLastError();
}

#ifndef SA_PEH_TPB  // (A/B builds)
#define SA_PEH_TPB 1
#endif
#ifndef SA_PEH_NW
#define SA_PEH_NW 4
#endif
hipError_t launch_pack_emit_hist(const DevReads &r, const EmitParams &p, uint64_t n, hipStream_t s) {
    constexpr uint32_t T = 8192;  // = radix_key_tile() (sort_scan.hip; checked by the caller)
    if (r.n == 0 || n == 0) return hipSuccess;
    if (!p.npr || !p.hist || p.hist_shift < 32 || radix_key_tile() != T) return hipErrorInvalidValue;
    constexpr int TPB = SA_PEH_TPB, NW = SA_PEH_NW;
    hipLaunchKernelGGL((pack_emit_hist_kernel<T, TPB, NW>),
                       dim3((uint32_t)((n + (uint64_t)TPB * T - 1) / ((uint64_t)TPB * T))), dim3(NW * 64), 0, s, r, p, n);
    return hipGetLastError();
}

hipError_t launch_pack_emit(const DevReads &r, const EmitParams &p, uint64_t *keys, hipStream_t s) {
    if (r.n == 0) return hipSuccess;
    hipLaunchKernelGGL(pack_emit_kernel, dim3(grid_for_waves(r.n)), dim3(256), 0, s, r, p, keys);
    return hipGetLastError();
}

}  // namespace sa
