// local_align.hip -- batched full-matrix affine local alignment (gfx950): the
// `--quadratic-align` aligner, BioLibs.generateLocalAlignmentSet
// (BioLibs.scala:267-368) for every dispatched (lead A, trail B) pair, with the
// Alignment / Overlap validity of ObjectStore.scala:99-141.
//
// Mapping (local_dp_kernel): one wavefront per pair; lane l owns the S columns
// j = l*S+1 .. l*S+S of B and keeps their previous-row state in registers.  The
// lanes sweep the matrix as a skewed wavefront: at step t lane l computes row
// i = t - l + 1 of its columns, so the row's left neighbour (lane l-1) finished
// the same row one step earlier and hands its right-edge state over with one
// DPP wave_shr:1 per value.  |A| + ceil(|B|/S) - 1 steps per pair; integer
// max-plus VALU only (MFMA has no use here).  Per cell:
//   M = c(A[i-1], B[j-1]) + max(T(i-1, j-1), 0)
//   X = gE + max(max(M, Y)(i, j-1) + gO, X(i, j-1), 0)
//   Y = gE + max(max(M, X)(i-1, j) + gO, Y(i-1, j), 0)
// (BioLibs.scala:303-316, the bracketed maxima regrouped; boundary cells never
// win against the inner 0 for gap costs <= 0, so they enter as zeros).  Each
// cell leaves a 2-bit code for the greedy backtrack (:334-360): 0 when
// max(M, X, Y) <= 0 (the walk stops there), else 1 / 2 / 3 for the first of
// M / X / Y equal to the cell max.  A lane appends its codes step after step
// to its own stream in HBM (2S bits per step), in whole 64-byte segments.  The argmax is the first strict '>'
// in row-major order (:318-321): per-lane first best, then a (value desc,
// i asc, j asc) reduce across the wave.
//
// local_walk_kernel: one lane per pair replays the greedy walk from the argmax
// over the stored codes, counting matches (A[i-1] == B[j-1] on M steps) and
// errors (every other step), and writes the Alignment record.
#include "../sa_internal.h"

namespace sa {

namespace {

__device__ __forceinline__ void set_err(int32_t *err, int32_t code) { atomicCAS(err, 0, code); }

// wave-uniform value held in a VGPR: a VALU op with an SGPR operand issues at
// half rate on gfx950 (tools/valu_rate.hip)
__device__ __forceinline__ int32_t in_vgpr(int32_t x) {
    int32_t r;
    asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
}

__device__ __forceinline__ uint32_t gld(const uint32_t *p, int64_t i) {
    return ((const __attribute__((address_space(1))) uint32_t *)p)[i];
}

// lane l <- lane l-1 (DPP wave_shr:1, GFX9 family); lane 0 gets 0 (column 0)
__device__ __forceinline__ int32_t from_left(int32_t v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t base_at(const uint32_t *w, int32_t p) {
    return (gld(w, p >> 4) >> (30 - 2 * (p & 15))) & 3u;
}

}  // namespace

template <int S, class C>
__global__ __launch_bounds__(256) void local_dp_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                       uint64_t p0, uint64_t np, AlignParams P, uint32_t wpl,
                                                       uint32_t *tb, int4 *lmax, int32_t *err,
                                                       unsigned long long *cells_total) {
    constexpr int BPS = 2 * S;                    // code bits per lane-row
    constexpr int K = BPS >= 32 ? 1 : 32 / BPS;   // rows per code word (S < 16)
    constexpr int NW = S >= 16 ? S / 16 : 1;      // code words per row (S >= 16)
    const int lane = threadIdx.x & 63;
    const uint64_t q = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    unsigned long long my_cells = 0;
    if (q < np) {  // wave-uniform
        const uint64_t pair = p0 + q;
        const int32_t a = lead[pair] - 1, b = trail[pair] - 1;
        const int32_t LA = rd.len[a], LB = rd.len[b];
        int32_t status = 0;
        if (LB > 64 * S || LA >= (1 << 20) || (uint64_t)(LA + 63) * BPS > (uint64_t)wpl * 32) status = -11;
        else if (rd.bad[a] < LA || rd.bad[b] < LB) status = -3;  // every cell calls the cost closure
        if (status != 0) {
            if (lane == 0) {
                set_err(err, status);
                lmax[q] = make_int4(0, 0, 0, status);
            }
        } else {
            const uint32_t *Aw = rd.codes + rd.woff[a];
            const uint32_t *Bw = rd.codes + rd.woff[b];
            const int32_t gO = in_vgpr(P.gap_open), gE = in_vgpr(P.gap_extend);
            const int32_t nl = (LB + S - 1) / S;
            // cost packs of my columns: entry x = cost(x, B[j-1]); columns past |B|
            // get 0 (they can then never raise the lane's running best)
            C cb[S];
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int32_t pos = lane * S + s;
                cb[s] = C::make(0, 0, 0, 0);
                if (pos < LB) {
                    const uint32_t bc = base_at(Bw, pos);
                    cb[s] = C::make(P.cost[0 * 4 + bc], P.cost[1 * 4 + bc], P.cost[2 * 4 + bc], P.cost[3 * 4 + bc]);
                }
            }
            int32_t Pv[S], Qv[S];  // previous row: max(T, 0), max(max(M, X) + gO, Y, 0)
#pragma unroll
            for (int s = 0; s < S; ++s) { Pv[s] = 0; Qv[s] = 0; }
            int32_t Rout = 0, Pout = 0, Pl = 0;  // right edge of my last row; P(i-1, j0-1) from the left lane
            int32_t best = 0, bi = 0, bs = 0;
            // My code stream is indexed by step t (row t - lane + 1; idle steps
            // hold zeros) and leaves in whole, aligned 64-byte segments: 16 words
            // gathered in registers (uniform slot index -> scalar branches), then
            // four 16-byte stores, so no partially written line reaches HBM.
            uint32_t acc = 0, sb[16];
#pragma unroll
            for (int w = 0; w < 16; ++w) sb[w] = 0;
            int32_t widx = 0;
            uint4 *tl = reinterpret_cast<uint4 *>(tb + (q * 64 + (uint64_t)lane) * wpl);
            const bool mine = lane < nl;
            const int32_t steps = LA + nl - 1;
            // A words: aw holds A[i-1] of the current row, an the next word
            uint32_t aw = gld(Aw, 0), an = LA > 16 ? gld(Aw, 1) : 0u;
            for (int32_t t = 0; t < steps; ++t) {
                const int32_t Rin = from_left(Rout);
                const int32_t Pin = from_left(Pout);
                const int32_t i = t - lane + 1;
                uint32_t bits[NW];
#pragma unroll
                for (int w = 0; w < NW; ++w) bits[w] = 0;
                if (mine && i >= 1 && i <= LA) {
                    const uint32_t a8 = ((aw >> (30 - 2 * ((i - 1) & 15))) & 3u) * 8u;
                    int32_t Pd = Pl;
                    int32_t R = Rin;
                    int32_t rk = INT32_MIN;  // row argmax key (T << 5 | 31 - s)
#pragma unroll
                    for (int s = 0; s < S; ++s) {
                        const int32_t c = cb[s].at(a8);
                        const int32_t M = c + Pd;
                        const int32_t Y = gE + Qv[s];
                        const int32_t X = gE + R;
                        const int32_t MY = max(M, Y);
                        const int32_t MX = max(M, X);
                        const int32_t T = max(MY, X);
                        R = max(max(MY + gO, X), 0);
                        Pd = Pv[s];
                        Pv[s] = max(T, 0);
                        Qv[s] = max(max(MX + gO, Y), 0);
                        const uint32_t code = T <= 0 ? 0u : (M == T ? 1u : (X == T ? 2u : 3u));
                        // shift-in (inline-constant codes, no shifted literals):
                        // column s of a word ends at bits 2 * (15 - (s & 15)) (S >= 16)
                        // or 2 * (S - 1 - s) (S < 16)
                        bits[s >> 4] = (bits[s >> 4] << 2) | code;
                        rk = max(rk, (T << 5) | (31 - s));  // row max, first column among ties
                    }
                    // first strict '>' in row-major order: a later row must beat the best
                    if ((rk >> 5) > best) { best = rk >> 5; bi = i; bs = 31 - (rk & 31); }
                    Rout = R;
                    Pout = Pv[S - 1];
                    if ((i & 15) == 0 && i < LA) {  // next row starts a new A word
                        aw = an;
                        if (((i >> 4) + 1) * 16 < LA) an = gld(Aw, (i >> 4) + 1);
                    }
                }
                Pl = Pin;
                // this step's codes into the segment buffer (t is wave-uniform)
                auto put = [&](uint32_t v) {
                    switch (__builtin_amdgcn_readfirstlane(widx)) {  // uniform: scalar branches
#define SA_PUT(W) case W: sb[W] = v; break;
                    SA_PUT(0) SA_PUT(1) SA_PUT(2) SA_PUT(3) SA_PUT(4) SA_PUT(5) SA_PUT(6) SA_PUT(7)
                    SA_PUT(8) SA_PUT(9) SA_PUT(10) SA_PUT(11) SA_PUT(12) SA_PUT(13) SA_PUT(14) SA_PUT(15)
#undef SA_PUT
                    }
                    ++widx;
                };
                if constexpr (S >= 16) {
#pragma unroll
                    for (int w = 0; w < NW; ++w) put(bits[w]);
                } else {
                    acc |= bits[0] << ((t % K) * BPS);
                    if (t % K == K - 1 || t == steps - 1) { put(acc); acc = 0; }
                }
                if (widx == 16 || t == steps - 1) {
                    const int32_t seg = (t * NW / K) >> 4;  // 16-word segment of this step's last word
                    tl[4 * seg + 0] = make_uint4(sb[0], sb[1], sb[2], sb[3]);
                    tl[4 * seg + 1] = make_uint4(sb[4], sb[5], sb[6], sb[7]);
                    tl[4 * seg + 2] = make_uint4(sb[8], sb[9], sb[10], sb[11]);
                    tl[4 * seg + 3] = make_uint4(sb[12], sb[13], sb[14], sb[15]);
                    widx = 0;
                }
            }
            my_cells = lane == 0 ? (unsigned long long)LA * LB : 0ull;
            // first row-major argmax: value desc, i asc, j asc
            const int32_t jj = lane * S + bs + 1;
            unsigned long long key = (mine && best > 0)
                ? (((unsigned long long)(uint32_t)best << 32) | ((unsigned long long)(0xFFFFFu - (uint32_t)bi) << 12) |
                   (unsigned long long)(0xFFFu - (uint32_t)jj))
                : 0ull;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const unsigned long long o = __shfl_xor(key, off, 64);
                key = o > key ? o : key;
            }
            if (lane == 0) {
                const int32_t vb = (int32_t)(key >> 32);
                if (vb <= 0) {  // the reference's backtrack reads A.charAt(-1)
                    set_err(err, -6);
                    lmax[q] = make_int4(0, 0, 0, -6);
                } else {
                    const int32_t mi = (int32_t)(0xFFFFFu - ((key >> 12) & 0xFFFFFu));
                    const int32_t mj = (int32_t)(0xFFFu - (key & 0xFFFu));
                    lmax[q] = make_int4(vb, mi, mj, 0);
                }
            }
        }
    }
    // DP cells for statistics: block-reduced, one sharded atomic per block
    __shared__ unsigned long long cell_sum;
    if (threadIdx.x == 0) cell_sum = 0;
    __syncthreads();
    if (my_cells) atomicAdd(&cell_sum, my_cells);
    __syncthreads();
    if (threadIdx.x == 0 && cell_sum) atomicAdd(&cells_total[blockIdx.x % NSHARD], cell_sum);
}

template <int S>
__global__ __launch_bounds__(256) void local_walk_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                         uint64_t p0, uint64_t np, AlignParams P, uint32_t wpl,
                                                         const uint32_t *tb, const int4 *lmax, DevAlignment *out) {
    constexpr int BPS = 2 * S;
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= np) return;
    const uint64_t pair = p0 + q;
    const int32_t a = lead[pair] - 1, b = trail[pair] - 1;
    const int4 mx = lmax[q];
    DevAlignment o;
    o.lead = a + 1;
    o.trail = b + 1;
    o.reserved = 0;
    if (mx.w != 0) {  // error (the call fails with it)
        o.start_i = o.start_j = o.end_i = o.end_j = 0;
        o.correct = o.error = o.ahg = o.bhg = 0;
        o.flags = 0x100;
        out[pair] = o;
        return;
    }
    const int32_t LA = rd.len[a], LB = rd.len[b];
    const uint32_t *Aw = rd.codes + rd.woff[a];
    const uint32_t *Bw = rd.codes + rd.woff[b];
    const uint32_t *tq = tb + q * 64 * (uint64_t)wpl;
    auto code_at = [&](int32_t i, int32_t j) -> uint32_t {
        const int32_t l = (j - 1) / S, s = (j - 1) - l * S;
        // step t = row - 1 + lane; column s sits at 2 * (last - s) within its word
        const int32_t sp = S >= 16 ? (s & ~15) + (15 - (s & 15)) : (S - 1 - s);
        const uint64_t bit = (uint64_t)(i - 1 + l) * BPS + 2 * sp;
        return (gld(tq, (int64_t)l * wpl + (int64_t)(bit >> 5)) >> (bit & 31)) & 3u;
    };
    int32_t i = mx.y, j = mx.z, c = 0, e = 0;
    uint32_t code = code_at(i, j);  // != 0: the argmax cell is positive
    int32_t awi = -1, bwi = -1;
    uint32_t aw = 0, bw = 0;
    while (true) {
        if (code == 1) {
            const int32_t pa = i - 1, pb = j - 1;
            if ((pa >> 4) != awi) { awi = pa >> 4; aw = gld(Aw, awi); }
            if ((pb >> 4) != bwi) { bwi = pb >> 4; bw = gld(Bw, bwi); }
            const uint32_t ca = (aw >> (30 - 2 * (pa & 15))) & 3u, cbb = (bw >> (30 - 2 * (pb & 15))) & 3u;
            if (ca == cbb) ++c; else ++e;
            --i; --j;
        } else if (code == 2) { ++e; --j; }   // A[i-1] against '-'
        else { ++e; --i; }                     // '-' against B[j-1]
        if (i == 0 || j == 0) break;           // boundary row / column: cell max 0
        code = code_at(i, j);
        if (code == 0) break;
    }
    // Alignment(seqA, seqB, xSeq, ySeq, (i, j), opt, c, e) (:364) + validity
    const int32_t si = i, sj = j, ei = mx.y, ej = mx.z, alen = c + e;
    const float ratio = __fdiv_rn((float)c, (float)c + (float)e);
    const bool valid = (ratio >= P.min_identity) && (alen >= P.min_overlap) &&
                       ((si == 0 && LB == ej) || (sj == 0 && LA == ei));
    const int32_t ahg = si - sj;
    const int32_t bhg = LB - LA + ahg;
    const bool ovl = valid && ((float)abs(ahg) < P.max_ignore) && ((float)abs(bhg) < P.max_ignore);
    o.start_i = si; o.start_j = sj; o.end_i = ei; o.end_j = ej;
    o.correct = c; o.error = e; o.ahg = ahg; o.bhg = bhg;
    o.flags = (valid ? 2 : 0) | (ovl ? 4 : 0);
    out[pair] = o;
}

int local_align_stripe(int32_t max_len) {
    return max_len <= 256 ? 4 : (max_len <= 512 ? 8 : (max_len <= 1024 ? 16 : 32));
}

uint32_t local_align_wpl(int stripe, int32_t max_len) {
    // a lane's stream: one entry of 2*stripe bits per step, |A| + 63 steps at
    // most, whole 16-word (64-byte) segments
    const uint64_t bits = (uint64_t)(max_len + 63) * 2 * stripe;
    return (uint32_t)(((bits + 31) / 32 + 15) & ~15ull);
}

hipError_t launch_local_align(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t p0,
                              uint64_t np, const AlignParams &p, int stripe, uint32_t wpl, uint32_t *tb, int4 *lmax,
                              DevAlignment *out, int32_t *err, unsigned long long *cells, hipStream_t s) {
    if (!np) return hipSuccess;
    const dim3 g1((uint32_t)((np + 3) / 4)), g2((uint32_t)((np + 255) / 256));
#define SA_LOCAL(SS)                                                                                           \
    if (p.cost_bits == 16)                                                                                     \
        hipLaunchKernelGGL((local_dp_kernel<SS, Cost16>), g1, dim3(256), 0, s, r, lead, trail, p0, np, p, wpl, tb, \
                           lmax, err, cells);                                                                  \
    else                                                                                                       \
        hipLaunchKernelGGL((local_dp_kernel<SS, Cost8>), g1, dim3(256), 0, s, r, lead, trail, p0, np, p, wpl, tb,  \
                           lmax, err, cells);                                                                  \
    hipLaunchKernelGGL(local_walk_kernel<SS>, g2, dim3(256), 0, s, r, lead, trail, p0, np, p, wpl, tb, lmax, out)
    switch (stripe) {
    case 4: SA_LOCAL(4); break;
    case 8: SA_LOCAL(8); break;
    case 16: SA_LOCAL(16); break;
    case 32: SA_LOCAL(32); break;
    default: return hipErrorInvalidValue;
    }
#undef SA_LOCAL
    return hipGetLastError();
}

}  // namespace sa
