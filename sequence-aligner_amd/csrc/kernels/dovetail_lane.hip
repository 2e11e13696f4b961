// dovetail_lane.hip -- one (lead, trail) pair per lane, no traceback storage (gfx950).
//
// Same contract as dovetail.hip (BioLibs.generateFastDovetailAlignmentSet,
// BioLibs.scala:596-822, plus the ObjectStore.scala:99-141 validity), for pairs
// whose band has at most 15 columns (w <= 15: the k = 15, 500 bp workload and
// every read shorter than ~750 bp at min identity 0.98).
//
// Mapping: lane = pair.  The lane walks its DP matrix row by row and keeps the
// band row (<= 16 cells) in registers, fully unrolled over columns, so a cell
// is ~22-30 straight-line VALU ops with no cross-lane traffic, no LDS and no
// barriers.  The two greedy backtracks of the reference (phase 1 :673-689,
// phase 2 :768-819) are NOT replayed: the path out of every cell is fixed by
// that cell's winning term (M first, then X, then Y; stop when the cell max is
// <= 0), so each cell forwards the summary of the path that leaves it --
//   phase 1: the stop cell's row and whether its column is 0 (dud test)
//   phase 2: the stop cell (u, k) and the (matches, errors) counted on the way
// -- from the predecessor the walk would step to.  The best cell's summary is
// then exactly what the walk would have produced.  Bound: VALU issue (integer
// max-plus; no MFMA, no HBM traffic beyond the packed reads).
#include "../sa_internal.h"

namespace sa {

namespace {

constexpr int LW = 16;  // band cells per row held in registers (w <= LW - 1)

__device__ __forceinline__ int32_t bfe_s8(uint32_t packed, uint32_t shift) {
    return __builtin_amdgcn_sbfe((int32_t)packed, shift, 8);
}

__device__ __forceinline__ uint32_t code_of(const uint32_t *w, int32_t p) {
    return (w[p >> 4] >> (30 - 2 * (p & 15))) & 3u;
}

__device__ __forceinline__ void set_err(int32_t *err, int32_t code) { atomicCAS(err, 0, code); }

// One phase-2 cell (u, k) of the band (BioLibs.scala:725-764) plus the forward
// summary of the greedy backtrack out of it (:768-809): stop cell and
// (matches << 16 | errors).  MASKED rows test 1 <= j <= |B| per cell; EXACT
// launches have w == LW - 1 for every pair (no per-lane column tests).
template <bool MASKED, bool EXACT>
__device__ __forceinline__ void band_cell(const int k, const int32_t u6, const int32_t jb, const int32_t LB,
                                          const int32_t w, const uint32_t cp, const uint32_t a8, const int32_t gO,
                                          const int32_t gE, const uint32_t (&b8)[LW], int32_t (&Tk)[LW],
                                          int32_t (&Qk)[LW], int32_t (&Pk)[LW], int32_t (&Ck)[LW], int32_t &Zl,
                                          int32_t &Xl, int32_t &Pl, int32_t &Cl, int32_t &best, int32_t &bpos,
                                          int32_t &bstop, int32_t &bce) {
    const bool last = EXACT ? (k == LW - 1) : (k == LW - 1 || k == w);  // Y = 0 at k == width
    int32_t M = bfe_s8(cp, b8[k]) + Tk[k];
    int32_t Y = last ? 0 : gE + max(Qk[k < LW - 1 ? k + 1 : k], 0);
    int32_t X = k == 0 ? 0 : gE + max(max(Zl, Xl), 0);
    if (MASKED) {
        const bool valid = (uint32_t)(jb + k) < (uint32_t)LB;
        M = valid ? M : 0;
        X = valid ? X : 0;
        Y = valid ? Y : 0;
    }
    const int32_t T = max(max(M, X), Y);
    const bool isM = M == T, isX = X == T, pos = T > 0;
    const int32_t Pu = k == LW - 1 ? 0 : Pk[k < LW - 1 ? k + 1 : k];
    const int32_t Cu = k == LW - 1 ? 0 : Ck[k < LW - 1 ? k + 1 : k];
    const int32_t pxy = isX ? Pl : Pu;
    const int32_t cxy = (isX ? Cl : Cu) + 1;
    const int32_t cm = Ck[k] + (b8[k] == a8 ? 0x10000 : 1);
    const int32_t self = u6 | k;
    const int32_t pn = pos ? (isM ? Pk[k] : pxy) : self;
    const int32_t cn = pos ? (isM ? cm : cxy) : 0;
    Tk[k] = max(T, 0);
    Qk[k] = max(max(M, X) + gO, Y);
    Pk[k] = pn;
    Ck[k] = cn;
    const bool nb = T > best && (EXACT || k <= w);
    best = nb ? T : best;
    bpos = nb ? self : bpos;
    bstop = nb ? pn : bstop;
    bce = nb ? cn : bce;
    Zl = max(M, Y) + gO;
    Xl = X;
    Pl = pn;
    Cl = cn;
}

}  // namespace

template <bool EXACT>
__global__ __launch_bounds__(256) void dovetail_lane_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                            uint64_t npairs, AlignParams P, DevAlignment *out,
                                                            int32_t *err, unsigned long long *cells_total) {
    const uint64_t pair = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool have = pair < npairs;
    const int32_t gO = P.gap_open, gE = P.gap_extend;

    int32_t a = 0, b = 0, LA = 0, LB = 0, w = 0;
    const uint32_t *Aw = rd.codes, *Bw = rd.codes;
    int32_t status = have ? 0 : -100;  // 0 ok, 1 dud, < 0 error / no pair
    if (have) {
        a = lead[pair] - 1;
        b = trail[pair] - 1;
        LA = rd.len[a];
        LB = rd.len[b];
        Aw = rd.codes + rd.woff[a];
        Bw = rd.codes + rd.woff[b];
        // width = max(k, floor(|A| * (1 - minId)).toInt + 1)   (BioLibs.scala:619-620)
        const float prod = (float)LA * P.one_minus_minid;
        w = max(P.k, (int32_t)floorf(prod) + 1);
        if (w > LW - 1 || (EXACT && w != LW - 1) || LA > 30000) status = -11;  // (c << 16 | e) packing
        else if (LB < w) status = -5;
        else if (rd.bad[a] < LA || rd.bad[b] < w) status = -3;
        if (status < 0) set_err(err, status);
    }

    // ---------------- phase 1: A vs B[0 .. w)   (BioLibs.scala:644-668) ------
    // column j (1..w) costs for A base x = 0..3 against B[j-1], as int8 bytes
    uint32_t cb[LW - 1];
#pragma unroll
    for (int j = 1; j < LW; ++j) {
        const uint32_t bj = (status == 0 && j <= w) ? code_of(Bw, j - 1) : 0u;
        uint32_t v = 0;
#pragma unroll
        for (int x = 0; x < 4; ++x) v |= ((uint32_t)(uint8_t)(int8_t)P.cost[x * 4 + bj]) << (8 * x);
        cb[j - 1] = v;
    }
    // row-0 state: every cell 0; Q = max(max(M, X) + gO, Y) feeds the next row's Y
    const int32_t Q0 = max(gO, 0);
    int32_t Tc[LW - 1], Q[LW - 1], O[LW - 1];  // clamped cell max, Q, origin
#pragma unroll
    for (int j = 0; j < LW - 1; ++j) { Tc[j] = 0; Q[j] = Q0; O[j] = 1; }  // origin (row 0, col != 0)
    int32_t best = 0, borg = 0;
    const int32_t rows1 = status == 0 ? LA : 0;
    int32_t rmax = rows1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) rmax = max(rmax, __shfl_xor(rmax, off, 64));
    rmax = __builtin_amdgcn_readfirstlane(rmax);  // wave-uniform loop bound
    uint32_t aw = 0;
    for (int32_t i = 1; i <= rmax; ++i) {
        if (((i - 1) & 15) == 0) aw = (i <= rows1) ? Aw[(i - 1) >> 4] : 0u;
        if (i > rows1) continue;
        const uint32_t a8 = ((aw >> (30 - 2 * ((i - 1) & 15))) & 3u) << 3;
        // origin = (stop row << 1) | (stop col != 0); column 0 cells stop with col 0
        int32_t Tdiag = 0, Odiag = (i - 1) << 1;
        int32_t Zl = gO, Xl = 0, Ol = i << 1;
        const int32_t self = (i << 1) | 1;
#pragma unroll
        for (int j = 0; j < LW - 1; ++j) {
            const int32_t M = bfe_s8(cb[j], a8) + Tdiag;
            const int32_t Y = gE + max(Q[j], 0);
            const int32_t X = gE + max(max(Zl, Xl), 0);
            const int32_t T = max(max(M, X), Y);
            const int32_t Oup = O[j];
            const int32_t on = T > 0 ? (M == T ? Odiag : (X == T ? Ol : Oup)) : self;
            Tdiag = Tc[j];
            Odiag = Oup;
            Tc[j] = max(T, 0);
            Q[j] = max(max(M, X) + gO, Y);
            O[j] = on;
            // first strict '>' in row-major order; columns > w never win
            const bool nb = T > best && (EXACT || j < w);
            best = nb ? T : best;
            borg = nb ? on : borg;
            Zl = max(M, Y) + gO;
            Xl = X;
            Ol = on;
        }
    }
    int32_t ds = 0;
    const bool p1ok = status == 0;
    if (status == 0) {
        if (best <= 0) { status = -6; set_err(err, -6); }  // reference walks off (0,0)
        else { ds = borg >> 1; status = (borg & 1) ? 1 : 0; }
    }

    // ---------------- phase 2: band (u, k), i = u + ds, j = k - zr + u (:696-764)
    const int32_t st1 = status;
    const int32_t zr = w / 2;
    const int32_t dL = LA - ds;
    if (status == 0) {
        // every B base touched by phase 2 must be ACGT (MatchError otherwise)
        const int32_t touched = max(w, min(LB, dL - zr + w));
        if (rd.bad[b] < touched) { status = -3; set_err(err, -3); }
    }
    const bool p2 = status == 0;
    const int32_t rows2 = p2 ? dL : 0;
    // rows where every cell k <= w is inside B (1 <= j <= LB) run without masks
    int32_t lo = p2 ? zr + 1 : 0, hi = p2 ? LB + zr - w : 0x7fffffff;
    rmax = rows2;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        rmax = max(rmax, __shfl_xor(rmax, off, 64));
        lo = max(lo, __shfl_xor(lo, off, 64));
        hi = min(hi, __shfl_xor(hi, off, 64));
    }
    rmax = __builtin_amdgcn_readfirstlane(rmax);
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    const uint32_t cpa[4] = {
        (uint32_t)(uint8_t)(int8_t)P.cost[0] | ((uint32_t)(uint8_t)(int8_t)P.cost[1] << 8) |
            ((uint32_t)(uint8_t)(int8_t)P.cost[2] << 16) | ((uint32_t)(uint8_t)(int8_t)P.cost[3] << 24),
        (uint32_t)(uint8_t)(int8_t)P.cost[4] | ((uint32_t)(uint8_t)(int8_t)P.cost[5] << 8) |
            ((uint32_t)(uint8_t)(int8_t)P.cost[6] << 16) | ((uint32_t)(uint8_t)(int8_t)P.cost[7] << 24),
        (uint32_t)(uint8_t)(int8_t)P.cost[8] | ((uint32_t)(uint8_t)(int8_t)P.cost[9] << 8) |
            ((uint32_t)(uint8_t)(int8_t)P.cost[10] << 16) | ((uint32_t)(uint8_t)(int8_t)P.cost[11] << 24),
        (uint32_t)(uint8_t)(int8_t)P.cost[12] | ((uint32_t)(uint8_t)(int8_t)P.cost[13] << 8) |
            ((uint32_t)(uint8_t)(int8_t)P.cost[14] << 16) | ((uint32_t)(uint8_t)(int8_t)P.cost[15] << 24)};
    // b8[k] = 8 * B[k - zr + u - 1] for the current row u (0 outside B)
    uint32_t b8[LW];
#pragma unroll
    for (int k = 0; k < LW; ++k) {
        const int32_t p = k - zr;
        b8[k] = (p2 && p >= 0 && p < LB) ? code_of(Bw, p) << 3 : 0u;
    }
    int32_t Tk[LW], Qk[LW], Pk[LW], Ck[LW];  // clamped max, Q, stop cell (u << 6 | k), (c << 16 | e)
#pragma unroll
    for (int k = 0; k < LW; ++k) { Tk[k] = 0; Qk[k] = Q0; Pk[k] = k; Ck[k] = 0; }
    int32_t best2 = 0, bpos = 0, bstop = 0, bce = 0;
    int32_t bp = LW - zr;           // B position entering column LW-1 at the next row
    uint32_t bw = (p2 && bp < LB) ? Bw[bp >> 4] : 0u;
    int32_t ap = ds;                 // A position of row u + 1
    uint32_t awd = p2 ? Aw[ap >> 4] : 0u;
    for (int32_t u = 1; u <= rmax; ++u) {
        if (u > rows2) continue;
        const uint32_t a8 = ((awd >> (30 - 2 * (ap & 15))) & 3u) << 3;
        const uint32_t c01 = (a8 & 8) ? cpa[1] : cpa[0], c23 = (a8 & 8) ? cpa[3] : cpa[2];
        const uint32_t cp = (a8 & 16) ? c23 : c01;
        const int32_t u6 = u << 6;
        int32_t Zl = 0, Xl = 0, Pl = 0, Cl = 0;
        if (u >= lo && u <= hi) {
#pragma unroll
            for (int k = 0; k < LW; ++k)
                band_cell<false, EXACT>(k, u6, 0, LB, w, cp, a8, gO, gE, b8, Tk, Qk, Pk, Ck, Zl, Xl, Pl, Cl, best2,
                                        bpos, bstop, bce);
        } else {
            const int32_t jb = u - zr - 1;  // j - 1 of column 0
#pragma unroll
            for (int k = 0; k < LW; ++k)
                band_cell<true, EXACT>(k, u6, jb, LB, w, cp, a8, gO, gE, b8, Tk, Qk, Pk, Ck, Zl, Xl, Pl, Cl, best2,
                                       bpos, bstop, bce);
        }
        // advance the A and B windows one base
        ++ap;
        if ((ap & 15) == 0 && u < rows2) awd = Aw[ap >> 4];
#pragma unroll
        for (int k = 0; k < LW - 1; ++k) b8[k] = b8[k + 1];
        b8[LW - 1] = bp < LB ? ((bw >> (30 - 2 * (bp & 15))) & 3u) << 3 : 0u;
        ++bp;
        if ((bp & 15) == 0 && bp < LB) bw = Bw[bp >> 4];
    }

    // DP cells for statistics (same count as dovetail.hip): block-reduced, sharded
    {
        __shared__ unsigned long long cell_sum;
        if (threadIdx.x == 0) cell_sum = 0;
        __syncthreads();
        if (p1ok) {
            unsigned long long cells = (unsigned long long)LA * w;
            if (st1 == 0) cells += (unsigned long long)(dL + 1) * (w + 1);
            atomicAdd(&cell_sum, cells);
        }
        __syncthreads();
        if (threadIdx.x == 0 && cell_sum) atomicAdd(&cells_total[blockIdx.x % NSHARD], cell_sum);
    }
    if (!have) return;
    if (p2 && best2 <= 0) { status = -6; set_err(err, -6); }

    DevAlignment o;
    o.lead = a + 1; o.trail = b + 1;
    o.reserved = 0;
    if (status < 0) {
        o.start_i = o.start_j = o.end_i = o.end_j = 0; o.correct = 0; o.error = 0;
        o.ahg = o.bhg = 0; o.flags = 0x100;  // error marker
        out[pair] = o;
        return;
    }
    int32_t si = 0, sj = 0, ei = 0, ej = 0, c = 0, e = 1, la = 0, lb = 0, alen = 0;
    const bool dud = status == 1;
    if (!dud) {
        const int32_t su = bstop >> 6, sk = bstop & 63;
        const int32_t eu = bpos >> 6, ek = bpos & 63;
        si = su + ds; sj = sk - zr + su;
        ei = eu + ds; ej = ek - zr + eu;
        c = bce >> 16; e = bce & 0xFFFF;
        la = LA; lb = LB;
        alen = c + e;
    }
    // Alignment.valid / Overlap.valid (ObjectStore.scala:99-141)
    const float ratio = __fdiv_rn((float)c, (float)c + (float)e);
    const bool valid = (ratio >= P.min_identity) && (alen >= P.min_overlap) &&
                       ((si == 0 && lb == ej) || (sj == 0 && la == ei));
    const int32_t ahg = si - sj;
    const int32_t bhg = lb - la + ahg;
    const bool ovl = valid && ((float)abs(ahg) < P.max_ignore) && ((float)abs(bhg) < P.max_ignore);
    o.start_i = si; o.start_j = sj; o.end_i = ei; o.end_j = ej;
    o.correct = c; o.error = e; o.ahg = ahg; o.bhg = bhg;
    o.flags = (dud ? 1 : 0) | (valid ? 2 : 0) | (ovl ? 4 : 0);
    out[pair] = o;
}

hipError_t launch_dovetail_lane(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                                const AlignParams &p, bool exact, DevAlignment *out, int32_t *err,
                                unsigned long long *cells, hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 grid((uint32_t)((n + 255) / 256));
    if (exact)
        hipLaunchKernelGGL(dovetail_lane_kernel<true>, grid, dim3(256), 0, s, r, lead, trail, n, p, out, err, cells);
    else
        hipLaunchKernelGGL(dovetail_lane_kernel<false>, grid, dim3(256), 0, s, r, lead, trail, n, p, out, err, cells);
    return hipGetLastError();
}

}  // namespace sa
