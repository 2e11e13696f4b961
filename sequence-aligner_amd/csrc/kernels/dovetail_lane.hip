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

// LW = band cells per row held in registers (w <= LW - 1): 16 for every read up
// to ~750 bp at min identity 0.98 (the bench), 24 / 32 for longer reads

__device__ __forceinline__ void set_err(int32_t *err, int32_t code) { atomicCAS(err, 0, code); }

// A wave-uniform value copied into a VGPR the compiler cannot see through: on
// gfx950 a VALU add with an SGPR operand issues at half rate (~4.4 cycles per
// wave64 instruction vs ~2.4 with VGPR / inline operands; tools/valu_rate.hip).
__device__ __forceinline__ int32_t in_vgpr(int32_t x) {
    int32_t r;
    asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
}

// read-window loads through the global address space (plain pointers held in
// structs otherwise lower to flat loads, which also count against lgkmcnt)
__device__ __forceinline__ uint32_t gld(const uint32_t *p, int32_t i) {
    return ((const __attribute__((address_space(1))) uint32_t *)p)[i];
}

// Phase-2 lane state: the band row in registers plus the A / B read windows.
template <int LW>
struct Band {
    uint32_t b8[LW];                            // 8 * B[k - zr + u - 1] for the current row u (0 outside B)
    int32_t Tk[LW], Qk[LW], Pk[LW], Ck[LW];     // max(T,0), max(Q,0), stop cell (u << 6 | k), (c << 16 | e)
    int32_t best, bpos, bstop, bce;             // first row-major argmax and its path summary
    int32_t ap, bp;                             // A position of the next row; B position entering column LW-1
    uint32_t awd, bw;                           // packed words holding A[ap], B[bp]
    uint32_t pa, pb;                            // next words, fetched the row before a window crosses
};

// One phase-2 cell (u, k) of the band (BioLibs.scala:725-764) plus the forward
// summary of the greedy backtrack out of it (:768-809): stop cell and
// (matches << 16 | errors).  MASKED rows test 1 <= j <= |B| per cell; EXACT
// launches have w == LW - 1 for every pair (no per-lane column tests).
// Q = max(max(M, X) + gO, Y) is kept clamped at 0: the next row's Y is gE + Q.
template <int LW, bool MASKED, bool EXACT, class C>
__device__ __forceinline__ void band_cell(Band<LW> &S, const int k, const int32_t u6, const int32_t jb, const int32_t LB,
                                          const int32_t w, const C &cp, const uint32_t eqsh, const int32_t gO,
                                          const int32_t gE, const bool act, int32_t &Zl, int32_t &Xl, int32_t &Pl,
                                          int32_t &Cl) {
    const bool last = EXACT ? (k == LW - 1) : (k == LW - 1 || k == w);  // Y = 0 at k == width
    const int kn = k < LW - 1 ? k + 1 : k;
    int32_t M = cp.at(S.b8[k]) + S.Tk[k];
    int32_t Y = last ? 0 : gE + S.Qk[kn];
    int32_t X = k == 0 ? 0 : gE + max(max(Zl, Xl), 0);
    if (MASKED) {
        const bool valid = (uint32_t)(jb + k) < (uint32_t)LB;
        M = valid ? M : 0;
        X = valid ? X : 0;
        Y = valid ? Y : 0;
    }
    const int32_t T = max(max(M, X), Y);
    const bool isM = M == T, isX = X == T, pos = T > 0;
    const int32_t Pu = k == LW - 1 ? 0 : S.Pk[kn];
    const int32_t Cu = k == LW - 1 ? 0 : S.Ck[kn];
    const int32_t pxy = isX ? Pl : Pu;
    const int32_t cxy = (isX ? Cl : Cu) + 1;
    // + (1 << 16) on a match, + 1 on a mismatch: byte b of eqsh is 16 iff b == A[i-1]
    const int32_t cm = (int32_t)((1u << __builtin_amdgcn_ubfe(eqsh, S.b8[k], 8)) + (uint32_t)S.Ck[k]);
    const int32_t self = u6 | k;
    const int32_t pn = pos ? (isM ? S.Pk[k] : pxy) : self;
    const int32_t cn = pos ? (isM ? cm : cxy) : 0;
    S.Tk[k] = max(T, 0);
    S.Qk[k] = max(max(max(M, X) + gO, Y), 0);
    S.Pk[k] = pn;
    S.Ck[k] = cn;
    const bool nb = T > S.best && act && (EXACT || k <= w);
    S.best = nb ? T : S.best;
    S.bpos = nb ? self : S.bpos;
    S.bstop = nb ? pn : S.bstop;
    S.bce = nb ? cn : S.bce;
    Zl = max(M, Y) + gO;
    Xl = X;
    Pl = pn;
    Cl = cn;
}

// One phase-2 row u, then advance the A / B windows one base.  Branch-free:
// lanes past their last row (u > rows2) keep computing but no longer update the
// argmax, and the window loads are unconditional (clamped to the read).
template <int LW, bool MASKED, bool EXACT, class C>
__device__ __forceinline__ void band_row(Band<LW> &S, const int32_t u, const int32_t rows2, const int32_t zr,
                                         const int32_t LB, const int32_t w, const C c0, const C c1,
                                         const C c2, const C c3,
                                         const int32_t gO, const int32_t gE, const uint32_t *Aw, const int32_t awl,
                                         const uint32_t *Bw, const int32_t bwl, const uint32_t *dummy) {
    const uint32_t a8 = ((S.awd >> (30 - 2 * (S.ap & 15))) & 3u) << 3;
    const C c01 = (a8 & 8) ? c1 : c0, c23 = (a8 & 8) ? c3 : c2;
    const C cp = (a8 & 16) ? c23 : c01;
    const uint32_t eqsh = 16u << a8;
    const int32_t u6 = u << 6;
    const int32_t jb = u - zr - 1;  // j - 1 of column 0
    const bool act = u <= rows2;
    int32_t Zl = 0, Xl = 0, Pl = 0, Cl = 0;
#pragma unroll
    for (int k = 0; k < LW; ++k) band_cell<LW, MASKED, EXACT, C>(S, k, u6, jb, LB, w, cp, eqsh, gO, gE, act, Zl, Xl, Pl, Cl);
    // two-word windows: the word after the current one was loaded at least one
    // row earlier, so the loads issued here are not waited on until next row
    // Window words are fetched the row before a window crosses into them, so a
    // load is consumed one row of compute after it is issued.  The load is
    // unconditional (no merge copy, which would wait at once) but lanes that are
    // not about to cross all read `dummy`: one shared line instead of 64.
    ++S.ap;
    S.awd = (S.ap & 15) == 0 ? S.pa : S.awd;
    S.pa = gld((((S.ap + 1) & 15) == 0) ? Aw + min((S.ap + 1) >> 4, awl) : dummy, 0);
#pragma unroll
    for (int k = 0; k < LW - 1; ++k) S.b8[k] = S.b8[k + 1];
    S.b8[LW - 1] = S.bp < LB ? ((S.bw >> (30 - 2 * (S.bp & 15))) & 3u) << 3 : 0u;
    ++S.bp;
    S.bw = (S.bp & 15) == 0 ? S.pb : S.bw;
    S.pb = gld((((S.bp + 1) & 15) == 0) ? Bw + min((S.bp + 1) >> 4, bwl) : dummy, 0);
}

// Pair setup shared by both phases: ids, lengths, band width, input checks.
struct LanePair {
    int32_t a, b, LA, LB, w, status;
    const uint32_t *Aw, *Bw;
};

template <int LW, bool EXACT>
__device__ __forceinline__ LanePair lane_pair(const DevReads &rd, const int32_t *lead, const int32_t *trail,
                                              uint64_t pair, const AlignParams &P) {
    LanePair q;
    q.a = lead[pair] - 1;
    q.b = trail[pair] - 1;
    q.LA = rd.len[q.a];
    q.LB = rd.len[q.b];
    q.Aw = rd.codes + rd.woff[q.a];
    q.Bw = rd.codes + rd.woff[q.b];
    // width = max(k, floor(|A| * (1 - minId)).toInt + 1)   (BioLibs.scala:619-620)
    const float prod = (float)q.LA * P.one_minus_minid;
    q.w = max(P.k, (int32_t)floorf(prod) + 1);
    q.status = 0;
    if (q.w > LW - 1 || (EXACT && q.w != LW - 1) || q.LA > 30000) q.status = -11;  // (c << 16 | e) packing
    else if (q.LB < q.w) q.status = -5;
    else if (rd.bad[q.a] < q.LA || rd.bad[q.b] < q.w) q.status = -3;
    return q;
}

__device__ __forceinline__ void add_cells(unsigned long long cells, unsigned long long *cells_total) {
    // block-reduced, one sharded atomic per block
    __shared__ unsigned long long cell_sum;
    if (threadIdx.x == 0) cell_sum = 0;
    __syncthreads();
    if (cells) atomicAdd(&cell_sum, cells);
    __syncthreads();
    if (threadIdx.x == 0 && cell_sum) atomicAdd(&cells_total[blockIdx.x % NSHARD], cell_sum);
}

// Alignment record from the phase-2 argmax and its path summary (stop cell
// (u << 6 | k), matches << 16 | errors), with Alignment / Overlap validity
// (ObjectStore.scala:99-141).  r1 = phase-1 result ((ds << 1) | dud or error).
__device__ __forceinline__ void finish_alignment(const AlignParams &P, const LanePair &q, int32_t r1, int32_t ds,
                                                 int32_t zr, int32_t best2, int32_t bpos, int32_t bstop, int32_t bce,
                                                 DevAlignment *out, int32_t *err) {
    const bool p2 = r1 >= 0 && !(r1 & 1);
    int32_t status = r1 < 0 ? r1 : (r1 & 1);
    if (p2 && best2 <= 0) { status = -6; set_err(err, -6); }
    DevAlignment o;
    o.lead = q.a + 1; o.trail = q.b + 1;
    o.reserved = 0;
    if (status < 0) {
        o.start_i = o.start_j = o.end_i = o.end_j = 0; o.correct = 0; o.error = 0;
        o.ahg = o.bhg = 0; o.flags = 0x100;  // error marker
        *out = o;
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
        la = q.LA; lb = q.LB;
        alen = c + e;
    }
    const float ratio = __fdiv_rn((float)c, (float)c + (float)e);
    const bool valid = (ratio >= P.min_identity) && (alen >= P.min_overlap) &&
                       ((si == 0 && lb == ej) || (sj == 0 && la == ei));
    const int32_t ahg = si - sj;
    const int32_t bhg = lb - la + ahg;
    const bool ovl = valid && ((float)abs(ahg) < P.max_ignore) && ((float)abs(bhg) < P.max_ignore);
    o.start_i = si; o.start_j = sj; o.end_i = ei; o.end_j = ej;
    o.correct = c; o.error = e; o.ahg = ahg; o.bhg = bhg;
    o.flags = (dud ? 1 : 0) | (valid ? 2 : 0) | (ovl ? 4 : 0);
    *out = o;
}

// ---- phase 2 with stored traceback codes (the cheaper variant) ------------
// Per cell only the DP, a 2-bit code (0: cell max <= 0, 1: M, 2: X, 3: Y --
// what the reference's greedy walk reads, BioLibs.scala:780-809) OR-ed into a
// per-column word of 16 rows, and the argmax; every 16 rows the 16 words go
// to HBM lane-interleaved (one coalesced 256-B store per column).  The walk
// then runs per lane from the argmax over those words, 16 diagonal steps per
// word load, counting matches with a 2-bit XOR / popcount.
template <int LW>
struct BandTb {
    uint32_t b8[LW];
    int32_t Tk[LW], Qk[LW];
    uint32_t acc[LW];
    int32_t best, bpos;
    int32_t ap, bp;
    uint32_t awd, bw, pa, pb;
};

template <int LW, bool MASKED, bool EXACT, class C>
__device__ __forceinline__ void band_cell_tb(BandTb<LW> &S, const int k, const int32_t u6, const int32_t jb,
                                             const int32_t LB, const int32_t w, const C &cp, const int32_t gO,
                                             const int32_t gE, const bool act, const uint32_t c1, const uint32_t c2,
                                             const uint32_t c3, int32_t &Zl, int32_t &Xl) {
    const bool last = EXACT ? (k == LW - 1) : (k == LW - 1 || k == w);
    const int kn = k < LW - 1 ? k + 1 : k;
    int32_t M = cp.at(S.b8[k]) + S.Tk[k];
    int32_t Y = last ? 0 : gE + S.Qk[kn];
    int32_t X = k == 0 ? 0 : gE + max(max(Zl, Xl), 0);
    if (MASKED) {
        const bool valid = (uint32_t)(jb + k) < (uint32_t)LB;
        M = valid ? M : 0;
        X = valid ? X : 0;
        Y = valid ? Y : 0;
    }
    const int32_t T = max(max(M, X), Y);
    const uint32_t code = T > 0 ? (M == T ? c1 : (X == T ? c2 : c3)) : 0u;
    S.acc[k] |= code;
    S.Tk[k] = max(T, 0);
    S.Qk[k] = max(max(max(M, X) + gO, Y), 0);
    const bool nb = T > S.best && act && (EXACT || k <= w);
    S.best = nb ? T : S.best;
    S.bpos = nb ? (u6 | k) : S.bpos;
    Zl = max(M, Y) + gO;
    Xl = X;
}

template <int LW, bool MASKED, bool EXACT, class C>
__device__ __forceinline__ void band_row_tb(BandTb<LW> &S, const int32_t u, const int32_t rows2, const int32_t zr,
                                            const int32_t LB, const int32_t w, const C c0, const C cq1,
                                            const C cq2, const C cq3, const int32_t gO, const int32_t gE,
                                            const uint32_t *Aw, const int32_t awl, const uint32_t *Bw,
                                            const int32_t bwl, const uint32_t *dummy, uint32_t *tb, uint64_t nt) {
    const uint32_t a8 = ((S.awd >> (30 - 2 * (S.ap & 15))) & 3u) << 3;
    const C c01 = (a8 & 8) ? cq1 : c0, c23 = (a8 & 8) ? cq3 : cq2;
    const C cp = (a8 & 16) ? c23 : c01;
    const int32_t u6 = u << 6;
    const int32_t jb = u - zr - 1;
    const bool act = u <= rows2;
    const int sh = 2 * (u & 15);
    const uint32_t k1 = in_vgpr((int32_t)(1u << sh)), k2 = in_vgpr((int32_t)(2u << sh)),
                   k3 = in_vgpr((int32_t)(3u << sh));
    int32_t Zl = 0, Xl = 0;
#pragma unroll
    for (int k = 0; k < LW; ++k) band_cell_tb<LW, MASKED, EXACT, C>(S, k, u6, jb, LB, w, cp, gO, gE, act, k1, k2, k3, Zl, Xl);
    if ((u & 15) == 15) {  // a full 16-row word per column: out, lane-interleaved
        uint32_t *base = tb + (uint64_t)(u >> 4) * LW * nt;
#pragma unroll
        for (int k = 0; k < LW; ++k) {
            base[(uint64_t)k * nt] = S.acc[k];
            S.acc[k] = 0;
        }
    }
    ++S.ap;
    S.awd = (S.ap & 15) == 0 ? S.pa : S.awd;
    S.pa = gld((((S.ap + 1) & 15) == 0) ? Aw + min((S.ap + 1) >> 4, awl) : dummy, 0);
#pragma unroll
    for (int k = 0; k < LW - 1; ++k) S.b8[k] = S.b8[k + 1];
    S.b8[LW - 1] = S.bp < LB ? ((S.bw >> (30 - 2 * (S.bp & 15))) & 3u) << 3 : 0u;
    ++S.bp;
    S.bw = (S.bp & 15) == 0 ? S.pb : S.bw;
    S.pb = gld((((S.bp + 1) & 15) == 0) ? Bw + min((S.bp + 1) >> 4, bwl) : dummy, 0);
}

__device__ __forceinline__ uint32_t win16_g(const uint32_t *w, int32_t p) {
    const uint32_t a = gld(w, p >> 4);
    const int s = p & 15;
    if (s == 0) return a;
    return (a << (2 * s)) | (gld(w, (p >> 4) + 1) >> (32 - 2 * s));
}

}  // namespace

// Phase 1 (BioLibs.scala:644-689): per pair the start row ds of the phase-1
// backtrack and the dud test.  p1[pair] = (ds << 1 | dud) or a negative error;
// rows2[pair] = phase-2 row count (0 when phase 2 does not run) -- the key the
// host sorts by so each wave of the phase-2 kernel gets pairs of similar length.
template <int LW, bool EXACT, class C>
__global__ __launch_bounds__(256) void dovetail_p1_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                          uint64_t npairs, AlignParams P, int32_t *p1,
                                                          uint64_t *rows2_key, uint32_t *order, int32_t *err,
                                                          unsigned long long *cells_total) {
    const uint64_t pair = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool have = pair < npairs;
    const int32_t gO = in_vgpr(P.gap_open), gE = in_vgpr(P.gap_extend);
    LanePair q{0, 0, 0, 0, 0, -100, rd.codes, rd.codes};
    if (have) {
        q = lane_pair<LW, EXACT>(rd, lead, trail, pair, P);
        if (q.status < 0) set_err(err, q.status);
    }
    const int32_t w = q.w;
    // column j (1..w) costs for A base x = 0..3 against B[j-1] (cost packs);
    // the four column packs as scalars: selects over an array index would be
    // lowered to an LDS table
    auto colpack = [&](int bb) {
        return C::make(P.cost[0 * 4 + bb], P.cost[1 * 4 + bb], P.cost[2 * 4 + bb], P.cost[3 * 4 + bb]);
    };
    const C cq0 = colpack(0), cq1 = colpack(1), cq2 = colpack(2), cq3 = colpack(3);
    // B[0 .. LW - 1) covers every column j <= w <= LW - 1 (LB >= w, else status -5)
    const uint32_t bw0 = q.status == 0 ? gld(q.Bw, 0) : 0u;
    const uint32_t bw1 = (LW > 17 && q.status == 0 && q.LB > 16) ? gld(q.Bw, 1) : 0u;
    C cb[LW - 1];
#pragma unroll
    for (int j = 1; j < LW; ++j) {
        const uint32_t bwj = (j - 1) < 16 ? bw0 : bw1;
        const uint32_t bj = (bwj >> (30 - 2 * ((j - 1) & 15))) & 3u;
        const C c01 = (bj & 1) ? cq1 : cq0, c23 = (bj & 1) ? cq3 : cq2;
        cb[j - 1] = (bj & 2) ? c23 : c01;
    }
    // row-0 state: every cell 0; Q = max(max(M, X) + gO, Y) feeds the next row's Y
    const int32_t Q0 = max(gO, 0);
    int32_t Tc[LW - 1], Q[LW - 1], O[LW - 1];  // clamped cell max, Q, origin
#pragma unroll
    for (int j = 0; j < LW - 1; ++j) { Tc[j] = 0; Q[j] = Q0; O[j] = 1; }  // origin (row 0, col != 0)
    int32_t best = 0, borg = 0;
    const int32_t rows1 = q.status == 0 ? q.LA : 0;
    int32_t rmax = rows1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) rmax = max(rmax, __shfl_xor(rmax, off, 64));
    rmax = __builtin_amdgcn_readfirstlane(rmax);  // wave-uniform loop bound
    // A window: current word + the next one, loaded a row ahead of use;
    // branch-free rows (lanes past their last row stop updating the argmax)
    const int32_t awl = max((q.LA + 15) / 16 - 1, 0);
    uint32_t aw = q.Aw[0], awn = q.Aw[min(1, awl)];
    __builtin_amdgcn_s_waitcnt(0);  // (see phase 2)
#pragma unroll 2
    for (int32_t i = 1; i <= rmax; ++i) {
        const bool act = i <= rows1;
        const uint32_t a8 = ((aw >> (30 - 2 * ((i - 1) & 15))) & 3u) << 3;
        // origin = (stop row << 1) | (stop col != 0); column 0 cells stop with col 0
        int32_t Tdiag = 0, Odiag = (i - 1) << 1;
        int32_t Zl = gO, Xl = 0, Ol = i << 1;
        const int32_t self = (i << 1) | 1;
#pragma unroll
        for (int j = 0; j < LW - 1; ++j) {
            const int32_t M = cb[j].at(a8) + Tdiag;
            const int32_t Y = gE + Q[j];
            const int32_t X = gE + max(max(Zl, Xl), 0);
            const int32_t T = max(max(M, X), Y);
            const int32_t Oup = O[j];
            const int32_t on = T > 0 ? (M == T ? Odiag : (X == T ? Ol : Oup)) : self;
            Tdiag = Tc[j];
            Odiag = Oup;
            Tc[j] = max(T, 0);
            Q[j] = max(max(max(M, X) + gO, Y), 0);  // clamped: next row's Y = gE + Q
            O[j] = on;
            // first strict '>' in row-major order; columns > w never win
            const bool nb = T > best && act && (EXACT || j < w);
            best = nb ? T : best;
            borg = nb ? on : borg;
            Zl = max(M, Y) + gO;
            Xl = X;
            Ol = on;
        }
        aw = (i & 15) == 0 ? awn : aw;
        awn = gld(q.Aw, min((i >> 4) + 1, awl));
    }
    unsigned long long cells = 0;
    if (have) {
        int32_t r = q.status, rows2 = 0;
        if (r == 0) {
            cells = (unsigned long long)q.LA * w;
            if (best <= 0) { r = -6; set_err(err, -6); }  // the reference walks off (0,0)
            else {
                r = borg;  // (ds << 1) | dud
                if (!(borg & 1)) {
                    const int32_t ds = borg >> 1, zr = w / 2, dL = q.LA - ds;
                    cells += (unsigned long long)(dL + 1) * (w + 1);
                    // every B base touched by phase 2 must be ACGT (MatchError otherwise)
                    const int32_t touched = max(w, min(q.LB, dL - zr + w));
                    if (rd.bad[q.b] < touched) { r = -3; set_err(err, -3); }
                    else rows2 = dL;
                }
            }
        }
        p1[pair] = r;
        // descending row count: the longest waves launch first, so the grid's
        // tail is made of short ones (longest-processing-time-first)
        rows2_key[pair] = (uint64_t)(0xFFFFFu - (uint32_t)min(rows2, 0xFFFFF));
        order[pair] = (uint32_t)pair;
    }
    add_cells(cells, cells_total);
}

// Phase 1 with TWO pairs per lane in packed 16-bit halves (pair 2t in the low
// half, 2t + 1 in the high half): v_pk_{add,sub,max}_u16 run both pairs' cells
// in one instruction.  All values are kept saturated at 0 from below, which is
// exact here: every recurrence takes max(.., 0) (or compares with a positive
// maximum) before a negative value could matter -- T > 0 tests, M == T / X == T
// when T > 0, best starts at 0 -- and the host launches this kernel only when
// every score fits 16 bits (largest cost x |A| + 255 < 2^16), gap costs are
// <= 0 and every band is exactly 16 cells (EXACT).  Costs are int8 bytes biased
// by +128 so one v_perm_b32 per cell builds both pairs' (cost + 128).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 pk(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t upk(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ u16x2 pk_max(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ u16x2 pk_subs(u16x2 a, u16x2 b) { return __builtin_elementwise_sub_sat(a, b); }
// 0xFFFF in each half where x == 0 / where x > 0
__device__ __forceinline__ uint32_t pk_is0(u16x2 x, u16x2 one) { return upk((u16x2)0 - pk_subs(one, x)); }
__device__ __forceinline__ uint32_t pk_gt0(u16x2 x, u16x2 one) {
    return upk((u16x2)0 - __builtin_elementwise_min(x, one));
}
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
// Issue costs measured on gfx950 (tools/valu_rate.hip, profiles/r02/valu_rate_v9.txt): v_add_u32,
// v_sub_u32, v_and/or/xor_b32 and v_bitop3_b32 issue in ~2.5 cycles per wave per SIMD, every
// v_pk_* op, v_max/min, v_perm_b32, v_bfi_b32 and v_lshl_or_b32 in ~4.4.  So: plain u32
// add/sub wherever no half can carry or borrow, and selects as v_bitop3_b32 (S0 ? S1 : S2 is
// truth table 0xCA; the compiler would pick v_bfi_b32).
// (the builtin, not inline asm: an asm statement bounds the scheduling region,
// which left dependent packed ops back to back, each pair split by a hazard
// s_nop -- 146 of them in the phase-2 row loop)
__device__ __forceinline__ uint32_t bsel3(uint32_t m, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}
// a - b per half where a >= b in both halves (no borrow crosses)
__device__ __forceinline__ u16x2 pk_dif(u16x2 a, u16x2 b) { return pk(upk(a) - upk(b)); }
// a + b per half where neither half reaches 2^16 (no carry crosses)
__device__ __forceinline__ u16x2 pk_sum(u16x2 a, u16x2 b) { return pk(upk(a) + upk(b)); }

// Phase-1 lane state between row segments (dovetail_p1x2_seg_kernel): Tc, Q, O per
// column, best, borg -- u32 words, word r of lane l at [r * 64 + l] of the wave's slot.
// The next segment may run on another XCD (its own L2): the words move as device-scope
// relaxed atomics -- loads and stores that go past the non-coherent L2 one instruction at
// a time -- instead of release / acquire fences, whose L2 write-back and invalidate of the
// whole cache per hand-off cost more than the segments saved.
// Hardware assumption (gfx950), not a C++ memory-model guarantee: the producer's
// s_waitcnt(0) before its flag store means every sc1 state store has been acknowledged by
// the device-coherent level, and the consumer issues its sc1 state loads only after it
// has seen the flag, so they cannot return older values.  A later compiler or target
// could weaken that, so the hand-off is checked: word 47 of a lane's slot is a checksum
// of the other 47 words and of the segment they are for, and a consumer that reads a
// mismatch reports SA_E_HIP (err -7) instead of aligning from stale state.
constexpr int P1X2_WORDS = 3 * 15 + 2;
constexpr int P1X2_STATE = P1X2_WORDS + 1;
__device__ __forceinline__ uint32_t p1x2_seal(uint32_t h, uint32_t w) { return ((h << 5) | (h >> 27)) ^ w; }
__device__ __forceinline__ uint32_t p1x2_seal_init(int32_t seg) { return 0x9E3779B1u * (uint32_t)(seg + 1); }
__device__ __forceinline__ uint32_t st_ld(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_st(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Lane t's two pairs over rows [seg * R + 1, (seg + 1) * R] of its wave's rmax rows
// (R = rmax / nseg rounded up to even); st = the wave's state slot when nseg > 1.
__device__ __forceinline__ void p1x2_run(const DevReads &rd, const int32_t *lead, const int32_t *trail,
                                         uint64_t npairs, const AlignParams &P, int32_t *p1, uint64_t *rows2_key,
                                         uint32_t *order, int32_t *err, unsigned long long *cells_total,
                                         const uint64_t t, const int32_t seg, const int32_t nseg, uint32_t *st) {
    constexpr int LW = 16;
    const int lane = threadIdx.x & 63;
    const uint64_t pairA = 2 * t, pairB = 2 * t + 1;
    const bool haveA = pairA < npairs, haveB = pairB < npairs;
    const bool last = seg == nseg - 1;
    LanePair qa{0, 0, 0, 0, 0, -100, rd.codes, rd.codes}, qb = qa;
    if (haveA) {
        qa = lane_pair<LW, true>(rd, lead, trail, pairA, P);
        if (qa.status < 0 && last) set_err(err, qa.status);
    }
    if (haveB) {
        qb = lane_pair<LW, true>(rd, lead, trail, pairB, P);
        if (qb.status < 0 && last) set_err(err, qb.status);
    }
    // biased row packs (uniform): byte b = cost(a, b) + 128 for A base a of the row.  Each
    // row picks its pack per pair; each column's v_perm selector (a per-lane constant) picks
    // byte b_j of pair A's pack and byte b_j' of pair B's -- 15 selector registers, not 30
    // column packs, which keeps the kernel at <= 128 VGPRs (4 waves per SIMD).
    auto rowpack = [&](int a) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) v |= (uint32_t)((P.cost[a * 4 + b] + 128) & 255) << (8 * b);
        return v;
    };
    const uint32_t cr0 = rowpack(0), cr1 = rowpack(1), cr2 = rowpack(2), cr3 = rowpack(3);
    const uint32_t bwA = qa.status == 0 ? gld(qa.Bw, 0) : 0u, bwB = qb.status == 0 ? gld(qb.Bw, 0) : 0u;
    uint32_t csel[LW - 1];  // [bA_j, 0, 4 + bB_j, 0] (0x0C selects a zero byte)
#pragma unroll
    for (int j = 1; j < LW; ++j) {
        const uint32_t ba = (bwA >> (30 - 2 * (j - 1))) & 3u, bb = (bwB >> (30 - 2 * (j - 1))) & 3u;
        csel[j - 1] = ba | 0x00000C00u | ((4u + bb) << 16) | 0x0C000000u;
    }
    const u16x2 gO = pk((uint32_t)in_vgpr((int32_t)((uint32_t)(-P.gap_open) * 0x10001u)));
    const u16x2 gE = pk((uint32_t)in_vgpr((int32_t)((uint32_t)(-P.gap_extend) * 0x10001u)));
    const u16x2 bias = pk((uint32_t)in_vgpr((int32_t)0x00800080));
    const u16x2 one = pk((uint32_t)in_vgpr((int32_t)0x00010001));
    u16x2 Tc[LW - 1], Q[LW - 1];
    uint32_t O[LW - 1];
    u16x2 best = 0;
    uint32_t borg = 0;
    if (seg == 0) {
#pragma unroll
        for (int j = 0; j < LW - 1; ++j) { Tc[j] = 0; Q[j] = 0; O[j] = 0x00010001u; }  // origin (row 0, col != 0)
    } else {
        uint32_t hT = p1x2_seal_init(seg), hQ = 0, hO = 0;
#pragma unroll
        for (int j = 0; j < LW - 1; ++j) {
            const uint32_t t = st_ld(st + j * 64 + lane), q = st_ld(st + (15 + j) * 64 + lane);
            O[j] = st_ld(st + (30 + j) * 64 + lane);
            Tc[j] = pk(t);
            Q[j] = pk(q);
            hT = p1x2_seal(hT, t);
            hQ = p1x2_seal(hQ, q);
            hO = p1x2_seal(hO, O[j]);
        }
        best = pk(st_ld(st + 45 * 64 + lane));
        borg = st_ld(st + 46 * 64 + lane);
        const uint32_t chk = st_ld(st + P1X2_WORDS * 64 + lane);
        if (p1x2_seal(p1x2_seal(hT ^ hQ ^ hO, upk(best)), borg) != chk) set_err(err, -7);  // SA_E_HIP
    }
    const int32_t rowsA = qa.status == 0 ? qa.LA : 0, rowsB = qb.status == 0 ? qb.LA : 0;
    int32_t rmax = max(rowsA, rowsB);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) rmax = max(rmax, __shfl_xor(rmax, off, 64));
    rmax = __builtin_amdgcn_readfirstlane(rmax);
    const int32_t R = nseg == 1 ? rmax : (((rmax + nseg - 1) / nseg) + 1) & ~1;
    const int32_t i0 = seg * R + 1, i1 = min(rmax, (seg + 1) * R);
    const int32_t awlA = max((qa.LA + 15) / 16 - 1, 0), awlB = max((qb.LA + 15) / 16 - 1, 0);
    const int32_t w0 = (i0 - 1) >> 4;  // the A word of row i0, and the next
    uint32_t awA = qa.Aw[min(w0, awlA)], awnA = qa.Aw[min(w0 + 1, awlA)];
    uint32_t awB = qb.Aw[min(w0, awlB)], awnB = qb.Aw[min(w0 + 1, awlB)];
    __builtin_amdgcn_s_waitcnt(0);
    // rows every lane's pairs still have (i <= rmin, the wave's shortest) skip the row mask
    int32_t rmin = min(rowsA, rowsB);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) rmin = min(rmin, __shfl_xor(rmin, off, 64));
    rmin = __builtin_amdgcn_readfirstlane(rmin);
    auto row = [&](const int32_t i, auto masked) {
        const uint32_t act = !decltype(masked)::value ? 0xFFFFFFFFu
                             : (i <= rowsA ? 0x0000FFFFu : 0u) | (i <= rowsB ? 0xFFFF0000u : 0u);
        const uint32_t sh = 30 - 2 * ((i - 1) & 15);
        const uint32_t aA = (awA >> sh) & 3u, aB = (awB >> sh) & 3u;
        // bit-selects, not a ternary chain: that became a private lookup table (scratch)
        const uint32_t mA1 = 0u - (aA & 1u), mA2 = 0u - (aA >> 1), mB1 = 0u - (aB & 1u), mB2 = 0u - (aB >> 1);
        const uint32_t rA = bsel3(mA2, bsel3(mA1, cr3, cr2), bsel3(mA1, cr1, cr0));
        const uint32_t rB = bsel3(mB2, bsel3(mB1, cr3, cr2), bsel3(mB1, cr1, cr0));
        u16x2 Tdiag = 0, Zl = 0, Xl = 0;
        uint32_t Odiag = (uint32_t)((i - 1) << 1) * 0x10001u;
        uint32_t Ol = (uint32_t)(i << 1) * 0x10001u;
        const uint32_t self = (uint32_t)((i << 1) | 1) * 0x10001u;
#pragma unroll
        for (int j = 0; j < LW - 1; ++j) {
            const u16x2 cpk = pk(__builtin_amdgcn_perm(rB, rA, csel[j]));
            const u16x2 M = pk_subs(pk_sum(Tdiag, cpk), bias);
            const u16x2 Y = pk_subs(Q[j], gE);
            const u16x2 X = pk_subs(pk_max(Zl, Xl), gE);
            const u16x2 T = pk_max(pk_max(M, X), Y);
            const uint32_t Oup = O[j];
            const uint32_t mM = pk_is0(pk_dif(T, M), one), mX = pk_is0(pk_dif(T, X), one);
            const uint32_t on = bsel3(pk_gt0(T, one), bsel3(mM, Odiag, bsel3(mX, Ol, Oup)), self);
            Tdiag = Tc[j];
            Odiag = Oup;
            Tc[j] = T;
            Q[j] = pk_max(pk_subs(pk_max(M, X), gO), Y);
            O[j] = on;
            const uint32_t nb = pk_gt0(pk_subs(T, best), one) & act;  // first strict '>' in row-major order
            best = pk(bsel3(nb, upk(T), upk(best)));
            borg = bsel3(nb, on, borg);
            Zl = pk_subs(pk_max(M, Y), gO);
            Xl = X;
            Ol = on;
        }
        awA = (i & 15) == 0 ? awnA : awA;
        awB = (i & 15) == 0 ? awnB : awB;
        awnA = gld(qa.Aw, min((i >> 4) + 1, awlA));
        awnB = gld(qb.Aw, min((i >> 4) + 1, awlB));
    };
    int32_t i = i0;
    const int32_t iu = min(i1, rmin);  // rows [i0, iu] unmasked, (iu, i1] masked
    const std::false_type unm{};
    const std::true_type msk{};
    for (; i < iu; i += 2) {  // two rows per iteration (by hand: #pragma unroll gives up here)
        row(i, unm);
        row(i + 1, unm);
    }
    if (i == iu) { row(i, unm); ++i; }
    for (; i <= i1; ++i) row(i, msk);
    if (!last) {
        uint32_t hT = p1x2_seal_init(seg + 1), hQ = 0, hO = 0;
#pragma unroll
        for (int j = 0; j < LW - 1; ++j) {
            st_st(st + j * 64 + lane, upk(Tc[j]));
            st_st(st + (15 + j) * 64 + lane, upk(Q[j]));
            st_st(st + (30 + j) * 64 + lane, O[j]);
            hT = p1x2_seal(hT, upk(Tc[j]));
            hQ = p1x2_seal(hQ, upk(Q[j]));
            hO = p1x2_seal(hO, O[j]);
        }
        st_st(st + 45 * 64 + lane, upk(best));
        st_st(st + 46 * 64 + lane, borg);
        st_st(st + P1X2_WORDS * 64 + lane, p1x2_seal(p1x2_seal(hT ^ hQ ^ hO, upk(best)), borg));
        return;
    }
    unsigned long long cells = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const bool have = h ? haveB : haveA;
        const LanePair &q = h ? qb : qa;
        const uint64_t pair = h ? pairB : pairA;
        if (!have) continue;
        const int32_t bst = (int32_t)((upk(best) >> (16 * h)) & 0xFFFFu);
        const int32_t org = (int32_t)((borg >> (16 * h)) & 0xFFFFu);
        int32_t r = q.status, rows2 = 0;
        if (r == 0) {
            cells += (unsigned long long)q.LA * q.w;
            if (bst <= 0) { r = -6; set_err(err, -6); }  // the reference walks off (0,0)
            else {
                r = org;  // (ds << 1) | dud
                if (!(org & 1)) {
                    const int32_t ds = org >> 1, zr = q.w / 2, dL = q.LA - ds;
                    cells += (unsigned long long)(dL + 1) * (q.w + 1);
                    const int32_t touched = max(q.w, min(q.LB, dL - zr + q.w));
                    if (rd.bad[q.b] < touched) { r = -3; set_err(err, -3); }
                    else rows2 = dL;
                }
            }
        }
        p1[pair] = r;
        rows2_key[pair] = (uint64_t)(0xFFFFFu - (uint32_t)min(rows2, 0xFFFFF));
        order[pair] = (uint32_t)pair;
    }
    add_cells(cells, cells_total);
}

__global__ __launch_bounds__(256) void dovetail_p1x2_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                            uint64_t npairs, AlignParams P, int32_t *p1,
                                                            uint64_t *rows2_key, uint32_t *order, int32_t *err,
                                                            unsigned long long *cells_total) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    p1x2_run(rd, lead, trail, npairs, P, p1, rows2_key, order, err, cells_total, t, 0, 1, nullptr);
}

// Phase 1 in row segments (tail balance).  Every lane does the same instruction stream, so a
// wave of 128 pairs costs the same issue time however many pairs it holds: ~5,350 waves over
// 1,024 SIMDs quantize to 6 rounds for 5.23 of work.  Here each one-wave workgroup takes a
// ticket u (one device atomic): wave group g = u % ngroups, row segment s = u / ngroups.
// Tickets are handed out in order, so every segment-(s - 1) ticket went to a resident or
// finished workgroup before any segment-s ticket exists -- the wait below cannot deadlock.
// Segment s > 0 waits for flags[g] == s (bounded: SA_E_HIP after ~2^24 polls), loads the
// lanes' state, runs its rows and hands on; the last segment writes the results.  Units of
// 1 / nseg of a wave let the dispatcher even out the SIMDs' issue time.
__global__ __launch_bounds__(64) void dovetail_p1x2_seg_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                               uint64_t npairs, AlignParams P, int32_t *p1,
                                                               uint64_t *rows2_key, uint32_t *order, int32_t *err,
                                                               unsigned long long *cells_total, uint32_t ngroups,
                                                               int32_t nseg, uint32_t *ticket, uint32_t *flags,
                                                               uint32_t *state) {
    const int lane = threadIdx.x;
    uint32_t u = 0;
    if (lane == 0) u = atomicAdd(ticket, 1u);
    u = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)__shfl((int)u, 0, 64));
    const uint32_t g = u % ngroups;
    const int32_t s = (int32_t)(u / ngroups);
    uint32_t *st = state + (uint64_t)g * P1X2_STATE * 64;
    if (s > 0) {
        if (lane == 0) {
            uint32_t polls = 0;
            while (st_ld(flags + g) < (uint32_t)s) {
                __builtin_amdgcn_s_sleep(4);
                if (++polls > (1u << 24)) { set_err(err, -7); break; }  // SA_E_HIP
            }
        }
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the state loads stay after the flag's
    }
    p1x2_run(rd, lead, trail, npairs, P, p1, rows2_key, order, err, cells_total, (uint64_t)g * 64 + lane, s, nseg,
             st);
    if (s < nseg - 1) {
        __builtin_amdgcn_s_waitcnt(0);  // every state store acknowledged at device scope ...
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (lane == 0) st_st(flags + g, (uint32_t)(s + 1));  // ... before the flag
    }
}

// Phase 2 (BioLibs.scala:691-819) + Alignment/Overlap validity, one pair per
// lane, pairs taken in the order `order` (grouped by phase-2 row count).
template <int LW, bool EXACT, class C>
__global__ __launch_bounds__(256) void dovetail_p2_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                          uint64_t npairs, AlignParams P, const int32_t *p1,
                                                          const uint32_t *order, DevAlignment *out, int32_t *err) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool have = t < npairs;
    const uint64_t pair = have ? order[t] : 0;
    const int32_t gO = in_vgpr(P.gap_open), gE = in_vgpr(P.gap_extend);
    LanePair q{0, 0, 0, 0, 0, -100, rd.codes, rd.codes};
    int32_t r1 = -100;
    if (have) {
        q = lane_pair<LW, EXACT>(rd, lead, trail, pair, P);
        r1 = p1[pair];
    }
    const int32_t w = q.w;
    const bool p2 = r1 >= 0 && !(r1 & 1);
    const int32_t ds = r1 >= 0 ? r1 >> 1 : 0;
    const int32_t zr = w / 2;
    const int32_t dL = q.LA - ds;
    const int32_t LB = q.LB;
    const int32_t rows2 = p2 ? dL : 0;
    // rows where every cell k <= w is inside B (1 <= j <= LB) run without masks
    int32_t lo = p2 ? zr + 1 : 0, hi = p2 ? LB + zr - w : 0x7fffffff;
    int32_t rmax = rows2;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        rmax = max(rmax, __shfl_xor(rmax, off, 64));
        lo = max(lo, __shfl_xor(lo, off, 64));
        hi = min(hi, __shfl_xor(hi, off, 64));
    }
    rmax = __builtin_amdgcn_readfirstlane(rmax);
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    C cpa[4];  // row packs: costs of A base x against B bases 0..3
#pragma unroll
    for (int x = 0; x < 4; ++x) cpa[x] = C::make(P.cost[x * 4], P.cost[x * 4 + 1], P.cost[x * 4 + 2], P.cost[x * 4 + 3]);
    Band<LW> S;
    const uint32_t bw0 = p2 ? gld(q.Bw, 0) : 0u;  // k - zr < LW: B[0 .. 32)
    const uint32_t bw1 = (LW > 16 && p2 && LB > 16) ? gld(q.Bw, 1) : 0u;
#pragma unroll
    for (int k = 0; k < LW; ++k) {
        const int32_t p = k - zr;
        const uint32_t bwp = p < 16 ? bw0 : bw1;
        S.b8[k] = (p >= 0 && p < LB) ? ((bwp >> (30 - 2 * (p & 15))) & 3u) << 3 : 0u;
    }
    const int32_t Q0 = max(gO, 0);
#pragma unroll
    for (int k = 0; k < LW; ++k) { S.Tk[k] = 0; S.Qk[k] = Q0; S.Pk[k] = k; S.Ck[k] = 0; }
    S.best = 0; S.bpos = 0; S.bstop = 0; S.bce = 0;
    S.bp = LW - zr;
    const int32_t awl = max((q.LA + 15) / 16 - 1, 0), bwl = max((LB + 15) / 16 - 1, 0);
    S.bw = q.Bw[min(S.bp >> 4, bwl)];
    S.pb = q.Bw[min((S.bp >> 4) + 1, bwl)];
    S.ap = ds;
    S.awd = q.Aw[min(S.ap >> 4, awl)];
    S.pa = q.Aw[min((S.ap >> 4) + 1, awl)];
    // rows [lo, hi] run unmasked; the first zr rows and the rows past the end
    // of some lane's B test every cell (separate loops keep each body one block)
    // drain the setup loads here: otherwise the wait the loop needs on entry is
    // emitted inside it and also waits on each row's fresh prefetch
    __builtin_amdgcn_s_waitcnt(0);
    int32_t u = 1;
    const int32_t e1 = min(lo - 1, rmax), e2 = min(hi, rmax);
    for (; u <= e1; ++u) band_row<LW, true, EXACT, C>(S, u, rows2, zr, LB, w, cpa[0], cpa[1], cpa[2], cpa[3], gO, gE, q.Aw, awl,
                                                    q.Bw, bwl, rd.codes);
    for (; u <= e2; ++u) band_row<LW, false, EXACT, C>(S, u, rows2, zr, LB, w, cpa[0], cpa[1], cpa[2], cpa[3], gO, gE, q.Aw,
                                                     awl, q.Bw, bwl, rd.codes);
    for (; u <= rmax; ++u) band_row<LW, true, EXACT, C>(S, u, rows2, zr, LB, w, cpa[0], cpa[1], cpa[2], cpa[3], gO, gE, q.Aw, awl,
                                                    q.Bw, bwl, rd.codes);

    if (!have) return;
    finish_alignment(P, q, r1, ds, zr, S.best, S.bpos, S.bstop, S.bce, out + pair, err);
}

// Phase 2 with stored traceback codes: same contract as dovetail_p2_kernel;
// tb holds 16 columns x rw words for each of the nt lanes of this launch,
// which covers pairs order[t0 .. t0 + nt).
template <int LW, bool EXACT, class C>
__global__ __launch_bounds__(256) void dovetail_p2tb_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                            uint64_t npairs, uint64_t t0, uint64_t nt, AlignParams P,
                                                            const int32_t *p1, const uint32_t *order,
                                                            DevAlignment *out, int32_t *err, uint32_t *tbbuf) {
    const uint64_t tl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // lane within this launch
    const uint64_t t = t0 + tl;
    const bool have = tl < nt && t < npairs;
    const uint64_t pair = have ? order[t] : 0;
    const int32_t gO = in_vgpr(P.gap_open), gE = in_vgpr(P.gap_extend);
    LanePair q{0, 0, 0, 0, 0, -100, rd.codes, rd.codes};
    int32_t r1 = -100;
    if (have) {
        q = lane_pair<LW, EXACT>(rd, lead, trail, pair, P);
        r1 = p1[pair];
    }
    const int32_t w = q.w;
    const bool p2 = r1 >= 0 && !(r1 & 1);
    const int32_t ds = r1 >= 0 ? r1 >> 1 : 0;
    const int32_t zr = w / 2;
    const int32_t dL = q.LA - ds;
    const int32_t LB = q.LB;
    const int32_t rows2 = p2 ? dL : 0;
    int32_t lo = p2 ? zr + 1 : 0, hi = p2 ? LB + zr - w : 0x7fffffff;
    int32_t rmax = rows2;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        rmax = max(rmax, __shfl_xor(rmax, off, 64));
        lo = max(lo, __shfl_xor(lo, off, 64));
        hi = min(hi, __shfl_xor(hi, off, 64));
    }
    rmax = __builtin_amdgcn_readfirstlane(rmax);
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    C cpa[4];  // row packs: costs of A base x against B bases 0..3
#pragma unroll
    for (int x = 0; x < 4; ++x) cpa[x] = C::make(P.cost[x * 4], P.cost[x * 4 + 1], P.cost[x * 4 + 2], P.cost[x * 4 + 3]);
    BandTb<LW> S;
    const uint32_t bw0 = p2 ? gld(q.Bw, 0) : 0u;  // k - zr < LW: B[0 .. 32)
    const uint32_t bw1 = (LW > 16 && p2 && LB > 16) ? gld(q.Bw, 1) : 0u;
#pragma unroll
    for (int k = 0; k < LW; ++k) {
        const int32_t p = k - zr;
        const uint32_t bwp = p < 16 ? bw0 : bw1;
        S.b8[k] = (p >= 0 && p < LB) ? ((bwp >> (30 - 2 * (p & 15))) & 3u) << 3 : 0u;
    }
    const int32_t Q0 = max(gO, 0);
#pragma unroll
    for (int k = 0; k < LW; ++k) { S.Tk[k] = 0; S.Qk[k] = Q0; S.acc[k] = 0; }
    S.best = 0; S.bpos = 0;
    S.bp = LW - zr;
    const int32_t awl = max((q.LA + 15) / 16 - 1, 0), bwl = max((LB + 15) / 16 - 1, 0);
    S.bw = q.Bw[min(S.bp >> 4, bwl)];
    S.pb = q.Bw[min((S.bp >> 4) + 1, bwl)];
    S.ap = ds;
    S.awd = q.Aw[min(S.ap >> 4, awl)];
    S.pa = q.Aw[min((S.ap >> 4) + 1, awl)];
    uint32_t *tb = tbbuf + tl;  // lane column; word (row block rb, column k) at (rb * LW + k) * nt
    __builtin_amdgcn_s_waitcnt(0);
    int32_t u = 1;
    const int32_t e1 = min(lo - 1, rmax), e2 = min(hi, rmax);
    for (; u <= e1; ++u)
        band_row_tb<LW, true, EXACT, C>(S, u, rows2, zr, LB, w, cpa[0], cpa[1], cpa[2], cpa[3], gO, gE, q.Aw, awl, q.Bw,
                                 bwl, rd.codes, tb, nt);
    for (; u <= e2; ++u)
        band_row_tb<LW, false, EXACT, C>(S, u, rows2, zr, LB, w, cpa[0], cpa[1], cpa[2], cpa[3], gO, gE, q.Aw, awl, q.Bw,
                                  bwl, rd.codes, tb, nt);
    for (; u <= rmax; ++u)
        band_row_tb<LW, true, EXACT, C>(S, u, rows2, zr, LB, w, cpa[0], cpa[1], cpa[2], cpa[3], gO, gE, q.Aw, awl, q.Bw,
                                 bwl, rd.codes, tb, nt);
    if ((rmax & 15) != 15) {  // the last, partial row block
        uint32_t *base = tb + (uint64_t)(rmax >> 4) * LW * nt;
#pragma unroll
        for (int k = 0; k < LW; ++k) base[(uint64_t)k * nt] = S.acc[k];
    }
    if (!have) return;
    // ---- greedy walk from the argmax (BioLibs.scala:768-809) ---------------
    int32_t bstop = 0, bce = 0;
    if (p2 && S.best > 0) {
        int32_t uu = S.bpos >> 6, k = S.bpos & 63;
        int32_t c = 0, e = 0;
        uint32_t word = tb[((uint64_t)(uu >> 4) * LW + k) * nt];
        uint32_t code = (word >> (2 * (uu & 15))) & 3u;
        while (code != 0) {
            if (code == 1) {
                // run of M codes in column k from row uu down, inside this word
                const int r = uu & 15;
                uint32_t x = word ^ 0x55555555u;
                x &= (r == 15) ? 0xFFFFFFFFu : ((1u << (2 * r + 2)) - 1u);
                const int32_t n = x == 0 ? r + 1 : r - ((31 - __clz(x)) >> 1);
                const int32_t i = uu + ds, j = k - zr + uu;
                // compare A[i-n .. i) with B[j-n .. j)
                const uint32_t sh = 32 - 2 * n;
                const uint32_t xa = win16_g(q.Aw, i - n), xb = win16_g(q.Bw, j - n);
                uint32_t d = (sh == 0) ? (xa ^ xb) : ((xa ^ xb) >> sh);
                d = (d | (d >> 1)) & 0x55555555u;
                const int32_t mism = __popc(d);
                c += n - mism;
                e += mism;
                uu -= n;
            } else if (code == 2) {
                ++e; --k;
            } else {
                ++e; --uu; ++k;
            }
            word = tb[((uint64_t)(uu >> 4) * LW + k) * nt];
            code = (word >> (2 * (uu & 15))) & 3u;
        }
        bstop = (uu << 6) | k;
        bce = (c << 16) | e;
    }
    finish_alignment(P, q, r1, ds, zr, S.best, S.bpos, bstop, bce, out + pair, err);
}

// Phase 2 with stored traceback codes, TWO pairs per lane in packed 16-bit
// halves (pairs order[t0 + 2 tl] and order[t0 + 2 tl + 1]: adjacent in the
// row-count order, so of similar length), same conditions and saturation
// argument as dovetail_p1x2_kernel.  Each column word holds 8 rows of 2-bit
// codes per pair (low half: the first pair), word (rb8, k) of lane tl at
// (rb8 * 16 + k) * nl; the walks run per pair over the halves.
struct BandX2 {
    uint32_t sel[16];          // v_perm selector per column: [B code of pair 0, 0, 4 + B code of pair 1, 0]
    u16x2 Tk[16], Qk[16];
    uint32_t acc[16];
    u16x2 best;
    uint32_t bpos;
    // A words realigned to the pair's phase-2 start ds: ra = A bases [ds + 16 m, +16) for the
    // rows 16 m + 1 .. 16 m + 16, so every lane changes word on the same rows; aw1 / aw2 the
    // next two aligned words (aw2's load issued 16 rows before it is used), as = ds mod 16,
    // aj the next aligned word to load.  B positions (9 + u - 1 on row u) are the same for
    // every lane: bw the current word, bw1 the next (loaded 16 rows ahead).  No word load is
    // waited on within 16 rows of its issue -- the row loop's loads were once every row and
    // their vmcnt waits also drained the code stores issued before them.
    uint32_t ra[2], aw1[2], aw2[2], bw[2], bw1[2];
    int32_t as[2], aj[2];
};

__device__ __forceinline__ uint32_t x2_sel(uint32_t b0, uint32_t b1) {
    return b0 | 0x00000C00u | ((4u + b1) << 16) | 0x0C000000u;
}

// after row u: every 8 rows the half-words go out, lane-interleaved
__device__ __forceinline__ void store_x2(BandX2 &S, const int32_t u, uint32_t *tb, uint64_t nl) {
    if ((u & 7) == 7) {
        uint32_t *base = tb + (uint64_t)(u >> 3) * 16 * nl;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            base[(uint64_t)k * nl] = S.acc[k];
            S.acc[k] = 0;
        }
    }
}

template <bool MASKED>
__device__ __forceinline__ void band_row_x2(BandX2 &S, const int32_t u, const uint32_t act, const int32_t zr,
                                            const int32_t LB0, const int32_t LB1, const uint32_t *cpa, const u16x2 gO,
                                            const u16x2 gE, const u16x2 bias, const u16x2 one, const LanePair &q0, const LanePair &q1,
                                            const int32_t awl0, const int32_t awl1, const int32_t bwl0,
                                            const int32_t bwl1, const uint32_t *dummy, uint32_t *tb, uint64_t nl) {
    uint32_t cp[2];
    const int ash = 30 - 2 * ((u - 1) & 15);  // (uniform)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t a = (S.ra[h] >> ash) & 3u;
        const uint32_t c01 = (a & 1) ? cpa[1] : cpa[0], c23 = (a & 1) ? cpa[3] : cpa[2];
        cp[h] = (a & 2) ? c23 : c01;
    }
    const uint32_t u4 = (uint32_t)(u << 4) * 0x10001u;  // argmax cell (u << 4 | k) per half: u < 4096
    const int32_t jb = u - zr - 1;
    const int sh = 2 * (u & 7);
    u16x2 Zl = 0, Xl = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const u16x2 cpk = pk(__builtin_amdgcn_perm(cp[1], cp[0], S.sel[k]));
        u16x2 M = pk_subs(pk_sum(S.Tk[k], cpk), bias);
        u16x2 Y = k == 15 ? (u16x2)0 : pk_subs(S.Qk[k + 1], gE);
        u16x2 X = k == 0 ? (u16x2)0 : pk_subs(pk_max(Zl, Xl), gE);
        if (MASKED) {
            const uint32_t v = ((uint32_t)(jb + k) < (uint32_t)LB0 ? 0x0000FFFFu : 0u) |
                               ((uint32_t)(jb + k) < (uint32_t)LB1 ? 0xFFFF0000u : 0u);
            M = pk(upk(M) & v);
            X = pk(upk(X) & v);
            Y = pk(upk(Y) & v);
        }
        const u16x2 MX = pk_max(M, X);
        const u16x2 T = pk_max(MX, Y);
        // [T > 0] + [M < T] + [max(M, X) < T]: 0 (T = 0: then M = X = Y = 0), 1 M, 2 X, 3 Y
        const uint32_t code = upk(__builtin_elementwise_min(T, one)) +
                              upk(__builtin_elementwise_min(pk_dif(T, M), one)) +
                              upk(__builtin_elementwise_min(pk_dif(T, MX), one));
        S.acc[k] |= code << sh;
        S.Tk[k] = T;
        S.Qk[k] = pk_max(pk_subs(MX, gO), Y);
        const uint32_t nb = pk_gt0(pk_subs(T, S.best), one) & act;  // first strict '>' in row-major order
        S.best = pk(bsel3(nb, upk(T), upk(S.best)));
        S.bpos = bsel3(nb, u4 | (uint32_t)k * 0x10001u, S.bpos);
        Zl = pk_subs(pk_max(M, Y), gO);
        Xl = X;
    }
    uint32_t bnew[2];
    const int32_t bp = 8 + u;  // this row's new B position (uniform)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int32_t LB = h ? LB1 : LB0;
        bnew[h] = bp < LB ? (S.bw[h] >> (30 - 2 * (bp & 15))) & 3u : 0u;
    }
    if (((bp + 1) & 15) == 0) {  // (uniform) the next row starts B word (bp + 1) >> 4
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const LanePair &q = h ? q1 : q0;
            S.bw[h] = S.bw1[h];
            S.bw1[h] = gld(q.Bw, min(((bp + 1) >> 4) + 1, h ? bwl1 : bwl0));
        }
    }
    if ((u & 15) == 0) {  // (uniform) the next row starts realigned A word u >> 4
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const LanePair &q = h ? q1 : q0;
            S.ra[h] = S.as[h] == 0 ? S.aw1[h] : __builtin_amdgcn_alignbit(S.aw1[h], S.aw2[h], 32 - 2 * S.as[h]);
            S.aw1[h] = S.aw2[h];
            S.aw2[h] = gld(q.Aw, min(S.aj[h], h ? awl1 : awl0));
            ++S.aj[h];
        }
    }
    (void)dummy;
#pragma unroll
    for (int k = 0; k < 15; ++k) S.sel[k] = S.sel[k + 1];
    S.sel[15] = x2_sel(bnew[0], bnew[1]);
}

#ifndef SA_P2_WAVES  // (A/B builds: a minimum of waves per SIMD for the packed phase 2)
#define SA_P2_WAVES 1
#endif
__global__ __launch_bounds__(256, SA_P2_WAVES) void dovetail_p2tbx2_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                              uint64_t npairs, uint64_t t0, uint64_t nt, AlignParams P,
                                                              const int32_t *p1, const uint32_t *order,
                                                              DevAlignment *out, int32_t *err, uint32_t *tbbuf) {
    constexpr int LW = 16;
    const uint64_t nl = (nt + 1) / 2;  // lanes of this launch
    const uint64_t tl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool have[2];
    uint64_t pair[2];
    LanePair q[2];
    int32_t r1[2], ds[2], rows2[2], LBh[2];
    bool p2[2];
    int32_t lo = 0, hi = 0x7fffffff, rmax = 0;
    constexpr int32_t zr = (LW - 1) / 2;  // every band 16 cells (EXACT)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint64_t t = t0 + 2 * tl + h;
        have[h] = tl < nl && 2 * tl + h < nt && t < npairs;
        pair[h] = have[h] ? order[t] : 0;
        q[h] = LanePair{0, 0, 0, 0, 0, -100, rd.codes, rd.codes};
        r1[h] = -100;
        if (have[h]) {
            q[h] = lane_pair<LW, true>(rd, lead, trail, pair[h], P);
            r1[h] = p1[pair[h]];
        }
        p2[h] = r1[h] >= 0 && !(r1[h] & 1);
        ds[h] = r1[h] >= 0 ? r1[h] >> 1 : 0;
        LBh[h] = q[h].LB;
        rows2[h] = p2[h] ? q[h].LA - ds[h] : 0;
        if (p2[h]) {
            lo = max(lo, zr + 1);
            hi = min(hi, LBh[h] + zr - (LW - 1));
        }
        rmax = max(rmax, rows2[h]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        rmax = max(rmax, __shfl_xor(rmax, off, 64));
        lo = max(lo, __shfl_xor(lo, off, 64));
        hi = min(hi, __shfl_xor(hi, off, 64));
    }
    rmax = __builtin_amdgcn_readfirstlane(rmax);
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    uint32_t cpa[4];  // biased row packs: byte y = cost(x, y) + 128
#pragma unroll
    for (int x = 0; x < 4; ++x) {
        cpa[x] = 0;
#pragma unroll
        for (int y = 0; y < 4; ++y) cpa[x] |= (uint32_t)((P.cost[x * 4 + y] + 128) & 255) << (8 * y);
    }
    const u16x2 gO = pk((uint32_t)in_vgpr((int32_t)((uint32_t)(-P.gap_open) * 0x10001u)));
    const u16x2 gE = pk((uint32_t)in_vgpr((int32_t)((uint32_t)(-P.gap_extend) * 0x10001u)));
    const u16x2 bias = pk((uint32_t)in_vgpr((int32_t)0x00800080));
    const u16x2 one = pk((uint32_t)in_vgpr((int32_t)0x00010001));
    BandX2 S;
    uint32_t bw0[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) bw0[h] = p2[h] ? gld(q[h].Bw, 0) : 0u;  // k - zr < 16: B[0 .. 16)
#pragma unroll
    for (int k = 0; k < LW; ++k) {
        const int32_t p = k - zr;
        uint32_t b[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) b[h] = (p >= 0 && p < LBh[h]) ? (bw0[h] >> (30 - 2 * (p & 15))) & 3u : 0u;
        S.sel[k] = x2_sel(b[0], b[1]);
        S.Tk[k] = 0;
        S.Qk[k] = 0;
        S.acc[k] = 0;
    }
    S.best = 0;
    S.bpos = 0;
    int32_t awl[2], bwl[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        awl[h] = max((q[h].LA + 15) / 16 - 1, 0);
        bwl[h] = max((LBh[h] + 15) / 16 - 1, 0);
        // row 1's B position LW - zr = 9 lies in word 0
        S.bw[h] = q[h].Bw[0];
        S.bw1[h] = q[h].Bw[min(1, bwl[h])];
        // realigned A word 0 = bases [ds, ds + 16) from aligned words j0, j0 + 1
        const int32_t j0 = ds[h] >> 4;
        S.as[h] = ds[h] & 15;
        const uint32_t w0 = q[h].Aw[min(j0, awl[h])];
        S.aw1[h] = q[h].Aw[min(j0 + 1, awl[h])];
        S.aw2[h] = q[h].Aw[min(j0 + 2, awl[h])];
        S.aj[h] = j0 + 3;
        S.ra[h] = S.as[h] == 0 ? w0 : __builtin_amdgcn_alignbit(w0, S.aw1[h], 32 - 2 * S.as[h]);
    }
    uint32_t *tb = tbbuf + tl;
    __builtin_amdgcn_s_waitcnt(0);
    int32_t u = 1;
    const int32_t e1 = min(lo - 1, rmax), e2 = min(hi, rmax);
#define X2_ROW(MASKED)                                                                                          \
    band_row_x2<MASKED>(S, u, (u <= rows2[0] ? 0x0000FFFFu : 0u) | (u <= rows2[1] ? 0xFFFF0000u : 0u), zr, LBh[0], \
                        LBh[1], cpa, gO, gE, bias, one, q[0], q[1], awl[0], awl[1], bwl[0], bwl[1],   \
                        rd.codes, tb, nl)
    for (; u <= e1; ++u) { X2_ROW(true); store_x2(S, u, tb, nl); }
    if ((u & 1) && u <= e2) { X2_ROW(false); store_x2(S, u, tb, nl); ++u; }
    for (; u < e2; u += 2) {  // two rows (even, odd) per iteration: one basic block
        X2_ROW(false);
        ++u;
        X2_ROW(false);
        store_x2(S, u, tb, nl);
        --u;
    }
    for (; u <= e2; ++u) { X2_ROW(false); store_x2(S, u, tb, nl); }
    for (; u <= rmax; ++u) { X2_ROW(true); store_x2(S, u, tb, nl); }
#undef X2_ROW
    if ((rmax & 7) != 7) {  // the last, partial row block
        uint32_t *base = tb + (uint64_t)(rmax >> 3) * 16 * nl;
#pragma unroll
        for (int k = 0; k < LW; ++k) base[(uint64_t)k * nl] = S.acc[k];
    }
    // ---- greedy walks from the argmaxes (BioLibs.scala:768-809) ------------
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (!have[h]) continue;
        const int32_t best = (int32_t)((upk(S.best) >> (16 * h)) & 0xFFFFu);
        const int32_t bp4 = (int32_t)((S.bpos >> (16 * h)) & 0xFFFFu);
        const int32_t bpos = ((bp4 >> 4) << 6) | (bp4 & 15);
        int32_t bstop = 0, bce = 0;
        if (p2[h] && best > 0) {
            int32_t uu = bpos >> 6, k = bpos & 63;
            int32_t c = 0, e = 0;
            uint32_t hw = (tb[((uint64_t)(uu >> 3) * LW + k) * nl] >> (16 * h)) & 0xFFFFu;
            uint32_t code = (hw >> (2 * (uu & 7))) & 3u;
            while (code != 0) {
                if (code == 1) {
                    // run of M codes in column k from row uu down, inside this half-word
                    const int r = uu & 7;
                    uint32_t x = hw ^ 0x5555u;
                    x &= (r == 7) ? 0xFFFFu : ((1u << (2 * r + 2)) - 1u);
                    const int32_t n = x == 0 ? r + 1 : r - ((31 - __clz(x)) >> 1);
                    const int32_t i = uu + ds[h], j = k - zr + uu;
                    const uint32_t shn = 32 - 2 * n;
                    const uint32_t xa = win16_g(q[h].Aw, i - n), xb = win16_g(q[h].Bw, j - n);
                    uint32_t d = (shn == 0) ? (xa ^ xb) : ((xa ^ xb) >> shn);
                    d = (d | (d >> 1)) & 0x55555555u;
                    const int32_t mism = __popc(d);
                    c += n - mism;
                    e += mism;
                    uu -= n;
                } else if (code == 2) {
                    ++e; --k;
                } else {
                    ++e; --uu; ++k;
                }
                hw = (tb[((uint64_t)(uu >> 3) * LW + k) * nl] >> (16 * h)) & 0xFFFFu;
                code = (hw >> (2 * (uu & 7))) & 3u;
            }
            bstop = (uu << 6) | k;
            bce = (c << 16) | e;
        }
        finish_alignment(P, q[h], r1[h], ds[h], zr, best, bpos, bstop, bce, out + pair[h], err);
    }
}

// LW = 16 (with the EXACT variant: every band exactly 16 cells), 24 or 32
#define SA_LANE_DISPATCH_C(KERNEL, C, GRID, ...)                                                            \
    do {                                                                                                    \
        if (lw == 16 && exact) hipLaunchKernelGGL((KERNEL<16, true, C>), GRID, dim3(256), 0, s, __VA_ARGS__); \
        else if (lw == 16) hipLaunchKernelGGL((KERNEL<16, false, C>), GRID, dim3(256), 0, s, __VA_ARGS__);     \
        else if (lw == 24) hipLaunchKernelGGL((KERNEL<24, false, C>), GRID, dim3(256), 0, s, __VA_ARGS__);     \
        else if (lw == 32) hipLaunchKernelGGL((KERNEL<32, false, C>), GRID, dim3(256), 0, s, __VA_ARGS__);     \
        else return hipErrorInvalidValue;                                                                   \
    } while (0)
// cost packs: int8 bytes unless the (reduced) matrix needs int16 halves
#define SA_LANE_DISPATCH(KERNEL, GRID, ...)                                                                 \
    do {                                                                                                    \
        if (p.cost_bits == 16) SA_LANE_DISPATCH_C(KERNEL, Cost16, GRID, __VA_ARGS__);                       \
        else SA_LANE_DISPATCH_C(KERNEL, Cost8, GRID, __VA_ARGS__);                                          \
    } while (0)

int dovetail_lane_width(int32_t wmax) {
    return wmax <= 15 ? 16 : (wmax <= 23 ? 24 : (wmax <= 31 ? 32 : 0));
}

hipError_t launch_dovetail_p1(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                              const AlignParams &p, int lw, bool exact, int32_t *p1, uint64_t *rows2_key,
                              uint32_t *order, int32_t *err, unsigned long long *cells, hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 grid((uint32_t)((n + 255) / 256));
    SA_LANE_DISPATCH(dovetail_p1_kernel, grid, r, lead, trail, n, p, p1, rows2_key, order, err, cells);
    return hipGetLastError();
}

hipError_t launch_dovetail_p2(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                              const AlignParams &p, int lw, bool exact, const int32_t *p1, const uint32_t *order,
                              DevAlignment *out, int32_t *err, hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 grid((uint32_t)((n + 255) / 256));
    SA_LANE_DISPATCH(dovetail_p2_kernel, grid, r, lead, trail, n, p, p1, order, out, err);
    return hipGetLastError();
}

hipError_t launch_dovetail_p1x2(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                                const AlignParams &p, int32_t *p1, uint64_t *rows2_key, uint32_t *order, int32_t *err,
                                unsigned long long *cells, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint64_t lanes = (n + 1) / 2;
    hipLaunchKernelGGL(dovetail_p1x2_kernel, dim3((uint32_t)((lanes + 255) / 256)), dim3(256), 0, s, r, lead, trail,
                       n, p, p1, rows2_key, order, err, cells);
    return hipGetLastError();
}

uint32_t dovetail_p1x2_groups(uint64_t n) { return (uint32_t)(((n + 1) / 2 + 63) / 64); }
size_t dovetail_p1x2_state_words(uint64_t n) { return (size_t)dovetail_p1x2_groups(n) * P1X2_STATE * 64; }

hipError_t launch_dovetail_p1x2_seg(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                                    const AlignParams &p, int32_t *p1, uint64_t *rows2_key, uint32_t *order,
                                    int32_t *err, unsigned long long *cells, int32_t nseg, uint32_t *ticket_flags,
                                    uint32_t *state, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t ng = dovetail_p1x2_groups(n);
    // ticket_flags: 1 + ng words, zeroed here
    hipError_t e = hipMemsetAsync(ticket_flags, 0, (size_t)(1 + ng) * 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(dovetail_p1x2_seg_kernel, dim3((uint32_t)((uint64_t)ng * nseg)), dim3(64), 0, s, r, lead,
                       trail, n, p, p1, rows2_key, order, err, cells, ng, nseg, ticket_flags, ticket_flags + 1, state);
    return hipGetLastError();
}

size_t dovetail_tbx2_words(uint64_t nt, int32_t max_len) {
    const uint64_t rb8 = (uint64_t)(max_len + 1 + 7) / 8 + 1;
    return rb8 * 16 * ((nt + 1) / 2);
}

hipError_t launch_dovetail_p2tbx2(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                                  uint64_t t0, uint64_t nt, const AlignParams &p, const int32_t *p1,
                                  const uint32_t *order, DevAlignment *out, int32_t *err, uint32_t *tb,
                                  hipStream_t s) {
    if (!n || !nt) return hipSuccess;
    const uint64_t lanes = (nt + 1) / 2;
    hipLaunchKernelGGL(dovetail_p2tbx2_kernel, dim3((uint32_t)((lanes + 255) / 256)), dim3(256), 0, s, r, lead, trail,
                       n, t0, nt, p, p1, order, out, err, tb);
    return hipGetLastError();
}

size_t dovetail_tb_words(uint64_t nt, int32_t max_len, int lw) {
    const uint64_t rw = (uint64_t)(max_len + 1 + 15) / 16 + 1;
    return rw * (uint64_t)lw * nt;
}

hipError_t launch_dovetail_p2tb(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                                uint64_t t0, uint64_t nt, const AlignParams &p, int lw, bool exact, const int32_t *p1,
                                const uint32_t *order, DevAlignment *out, int32_t *err, uint32_t *tb,
                                hipStream_t s) {
    if (!n || !nt) return hipSuccess;
    const dim3 grid((uint32_t)((nt + 255) / 256));
    SA_LANE_DISPATCH(dovetail_p2tb_kernel, grid, r, lead, trail, n, t0, nt, p, p1, order, out, err, tb);
    return hipGetLastError();
}
#undef SA_LANE_DISPATCH

}  // namespace sa
