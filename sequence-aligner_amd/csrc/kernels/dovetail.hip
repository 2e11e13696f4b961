// dovetail.hip -- batched two-phase banded affine dovetail alignment (gfx950).
//
// Device replacement of BioLibs.generateFastDovetailAlignmentSet
// (BioLibs.scala:596-822) for every dispatched (lead A, trail B) pair, with the
// Alignment / Overlap validity of ObjectStore.scala:99-141.
//
// Mapping: a group of G lanes (G = 16, one DPP row) aligns one pair; lane j
// owns band column j, so a DP row is one step for the whole group:
//   M  : diagonal -> DPP row_shr:1 of the previous row's cell max (phase 1) or
//        the same lane (phase 2, band coordinates)
//   Y  : vertical -> same lane (phase 1) or DPP row_shl:1 (phase 2)
//   X  : horizontal recurrence X_j = gE + max(Z_{j-1}, X_{j-1}, 0) solved as a
//        max-plus prefix scan with decay gE over the row (4 DPP steps)
// Integer VALU only -- the recurrences are max-plus, not a dense contraction,
// so MFMA is deliberately unused.  Each cell also yields a 2-bit traceback
// code (0 = cell max <= 0, i.e. backtrack stops; 1 = M; 2 = X; 3 = Y --
// exactly the information the reference's greedy do/while backtracks read,
// BioLibs.scala:679-689 and :780-809), packed 16 rows per dword in LDS,
// column-major, so the phase-2 walk skips runs of diagonal steps 16 rows at a
// time and counts matches with a 2-bit XOR/popcount.
// The maxLoc tie-break is the first strict '>' in row-major order: per-lane
// first best row, then a lexicographic (value desc, row asc, lane asc) reduce.
#include "../sa_internal.h"

namespace sa {

constexpr int32_t NEG = -(1 << 29);

template <int G>
__device__ __forceinline__ int glane_of() { return threadIdx.x & (G - 1); }

// lane j <- lane j-S of the same group; lanes j < S get `fill`
template <int G, int S>
__device__ __forceinline__ int32_t shr_g(int32_t v, int32_t fill) {
    if constexpr (G == 16) {
        return __builtin_amdgcn_update_dpp(fill, v, 0x110 + S, 0xF, 0xF, false);
    } else {
        const int32_t t = __shfl_up(v, S, G);
        return (int)(threadIdx.x & (G - 1)) >= S ? t : fill;
    }
}
// lane j <- lane j+1 of the same group; the last lane gets `fill`
template <int G>
__device__ __forceinline__ int32_t shl1_g(int32_t v, int32_t fill) {
    if constexpr (G == 16) {
        return __builtin_amdgcn_update_dpp(fill, v, 0x101, 0xF, 0xF, false);
    } else {
        const int32_t t = __shfl_down(v, 1, G);
        return (int)(threadIdx.x & (G - 1)) < G - 1 ? t : fill;
    }
}

// X_j = max(V_j, X_{j-1} + gE) over the group's lanes (max-plus scan, decay gE)
template <int G>
__device__ __forceinline__ int32_t xscan(int32_t v, int32_t gE) {
    v = max(v, shr_g<G, 1>(v, NEG) + gE);
    v = max(v, shr_g<G, 2>(v, NEG) + 2 * gE);
    v = max(v, shr_g<G, 4>(v, NEG) + 4 * gE);
    v = max(v, shr_g<G, 8>(v, NEG) + 8 * gE);
    if constexpr (G >= 32) v = max(v, shr_g<G, 16>(v, NEG) + 16 * gE);
    if constexpr (G >= 64) v = max(v, shr_g<G, 32>(v, NEG) + 32 * gE);
    return v;
}

__device__ __forceinline__ uint32_t code_at(const uint32_t *w, int32_t p) {
    return (w[p >> 4] >> (30 - 2 * (p & 15))) & 3u;
}

__device__ __forceinline__ uint32_t win16(const uint32_t *w, int32_t p) {
    const uint32_t a = w[p >> 4];
    const int s = p & 15;
    if (s == 0) return a;
    return (a << (2 * s)) | (w[(p >> 4) + 1] >> (32 - 2 * s));
}

// 64-bit argmax key: value desc, row asc, lane asc
__device__ __forceinline__ unsigned long long amax_key(int32_t best, int32_t row, int lane) {
    return ((unsigned long long)(uint32_t)best << 32) | ((unsigned long long)(0xFFFFFu - (uint32_t)row) << 8) |
           (unsigned long long)(0xFFu - (uint32_t)lane);
}

template <int G>
__device__ __forceinline__ unsigned long long group_max_u64(unsigned long long v) {
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off, G);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ void set_err(int32_t *err, int32_t code) { atomicCAS(err, 0, code); }

template <int G, class C>
__global__ __launch_bounds__(256) void dovetail_kernel(DevReads rd, const int32_t *lead, const int32_t *trail,
                                                       uint64_t npairs, AlignParams P, DevAlignment *out,
                                                       int32_t *err, unsigned long long *cells_total) {
    extern __shared__ __align__(16) uint32_t tb_all[];
    constexpr int GPB = 256 / G;  // groups (pairs) per block
    const int lane = glane_of<G>();
    const int grp = threadIdx.x / G;
    const uint64_t pair = (uint64_t)blockIdx.x * GPB + grp;
    const bool have = pair < npairs;
    const uint32_t RW = P.rw;
    uint32_t *tb = tb_all + (size_t)grp * G * RW;  // [col][RW]
    const int32_t gO = P.gap_open, gE = P.gap_extend;

    int32_t a = 0, b = 0, LA = 0, LB = 0, w = 0;
    const uint32_t *Aw = rd.codes, *Bw = rd.codes;
    bool ok = have;
    if (have) {
        a = lead[pair] - 1;
        b = trail[pair] - 1;
        LA = rd.len[a];
        LB = rd.len[b];
        Aw = rd.codes + rd.woff[a];
        Bw = rd.codes + rd.woff[b];
        // width = max(k, floor(|A| * (1 - minId)).toInt + 1)   (BioLibs.scala:619-620)
        const float prod = (float)LA * P.one_minus_minid;
        const int32_t fl = (int32_t)floorf(prod);
        w = max(P.k, fl + 1);
        if (w > G - 1 || (uint32_t)(LA + 1) > RW * 16u) { if (lane == 0) set_err(err, -11); ok = false; }
        else if (LB < w) { if (lane == 0) set_err(err, -5); ok = false; }
        else if (rd.bad[a] < LA || rd.bad[b] < w) { if (lane == 0) set_err(err, -3); ok = false; }
    }
    // wave-uniform loop bounds (DPP must run with all lanes of the wave on)
    int32_t rows1 = ok ? LA : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) rows1 = max(rows1, __shfl_xor(rows1, off, 64));

    // ---------------- phase 1: A vs B[0 .. w)   (BioLibs.scala:645-668) ------
    const int32_t bj = (ok && lane >= 1 && lane <= w) ? (int32_t)code_at(Bw, lane - 1) : 0;
    const C cb = C::make(P.cost[0 * 4 + bj], P.cost[1 * 4 + bj], P.cost[2 * 4 + bj], P.cost[3 * 4 + bj]);  // (a, B[j-1])
    int32_t Mp = 0, Xp = 0, Yp = 0, Tp = 0;
    int32_t best = 0, brow = 0;
    uint32_t acc = 0, aw = 0;
    const bool col_ok = ok && lane <= w;
    for (int32_t i = 1; i <= rows1; ++i) {
        if (((i - 1) & 15) == 0) aw = (ok && i <= LA) ? Aw[(i - 1) >> 4] : 0u;
        const uint32_t ac = (aw >> (30 - 2 * ((i - 1) & 15))) & 3u;
        const int32_t c = cb.at(ac << 3);
        const int32_t diag = shr_g<G, 1>(Tp, 0);
        // lane 0 is the boundary column j = 0: M = X = 0 and Y <= 0 there, so it
        // must feed 0 (not a computed cell) into the diagonal and the X scan
        const int32_t M = lane == 0 ? 0 : c + max(diag, 0);
        const int32_t Y = lane == 0 ? 0 : gE + max(max(max(Mp, Xp) + gO, Yp), 0);
        const int32_t Z = max(M, Y) + gO;
        const int32_t Zs = shr_g<G, 1>(Z, NEG);
        const int32_t V = lane == 0 ? 0 : gE + max(Zs, 0);
        int32_t X = xscan<G>(V, gE);
        if (lane == 0) X = 0;
        const int32_t T = max(M, max(X, Y));
        const bool row_ok = col_ok && i <= LA;
        if (row_ok && lane >= 1 && T > best) { best = T; brow = i; }
        const uint32_t code = T <= 0 ? 0u : (M == T ? 1u : (X == T ? 2u : 3u));
        acc |= code << (2 * (i & 15));
        if (((i & 15) == 15 || i == LA) && row_ok) tb[lane * RW + (i >> 4)] = acc;
        if ((i & 15) == 15) acc = 0;
        if (row_ok) { Mp = M; Xp = X; Yp = Y; Tp = T; }
    }
    if (col_ok && LA < 15) { /* rows < 16 already stored by the i == LA branch */ }
    if (col_ok && LA == 0) tb[lane * RW] = 0;
    unsigned long long mk = group_max_u64<G>(col_ok && lane >= 1 ? amax_key(best, brow, lane) : 0ull);
    __syncthreads();

    // phase-1 greedy backtrack (BioLibs.scala:673-689) by lane 0 of the group
    int32_t ds = 0;
    int32_t status = 0;  // 0 ok, 1 dud, <0 error
    if (ok && lane == 0) {
        const int32_t vbest = (int32_t)(mk >> 32);
        if (vbest <= 0) { status = -6; set_err(err, -6); }
        else {
            int32_t i = (int32_t)(0xFFFFFu - ((mk >> 8) & 0xFFFFFu));
            int32_t j = (int32_t)(0xFFu - (mk & 0xFFu));
            uint32_t code = (tb[j * RW + (i >> 4)] >> (2 * (i & 15))) & 3u;
            while (code != 0) {
                if (code == 1) { --i; --j; }
                else if (code == 2) { --j; }
                else { --i; }
                code = (tb[j * RW + (i >> 4)] >> (2 * (i & 15))) & 3u;
            }
            if (j != 0) status = 1;  // dud
            ds = i;
        }
    }
    ds = __shfl(ds, 0, G);
    status = __shfl(status, 0, G);
    const bool p2 = ok && status == 0;
    const int32_t zr = w / 2;
    const int32_t dL = LA - ds;
    if (p2 && lane == 0) {
        // every B base touched by phase 2 must be ACGT (MatchError otherwise)
        const int32_t touched = max(w, min(LB, dL - zr + w));
        if (rd.bad[b] < touched) set_err(err, -3);
    }
    __syncthreads();

    // ---------------- phase 2: band (u, k), i = u + ds, j = k - zr + u (:725-764)
    int32_t rows2 = p2 ? dL : -1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) rows2 = max(rows2, __shfl_xor(rows2, off, 64));
    const bool col2 = p2 && lane <= w;
    // B code of lane k at row u is B[k - zr + u - 1]; start at u = 0, shift left each row
    int32_t bq = 0;
    {
        const int32_t pos = lane - zr - 1;
        if (col2 && pos >= 0 && pos < LB) bq = (int32_t)code_at(Bw, pos);
    }
    C cpack[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) cpack[x] = C::make(P.cost[x * 4], P.cost[x * 4 + 1], P.cost[x * 4 + 2], P.cost[x * 4 + 3]);
    Mp = 0; Xp = 0; Yp = 0; Tp = 0;
    int32_t Qp = NEG;  // max(max(M,X)+gO, Y) of the previous row (feeds Y of lane k-1)
    best = 0; brow = 0; acc = 0;
    uint32_t aw2 = 0, bw2 = 0;
    for (int32_t u = 0; u <= rows2; ++u) {
        const bool row_ok = col2 && u <= dL;
        const int32_t i = u + ds, j = lane - zr + u;
        if (u >= 1) {
            const int32_t ap = i - 1;  // A position of this row
            if (u == 1 || (ap & 15) == 0) aw2 = (p2 && u <= dL) ? Aw[ap >> 4] : 0u;
            bq = shl1_g<G>(bq, 0);
            const int32_t bpos = w - zr + u - 1;  // new code entering at lane w
            if (u == 1 || (bpos & 15) == 0) bw2 = (p2 && bpos < LB) ? Bw[bpos >> 4] : 0u;
            if (lane == w) bq = bpos < LB ? (int32_t)((bw2 >> (30 - 2 * (bpos & 15))) & 3u) : 0;
        }
        const uint32_t ac = (aw2 >> (30 - 2 * ((i - 1) & 15))) & 3u;
        const bool valid = row_ok && u >= 1 && j >= 1 && j <= LB;
        const C cp = ac == 0 ? cpack[0] : (ac == 1 ? cpack[1] : (ac == 2 ? cpack[2] : cpack[3]));
        const int32_t c = cp.at((uint32_t)bq << 3);
        int32_t M = valid ? c + max(Tp, 0) : 0;
        const int32_t Ys = shl1_g<G>(Qp, NEG);
        int32_t Y = (valid && lane != w) ? gE + max(Ys, 0) : 0;
        const int32_t Z = max(M, Y) + gO;
        const int32_t Zs = shr_g<G, 1>(Z, NEG);
        const int32_t V = (valid && lane != 0) ? gE + max(Zs, 0) : 0;
        int32_t X = xscan<G>(V, gE);
        if (!valid) X = 0;
        const int32_t T = max(M, max(X, Y));
        if (row_ok && T > best) { best = T; brow = u; }
        const uint32_t code = T <= 0 ? 0u : (M == T ? 1u : (X == T ? 2u : 3u));
        acc |= code << (2 * (u & 15));
        if (((u & 15) == 15 || u == dL) && row_ok) tb[lane * RW + (u >> 4)] = acc;
        if ((u & 15) == 15) acc = 0;
        if (row_ok) { Mp = M; Xp = X; Yp = Y; Tp = T; Qp = max(max(Mp, Xp) + gO, Yp); }
    }
    mk = group_max_u64<G>(col2 ? amax_key(best, brow, lane) : 0ull);
    __syncthreads();

    // phase-2 greedy backtrack with match counting (BioLibs.scala:768-819)
    if (have && lane == 0) {
        DevAlignment o;
        o.lead = a + 1; o.trail = b + 1;
        o.reserved = 0;
        if (!ok || status < 0) {
            o.start_i = o.start_j = o.end_i = o.end_j = 0; o.correct = 0; o.error = 0;
            o.ahg = o.bhg = 0; o.flags = 0x100;  // error marker
            out[pair] = o;
        } else {
            int32_t si = 0, sj = 0, ei = 0, ej = 0, c = 0, e = 1, la = 0, lb = 0, alen = 0;
            bool dud = status == 1;
            if (!dud) {
                const int32_t vbest = (int32_t)(mk >> 32);
                int32_t u = (int32_t)(0xFFFFFu - ((mk >> 8) & 0xFFFFFu));
                int32_t k = (int32_t)(0xFFu - (mk & 0xFFu));
                const int32_t u0 = u, k0 = k;
                c = 0; e = 0;
                if (vbest <= 0) { set_err(err, -6); }
                uint32_t code = (tb[k * RW + (u >> 4)] >> (2 * (u & 15))) & 3u;
                while (code != 0) {
                    if (code == 1) {
                        // run of M codes in column k from row u down, inside this word
                        const uint32_t word = tb[k * RW + (u >> 4)];
                        const int r = u & 15;
                        uint32_t x = word ^ 0x55555555u;
                        x &= (r == 15) ? 0xFFFFFFFFu : ((1u << (2 * r + 2)) - 1u);
                        const int32_t n = x == 0 ? r + 1 : r - ((31 - __clz(x)) >> 1);
                        const int32_t i = u + ds, j = k - zr + u;
                        // compare A[i-n .. i) with B[j-n .. j)
                        const uint32_t sh = 32 - 2 * n;
                        const uint32_t xa = win16(Aw, i - n), xb = win16(Bw, j - n);
                        uint32_t d = (sh == 0) ? (xa ^ xb) : ((xa ^ xb) >> sh);
                        d = (d | (d >> 1)) & 0x55555555u;
                        const int32_t mism = __popc(d);
                        c += n - mism;
                        e += mism;
                        u -= n;
                    } else if (code == 2) { ++e; --k; }
                    else { ++e; --u; ++k; }
                    code = (tb[k * RW + (u >> 4)] >> (2 * (u & 15))) & 3u;
                }
                si = u + ds; sj = k - zr + u;
                ei = u0 + ds; ej = k0 - zr + u0;
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
    }
    // DP cells for statistics: block-reduced, one sharded atomic per block
    {
        __shared__ unsigned long long cell_sum;
        if (threadIdx.x == 0) cell_sum = 0;
        __syncthreads();
        if (lane == 0 && have && ok) {
            unsigned long long cells = (unsigned long long)LA * w;
            if (status == 0) cells += (unsigned long long)(dL + 1) * (w + 1);
            atomicAdd(&cell_sum, cells);
        }
        __syncthreads();
        if (threadIdx.x == 0 && cell_sum) atomicAdd(&cells_total[blockIdx.x % NSHARD], cell_sum);
    }
}

hipError_t launch_dovetail(const DevReads &r, const int32_t *lead, const int32_t *trail, uint64_t n,
                           const AlignParams &p, int group_lanes, DevAlignment *out, int32_t *err,
                           unsigned long long *cells, hipStream_t s) {
    if (!n) return hipSuccess;
    const size_t lds = (size_t)256 * p.rw * sizeof(uint32_t);  // (256/G groups) * G cols * rw
#define SA_GROUP_LAUNCH(GV, C, BLOCKS)                                                                   \
    do {                                                                                                 \
        (void)hipFuncSetAttribute((const void *)dovetail_kernel<GV, C>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)lds);                                                             \
        hipLaunchKernelGGL((dovetail_kernel<GV, C>), dim3(BLOCKS), dim3(256), lds, s, r, lead, trail, n, p, out, err, \
                           cells);                                                                       \
    } while (0)
    const bool c16 = p.cost_bits == 16;  // int16 cost packs (sa_internal.h)
    if (group_lanes == 16) {
        if (c16) SA_GROUP_LAUNCH(16, Cost16, (uint32_t)((n + 15) / 16));
        else SA_GROUP_LAUNCH(16, Cost8, (uint32_t)((n + 15) / 16));
    } else if (group_lanes == 32) {
        if (c16) SA_GROUP_LAUNCH(32, Cost16, (uint32_t)((n + 7) / 8));
        else SA_GROUP_LAUNCH(32, Cost8, (uint32_t)((n + 7) / 8));
    } else {
        if (c16) SA_GROUP_LAUNCH(64, Cost16, (uint32_t)((n + 3) / 4));
        else SA_GROUP_LAUNCH(64, Cost8, (uint32_t)((n + 3) / 4));
    }
#undef SA_GROUP_LAUNCH
    return hipGetLastError();
}

}  // namespace sa
