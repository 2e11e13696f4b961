// CPU emulation of csrc/kernels/trove_replay.hip's eviction-chain reservations (test
// infrastructure): the rehash chain's tables from the same level plan, each table built by
// "threads" run one after another in a shuffled order, every thread carrying keys down their
// probe sequences with the kernel's atomicMin rule -- checked against the sequential replay
// (csrc/host/trove.h).  Prints one line per case: m, tables, equal (1/0).
#include <algorithm>
#include <cstdio>
#include <random>
#include <unordered_set>
#include <vector>

#include "trove.h"

using sa::TroveLayout;

static void levels(uint32_t m, std::vector<uint32_t> &cap, std::vector<uint32_t> &n_re, std::vector<uint32_t> &a0,
                   std::vector<uint32_t> &na) {
    const float f = 10.0f / 0.5f;
    int32_t c0 = (int32_t)f;
    if (f - (float)c0 > 0.0f) ++c0;
    int32_t c = TroveLayout::next_prime(c0);
    uint32_t size = 0, arrived = 0;
    for (;;) {
        const int32_t lf = (int32_t)((float)c * 0.5f);
        const uint32_t maxs = (uint32_t)(c - 1 < lf ? c - 1 : lf);
        const uint32_t take = std::min<uint32_t>(m - arrived, maxs + 1 - size);
        cap.push_back((uint32_t)c); n_re.push_back(size); a0.push_back(arrived); na.push_back(take);
        arrived += take;
        size += take;
        if (size <= maxs) break;
        c = TroveLayout::next_prime(c << 1);
    }
}

int main(int argc, char **argv) {
    const unsigned seed = argc > 1 ? (unsigned)atoi(argv[1]) : 1u;
    std::mt19937_64 rng(seed);
    int bad = 0;
    for (uint32_t m : {0u, 1u, 11u, 12u, 13u, 24u, 47u, 100u, 1000u, 65536u, 300000u}) {
        std::vector<int32_t> keys;
        std::unordered_set<int32_t> seen;
        while (keys.size() < m) {  // distinct keys, half of them PairData-shaped (fst << 16) ^ snd
            const int32_t k = keys.size() % 2 ? (int32_t)rng()
                                              : (int32_t)((uint32_t)(1 + rng() % 32000) << 16 ^ (uint32_t)(1 + rng() % 32000));
            if (seen.insert(k).second) keys.push_back(k);
        }
        TroveLayout t;
        for (uint32_t i = 0; i < m; ++i) t.insert(keys[i], (int32_t)i);
        std::vector<uint32_t> ref;
        t.for_each_kv([&](int32_t, int32_t v) { ref.push_back((uint32_t)v); });
        std::vector<uint32_t> cap, n_re, a0, na;
        levels(m, cap, n_re, a0, na);
        std::vector<uint32_t> ord, out;
        for (size_t l = 0; l < cap.size(); ++l) {
            const uint32_t C = cap[l], n = n_re[l] + na[l];
            ord.resize(n_re[l]);
            for (uint32_t j = 0; j < na[l]; ++j) ord.push_back(a0[l] + j);
            std::vector<uint32_t> owner(C, 0xFFFFFFFFu), perm(n);
            for (uint32_t p = 0; p < n; ++p) perm[p] = p;
            std::shuffle(perm.begin(), perm.end(), rng);
            for (uint32_t p0 : perm) {  // tr_chain_kernel, one thread after another
                uint32_t cur = p0, h = (uint32_t)(keys[ord[cur]] & 0x7fffffff), s = h % C;
                for (;;) {
                    const uint32_t old = owner[s];
                    owner[s] = std::min(old, cur);
                    if (old == 0xFFFFFFFFu) break;
                    if (old > cur) { cur = old; h = (uint32_t)(keys[ord[cur]] & 0x7fffffff); }
                    const uint32_t step = 1u + h % (C - 2u);
                    s = s >= step ? s - step : s + C - step;
                }
            }
            out.clear();
            for (uint32_t j = 0; j < C; ++j)
                if (owner[C - 1 - j] != 0xFFFFFFFFu) out.push_back(ord[owner[C - 1 - j]]);
            ord = out;
        }
        const bool same = (m == 0 && ref.empty()) || ref == out;
        bad += !same;
        printf("%u %zu %d\n", m, cap.size(), (int)same);
    }
    return bad ? 1 : 0;
}
