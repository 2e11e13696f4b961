// host_san.cpp -- drives the library's host-side parsers and the Trove replay
// (sequence-aligner_amd/csrc/host/fasta.cpp, trove.h) in a CPU-only build with
// AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_sanitizers.py).
//   host_san fasta FILE     -> "n <reads> bases <total> sum <checksum>" or "rc <code>"
//   host_san hoxd FILE      -> the 16 costs or "rc <code>"
//   host_san trove N SEED   -> N pseudo-random keys inserted (with repeats), the
//                              iteration order, one key per line
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../sequence-aligner_amd/csrc/host/trove.h"

namespace sa {
int read_fasta(const char *path, std::vector<char> &bases, std::vector<uint64_t> &offsets);
int read_hoxd(const char *path, int32_t cost[16]);
}  // namespace sa

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    if (!strcmp(argv[1], "fasta")) {
        std::vector<char> b;
        std::vector<uint64_t> off;
        const int rc = sa::read_fasta(argv[2], b, off);
        if (rc) { printf("rc %d\n", rc); return 0; }
        uint64_t sum = 0;
        for (size_t i = 0; i < b.size(); ++i) sum = sum * 1000003u + (unsigned char)b[i];
        printf("n %zu bases %zu sum %llu\n", off.size() - 1, b.size(), (unsigned long long)sum);
        for (size_t i = 0; i + 1 < off.size(); ++i) printf("%.*s\n", (int)(off[i + 1] - off[i]), b.data() + off[i]);
        return 0;
    }
    if (!strcmp(argv[1], "hoxd")) {
        int32_t cost[16];
        for (int i = 0; i < 16; ++i) cost[i] = 12345;  // left untouched on failure
        const int rc = sa::read_hoxd(argv[2], cost);
        printf("rc %d\n", rc);
        for (int i = 0; i < 16; ++i) printf("%d%c", cost[i], i == 15 ? '\n' : ' ');
        return 0;
    }
    if (!strcmp(argv[1], "trove") && argc >= 4) {
        const long n = atol(argv[2]);
        uint64_t x = strtoull(argv[3], nullptr, 10) * 0x9E3779B97F4A7C15ull + 1;
        sa::TroveLayout t;
        for (long i = 0; i < n; ++i) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            const int32_t key = (int32_t)(uint32_t)(x % 4 == 0 ? (x >> 40) % 1000 : x >> 32);  // repeats too
            t.insert(key);
        }
        t.for_each([](int32_t k) { printf("%d\n", k); });
        return 0;
    }
    return 2;
}
