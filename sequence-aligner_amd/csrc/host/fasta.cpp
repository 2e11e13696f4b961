// fasta.cpp -- BioLibs.readSeq (BioLibs.scala:26-50) on the host.
//
// java.io.BufferedReader.readLine splits on "\n", "\r" and "\r\n"; the first
// line must start with '>' (else "Invalid Sequence File"); every later '>' line
// closes the current sequence (even an empty one); other lines are appended;
// the sequence is upper-cased; ids are the ordinals 1..N.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

namespace sa {

int read_fasta(const char *path, std::vector<char> &bases, std::vector<uint64_t> &offsets) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    std::vector<char> buf;
    {
        char tmp[1 << 16];
        size_t got;
        while ((got = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    }
    fclose(f);
    bases.clear();
    offsets.assign(1, 0);
    const size_t n = buf.size();
    size_t p = 0;
    bool first = true;
    if (n == 0) return -1;  // in.readLine() == null -> NPE on line.startsWith
    while (p < n) {
        size_t e = p;
        while (e < n && buf[e] != '\n' && buf[e] != '\r') ++e;
        size_t next = e;
        if (next < n) next += (buf[next] == '\r' && next + 1 < n && buf[next + 1] == '\n') ? 2 : 1;
        if (first) {
            if (e == p || buf[p] != '>') return -1;
            first = false;
        } else if (e > p && buf[p] == '>') {
            offsets.push_back(bases.size());
        } else {
            for (size_t q = p; q < e; ++q) {
                char ch = buf[q];
                if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
                bases.push_back(ch);
            }
        }
        p = next;
    }
    offsets.push_back(bases.size());
    return 0;
}

// BioLibs.readHOXD (BioLibs.scala:66-114): title line, column header line, then
// "X,v,v,v,v" rows; cost[A][B] with A/B in A0 C1 G2 T3.  Returns 0 or -1.
int read_hoxd(const char *path, int32_t cost[16]) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    std::vector<std::string> lines;
    std::string cur;
    int ch;
    while ((ch = fgetc(f)) != EOF) {
        if (ch == '\n' || ch == '\r') {
            lines.push_back(cur);
            cur.clear();
            if (ch == '\r') { int c2 = fgetc(f); if (c2 != '\n' && c2 != EOF) ungetc(c2, f); }
        } else cur.push_back((char)ch);
    }
    if (!cur.empty()) lines.push_back(cur);
    fclose(f);
    auto split = [](const std::string &s) {
        std::vector<std::string> out;
        std::string t;
        for (char c : s) { if (c == ',') { out.push_back(t); t.clear(); } else t.push_back(c); }
        out.push_back(t);
        return out;
    };
    auto trim_first = [](const std::string &s) -> int {
        size_t i = 0;
        while (i < s.size() && (unsigned char)s[i] <= ' ') ++i;
        if (i >= s.size()) return -1;
        char c = s[i];
        if (c >= 'a' && c <= 'z') c = (char)(c - 32);
        switch (c) { case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3; default: return -1; }
    };
    if (lines.size() < 2) return -1;
    const std::vector<std::string> col = split(lines[1]);
    for (size_t li = 2; li < lines.size() && !lines[li].empty(); ++li) {
        const std::vector<std::string> row = split(lines[li]);
        for (size_t i = 1; i < row.size(); ++i) {
            const int A = trim_first(row[0]);
            if (i >= col.size()) return -1;
            const int B = trim_first(col[i]);
            if (A < 0 || B < 0) return -1;  // MatchError
            char *end = nullptr;
            const long v = strtol(row[i].c_str(), &end, 10);  // Integer.parseInt
            if (end == row[i].c_str() || *end != 0) return -1;
            cost[A * 4 + B] = (int32_t)v;
        }
    }
    return 0;
}

}  // namespace sa
