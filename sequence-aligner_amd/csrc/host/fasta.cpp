// fasta.cpp -- BioLibs.readSeq (BioLibs.scala:26-50) on the host.
//
// java.io.BufferedReader.readLine splits on "\n", "\r" and "\r\n"; the first
// line must start with '>' (else "Invalid Sequence File"); every later '>' line
// closes the current sequence (even an empty one); other lines are appended;
// the sequence is upper-cased; ids are the ordinals 1..N.
#include <string.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

namespace sa {

int read_fasta(const char *path, std::vector<char> &bases, std::vector<uint64_t> &offsets) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    // the whole file in one read (then whatever a pipe or a growing file still holds)
    std::vector<char> buf;
    if (fseeko(f, 0, SEEK_END) == 0) {
        const off_t sz = ftello(f);
        if (sz > 0) buf.resize((size_t)sz);
        if (fseeko(f, 0, SEEK_SET) != 0) buf.clear();
    }
    buf.resize(buf.empty() ? 0 : fread(buf.data(), 1, buf.size(), f));
    {
        char tmp[1 << 16];
        size_t got;
        while ((got = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    }
    fclose(f);
    const size_t n = buf.size();
    if (n == 0) return -1;  // in.readLine() == null -> NPE on line.startsWith
    bases.resize(n);  // (an upper bound; trimmed below)
    offsets.assign(1, 0);
    const char *B = buf.data();
    char *D = bases.data();
    size_t nb = 0, p = 0;
    bool first = true;
    while (p < n) {
        // the line [p, e) and the start of the next: "\n", "\r" and "\r\n" end a line
        const char *nl = (const char *)memchr(B + p, '\n', n - p);
        size_t e = nl ? (size_t)(nl - B) : n;
        size_t next = nl ? e + 1 : n;
        if (const char *cr = (const char *)memchr(B + p, '\r', e - p)) {
            e = (size_t)(cr - B);
            next = e + ((e + 1 < n && B[e + 1] == '\n') ? 2 : 1);
        }
        if (first) {
            if (e == p || B[p] != '>') return -1;
            first = false;
        } else if (e > p && B[p] == '>') {
            offsets.push_back(nb);
        } else {  // sequence text, upper-cased (toUpperCase)
            char *d = D + nb;
            const size_t len = e - p;
            memcpy(d, B + p, len);
            for (size_t q = 0; q < len; ++q) d[q] = (char)(d[q] - ((d[q] >= 'a' && d[q] <= 'z') ? 32 : 0));
            nb += len;
        }
        p = next;
    }
    bases.resize(nb);
    offsets.push_back(nb);
    return 0;
}

// BioLibs.readHOXD (BioLibs.scala:66-114), with the JVM's semantics: the
// matrix starts zeroed (Array.ofDim(4,4), :68); BufferedReader.readLine line
// splitting (\n, \r, \r\n); the title line is skipped, the second line is the
// column header; rows follow until EOF or an empty line.  String.split(",")
// drops trailing empty fields; row(0).trim().charAt(0) / col(i).trim().charAt(0)
// pick A / B (A0 C1 G2 T3, MatchError otherwise); Integer.parseInt(row(i)) takes
// an optional sign and decimal digits only (no blanks) in the int32 range.
// Anything the reference would die on (NPE, StringIndexOutOfBounds,
// ArrayIndexOutOfBounds, MatchError, NumberFormatException) returns -1 and
// leaves cost[] untouched; on success all 16 entries are replaced.
namespace {
std::vector<std::string> java_split_comma(const std::string &s) {
    if (s.empty()) return {std::string()};  // no match: the whole (empty) string
    std::vector<std::string> out;
    std::string t;
    for (char c : s) {
        if (c == ',') { out.push_back(t); t.clear(); } else t.push_back(c);
    }
    out.push_back(t);
    while (!out.empty() && out.back().empty()) out.pop_back();  // trailing empty strings removed
    return out;
}

int java_base_of(const std::string &s) {  // s.trim().charAt(0).toUpper match {A,C,G,T}
    size_t b = 0, e = s.size();
    while (b < e && (unsigned char)s[b] <= ' ') ++b;
    while (e > b && (unsigned char)s[e - 1] <= ' ') --e;
    if (b >= e) return -1;  // charAt(0) of ""
    char c = s[b];
    if (c >= 'a' && c <= 'z') c = (char)(c - 32);
    switch (c) { case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3; default: return -1; }
}

bool java_parse_int(const std::string &s, int32_t *out) {  // Integer.parseInt(s, 10)
    size_t i = 0;
    bool neg = false;
    if (i < s.size() && (s[i] == '-' || s[i] == '+')) { neg = s[i] == '-'; ++i; }
    if (i >= s.size()) return false;
    int64_t v = 0;
    for (; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9') return false;
        v = v * 10 + (s[i] - '0');
        if (v > (int64_t)2147483648LL) return false;
    }
    if (neg) v = -v;
    if (v < INT32_MIN || v > INT32_MAX) return false;
    *out = (int32_t)v;
    return true;
}
}  // namespace

int read_hoxd(const char *path, int32_t cost[16]) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    std::vector<std::string> lines;  // BufferedReader.readLine
    std::string cur;
    bool pending = false;
    int ch;
    while ((ch = fgetc(f)) != EOF) {
        if (ch == '\n' || ch == '\r') {
            lines.push_back(cur);
            cur.clear();
            pending = false;
            if (ch == '\r') { int c2 = fgetc(f); if (c2 != '\n' && c2 != EOF) ungetc(c2, f); }
        } else { cur.push_back((char)ch); pending = true; }
    }
    if (pending) lines.push_back(cur);
    fclose(f);
    if (lines.size() < 2) return -1;  // readLine() == null -> .split: NullPointerException
    int32_t m[16] = {0};
    const std::vector<std::string> col = java_split_comma(lines[1]);
    for (size_t li = 2; li < lines.size() && !lines[li].empty(); ++li) {
        const std::vector<std::string> row = java_split_comma(lines[li]);
        for (size_t i = 1; i < row.size(); ++i) {
            const int A = java_base_of(row[0]);
            if (A < 0) return -1;
            if (i >= col.size()) return -1;  // ArrayIndexOutOfBounds
            const int B = java_base_of(col[i]);
            if (B < 0) return -1;
            int32_t v;
            if (!java_parse_int(row[i], &v)) return -1;  // NumberFormatException
            m[A * 4 + B] = v;
        }
    }
    memcpy(cost, m, sizeof(m));
    return 0;
}

}  // namespace sa
