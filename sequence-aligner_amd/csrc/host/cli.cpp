// cli.cpp -- `sa-overlap`, the process boundary AMOS sees.
//
// Same flags, defaults, sign normalisation and last-wins semantics as
// Project4.readArgs (Project4.scala:101-259); the default mode is
// calc-overlaps (Project4.scala:56-60): read FASTA -> candidates -> dovetail
// (or --quadratic-align) alignments -> AMOS {OVL} records to -o FILE or stdout.
// The developer modes (--test-* / --bench-*, :61-98) print what Project4
// prints, except --test-alignment / --test-overlaps (alignment strings).
// Diagnostics go to stderr so stdout stays a clean .ovl stream.
// Extra flags: --wide-ids / --strict-ids, --device N, --stats,
// --afg FILE [--afg-quality Q] [--afg-header-eids] (also an AMOS message file:
// the reads as {RED} messages, eid = the read ordinal as in the reference's
// c_ruddii bank map, or with --afg-header-eids the FASTA header's first word --
// which of the two toAmos_new writes is parity unpinned, INTEGRATION.md;
// then the {OVL} records --
// toAmos_new + bank-transact -m in one file),
// --gpus P (one process over devices 0..P-1, one shard each, RCCL exchanges;
// SURVEY.md 8(b)) and --shards S (S virtual shards on one device: the sharded
// path on one GPU).  The output is identical for any P and S.
#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "../../../include/sa_overlap.h"

static int parse_int(const char *s, int32_t *out) {  // Integer.parseInt
    if (!s || !*s) return -1;
    char *end = nullptr;
    const long long v = strtoll(s, &end, 10);
    if (*end != 0 || v < INT32_MIN || v > INT32_MAX) return -1;
    *out = (int32_t)v;
    return 0;
}
static int parse_float(const char *s, float *out) {  // Float.parseFloat
    if (!s || !*s) return -1;
    char *end = nullptr;
    const float v = strtof(s, &end);
    while (*end == ' ' || *end == '\t') ++end;
    if (*end == 'f' || *end == 'F' || *end == 'd' || *end == 'D') ++end;
    if (*end != 0) return -1;
    *out = v;
    return 0;
}
static int32_t iabs(int32_t v) { return v < 0 ? -v : v; }  // math.abs(Int) (wraps at MinValue like the JVM)

// ---------------------------------------------------------------------------
// The reference's developer modes (Project4.scala:61-98, bodies :272-504),
// printing what Project4 prints to stdout.  Timings are wall-clock around the
// device calls.
// ---------------------------------------------------------------------------
static double now_ms() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

// java.lang.Float.toString: the shortest decimal that reads back as the same
// float; plain notation in [1e-3, 1e7), else d.dddE<exp>; always a fraction digit
static std::string java_float(float f) {
    if (f != f) return "NaN";
    if (f == 0) return signbit(f) ? "-0.0" : "0.0";
    if (isinf(f)) return f > 0 ? "Infinity" : "-Infinity";
    char buf[64];
    for (int prec = 1; prec <= 9; ++prec) {
        snprintf(buf, sizeof(buf), "%.*e", prec - 1, (double)f);
        if (strtof(buf, nullptr) == f) break;
    }
    std::string m = buf, sign;
    if (m[0] == '-') { sign = "-"; m = m.substr(1); }
    const size_t epos = m.find('e');
    const int ex = atoi(m.c_str() + epos + 1);
    std::string digits;
    for (size_t i = 0; i < epos; ++i)
        if (m[i] != '.') digits.push_back(m[i]);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    const float a = fabsf(f);
    std::string out;
    if (a >= 1e-3f && a < 1e7f) {
        if (ex >= 0) {
            std::string ip = digits.substr(0, std::min<size_t>(digits.size(), (size_t)ex + 1));
            while ((int)ip.size() < ex + 1) ip.push_back('0');
            const std::string fp = (int)digits.size() > ex + 1 ? digits.substr((size_t)ex + 1) : "0";
            out = ip + "." + fp;
        } else {
            out = "0." + std::string((size_t)(-ex - 1), '0') + digits;
        }
    } else {
        out = digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "E" + std::to_string(ex);
    }
    return sign + out;
}

// FASTA header names in read order, under read_fasta's line rules (fasta.cpp):
// every '>' line opens a read; its eid is the text up to the first blank
static std::vector<std::string> fasta_eids(const std::string &path) {
    std::vector<std::string> out;
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return out;
    std::string line;
    int ch;
    bool more = true;
    while (more) {
        line.clear();
        while ((ch = fgetc(f)) != EOF && ch != '\n' && ch != '\r') line.push_back((char)ch);
        if (ch == '\r') {
            const int nx = fgetc(f);
            if (nx != '\n' && nx != EOF) ungetc(nx, f);
        }
        more = ch != EOF;
        if (!line.empty() && line[0] == '>') {
            size_t e = 1;
            while (e < line.size() && !isspace((unsigned char)line[e])) ++e;
            out.push_back(line.substr(1, e - 1));
        }
    }
    fclose(f);
    return out;
}

// --gpus / --shards: a sharded context (sa_ctx_create_multi) or one device
static int g_gpus = 1, g_shards = 1;
static int new_ctx(const sa_settings *s, int device, sa_ctx **ctx) {
    if (g_gpus > 1) return sa_ctx_create_multi(s, g_gpus, g_gpus, ctx);
    if (g_shards > 1) return sa_ctx_create_multi(s, 1, g_shards, ctx);
    return sa_ctx_create(s, device, ctx);
}

static void die_ctx(sa_ctx *ctx, int rc) {
    fprintf(stderr, "sa-overlap: %s (%d)\n", ctx ? sa_last_error(ctx) : "error", rc);
    if (ctx) sa_ctx_destroy(ctx);
    exit(1);
}

static sa_ctx *open_ctx(const sa_settings &s, int device, const std::string &input, int aligner) {
    sa_ctx *ctx = nullptr;
    const int rc0 = new_ctx(&s, device, &ctx);
    if (rc0 != SA_OK) {
        fprintf(stderr, "sa-overlap: no usable gfx950 device (%d)\n", rc0);
        exit(1);
    }
    int rc = sa_set_option(ctx, SA_OPT_ALIGNER, aligner);
    if (rc == SA_OK) rc = sa_read_fasta(ctx, input.c_str());
    if (rc != SA_OK) die_ctx(ctx, rc);
    return ctx;
}

// Project4.testFastaRead (:272-285): the first 10 sequences, then exit
static int mode_test_fasta_read(const sa_settings &s, int device, const std::string &input) {
    sa_ctx *ctx = open_ctx(s, device, input, SA_ALIGNER_LINEAR);
    printf("\n");
    const uint32_t n = sa_num_reads(ctx);
    for (uint32_t id = 1; id <= n && id <= 10; ++id) {
        const char *seq;
        size_t len;
        sa_get_read(ctx, id, &seq, &len);
        printf("id : %u\nseq: %.*s\n\n", id, (int)len, seq);
    }
    sa_ctx_destroy(ctx);
    return 0;
}

// Project4.benchFastaRead (:288-296)
static int mode_bench_fasta_read(const sa_settings &s, int device, const std::string &input) {
    sa_ctx *ctx = nullptr;
    if (new_ctx(&s, device, &ctx) != SA_OK) {
        fprintf(stderr, "sa-overlap: no usable gfx950 device\n");
        return 1;
    }
    const double t0 = now_ms();
    const int rc = sa_read_fasta(ctx, input.c_str());
    const double t1 = now_ms();
    if (rc != SA_OK) die_ctx(ctx, rc);
    printf(" Read %u sequences from %s in %lld milliseconds.\n", sa_num_reads(ctx), input.c_str(),
           (long long)(t1 - t0));
    sa_ctx_destroy(ctx);
    return 0;
}

// Project4.testKmerCover (:299-320): uniques, ratio to 4^k and the bucket-size
// histogram for k = 0 .. 25 (KmerTable.uniqueKmers / kmerCollisionHistogram)
static int mode_test_kmer_cover(sa_settings s, int device, const std::string &input) {
    for (int k = 0; k <= 25; ++k) {
        uint64_t uniques = 0;
        std::vector<std::pair<uint64_t, uint64_t>> hist;
        if (k == 0) {
            // every k-mer is "" (seqHash 0): one bucket of sum(L + 1) occurrences
            sa_settings s1 = s;
            s1.kmer_size = 1;
            sa_ctx *ctx = open_ctx(s1, device, input, SA_ALIGNER_LINEAR);
            uint64_t total = 0;
            for (uint32_t id = 1; id <= sa_num_reads(ctx); ++id) {
                const char *seq;
                size_t len;
                sa_get_read(ctx, id, &seq, &len);
                total += len + 1;
            }
            sa_ctx_destroy(ctx);
            if (total) { uniques = 1; hist.push_back({total, 1}); }
        } else {
            s.kmer_size = k;
            sa_ctx *ctx = open_ctx(s, device, input, SA_ALIGNER_LINEAR);
            const uint64_t *sz, *ct;
            size_t n;
            const int rc = sa_kmer_histogram(ctx, &uniques, &sz, &ct, &n);
            if (rc != SA_OK) die_ctx(ctx, rc);
            for (size_t i = 0; i < n; ++i) hist.push_back({sz[i], ct[i]});
            sa_ctx_destroy(ctx);
        }
        const double possible = pow(4.0, k);
        const float ratio = (float)(int32_t)uniques / (float)possible;
        printf("Kmer Size : %d\n", k);
        printf("  uniques : %llu\n", (unsigned long long)uniques);
        printf("  ratio   : %s\n", java_float(ratio).c_str());
        printf("  [ number of collisions -> count of seqs with that many collisions ] :\n");
        for (auto &h : hist) printf("          [%llu -> %llu]\n", (unsigned long long)h.first, (unsigned long long)h.second);
        printf("\n");
    }
    return 0;
}

// Project4.testDispatchCollisions / testBlockDispatch (:376-421): every
// dispatched pair in dispatch order (DispatchData lists hold distinct trails,
// so the reference's duplicate warning never fires), then the block histogram
static int mode_test_dispatch(const sa_settings &s, int device, const std::string &input, bool blocks) {
    sa_ctx *ctx = open_ctx(s, device, input, SA_ALIGNER_LINEAR);
    int rc = sa_build_candidates(ctx);
    if (rc != SA_OK) die_ctx(ctx, rc);
    const int32_t *lead, *trail, *count;
    size_t n;
    sa_get_dispatch(ctx, &lead, &trail, &count, &n);
    std::vector<std::pair<size_t, uint64_t>> hist;  // block size -> number of blocks
    size_t i = 0;
    while (i < n) {
        size_t j = i;
        while (j < n && lead[j] == lead[i]) {
            printf(" Dispatched Coll : %zu - %d <-> %d\n", j + 1, lead[j], trail[j]);
            ++j;
        }
        const size_t bs = j - i;
        auto it = std::lower_bound(hist.begin(), hist.end(), std::make_pair(bs, (uint64_t)0));
        if (it != hist.end() && it->first == bs) ++it->second;
        else hist.insert(it, {bs, 1});
        i = j;
    }
    if (blocks) {
        printf("\n Histogram Of Relations : [Number of Aligns -> Number of Seqs w/ that many Aligns]\n");
        for (auto &h : hist) printf("          [%zu -> %llu]\n", h.first, (unsigned long long)h.second);
        printf("\n");
    }
    sa_ctx_destroy(ctx);
    return 0;
}

// Project4.benchKmerGen / benchKmerAnalysis (:324-373)
static int mode_bench_kmer(const sa_settings &s, int device, const std::string &input, bool analysis) {
    if (!analysis) {
        for (int pass = 0; pass < 2; ++pass) {  // "sequentially", "in parellel": one device path
            sa_ctx *ctx = nullptr;
            if (new_ctx(&s, device, &ctx) != SA_OK) {
                fprintf(stderr, "sa-overlap: no usable gfx950 device\n");
                return 1;
            }
            const double t0 = now_ms();
            int rc = sa_read_fasta(ctx, input.c_str());
            uint64_t uniques = 0;
            const uint64_t *sz, *ct;
            size_t n;
            if (rc == SA_OK) rc = sa_kmer_histogram(ctx, &uniques, &sz, &ct, &n);
            const double t1 = now_ms();
            if (rc != SA_OK) die_ctx(ctx, rc);
            printf(pass == 0 ? "\nGenerated %llu unique kmers from %u sequences from %s sequentially in %lld milliseconds.\n\n"
                             : "Generated %llu unique kmers from %u sequences from %s in parellel in %lld milliseconds.\n\n",
                   (unsigned long long)uniques, sa_num_reads(ctx), input.c_str(), (long long)(t1 - t0));
            sa_ctx_destroy(ctx);
        }
        return 0;
    }
    printf("Starting kmer gen.\n");
    sa_ctx *ctx = open_ctx(s, device, input, SA_ALIGNER_LINEAR);
    sa_set_option(ctx, SA_OPT_TIMING, 1);
    printf("Finished kmer gen.\n");
    const double t0 = now_ms();
    const int rc = sa_build_candidates(ctx);
    const double t1 = now_ms();
    if (rc != SA_OK) die_ctx(ctx, rc);
    double ms[SA_NUM_STAGES];
    sa_get_stage_times(ctx, ms, nullptr, SA_NUM_STAGES);
    // calcPairData ~ everything up to the counted pairs, calcDispatchData ~ ordering
    const double disp = ms[SA_STAGE_ORDER];
    printf("\nCalculated pair data in %lld milliseconds.\n\n", (long long)(t1 - t0 - disp));
    printf("Calculated dispatch data in %lld milliseconds.\n\n", (long long)disp);
    sa_ctx_destroy(ctx);
    return 0;
}

// Project4.benchAlign / benchAlignQuick (:444-481): filter = false, so every
// dispatched pair counts.  The quick variant sets debugStop = 500, and the
// reference's guard `(debugStop < 0) || (aligns.size > debugStop)` then never
// lets a pair through: it reports 0 alignments, as here.
static int mode_bench_align(const sa_settings &s, int device, const std::string &input, bool quick) {
    static const char *names[8] = {"single threaded quad single", "single threaded quad block",
                                   "multi threaded quad single", "multi threaded quad block",
                                   "single threaded linear single", "single threaded linear block",
                                   "multi threaded linear single", "multi threaded linear block"};
    sa_ctx *ctx = open_ctx(s, device, input, SA_ALIGNER_LINEAR);
    int rc = sa_build_candidates(ctx);
    if (rc != SA_OK) die_ctx(ctx, rc);
    for (int v = 0; v < 8; ++v) {
        size_t n = 0;
        const double t0 = now_ms();
        if (!quick) {
            rc = sa_set_option(ctx, SA_OPT_ALIGNER, v < 4 ? SA_ALIGNER_QUADRATIC : SA_ALIGNER_LINEAR);
            if (rc == SA_OK) rc = sa_align(ctx);
            if (rc != SA_OK) {
                printf("\n%c%s Alignment Benchmark Failed : \n\n\n%s\n", (char)toupper(names[v][0]), names[v] + 1,
                       sa_last_error(ctx));
                continue;
            }
            const sa_alignment *al;
            sa_get_alignments(ctx, &al, &n);
        }
        const double t1 = now_ms();
        printf("\nCalculated %zu %s alignments in %lld milliseconds.\n\n", n, names[v], (long long)(t1 - t0));
    }
    sa_ctx_destroy(ctx);
    return 0;
}

int main(int argc, char **argv) {
    sa_settings s;
    sa_default_settings(&s);
    std::string input, output, hoxd, afg;
    int afg_quality = 20;
    bool afg_header_eids = false;
    int device = 0;
    bool stats = false;
    int aligner = SA_ALIGNER_LINEAR;
    std::string action = "calc-overlaps";
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto need = [&](int32_t *iv, float *fv) -> bool {
            if (i + 1 >= argc) {
                fprintf(stderr, "Missing value for %s\n", a.c_str());
                exit(1);
            }
            const char *v = argv[++i];
            if (iv && parse_int(v, iv) == 0) return true;
            if (fv && parse_float(v, fv) == 0) return true;
            fprintf(stderr, "Invalid value for %s : %s\n", a.c_str(), v);
            exit(1);
        };
        auto str = [&]() -> std::string {
            if (i + 1 >= argc) { fprintf(stderr, "Missing value for %s\n", a.c_str()); exit(1); }
            return std::string(argv[++i]);
        };
        int32_t iv;
        float fv;
        if (a == "-h" || a == "--help") {
            printf(" Rohit Ramesh :         Cmsc 423 \n Project 4 : Sequence Overlapper \n"
                   "                                 \n [Usage]                         \n"
                   "   See README file for details   \n");
            return 0;
        } else if (a == "-m" || a == "--matrix" || a == "-H" || a == "--HOXD-matrix") hoxd = str();
        else if (a == "-k" || a == "--kmer-size") { need(&iv, nullptr); s.kmer_size = iv; }
        else if (a == "-i" || a == "--input") input = str();
        else if (a == "-o" || a == "--output") output = str();
        else if (a == "--match") need(&iv, nullptr);      // parsed, never used (Project4.scala:243)
        else if (a == "--mismatch") need(&iv, nullptr);   // parsed, never used
        else if (a == "--min-overlap") { need(&iv, nullptr); s.min_overlap = iabs(iv); }
        else if (a == "--min-identity") {
            need(nullptr, &fv);
            if (fv >= 1) fv *= .01f;  // Project4.scala:143-146
            s.min_identity = fv;
        } else if (a == "--min-collisions") { need(&iv, nullptr); s.min_collisions = iabs(iv); }
        else if (a == "--max-collisions") { need(&iv, nullptr); s.max_collisions = iabs(iv); }
        else if (a == "--kmer-center") { need(nullptr, &fv); s.kmer_center = fabsf(fv); }
        else if (a == "--kmer-edge") { need(nullptr, &fv); s.kmer_edge = fabsf(fv); }
        else if (a == "-gO" || a == "--gap-open") { need(&iv, nullptr); s.gap_open = -iabs(iv); }
        else if (a == "-gE" || a == "--gap-extend") { need(&iv, nullptr); s.gap_extend = -iabs(iv); }
        else if (a == "--max-ignore") { need(&iv, nullptr); s.max_ignore = iabs(iv); }
        else if (a == "--st-hash" || a == "--mt-hash" || a == "--st-align" || a == "--mt-align" ||
                 a == "--block-align" || a == "--single-align" ||
                 a == "--sleep-for-debug") {
            // threading / dispatch variants give identical results and order
        } else if (a == "--linear-align") aligner = SA_ALIGNER_LINEAR;  // fdAlign = true (:190-192)
        else if (a == "--calc-overlaps") action = "calc-overlaps";
        else if (a == "--debug") stats = true;
        else if (a == "--quadratic-align") aligner = SA_ALIGNER_QUADRATIC;  // fdAlign = false (:187-189)
        else if (a == "--test-fasta-read" || a == "--bench-fasta-read" || a == "--test-kmer-cover" ||
                 a == "--test-dispatch-collisions" || a == "--test-block-dispatch" || a == "--bench-kmer-gen" ||
                 a == "--bench-kmer-analysis" || a == "--bench-align" || a == "--bench-align-quick" ||
                 a == "--test-alignment" || a == "--test-overlaps") {
            action = a.substr(2);  // last wins, like Project4's `action`
        } else if (a == "--wide-ids") s.id_mode = SA_IDS_WIDE;
        else if (a == "--strict-ids") s.id_mode = SA_IDS_STRICT;
        else if (a == "--device") { need(&iv, nullptr); device = iv; }
        else if (a == "--gpus" || a == "--shards") {
            need(&iv, nullptr);
            if (iv < 1 || iv > 256 || (iv & (iv - 1))) {
                fprintf(stderr, "Invalid value for %s : %d (a power of two <= 256)\n", a.c_str(), iv);
                return 1;
            }
            (a == "--gpus" ? g_gpus : g_shards) = iv;
        }
        else if (a == "--stats") stats = true;
        else if (a == "--afg") afg = str();
        else if (a == "--afg-header-eids") afg_header_eids = true;
        else if (a == "--afg-quality") {
            need(&iv, nullptr);
            if (iv < 0 || iv > 60) {
                fprintf(stderr, "Invalid value for %s : %d (0..60)\n", a.c_str(), iv);
                return 1;
            }
            afg_quality = iv;
        } else {
            fprintf(stderr, "Invalid Argument : %s\nExiting Program.\n", a.c_str());
            return 1;
        }
    }
    if (!hoxd.empty() && sa_load_hoxd(&s, hoxd.c_str()) != SA_OK) {
        fprintf(stderr, "Cannot read HOXD matrix %s\n", hoxd.c_str());
        return 1;
    }
    if (input.empty()) {
        fprintf(stderr, "No input file specified\n");
        return 255;  // System.exit(-1)
    }
    if (action == "test-fasta-read") return mode_test_fasta_read(s, device, input);
    if (action == "bench-fasta-read") return mode_bench_fasta_read(s, device, input);
    if (action == "test-kmer-cover") return mode_test_kmer_cover(s, device, input);
    if (action == "test-dispatch-collisions") return mode_test_dispatch(s, device, input, false);
    if (action == "test-block-dispatch") return mode_test_dispatch(s, device, input, true);
    if (action == "bench-kmer-gen") return mode_bench_kmer(s, device, input, false);
    if (action == "bench-kmer-analysis") return mode_bench_kmer(s, device, input, true);
    if (action == "bench-align") return mode_bench_align(s, device, input, false);
    if (action == "bench-align-quick") return mode_bench_align(s, device, input, true);
    if (action == "test-alignment" || action == "test-overlaps") {
        // these print alignA / alignB strings, which the device path never builds
        fprintf(stderr, "--%s: alignment strings are not materialised by this build\n", action.c_str());
        return 1;
    }
    sa_ctx *ctx = nullptr;
    int rc = new_ctx(&s, device, &ctx);
    if (rc != SA_OK) {
        fprintf(stderr, "sa-overlap: no usable gfx950 device (%d)\n", rc);
        return 1;
    }
    rc = sa_set_option(ctx, SA_OPT_ALIGNER, aligner);
    if (rc == SA_OK && (rc = sa_read_fasta(ctx, input.c_str())) == SA_OK && (rc = sa_build_candidates(ctx)) == SA_OK &&
        (rc = sa_align(ctx)) == SA_OK) {
        rc = sa_write_ovl(ctx, output.empty() ? nullptr : output.c_str());
    }
    if (rc == SA_OK && !afg.empty()) {
        // default eid = ordinal (the only bank the reference holds maps iid = bid =
        // eid = ordinal, amos/c_ruddii.bnk/RED.0.map -- which cannot tell ordinals
        // from header words, its .seq being a missing blob: the eid rule is parity
        // unpinned either way); header names are opt-in
        const std::vector<std::string> names = afg_header_eids ? fasta_eids(input) : std::vector<std::string>();
        std::vector<const char *> eids(sa_num_reads(ctx), nullptr);
        for (size_t i = 0; i < eids.size() && i < names.size(); ++i) eids[i] = names[i].c_str();
        rc = sa_write_afg(ctx, afg.c_str(), afg_header_eids ? eids.data() : nullptr, afg_quality);
    }
    if (rc != SA_OK) {
        fprintf(stderr, "sa-overlap: %s (%d)\n", sa_last_error(ctx), rc);
        sa_ctx_destroy(ctx);
        return 1;
    }
    if (stats) {
        sa_stats st;
        sa_get_stats(ctx, &st);
        fprintf(stderr,
                "reads %u kmers %llu buckets %llu role_pairs %llu pairs %llu dispatched %llu aligned %llu "
                "ovl %llu cells %llu ids %s\n",
                sa_num_reads(ctx), (unsigned long long)st.kmers, (unsigned long long)st.buckets,
                (unsigned long long)st.role_pairs, (unsigned long long)st.pairs, (unsigned long long)st.dispatched,
                (unsigned long long)st.aligned, (unsigned long long)st.ovl_records, (unsigned long long)st.dp_cells,
                st.id_mode == SA_IDS_STRICT ? "strict" : "wide");
    }
    sa_ctx_destroy(ctx);
    return 0;
}
