// cli.cpp -- `sa-overlap`, the process boundary AMOS sees.
//
// Same flags, defaults, sign normalisation and last-wins semantics as
// Project4.readArgs (Project4.scala:101-259); the default (and only supported)
// mode is calc-overlaps (Project4.scala:56-60): read FASTA -> candidates ->
// dovetail alignments -> AMOS {OVL} records to -o FILE or stdout.
// Diagnostics go to stderr so stdout stays a clean .ovl stream.
// Extra flags: --wide-ids / --strict-ids, --device N, --stats.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

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

int main(int argc, char **argv) {
    sa_settings s;
    sa_default_settings(&s);
    std::string input, output, hoxd;
    int device = 0;
    bool stats = false;
    int aligner = SA_ALIGNER_LINEAR;
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
                 a == "--block-align" || a == "--single-align" || a == "--calc-overlaps" ||
                 a == "--sleep-for-debug") {
            // threading / dispatch variants give identical results and order
        } else if (a == "--linear-align") aligner = SA_ALIGNER_LINEAR;  // fdAlign = true (:190-192)
        else if (a == "--debug") stats = true;
        else if (a == "--quadratic-align") aligner = SA_ALIGNER_QUADRATIC;  // fdAlign = false (:187-189)
        else if (a.rfind("--test-", 0) == 0 || a.rfind("--bench-", 0) == 0) {
            fprintf(stderr, "%s: developer test/bench modes are out of scope; use bench.py\n", a.c_str());
            return 1;
        } else if (a == "--wide-ids") s.id_mode = SA_IDS_WIDE;
        else if (a == "--strict-ids") s.id_mode = SA_IDS_STRICT;
        else if (a == "--device") { need(&iv, nullptr); device = iv; }
        else if (a == "--stats") stats = true;
        else {
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
    sa_ctx *ctx = nullptr;
    int rc = sa_ctx_create(&s, device, &ctx);
    if (rc != SA_OK) {
        fprintf(stderr, "sa-overlap: no usable gfx950 device (%d)\n", rc);
        return 1;
    }
    rc = sa_set_option(ctx, SA_OPT_ALIGNER, aligner);
    if (rc == SA_OK && (rc = sa_read_fasta(ctx, input.c_str())) == SA_OK && (rc = sa_build_candidates(ctx)) == SA_OK &&
        (rc = sa_align(ctx)) == SA_OK) {
        rc = sa_write_ovl(ctx, output.empty() ? nullptr : output.c_str());
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
