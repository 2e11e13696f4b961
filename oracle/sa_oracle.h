/*
 * sa_oracle.h -- CPU restatement of the reference hash-overlap path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may link or call it,
 * and only as the checker / CPU baseline -- never as the product path.
 *
 * It restates, single-threaded and in plain C99 with IEEE float32 arithmetic
 * (build with -ffp-contract=off, no fast-math):
 *   BioLibs.scala:26-61        readSeq, generateKmerSet
 *   BioLibs.scala:119-161      defaultHOXD
 *   BioLibs.scala:267-368      generateLocalAlignmentSet (--quadratic-align, per pair)
 *   BioLibs.scala:596-822      generateFastDovetailAlignmentSet (per pair)
 *   KmerTable.scala:41-187     addKmerSet, addKmerPair, calcPairData, calcDispatchData
 *   KmerTable.scala:246-273    dispatchCollisionBlocks
 *   ObjectStore.scala:17-142   AlignSettings, Kmer.seqHash, Alignment, Overlap
 *   Project4.scala:725-825     genBlockMTAlign (filter=true), calcOverlaps
 *   lib/trove.jar              TIntObjectHashMap 3.0.3 slot layout & iteration order
 *
 * Parity pinning: see oracle/README.md ("partially pinned").
 */
#ifndef SA_ORACLE_H
#define SA_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORC_OK = 0,
    ORC_E_INPUT = -1,      /* readSeq: file missing / first line not '>' */
    ORC_E_NPE = -2,        /* dispatch decoded an id with no SequenceData entry (E4) */
    ORC_E_MATCH = -3,      /* HOXD closure MatchError: non-ACGT char aligned */
    ORC_E_INDEX = -4,      /* StringIndexOutOfBounds (|B| < width) or degenerate backtrack */
    ORC_E_NOMEM = -5,
    ORC_E_TROVE = -6       /* Trove table full (cannot happen at load 0.5) */
};

typedef struct {
    int32_t kmer_size;       /* -k            default 12 */
    int32_t min_overlap;     /* --min-overlap default 40 */
    int32_t max_ignore;      /* --max-ignore  default 90 (compared as Float) */
    int32_t gap_open;        /* -gO           default -200 */
    int32_t gap_extend;      /* -gE           default -20 */
    int32_t min_collisions;  /* default 7 */
    int32_t max_collisions;  /* default 222 */
    float min_identity;      /* default 0.98f */
    float kmer_edge;         /* default 0.4f */
    float kmer_center;       /* default 0.4f */
    int32_t cost[16];        /* HOXD, index a*4+b, base order A0 C1 G2 T3 */
} orc_settings;

typedef struct {
    int32_t lead, trail;     /* dispatched pair (read ids, 1-based) */
    int32_t is_dud;          /* phase-1 backtrack did not end at j==0 */
    int32_t start_i, start_j, end_i, end_j;
    int32_t correct, error;  /* c, e */
    int32_t len_a, len_b;    /* 0 for a dud (dud carries empty sequences) */
    int32_t valid;           /* Alignment.valid */
    int32_t ovl_valid;       /* Overlap.valid (implies valid) */
    int32_t ahg, bhg;
} orc_align_t;

typedef struct orc_ctx orc_ctx;

void orc_default_settings(orc_settings *s);

/* Reads: FASTA file parsed like BioLibs.readSeq, or caller buffers (already
 * upper-cased bases, read r = bases[offsets[r] .. offsets[r+1])). */
int orc_create_from_fasta(const char *path, orc_ctx **out);
int orc_create_from_buffers(const char *bases, const uint64_t *offsets, uint32_t n, orc_ctx **out);
void orc_destroy(orc_ctx *c);
uint32_t orc_num_reads(const orc_ctx *c);

/* Run the whole calc-overlaps path.  flags bit 0 (wide) = 0: reference emulation
 * with 32-bit (fst<<16)^snd keys and Trove order (E1/E4); = 1: 64-bit (fst,snd)
 * keys, canonical order (lead descending, trail ascending).  flags bit 1: stop
 * after DispatchData (candidate stage only, for the CPU baseline).  flags bit 2:
 * `--quadratic-align` (generateLocalAlignmentSet, BioLibs.scala:267-368) instead
 * of the banded dovetail aligner. */
int orc_run(orc_ctx *c, const orc_settings *s, int flags);
/* Wide-id hash stage only (flags 1 | 2 of orc_run) on `threads` OpenMP threads
 * (0 = all): same pairs / dispatch; role pairs visited -> *role_pairs.  The
 * all-core CPU baseline of the hash stage (bench.py). */
int orc_run_wide_mt(orc_ctx *c, const orc_settings *s, int threads, uint64_t *role_pairs);

/* Sampled-lead PairData rows (checker for read sets whose whole PairData does
 * not fit host memory): for each lead of `leads` (1-based, strictly ascending)
 * every PairData entry whose fst is that lead -- snd ascending, count >= 1 --
 * in (*snd_out, *cnt_out)[row_off[i] .. row_off[i + 1]).  Same semantics as
 * orc_run's wide branch (KmerTable.scala:57-149); memory is bounded by the
 * sampled leads' buckets.  Free the outputs with orc_free. */
int orc_lead_rows(const char *bases, const uint64_t *offsets, uint32_t n_reads, const orc_settings *s,
                  const int32_t *leads, size_t n_leads, int threads, uint64_t *row_off, int32_t **snd_out,
                  int32_t **cnt_out);
/* Projection statistics of the sampled leads over reads cut from one genome (read r =
 * genome[starts[r] .. starts[r] + lens[r])): per lead 4 values in stats[4 i ..] --
 * distinct partners, role pairs with fst = the lead, partials (distinct (partner,
 * owner rank) over 2^log_ranks hash-range owners, log_ranks <= 6: what the sharded
 * count of that lead writes in all) and dispatched partners.  Same semantics as
 * orc_lead_rows. */
int orc_lead_stats(const char *genome, const uint64_t *starts, const int32_t *lens, uint32_t n_reads,
                   const orc_settings *s, const int32_t *leads, size_t n_leads, int threads, int log_ranks,
                   uint64_t *stats);
/* bench.synth_workload's genome (splitmix64 `seed`, GC fraction gc) into out[n] */
void orc_synth_genome(uint64_t seed, uint64_t n, double gc, char *out, int threads);
void orc_free(void *p);

/* Results of orc_run (arrays owned by ctx, valid until destroy/next run). */
size_t orc_num_kmers(const orc_ctx *c);
void orc_kmers(const orc_ctx *c, const int32_t **hash, const int32_t **read_id,
               const float **loc);
size_t orc_num_buckets(const orc_ctx *c);
/* distinct k-mer hashes in KmerData iteration order (descending Trove slot) */
const int32_t *orc_bucket_order(const orc_ctx *c);
size_t orc_num_pairs(const orc_ctx *c);
/* PairData in iteration order (strict) or sorted (fst asc, snd asc) (wide) */
void orc_pairs(const orc_ctx *c, const int32_t **fst, const int32_t **snd, const int32_t **count);
/* strict only: distinct pair keys in first-insertion order */
void orc_pairs_first_order(const orc_ctx *c, const int32_t **fst, const int32_t **snd);
size_t orc_num_dispatch(const orc_ctx *c);
void orc_dispatch(const orc_ctx *c, const int32_t **lead, const int32_t **trail);
const orc_align_t *orc_aligns(const orc_ctx *c); /* one per dispatched pair */
/* .ovl bytes for the run (records of ovl_valid alignments, dispatch order) */
size_t orc_ovl(const orc_ctx *c, const char **text);

/* One banded dovetail alignment (BioLibs.scala:613-820 for one trailer). */
int orc_align_pair(const char *A, int32_t len_a, const char *B, int32_t len_b,
                   int32_t id_a, int32_t id_b, const orc_settings *s, orc_align_t *out);

/* The dovetail aligner over a dispatch list on `threads` OpenMP threads (0 =
 * all): the aligner leg of the CPU baseline (genBlockMTAlign's actor pool,
 * Project4.scala:725-790; pairs are independent). */
int orc_align_batch(const char *bases, const uint64_t *offsets, uint32_t n_reads, const int32_t *lead,
                    const int32_t *trail, size_t n_pairs, const orc_settings *s, int threads, orc_align_t *out);
int orc_max_threads(void);

/* One full-matrix local alignment (BioLibs.scala:267-368 for one trailer). */
int orc_align_pair_local(const char *A, int32_t len_a, const char *B, int32_t len_b,
                         int32_t id_a, int32_t id_b, const orc_settings *s, orc_align_t *out);

/* Trove emulation probe (for fixtures): capacity after inserting n distinct
 * keys in order; and the descending-slot iteration order. */
int orc_trove_order(const int32_t *keys, size_t n, int32_t *order_out, int32_t *cap_out);

#ifdef __cplusplus
}
#endif
#endif
