/*
 * sa_overlap.h -- C ABI of the MI355X hash-overlap stage (libsa_overlap.so).
 *
 * Drop-in boundary for the reference's hot path (rohit507/Sequence-Aligner):
 *   KmerTable.scala   k-mer hashing, edge<->middle candidate-pair counting, filter
 *   BioLibs.scala     banded HOXD dovetail alignment (generateFastDovetailAlignmentSet)
 *   Project4.scala    calc-overlaps driver and AMOS .ovl writer
 * Plain pointers and sizes only; no torch or HIP types cross this boundary.
 * Each entry point names the reference interface it replaces (file:line,
 * /root/reference/src/...).  INTEGRATION.md shows the JNI / ctypes bindings.
 *
 * Ownership: the library owns device buffers and every array it returns by
 * pointer (valid until the next call on the same context or sa_ctx_destroy);
 * the caller owns its inputs.  One context per host thread.
 * Errors: every int-returning call returns SA_OK (0) or a negative SA_E_* code;
 * sa_last_error() gives the message.  The HIP path is the only compute path:
 * without a usable gfx950 device, sa_ctx_create fails with SA_E_HIP.
 */
#ifndef SA_OVERLAP_H
#define SA_OVERLAP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SA_ABI_VERSION 2

enum sa_status {
    SA_OK = 0,
    SA_E_ARG = -1,         /* bad argument / flag (Project4.readArgs exit 1) */
    SA_E_INPUT = -2,       /* unreadable FASTA / first line not '>' (BioLibs.scala:32-33) */
    SA_E_NON_ACGT = -3,    /* non-ACGT base reached the HOXD cost closure (BioLibs.scala:142-160 MatchError) */
    SA_E_ID_RANGE = -4,    /* strict ids: a dispatched id does not survive the 16-bit key packing (KmerTable.scala:73,169-170) */
    SA_E_SHORT_READ = -5,  /* |B| < band width: B.charAt(j-1) out of range (BioLibs.scala:648) */
    SA_E_DEGENERATE = -6,  /* no positive phase-1 cell: backtrack leaves the matrix (BioLibs.scala:679-689) */
    SA_E_HIP = -7,         /* HIP runtime failure or no gfx950 device */
    SA_E_NOMEM = -8,
    SA_E_RCCL = -9,
    SA_E_STATE = -10,      /* call out of order (e.g. sa_align before sa_build_candidates) */
    SA_E_OVERFLOW = -11    /* a size limit of this implementation was exceeded */
};

/* Id policy.  STRICT reproduces the reference's 32-bit
 * (fst<<16)^snd PairData keys and its GNU Trove iteration order, so the .ovl is
 * byte-identical; it is defined for < 32,768 reads (the reference crashes
 * beyond).  WIDE keys pairs by two 32-bit ids and orders records canonically
 * (lead descending, trail ascending).  AUTO = STRICT below 32,768 reads, else WIDE. */
enum sa_id_mode { SA_IDS_AUTO = 0, SA_IDS_STRICT = 1, SA_IDS_WIDE = 2 };

/* AlignSettings (ObjectStore.scala:17-36) with Project4 defaults (Project4.scala:104-114). */
typedef struct sa_settings {
    int32_t kmer_size;       /* -k, --kmer-size        12   */
    int32_t min_overlap;     /* --min-overlap          40   */
    int32_t max_ignore;      /* --max-ignore           90   (compared as Float) */
    int32_t gap_open;        /* -gO, --gap-open        -200 */
    int32_t gap_extend;      /* -gE, --gap-extend      -20  */
    int32_t min_collisions;  /* --min-collisions       7    */
    int32_t max_collisions;  /* --max-collisions       222  */
    float min_identity;      /* --min-identity         0.98f */
    float kmer_edge;         /* --kmer-edge            0.4f */
    float kmer_center;       /* --kmer-center          0.4f */
    int32_t cost[16];        /* HOXD matrix, [a*4+b], bases A0 C1 G2 T3 (BioLibs.scala:122-140) */
    int32_t id_mode;         /* enum sa_id_mode */
} sa_settings;

/* One alignment per dispatched pair (Alignment + Overlap, ObjectStore.scala:89-142). */
typedef struct sa_alignment {
    int32_t lead, trail;             /* read ids, 1-based (rds:lead,trail) */
    int32_t start_i, start_j;        /* Alignment.start */
    int32_t end_i, end_j;            /* Alignment.end */
    int32_t correct, error;          /* c, e (alignA.length == c + e) */
    int32_t ahg, bhg;                /* Overlap.ahg / bhg */
    int32_t flags;                   /* SA_ALN_* bits */
    int32_t reserved;
} sa_alignment;
#define SA_ALN_DUD 1        /* phase-1 backtrack missed j==0 -> BioLibs.dud (BioLibs.scala:694-695) */
#define SA_ALN_VALID 2      /* Alignment.valid (ObjectStore.scala:102-107) */
#define SA_ALN_OVL_VALID 4  /* Overlap.valid (ObjectStore.scala:137-141) -> written to the .ovl */

typedef struct sa_ctx sa_ctx;

/* Project4.readArgs defaults (Project4.scala:104-114) + defaultHOXD. */
void sa_default_settings(sa_settings *s);

/* new AlignSettings + new KmerTable (KmerTable.scala:26-37) on HIP device `device`. */
int sa_ctx_create(const sa_settings *s, int device, sa_ctx **out);
void sa_ctx_destroy(sa_ctx *ctx);
const char *sa_last_error(const sa_ctx *ctx);

/* BioLibs.readHOXD (BioLibs.scala:66-114): -m / --matrix FILE into s->cost. */
int sa_load_hoxd(sa_settings *s, const char *path);

/* Reads.  Ids are assigned 1..N in call order (BioLibs.readSeq ordinal ids,
 * BioLibs.scala:27-47).  Bases are copied; lower case is upper-cased as
 * readSeq's toUpperCase does.  Replaces KmerTable.addKmerSet (KmerTable.scala:41)
 * fed by BioLibs.generateKmerSet (BioLibs.scala:54). */
int sa_add_reads(sa_ctx *ctx, const char *bases, const uint64_t *offsets, uint32_t n);
/* BioLibs.readSeq (BioLibs.scala:26-50) + sa_add_reads. */
int sa_read_fasta(sa_ctx *ctx, const char *path);
uint32_t sa_num_reads(const sa_ctx *ctx);
/* SequenceData.get (KmerTable.scala:37): read `id` (1-based) as added
 * (upper-cased); library-owned, valid until reads change or destroy. */
int sa_get_read(const sa_ctx *ctx, uint32_t id, const char **seq, size_t *len);

/* KmerTable.calcPairData + calcDispatchData (KmerTable.scala:85-187): device
 * k-mer emission, bucket build, edge<->middle pair counting, collision filter. */
int sa_build_candidates(sa_ctx *ctx);
/* DispatchData in dispatch order (KmerTable.scala:251-271): one entry per
 * (lead, trail) with its collision count. */
int sa_get_dispatch(sa_ctx *ctx, const int32_t **lead, const int32_t **trail,
                    const int32_t **count, size_t *n);
/* PairData (every counted ordered pair, not only dispatched ones), in the
 * reference's iteration order (STRICT) or by (fst, snd) ascending (WIDE).
 * Requires sa_set_option(ctx, SA_OPT_KEEP_PAIRS, 1) before sa_build_candidates. */
int sa_get_pairs(sa_ctx *ctx, const int32_t **fst, const int32_t **snd,
                 const int32_t **count, size_t *n);

/* KmerTable.uniqueKmers + kmerCollisionHistogram (KmerTable.scala:189-221), what
 * `--test-kmer-cover` prints (Project4.scala:299-320): the number of distinct
 * k-mer hashes and, ascending by size, how many hashes have `size` occurrences.
 * Works on the added reads at this context's k; independent of
 * sa_build_candidates.  Arrays are library-owned. */
int sa_kmer_histogram(sa_ctx *ctx, uint64_t *uniques, const uint64_t **size, const uint64_t **count, size_t *n);

/* genBlockMTAlign -> generateFastDovetailAlignmentSet for every dispatched pair
 * (Project4.scala:725-790, BioLibs.scala:596-822), or generateLocalAlignmentSet
 * (BioLibs.scala:267-368) under SA_OPT_ALIGNER = SA_ALIGNER_QUADRATIC. */
int sa_align(sa_ctx *ctx);
int sa_get_alignments(sa_ctx *ctx, const sa_alignment **out, size_t *n);

/* calcOverlaps (Project4.scala:795-825): AMOS {OVL} records of valid overlaps in
 * dispatch order.  path == NULL writes to stdout; an existing file is replaced. */
int sa_write_ovl(sa_ctx *ctx, const char *path);
/* The same bytes into a library-owned buffer. */
int sa_get_ovl(sa_ctx *ctx, const char **text, size_t *len);
/* AMOS message file for `bank-transact -c -b X.bnk -m X.afg` (SURVEY.md 8(f)
 * rank 1): the bank toAmos_new builds from the .seq (Rakefile.rb:174) and the
 * .ovl that bank-transact -m loads into it (:180-184), in one file.  One {RED}
 * per read in id order (iid = read id, eid = eids[id - 1], or the id when eids
 * or the entry is NULL / empty -- the eid rule is parity unpinned: the reference
 * bank's RED.0.map cannot tell ordinal eids from header words; eids, when given, holds one entry per read and
 * an entry with whitespace, ':' or braces fails with SA_E_ARG; seq = the read as
 * the context holds it; qlt = '0' + quality on every base, quality 0..60; clr =
 * 0,len and no other range, as the reference bank's RED records hold), then the
 * {OVL} records of sa_write_ovl, byte for byte.  One-process contexts only
 * (SA_E_ARG in rank mode); SA_E_STATE before an alignment. */
int sa_write_afg(sa_ctx *ctx, const char *path, const char *const *eids, int quality);

/* Options. */
enum sa_option {
    SA_OPT_KEEP_PAIRS = 1,   /* also materialise PairData for sa_get_pairs */
    SA_OPT_TIMING = 2,       /* record HIP events per stage (sa_get_stage_times) */
    SA_OPT_ALIGN_KERNEL = 3, /* 0 auto (default): lane-per-pair kernels when every band
                                fits 15 columns, else lane-group kernel; 1 force the
                                lane-group kernel; 2 force lane-per-pair (SA_E_ARG if
                                a band or read does not fit it); 3 lane-per-pair with
                                per-cell path summaries instead of stored codes */
    SA_OPT_ALIGNER = 4,      /* enum sa_aligner: which reference aligner sa_align runs */
    SA_OPT_LOCAL_BATCH_MB = 5, /* quadratic aligner: MiB of traceback codes per launch (16384) */
    SA_OPT_SERIAL_SHARDS = 6,  /* sharded context: run the shards' compute one after another
                                  (measurement: clean per-shard stage times on one device) */
    SA_OPT_LAUNCH_SLICE = 7,   /* pair counter: at most this many workgroups per launch (0 =
                                  default: lists are sliced only where a dispatch's 32-bit
                                  work-item count would wrap; a test hook for that path).
                                  Applies to the launches that walk a read / item list
                                  (every build passes one); a list-less launch larger
                                  than the slice fails with SA_E_HIP */
    SA_OPT_FIRST_PASS = 8,     /* pair counter's first pass (wide ids): 0 auto (default: a
                                  sample of every 64th read runs it first when there are
                                  >= 2^18 reads; if >= 95 % of the sample overflows its
                                  256-slot tables, every read goes straight to the big
                                  recount tier), 1 always run it, 2 always skip it (a
                                  test hook for the dense path) */
    SA_OPT_PASS_BUDGET_MB = 9, /* sharded context: MiB of partial (lead, trail, count)
                                  entries (12 B each, counted by their upper bound) one
                                  shard may produce per lead-range pass; the shards then
                                  count, exchange and reduce 1/npass of every owner's leads
                                  per pass (sa_dist_plan).  0 (default): 60 % of the free
                                  device memory after the bucket build, shared by the
                                  shards on the device, at 67 B x rho per bound entry
                                  (rho = 1.5 x the partials / bound ratio of these reads,
                                  probed on their first build; one pass whenever the
                                  bound is far from the memory) */
    SA_OPT_LEAN_MEMORY = 10    /* virtual shards (one device): the shards' transients (sort
                                  and bucket-build scratch, pair-counter regions, reduce
                                  scratch) come from one pool that each shard borrows for
                                  the length of a call, instead of P copies, so that
                                  virtual shards of a large read set fit one device; the
                                  shards then run one after another */
};

/* Project4's fdAlign switch (Project4.scala:187-192, :585-604).
 * LINEAR     --linear-align (default): generateFastDovetailAlignmentSet, banded
 *            two-phase dovetail DP (BioLibs.scala:596-822).
 * QUADRATIC  --quadratic-align: generateLocalAlignmentSet, full-matrix affine
 *            local alignment + greedy backtrack (BioLibs.scala:267-368); trails
 *            up to 2,048 bp (longer ones fail with SA_E_OVERFLOW), gap costs <= 0. */
enum sa_aligner { SA_ALIGNER_LINEAR = 0, SA_ALIGNER_QUADRATIC = 1 };
int sa_set_option(sa_ctx *ctx, int option, int64_t value);

/* Statistics of the last sa_build_candidates / sa_align. */
typedef struct sa_stats {
    uint64_t kmers;            /* k-mer occurrences (Kmer objects) */
    uint64_t buckets;          /* distinct k-mer hashes (KmerData.size) */
    uint64_t role_pairs;       /* (st x md) + (en x md) occurrence pairs visited by calcPairData */
    uint64_t pairs;            /* distinct ordered read pairs (PairData.size) */
    uint64_t dispatched;       /* pairs with min <= count <= max */
    uint64_t aligned;          /* alignments computed */
    uint64_t ovl_records;      /* valid overlaps */
    uint64_t dp_cells;         /* DP cells evaluated (phase 1 + phase 2) */
    int32_t id_mode;           /* resolved mode (STRICT or WIDE) */
    int32_t flags;             /* SA_STATS_* bits of the last build (was `reserved`, always 0) */
} sa_stats;
/* the build kept each read's dispatched pairs in its own region (wide ids,
 * dispatched pairs only): the lead-descending order is a scan + copy */
#define SA_STATS_PER_READ_REGIONS 1
/* some reads had more distinct partners than the first pass's table: they were
 * recounted by the larger tiers (KmerTable.scala:85-149 semantics unchanged) */
#define SA_STATS_RECOUNTED 2
int sa_get_stats(const sa_ctx *ctx, sa_stats *out);

/* Per-stage device time accumulated since the last reset (SA_OPT_TIMING). */
enum sa_stage {
    SA_STAGE_PACK = 0, SA_STAGE_EMIT, SA_STAGE_SORT, SA_STAGE_BUCKETS, SA_STAGE_PAIRS,
    SA_STAGE_ORDER, SA_STAGE_ALIGN,
    SA_STAGE_EXCHANGE,  /* sharded contexts: inter-shard exchanges (host wall clock) */
    /* host wall clock of the calc-overlaps path around the device stages (any context) */
    SA_STAGE_UPLOAD,    /* read metadata + H2D of the reads (first build after reads change) */
    SA_STAGE_REPLAY,    /* strict ids: Trove replay of KmerData / PairData / DispatchData order,
                           with its D2H / H2D copies; wide ids + keep_pairs: PairData on the host */
    SA_STAGE_READBACK,  /* D2H of the dispatch (sa_build_candidates) and alignments */
    SA_STAGE_FORMAT,    /* .ovl record text (Overlap.print, ObjectStore.scala:127-135) */
    SA_STAGE_WRITE,     /* sa_write_ovl: the file write */
    SA_NUM_STAGES
};
int sa_get_stage_times(const sa_ctx *ctx, double *ms, uint64_t *launches, int n);
int sa_reset_stage_times(sa_ctx *ctx);

/* Benchmark hooks: reads stay resident on the device; each call re-runs the
 * hot path on them with no host<->device copies of bulk data. */
int sa_device_build(sa_ctx *ctx);   /* == sa_build_candidates without host readback */
int sa_device_align(sa_ctx *ctx);   /* == sa_align without host readback */
int sa_sync(sa_ctx *ctx);

/* ---- Sharded contexts: `--gpus P` ---------------------
 * One context over P shards of the read set: read ids are split into P
 * contiguous ranges; every shard emits its k-mers, an all-to-all sends each
 * record to the shard owning its hash range, that shard builds its buckets and
 * counts partial (lead, trail) pairs, a second all-to-all sends the partials to
 * the shard owning the lead, which sums them and applies [min, max]; for
 * alignment the 2-bit packed reads are all-gathered once and every shard aligns
 * its own leads.  Every call above works on a sharded context, and dispatch,
 * alignments and .ovl bytes are identical to a single-device context's for any
 * P (the shards' outputs, concatenated in descending shard order).  The
 * reference is one JVM process (Project4.scala:517-563, :725-790): sharding
 * has no reference counterpart beyond reproducing its output.
 * Inputs in the reference's own id domain (strict ids, < 32,768 reads) need one
 * PairData table for the Trove order: a sharded context runs them unsharded on
 * its first device.  SA_OPT_KEEP_PAIRS is refused on a sharded build. */

/* One process, devices 0 .. n_gpus-1 with one shard each (n_shards == n_gpus),
 * exchanges over RCCL (send/recv groups over xGMI), or n_gpus == 1 with
 * n_shards virtual shards on device 0 exchanged in HBM (the sharded path on one
 * GPU).  n_shards is a power of two <= 256.  Replaces the reference's
 * single-process genMTKmerTable / genBlockMTAlign drivers (Project4.scala:531-563,
 * :725-790) under `sa-overlap --gpus P`. */
int sa_ctx_create_multi(const sa_settings *s, int n_gpus, int n_shards, sa_ctx **out);

/* One process per GPU (e.g. launched by torchrun): rank `rank` of `nranks`
 * (power of two), joined by an RCCL unique id that one rank creates with
 * sa_rccl_unique_id and the caller broadcasts.  Each rank adds only its own
 * reads; ranks hold consecutive id ranges in rank order.  sa_build_candidates,
 * sa_device_build, sa_align, sa_device_align and sa_write_ovl are collective
 * (every rank calls them); sa_get_dispatch / sa_get_alignments / sa_get_ovl /
 * sa_get_stats cover this rank's leads; sa_write_ovl writes all ranks' records
 * from rank 0.  Wide ids only (SA_IDS_STRICT is refused). */
#define SA_RCCL_ID_BYTES 128
int sa_rccl_unique_id(void *id, size_t cap);
int sa_ctx_create_rank(const sa_settings *s, int device, int rank, int nranks, const void *id, sa_ctx **out);
/* Bytes this process's shards sent to other shards (exchanges 1 and 2, read
 * all-gather) since the context was created. */
uint64_t sa_exchanged_bytes(const sa_ctx *ctx);
/* The last sharded build of this process's shards: its lead-range passes (1 unless the
 * partials' bound passed SA_OPT_PASS_BUDGET_MB), the partial (lead, trail, count)
 * entries its shards counted over all passes (the exchange-2 volume, 12 B each), and
 * their upper bound (sa_dist_buckets).  Any pointer may be NULL; SA_E_ARG on a
 * single-device context. */
int sa_get_shard_info(const sa_ctx *ctx, uint32_t *npass, uint64_t *partials, uint64_t *bound);

/* ---- Per-shard entry points, one process (context) per GPU ----
 * What a sharded context runs on each shard; exposed for callers that move the
 * data between ranks themselves (e.g. with torch.distributed).
 * Rank r holds reads [starts[r], starts[r+1]) of the global read set (0-based,
 * global id = index + 1), added to its context with sa_add_reads as usual.
 * The caller moves data between ranks (all-to-all / all-gather, e.g. with
 * torch.distributed over RCCL); every buffer argument below is a DEVICE
 * pointer on this context's GPU.  Wide ids only.  The sequence per step is
 *   sa_dist_emit      -> exchange 1 (8-byte k-mer records, grouped by owner rank)
 *   sa_dist_count     -> sa_dist_partials -> exchange 2 (partial pair counts)
 *   sa_dist_reduce    (this rank's leads: sum, [min,max] filter, dispatch)
 * or, with the partials bounded per lead-range pass (read sets whose partials do
 * not fit HBM at once, e.g. configs[4] at k = 12):
 *   sa_dist_emit      -> exchange 1
 *   sa_dist_buckets   -> sa_dist_plan (every rank; npass = the max over ranks)
 *   for pass = npass - 1 down to 0:
 *     sa_dist_count_pass -> sa_dist_partials -> exchange 2 -> sa_dist_reduce_pass
 * and, for alignment, sa_dist_codes -> all-gather -> sa_dist_set_reads, then
 * sa_align / sa_device_align / sa_get_ovl over this rank's leads.  The
 * library works on its own non-blocking HIP stream: device buffers handed in
 * must be complete (synchronise the stream that produced them, e.g. the one a
 * collective ran on), and buffers it fills are complete when the call returns.  No
 * reference counterpart: the reference is single-process
 * (KmerTable.scala:41-187 is the semantics each rank restates).
 */
/* nranks is a power of two <= 256; starts has nranks + 1 entries;
 * lengths[i] is the length of global read i (all starts[nranks] reads). */
int sa_dist_init(sa_ctx *ctx, int rank, int nranks, const uint32_t *starts, const int32_t *lengths);
/* k-mer occurrences of this rank's reads (the size of the exchange-1 send buffers). */
int sa_dist_local_kmers(sa_ctx *ctx, uint64_t *n);
/* Emit this rank's k-mer records (u64[n]: mixed hash << 32 | occurrence index
 * local to this rank, so only each rank's k-mer count is bounded by 2^32) into
 * send_recs, grouped by owner rank; counts[nranks] = records per owner. */
int sa_dist_emit(sa_ctx *ctx, void *send_recs, uint64_t *counts);
/* Records received in exchange 1, concatenated in source-rank order with
 * recv_counts[s] (host, nranks entries) records from rank s (the buffer is
 * consumed and overwritten): build this rank's buckets and count partial pairs
 * for every read; counts[nranks] = partials per lead owner. */
int sa_dist_count(sa_ctx *ctx, void *recv_recs, const uint64_t *recv_counts, uint64_t *counts);
/* Copy the partials (u32 lead, trail, count; 0-based ids) grouped by lead owner. */
int sa_dist_partials(sa_ctx *ctx, void *fst, void *snd, void *cnt);
/* Partials received in exchange 2: sum, filter, dispatch this rank's leads
 * (wide canonical order: lead descending, trail ascending). */
int sa_dist_reduce(sa_ctx *ctx, const void *fst, const void *snd, const void *cnt, uint64_t n);
/* Lead-range passes.  sa_dist_buckets: the first half of sa_dist_count (the records
 * received in exchange 1 -> this rank's buckets, built once); *bound = an upper bound
 * of the partials this rank can produce (the partner-list elements of its
 * occurrences, KmerTable.scala:85-149).  sa_dist_plan: the fewest passes whose every
 * pass stays within `budget` partial entries on this rank (1 when the bound fits);
 * ranks must agree on one pass count -- take the max over ranks.  Pass p of npass
 * covers, for every owner rank r, leads [s_r + len_r * p / npass,
 * s_r + len_r * (p + 1) / npass) of its reads [s_r, s_r + len_r).
 * sa_dist_count_pass: that pass's partials (counts[nranks] per lead owner, then
 * sa_dist_partials as above).  sa_dist_reduce_pass: this rank's leads of the pass,
 * appended to the dispatch; run the passes from npass - 1 down to 0 (pass npass - 1
 * starts a new dispatch, pass 0 completes it), so the dispatch stays lead-descending.
 * sa_dist_count == sa_dist_buckets + sa_dist_count_pass(0, 1); sa_dist_reduce ==
 * sa_dist_reduce_pass(0, 1). */
int sa_dist_buckets(sa_ctx *ctx, void *recv_recs, const uint64_t *recv_counts, uint64_t *bound);
int sa_dist_plan(sa_ctx *ctx, uint64_t budget, uint32_t *npass);
int sa_dist_count_pass(sa_ctx *ctx, uint32_t pass, uint32_t npass, uint64_t *counts);
int sa_dist_reduce_pass(sa_ctx *ctx, const void *fst, const void *snd, const void *cnt, uint64_t n, uint32_t pass,
                        uint32_t npass);
/* This rank's packed reads (2-bit words, u32[*nwords]) and first-invalid
 * positions (int32 per read); NULL buffers query *nwords only. */
int sa_dist_codes(sa_ctx *ctx, void *codes, void *bad, uint64_t *nwords);
/* All ranks' packed words / bad positions in global read order (all-gathered). */
int sa_dist_set_reads(sa_ctx *ctx, const void *codes, const void *bad, uint64_t nwords);

#ifdef __cplusplus
}
#endif
#endif
