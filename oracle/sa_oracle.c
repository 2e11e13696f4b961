/*
 * sa_oracle.c -- CPU restatement of the reference hash-overlap path.
 * TEST INFRASTRUCTURE ONLY (see sa_oracle.h).  Single-threaded, float32 exact.
 * Every function cites the Scala line range (under /root/reference/src) it follows.
 */
#include "sa_oracle.h"
#ifdef _OPENMP
#include <omp.h>
#endif
#include "trove_primes.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* small growable arrays                                                     */
/* ------------------------------------------------------------------------ */
typedef struct { int32_t *v; size_t n, cap; } ivec;
static int iv_push(ivec *a, int32_t x) {
    if (a->n == a->cap) {
        size_t nc = a->cap ? a->cap * 2 : 4;
        int32_t *nv = (int32_t *)realloc(a->v, nc * sizeof(int32_t));
        if (!nv) return ORC_E_NOMEM;
        a->v = nv; a->cap = nc;
    }
    a->v[a->n++] = x;
    return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* GNU Trove 3.0.3 TIntObjectHashMap (values: int32).  lib/trove.jar:        */
/*   THash.<init>(10,0.5f) -> setUp(fastCeil(20.0f)) ; computeMaxSize        */
/*   TIntHash.insertKey / insertKeyRehash (double hashing, idx -= probe)     */
/*   THash.postInsertHook (grow to nextPrime(cap<<1) when size > maxSize)    */
/*   TIntObjectHashMap.rehash (reinsert old slots high -> low)               */
/*   THashPrimitiveIterator.nextIndex (slots cap-1 .. 0)                     */
/* ------------------------------------------------------------------------ */
typedef struct {
    int32_t *keys, *vals;
    uint8_t *states; /* 0 FREE, 1 FULL (REMOVED never produced) */
    int32_t cap, size, free_, max_size;
    int consume_free;
} trove_map;

static int32_t trove_next_prime(int32_t desired) {
    int lo = 0, hi = TROVE_NPRIMES - 1;
    while (lo <= hi) { /* java.util.Arrays.binarySearch */
        int mid = (lo + hi) >> 1;
        if (trove_primes[mid] < desired) lo = mid + 1;
        else if (trove_primes[mid] > desired) hi = mid - 1;
        else return trove_primes[mid];
    }
    return trove_primes[lo]; /* insertion point */
}

static void trove_compute_max_size(trove_map *m) {
    float f = (float)m->cap * 0.5f; /* (int)(capacity * _loadFactor), float32 */
    int32_t lf = (int32_t)f;
    m->max_size = (m->cap - 1 < lf) ? m->cap - 1 : lf;
    m->free_ = m->cap - m->size;
}

static int trove_alloc(trove_map *m, int32_t cap) {
    m->keys = (int32_t *)calloc((size_t)cap, sizeof(int32_t));
    m->vals = (int32_t *)calloc((size_t)cap, sizeof(int32_t));
    m->states = (uint8_t *)calloc((size_t)cap, 1);
    m->cap = cap;
    return (m->keys && m->vals && m->states) ? ORC_OK : ORC_E_NOMEM;
}

static int trove_init(trove_map *m) {
    memset(m, 0, sizeof(*m));
    float f = 10.0f / 0.5f; /* HashFunctions.fastCeil */
    int32_t c = (int32_t)f;
    if (f - (float)c > 0.0f) c++;
    int rc = trove_alloc(m, trove_next_prime(c));
    if (rc) return rc;
    m->size = 0;
    trove_compute_max_size(m);
    return ORC_OK;
}

static void trove_free(trove_map *m) {
    free(m->keys); free(m->vals); free(m->states);
    memset(m, 0, sizeof(*m));
}

/* returns slot >= 0 for a new key, -slot-1 for an existing one */
static int32_t trove_insert_key(trove_map *m, int32_t val) {
    int32_t length = m->cap;
    int32_t hash = val & 0x7fffffff; /* HashFunctions.hash(int) == value */
    int32_t index = hash % length;
    m->consume_free = 0;
    if (m->states[index] == 0) {
        m->consume_free = 1;
        m->keys[index] = val; m->states[index] = 1;
        return index;
    }
    if (m->keys[index] == val) return -index - 1;
    int32_t probe = 1 + (hash % (length - 2));
    int32_t loop = index;
    do {
        index -= probe;
        if (index < 0) index += length;
        if (m->states[index] == 0) {
            m->consume_free = 1;
            m->keys[index] = val; m->states[index] = 1;
            return index;
        }
        if (m->keys[index] == val) return -index - 1;
    } while (index != loop);
    return INT32_MIN; /* full: cannot happen */
}

static int32_t trove_index(const trove_map *m, int32_t val) {
    int32_t length = m->cap;
    int32_t hash = val & 0x7fffffff;
    int32_t index = hash % length;
    if (m->states[index] == 0) return -1;
    if (m->keys[index] == val) return index;
    int32_t probe = 1 + (hash % (length - 2));
    int32_t loop = index;
    do {
        index -= probe;
        if (index < 0) index += length;
        if (m->states[index] == 0) return -1;
        if (m->keys[index] == val) return index;
    } while (index != loop);
    return -1;
}

static int trove_rehash(trove_map *m, int32_t newcap) {
    trove_map old = *m;
    int rc = trove_alloc(m, newcap);
    if (rc) return rc;
    for (int32_t i = old.cap; i-- > 0;) {
        if (old.states[i] == 1) {
            int32_t idx = trove_insert_key(m, old.keys[i]);
            m->vals[idx] = old.vals[i];
        }
    }
    free(old.keys); free(old.vals); free(old.states);
    return ORC_OK;
}

/* put(key, value); returns slot of the key after any rehash is NOT tracked */
static int trove_put(trove_map *m, int32_t key, int32_t value) {
    int32_t index = trove_insert_key(m, key);
    if (index == INT32_MIN) return ORC_E_TROVE;
    if (index < 0) { m->vals[-index - 1] = value; return ORC_OK; }
    m->vals[index] = value;
    if (m->consume_free) m->free_--;
    if (++m->size > m->max_size || m->free_ == 0) {
        int32_t newcap = m->size > m->max_size ? trove_next_prime(m->cap << 1) : m->cap;
        int rc = trove_rehash(m, newcap);
        if (rc) return rc;
        trove_compute_max_size(m);
    }
    return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* wide-mode pair map: open addressing on 64-bit (fst,snd)                   */
/* ------------------------------------------------------------------------ */
typedef struct { uint64_t *keys; int32_t *cnt; size_t cap, size; } wmap;
static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}
static int wmap_init(wmap *m, size_t cap) {
    m->cap = 1; while (m->cap < cap) m->cap <<= 1;
    m->keys = (uint64_t *)malloc(m->cap * sizeof(uint64_t));
    m->cnt = (int32_t *)calloc(m->cap, sizeof(int32_t));
    m->size = 0;
    if (!m->keys || !m->cnt) return ORC_E_NOMEM;
    memset(m->keys, 0xff, m->cap * sizeof(uint64_t));
    return ORC_OK;
}
static int wmap_add(wmap *m, uint64_t key) {
    if ((m->size + 1) * 2 > m->cap) {
        wmap n;
        if (wmap_init(&n, m->cap * 2)) return ORC_E_NOMEM;
        for (size_t i = 0; i < m->cap; i++) {
            if (m->keys[i] == UINT64_MAX) continue;
            size_t j = mix64(m->keys[i]) & (n.cap - 1);
            while (n.keys[j] != UINT64_MAX) j = (j + 1) & (n.cap - 1);
            n.keys[j] = m->keys[i]; n.cnt[j] = m->cnt[i]; n.size++;
        }
        free(m->keys); free(m->cnt); *m = n;
    }
    size_t j = mix64(key) & (m->cap - 1);
    while (m->keys[j] != UINT64_MAX && m->keys[j] != key) j = (j + 1) & (m->cap - 1);
    if (m->keys[j] == UINT64_MAX) { m->keys[j] = key; m->size++; }
    m->cnt[j]++;
    return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* context                                                                   */
/* ------------------------------------------------------------------------ */
struct orc_ctx {
    char *bases;
    uint64_t *off;
    uint32_t n;
    /* k-mers, generation order (read 1..N, position 0..L-k) */
    size_t nk;
    int32_t *k_hash, *k_id;
    float *k_loc;
    /* buckets */
    size_t nb;
    int32_t *bucket_order;  /* hashes in KmerData iteration order */
    /* pairs */
    size_t np;
    int32_t *p_fst, *p_snd, *p_cnt;
    int32_t *pf_fst, *pf_snd; /* first-insertion order (strict) */
    /* dispatch */
    size_t nd;
    int32_t *d_lead, *d_trail;
    orc_align_t *aligns;
    char *ovl;
    size_t ovl_len;
};

void orc_default_settings(orc_settings *s) { /* Project4.scala:104-114, BioLibs.scala:122-140 */
    static const int32_t hoxd[16] = {91, -114, -31, -123, -114, 100, -125, -31,
                                     -31, -125, 100, -114, -123, -31, -114, 91};
    s->kmer_size = 12;
    s->min_overlap = 40;
    s->max_ignore = 90;
    s->gap_open = -200;
    s->gap_extend = -20;
    s->min_collisions = 7;
    s->max_collisions = 222;
    s->min_identity = 0.98f;
    s->kmer_edge = 0.4f;
    s->kmer_center = 0.4f;
    memcpy(s->cost, hoxd, sizeof(hoxd));
}

static void free_results(orc_ctx *c) {
    free(c->k_hash); free(c->k_id); free(c->k_loc);
    free(c->bucket_order);
    free(c->p_fst); free(c->p_snd); free(c->p_cnt); free(c->pf_fst); free(c->pf_snd);
    free(c->d_lead); free(c->d_trail); free(c->aligns); free(c->ovl);
    c->k_hash = c->k_id = NULL; c->k_loc = NULL; c->bucket_order = NULL;
    c->p_fst = c->p_snd = c->p_cnt = c->pf_fst = c->pf_snd = NULL;
    c->d_lead = c->d_trail = NULL; c->aligns = NULL; c->ovl = NULL;
    c->nk = c->nb = c->np = c->nd = c->ovl_len = 0;
}

void orc_destroy(orc_ctx *c) {
    if (!c) return;
    free_results(c);
    free(c->bases); free(c->off); free(c);
}

uint32_t orc_num_reads(const orc_ctx *c) { return c->n; }

int orc_create_from_buffers(const char *bases, const uint64_t *offsets, uint32_t n, orc_ctx **out) {
    orc_ctx *c = (orc_ctx *)calloc(1, sizeof(orc_ctx));
    if (!c) return ORC_E_NOMEM;
    size_t tot = offsets[n];
    c->bases = (char *)malloc(tot + 1);
    c->off = (uint64_t *)malloc((n + 1) * sizeof(uint64_t));
    if (!c->bases || !c->off) { orc_destroy(c); return ORC_E_NOMEM; }
    memcpy(c->bases, bases, tot);
    c->bases[tot] = 0;
    memcpy(c->off, offsets, (n + 1) * sizeof(uint64_t));
    c->n = n;
    *out = c;
    return ORC_OK;
}

/* BioLibs.readSeq :26-50.  java.io.BufferedReader.readLine splits on \n, \r,
 * \r\n; String.toUpperCase on ASCII. */
int orc_create_from_fasta(const char *path, orc_ctx **out) {
    FILE *f = fopen(path, "rb");
    if (!f) return ORC_E_INPUT;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = (char *)malloc((size_t)sz + 1);
    if (!buf) { fclose(f); return ORC_E_NOMEM; }
    if (fread(buf, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); free(buf); return ORC_E_INPUT; }
    fclose(f);
    buf[sz] = 0;
    char *bases = (char *)malloc((size_t)sz + 1);
    size_t cap_off = 1024, n = 0, nb = 0;
    uint64_t *off = (uint64_t *)malloc(cap_off * sizeof(uint64_t));
    if (!bases || !off) { free(buf); free(bases); free(off); return ORC_E_NOMEM; }
    long p = 0;
    int first = 1;
    off[0] = 0;
    while (p < sz || first) {
        if (p >= sz) { free(buf); free(bases); free(off); return ORC_E_INPUT; } /* readLine()==null -> NPE */
        long e = p;
        while (e < sz && buf[e] != '\n' && buf[e] != '\r') e++;
        long next = e;
        if (next < sz) { if (buf[next] == '\r' && next + 1 < sz && buf[next + 1] == '\n') next += 2; else next++; }
        if (first) {
            if (buf[p] != '>' || e == p) { free(buf); free(bases); free(off); return ORC_E_INPUT; }
            first = 0;
        } else if (e > p && buf[p] == '>') {
            if (n + 2 >= cap_off) { cap_off *= 2; off = (uint64_t *)realloc(off, cap_off * sizeof(uint64_t)); }
            off[++n] = nb;
        } else {
            for (long q = p; q < e; q++) {
                char ch = buf[q];
                if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
                bases[nb++] = ch;
            }
        }
        p = next;
        if (p >= sz) break;
    }
    if (n + 2 >= cap_off) { cap_off += 2; off = (uint64_t *)realloc(off, cap_off * sizeof(uint64_t)); }
    off[++n] = nb; /* act(new Sequence(i, s)) after EOF */
    free(buf);
    int rc = orc_create_from_buffers(bases, off, (uint32_t)n, out);
    free(bases); free(off);
    return rc;
}

/* Kmer.seqHash, ObjectStore.scala:48-67: A0 C1 T2 G3 over min(16,k) chars,
 * h = (h<<2) ^ code; other chars contribute 0 (a warning is printed). */
static int32_t seq_hash(const char *s, int k) {
    uint32_t h = 0;
    int n = k < 16 ? k : 16;
    for (int i = 0; i < n; i++) {
        char ch = s[i];
        if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
        h <<= 2;
        switch (ch) {
        case 'A': break;
        case 'C': h ^= 1; break;
        case 'T': h ^= 2; break;
        case 'G': h ^= 3; break;
        default: break;
        }
    }
    return (int32_t)h;
}

static int hx_code(char ch) { /* defaultHOXD closure, BioLibs.scala:142-160 */
    if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
    switch (ch) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    default: return -1; /* MatchError */
    }
}

/* ------------------------------------------------------------------------ */
/* BioLibs.generateFastDovetailAlignmentSet, one trailer (BioLibs.scala:613-820) */
/* ------------------------------------------------------------------------ */
typedef struct { int32_t *M, *X, *Y; size_t cap; } dp_buf;
static void judge(orc_align_t *o, const orc_settings *s);

static int align_one(dp_buf *b, const char *A, int32_t la, const char *B, int32_t lb,
                     int32_t ida, int32_t idb, const orc_settings *s, orc_align_t *o) {
    const int32_t gO = s->gap_open, gE = s->gap_extend;
    /* :619-620 width = max(k, floor(|A| * (1 - minId)).toInt + 1), Float product */
    float prod = (float)la * (1.0f - s->min_identity);
    int32_t fl = (int32_t)floor((double)prod);
    int32_t width = s->kmer_size > fl + 1 ? s->kmer_size : fl + 1;
    const int32_t W = width + 1;
    size_t need = (size_t)(la + 1) * (size_t)W;
    if (need > b->cap) {
        free(b->M); free(b->X); free(b->Y);
        b->M = (int32_t *)malloc(need * sizeof(int32_t));
        b->X = (int32_t *)malloc(need * sizeof(int32_t));
        b->Y = (int32_t *)malloc(need * sizeof(int32_t));
        b->cap = need;
        if (!b->M || !b->X || !b->Y) return ORC_E_NOMEM;
    }
    int32_t *M = b->M, *X = b->X, *Y = b->Y;
    memset(M, 0, need * sizeof(int32_t)); /* :622-624 fresh arrays */
    memset(X, 0, need * sizeof(int32_t));
    memset(Y, 0, need * sizeof(int32_t));
#define AT(P, i, j) P[(size_t)(i) * W + (j)]
    for (int32_t i = 0; i < la; i++) { AT(M, i, 0) = 0; AT(X, i, 0) = 0; AT(Y, i, 0) = gO + i * gE; }
    for (int32_t i = 0; i < width; i++) { AT(M, 0, i) = 0; AT(X, 0, i) = gO + i * gE; AT(Y, 0, i) = 0; }
    if (lb < width) return ORC_E_INDEX; /* B.charAt(j-1), j <= width */
    int32_t mx = 0, mi = 0, mj = 0;
    for (int32_t i = 1; i <= la; i++) { /* :645-668 */
        int ca = hx_code(A[i - 1]);
        for (int32_t j = 1; j <= width; j++) {
            int cb = hx_code(B[j - 1]);
            if (ca < 0 || cb < 0) return ORC_E_MATCH;
            int32_t d = AT(M, i - 1, j - 1);
            if (AT(Y, i - 1, j - 1) > d) d = AT(Y, i - 1, j - 1);
            int32_t d2 = AT(X, i - 1, j - 1) > 0 ? AT(X, i - 1, j - 1) : 0;
            AT(M, i, j) = s->cost[ca * 4 + cb] + (d > d2 ? d : d2);
            int32_t x1 = AT(M, i, j - 1) + gO, x2 = AT(Y, i, j - 1) + gO;
            int32_t x3 = AT(X, i, j - 1) > 0 ? AT(X, i, j - 1) : 0;
            int32_t xm = x1 > x2 ? x1 : x2;
            AT(X, i, j) = gE + (xm > x3 ? xm : x3);
            int32_t y1 = AT(M, i - 1, j) + gO, y2 = AT(Y, i - 1, j);
            int32_t y3 = AT(X, i - 1, j) + gO;
            if (y3 < 0) y3 = 0;
            int32_t ym = y1 > y2 ? y1 : y2;
            AT(Y, i, j) = gE + (ym > y3 ? ym : y3);
            int32_t t = AT(M, i, j);
            if (AT(X, i, j) > t) t = AT(X, i, j);
            if (AT(Y, i, j) > t) t = AT(Y, i, j);
            if (t > mx) { mx = t; mi = i; mj = j; }
        }
    }
    /* phase-1 greedy backtrack :673-689 */
    int32_t i = mi, j = mj;
#define CMAX(i_, j_) (AT(M, i_, j_) > AT(X, i_, j_) ? (AT(M, i_, j_) > AT(Y, i_, j_) ? AT(M, i_, j_) : AT(Y, i_, j_)) \
                                                    : (AT(X, i_, j_) > AT(Y, i_, j_) ? AT(X, i_, j_) : AT(Y, i_, j_)))
    mx = CMAX(i, j);
    do {
        if (AT(M, i, j) == mx) { i--; j--; }
        else if (AT(X, i, j) == mx) { j--; }
        else if (AT(Y, i, j) == mx) { i--; }
        if (i < 0 || j < 0) return ORC_E_INDEX;
        mx = CMAX(i, j);
    } while (mx > 0);
    memset(o, 0, sizeof(*o));
    o->lead = ida; o->trail = idb;
    if (j != 0) { /* :694-695 dud = Alignment(Sequence(0,""),Sequence(0,""),"","",(0,0),(0,0),0,1) */
        o->is_dud = 1;
        o->correct = 0; o->error = 1;
        o->len_a = 0; o->len_b = 0;
        return ORC_OK;
    }
    const int32_t doveStart = i, doveLength = la - doveStart, zeroRow = width / 2;
    mx = 0; mi = 0; mj = 0;
    for (int32_t u = 0; u <= doveLength; u++) { /* :725-764 */
        for (int32_t k = 0; k <= width; k++) {
            int32_t ii = u + doveStart, jj = k - zeroRow + u;
            if (ii <= doveStart || jj <= 0 || jj > lb) {
                AT(M, u, k) = 0; AT(X, u, k) = 0; AT(Y, u, k) = 0;
            } else {
                if (u != 0) {
                    int ca = hx_code(A[ii - 1]), cb = hx_code(B[jj - 1]);
                    if (ca < 0 || cb < 0) return ORC_E_MATCH;
                    int32_t d = AT(M, u - 1, k);
                    if (AT(Y, u - 1, k) > d) d = AT(Y, u - 1, k);
                    int32_t d2 = AT(X, u - 1, k) > 0 ? AT(X, u - 1, k) : 0;
                    AT(M, u, k) = s->cost[ca * 4 + cb] + (d > d2 ? d : d2);
                } else AT(M, u, k) = 0;
                if (k != 0) {
                    int32_t x1 = AT(M, u, k - 1) + gO, x2 = AT(Y, u, k - 1) + gO;
                    int32_t x3 = AT(X, u, k - 1) > 0 ? AT(X, u, k - 1) : 0;
                    int32_t xm = x1 > x2 ? x1 : x2;
                    AT(X, u, k) = gE + (xm > x3 ? xm : x3);
                } else AT(X, u, k) = 0;
                if (u != 0 && k != width) {
                    int32_t y1 = AT(M, u - 1, k + 1) + gO, y2 = AT(Y, u - 1, k + 1);
                    int32_t y3 = AT(X, u - 1, k + 1) + gO;
                    if (y3 < 0) y3 = 0;
                    int32_t ym = y1 > y2 ? y1 : y2;
                    AT(Y, u, k) = gE + (ym > y3 ? ym : y3);
                } else AT(Y, u, k) = 0;
            }
            int32_t t = CMAX(u, k);
            if (t > mx) { mx = t; mi = u; mj = k; }
        }
    }
    /* phase-2 greedy backtrack :768-809 */
    int32_t u = mi, k = mj, c = 0, e = 0;
    mx = CMAX(u, k);
    do {
        int32_t ii = u + doveStart, jj = k - zeroRow + u;
        char pa = ' ', pb = ' ';
        if (ii - 1 < 0 || ii - 1 >= la) return ORC_E_INDEX;
        if (AT(M, u, k) == mx) {
            if (jj - 1 < 0 || jj - 1 >= lb) return ORC_E_INDEX;
            pa = A[ii - 1]; pb = B[jj - 1]; u--;
        } else if (AT(X, u, k) == mx) {
            pa = A[ii - 1]; pb = '-'; k--;
        } else if (AT(Y, u, k) == mx) {
            if (jj - 1 < 0 || jj - 1 >= lb) return ORC_E_INDEX;
            pa = '-'; pb = B[jj - 1]; u--; k++;
        }
        if (pa != pb) e++; else c++;
        if (u < 0 || k < 0 || k > width) return ORC_E_INDEX;
        mx = CMAX(u, k);
    } while (mx > 0);
    o->start_i = u + doveStart;
    o->start_j = k - zeroRow + u;
    o->end_i = mi + doveStart;
    o->end_j = mj - zeroRow + mi;
    o->correct = c; o->error = e;
    o->len_a = la; o->len_b = lb;
    return ORC_OK;
#undef AT
#undef CMAX
}

/* ------------------------------------------------------------------------ */
/* BioLibs.generateLocalAlignmentSet, one trailer (BioLibs.scala:267-368):   */
/* the `--quadratic-align` aligner (full-matrix affine local alignment with  */
/* the same greedy backtrack).  The block variant reuses its matrices across  */
/* trailers, but every cell it reads for a trailer was written for that      */
/* trailer or is a boundary cell, so a per-pair matrix gives the same result. */
/* ------------------------------------------------------------------------ */
static int align_local(dp_buf *b, const char *A, int32_t la, const char *B, int32_t lb,
                       int32_t ida, int32_t idb, const orc_settings *s, orc_align_t *o) {
    const int32_t gO = s->gap_open, gE = s->gap_extend;
    const int32_t W = lb + 1;
    size_t need = (size_t)(la + 1) * (size_t)W;
    if (need > b->cap) {
        free(b->M); free(b->X); free(b->Y);
        b->M = (int32_t *)malloc(need * sizeof(int32_t));
        b->X = (int32_t *)malloc(need * sizeof(int32_t));
        b->Y = (int32_t *)malloc(need * sizeof(int32_t));
        b->cap = need;
        if (!b->M || !b->X || !b->Y) return ORC_E_NOMEM;
    }
    int32_t *M = b->M, *X = b->X, *Y = b->Y;
    memset(M, 0, need * sizeof(int32_t));
    memset(X, 0, need * sizeof(int32_t));
    memset(Y, 0, need * sizeof(int32_t));
#define AT(P, i, j) P[(size_t)(i) * W + (j)]
    for (int32_t i = 0; i < la; i++) { AT(Y, i, 0) = gO + i * gE; }  /* :281-285 */
    for (int32_t i = 0; i < lb; i++) { AT(X, 0, i) = gO + i * gE; }  /* :287-291 (maxL >= lb) */
    int32_t mx = 0, mi = 0, mj = 0;
    for (int32_t i = 1; i <= la; i++) { /* :301-324 */
        int ca = hx_code(A[i - 1]);
        for (int32_t j = 1; j <= lb; j++) {
            int cb = hx_code(B[j - 1]);
            if (ca < 0 || cb < 0) return ORC_E_MATCH;
            int32_t d = AT(M, i - 1, j - 1);
            if (AT(Y, i - 1, j - 1) > d) d = AT(Y, i - 1, j - 1);
            int32_t d2 = AT(X, i - 1, j - 1) > 0 ? AT(X, i - 1, j - 1) : 0;
            AT(M, i, j) = s->cost[ca * 4 + cb] + (d > d2 ? d : d2);
            int32_t x1 = AT(M, i, j - 1) + gO, x2 = AT(Y, i, j - 1) + gO;
            int32_t x3 = AT(X, i, j - 1) > 0 ? AT(X, i, j - 1) : 0;
            int32_t xm = x1 > x2 ? x1 : x2;
            AT(X, i, j) = gE + (xm > x3 ? xm : x3);
            int32_t y1 = AT(M, i - 1, j) + gO, y2 = AT(Y, i - 1, j);
            int32_t y3 = AT(X, i - 1, j) + gO;
            if (y3 < 0) y3 = 0;
            int32_t ym = y1 > y2 ? y1 : y2;
            AT(Y, i, j) = gE + (ym > y3 ? ym : y3);
            int32_t t = AT(M, i, j);
            if (AT(X, i, j) > t) t = AT(X, i, j);
            if (AT(Y, i, j) > t) t = AT(Y, i, j);
            if (t > mx) { mx = t; mi = i; mj = j; }
        }
    }
    /* greedy backtrack :326-362; A.charAt(-1) on a matrix with no positive cell */
#define CMAX(i_, j_) (AT(M, i_, j_) > AT(X, i_, j_) ? (AT(M, i_, j_) > AT(Y, i_, j_) ? AT(M, i_, j_) : AT(Y, i_, j_)) \
                                                    : (AT(X, i_, j_) > AT(Y, i_, j_) ? AT(X, i_, j_) : AT(Y, i_, j_)))
    int32_t i = mi, j = mj, c = 0, e = 0;
    mx = CMAX(i, j);
    do {
        char pa = ' ', pb = ' ';
        if (AT(M, i, j) == mx) {
            if (i < 1 || j < 1) return ORC_E_INDEX;
            pa = A[i - 1]; pb = B[j - 1]; i--; j--;
        } else if (AT(X, i, j) == mx) {
            if (i < 1 || j < 1) return ORC_E_INDEX;
            pa = A[i - 1]; pb = '-'; j--;
        } else if (AT(Y, i, j) == mx) {
            if (j < 1 || i < 1) return ORC_E_INDEX;
            pa = '-'; pb = B[j - 1]; i--;
        }
        if (pa != pb) e++; else c++;
        mx = CMAX(i, j);
    } while (mx > 0);
    memset(o, 0, sizeof(*o));
    o->lead = ida; o->trail = idb;
    o->start_i = i; o->start_j = j; /* Alignment(seqA, seqB, xSeq, ySeq, (i,j), opt, c, e) :364 */
    o->end_i = mi; o->end_j = mj;
    o->correct = c; o->error = e;
    o->len_a = la; o->len_b = lb;
    return ORC_OK;
#undef AT
#undef CMAX
}

int orc_align_pair_local(const char *A, int32_t la, const char *B, int32_t lb, int32_t ida, int32_t idb,
                         const orc_settings *s, orc_align_t *out) {
    dp_buf b = {0};
    int rc = align_local(&b, A, la, B, lb, ida, idb, s, out);
    free(b.M); free(b.X); free(b.Y);
    if (rc == ORC_OK) judge(out, s);
    return rc;
}

/* Alignment.valid / Overlap (ObjectStore.scala:99-141) */
static void judge(orc_align_t *o, const orc_settings *s) {
    float ratio = (float)o->correct / ((float)o->correct + (float)o->error);
    /* alignA.length: one char per backtrack step, but "" for the dud (BioLibs.scala:22) */
    int32_t alen = o->is_dud ? 0 : o->correct + o->error;
    o->valid = (ratio >= s->min_identity) && (alen >= s->min_overlap) &&
               ((o->start_i == 0 && o->len_b == o->end_j) || (o->start_j == 0 && o->len_a == o->end_i));
    o->ahg = o->start_i - o->start_j;
    o->bhg = o->len_b - o->len_a + o->ahg;
    float mi = (float)s->max_ignore;
    o->ovl_valid = o->valid && ((float)abs(o->ahg) < mi) && ((float)abs(o->bhg) < mi);
}

int orc_align_pair(const char *A, int32_t la, const char *B, int32_t lb, int32_t ida, int32_t idb,
                   const orc_settings *s, orc_align_t *out) {
    dp_buf b = {0};
    int rc = align_one(&b, A, la, B, lb, ida, idb, s, out);
    free(b.M); free(b.X); free(b.Y);
    if (rc == ORC_OK) judge(out, s);
    return rc;
}

/* all cores: OMP_NUM_THREADS when set (the GPU box sets it to this job's CPU
 * share), else every processor */
int orc_max_threads(void) {
    const char *e = getenv("OMP_NUM_THREADS");
    if (e && atoi(e) > 0) return atoi(e);
#ifdef _OPENMP
    return omp_get_num_procs();
#else
    return 1;
#endif
}

/* genBlockMTAlign's alignment work over a given dispatch list (Project4.scala:
 * 725-790 runs one future per block on the actor pool; pairs are independent):
 * the CPU baseline of the aligner, on `threads` OpenMP threads (0 = all).  The
 * reads are the caller's buffers (ids 1-based).  Returns the first error. */
int orc_align_batch(const char *bases, const uint64_t *offsets, uint32_t n_reads, const int32_t *lead,
                    const int32_t *trail, size_t n_pairs, const orc_settings *s, int threads, orc_align_t *out) {
    int err = ORC_OK;
    /* an explicit team size: omp_set_num_threads would leave the caller's
     * default changed for every later call (a 1-thread run then an all-core
     * run would both use one thread) */
    const int nt = threads > 0 ? threads : orc_max_threads();
    (void)nt;
#pragma omp parallel num_threads(nt)
    {
        dp_buf b = {0};
#pragma omp for schedule(dynamic, 256)
        for (size_t i = 0; i < n_pairs; ++i) {
            const uint32_t a = (uint32_t)lead[i] - 1u, t = (uint32_t)trail[i] - 1u;
            int rc = ORC_E_INPUT;
            if (a < n_reads && t < n_reads) {
                rc = align_one(&b, bases + offsets[a], (int32_t)(offsets[a + 1] - offsets[a]), bases + offsets[t],
                               (int32_t)(offsets[t + 1] - offsets[t]), lead[i], trail[i], s, &out[i]);
                if (rc == ORC_OK) judge(&out[i], s);
            }
            if (rc != ORC_OK) {
#pragma omp critical
                if (err == ORC_OK) err = rc;
            }
        }
        free(b.M); free(b.X); free(b.Y);
    }
    return err;
}


/* ------------------------------------------------------------------------ */
/* the calc-overlaps path                                                    */
/* ------------------------------------------------------------------------ */
static int cmp_wide_pair(const void *a, const void *b) {
    const int64_t *x = (const int64_t *)a, *y = (const int64_t *)b;
    return (*x > *y) - (*x < *y);
}

int orc_run(orc_ctx *c, const orc_settings *s, int flags) {
    const int wide = flags & 1, skip_align = flags & 2, quadratic = flags & 4;
    free_results(c);
    const int k = s->kmer_size;
    /* AlignSettings derived edges, ObjectStore.scala:30-35 */
    const float head = s->kmer_edge;
    const float tail = 1.0f - s->kmer_edge;
    const float midLead = 0.5f - (s->kmer_center * 0.5f);
    const float midTail = 0.5f + (s->kmer_center * 0.5f);
    int rc = ORC_OK;

    /* generateKmerSet (BioLibs.scala:54-61) for reads 1..N in order */
    size_t nk = 0;
    for (uint32_t r = 0; r < c->n; r++) {
        int64_t L = (int64_t)(c->off[r + 1] - c->off[r]);
        if (L - k + 1 > 0) nk += (size_t)(L - k + 1);
    }
    c->nk = nk;
    c->k_hash = (int32_t *)malloc((nk + 1) * sizeof(int32_t));
    c->k_id = (int32_t *)malloc((nk + 1) * sizeof(int32_t));
    c->k_loc = (float *)malloc((nk + 1) * sizeof(float));
    if (!c->k_hash || !c->k_id || !c->k_loc) return ORC_E_NOMEM;
    size_t g = 0;
    for (uint32_t r = 0; r < c->n; r++) {
        int64_t L = (int64_t)(c->off[r + 1] - c->off[r]);
        const char *sq = c->bases + c->off[r];
        float d = (float)(L - k);
        for (int64_t i = 0; i <= L - k; i++, g++) {
            c->k_hash[g] = seq_hash(sq + i, k);
            c->k_id[g] = (int32_t)(r + 1);
            c->k_loc[g] = (float)i / d;
        }
    }

    /* addKmerSet (KmerTable.scala:41-53): KmerData Trove map hash -> bucket */
    trove_map kd;
    if ((rc = trove_init(&kd))) return rc;
    ivec *buckets = NULL;
    size_t nb = 0, bcap = 0;
    for (size_t q = 0; q < nk; q++) {
        int32_t h = c->k_hash[q];
        int32_t idx = trove_index(&kd, h);
        int32_t bid;
        if (idx < 0) {
            if (nb == bcap) {
                bcap = bcap ? bcap * 2 : 1024;
                ivec *nbk = (ivec *)realloc(buckets, bcap * sizeof(ivec));
                if (!nbk) { rc = ORC_E_NOMEM; goto out_kd; }
                buckets = nbk;
            }
            memset(&buckets[nb], 0, sizeof(ivec));
            bid = (int32_t)nb++;
            if ((rc = trove_put(&kd, h, bid))) goto out_kd;
        } else bid = kd.vals[idx];
        if ((rc = iv_push(&buckets[bid], (int32_t)q))) goto out_kd;
    }
    c->nb = nb;
    c->bucket_order = (int32_t *)malloc((nb + 1) * sizeof(int32_t));
    int32_t *border = (int32_t *)malloc((nb + 1) * sizeof(int32_t));
    {
        size_t t = 0;
        for (int32_t i = kd.cap; i-- > 0;)
            if (kd.states[i] == 1) { c->bucket_order[t] = kd.keys[i]; border[t] = kd.vals[i]; t++; }
    }

    /* calcPairData (KmerTable.scala:85-149) + addKmerPair (:57-80) */
    {
        ivec st = {0}, md = {0}, en = {0};
        trove_map pd;
        wmap wm;
        ivec ffst = {0}, fsnd = {0};
        if (!wide) { if ((rc = trove_init(&pd))) goto out_b; }
        else if ((rc = wmap_init(&wm, 1 << 16))) goto out_b;
        for (size_t t = 0; t < nb; t++) {
            ivec *bk = &buckets[border[t]];
            st.n = md.n = en.n = 0;
            for (size_t q = 0; q < bk->n; q++) {
                float l = c->k_loc[bk->v[q]];
                if (l <= head) iv_push(&st, bk->v[q]);
                if (midLead <= l && l <= midTail) iv_push(&md, bk->v[q]);
                if (tail <= l) iv_push(&en, bk->v[q]);
            }
            for (int pass = 0; pass < 2; pass++) {
                ivec *ed = pass == 0 ? &st : &en;
                for (size_t x = 0; x < ed->n; x++) {
                    int32_t a = ed->v[x];
                    for (size_t y = 0; y < md.n; y++) {
                        int32_t b = md.v[y];
                        if (c->k_id[a] == c->k_id[b]) continue;
                        int32_t fst, snd;
                        if (c->k_loc[a] > c->k_loc[b]) { fst = c->k_id[a]; snd = c->k_id[b]; }
                        else { fst = c->k_id[b]; snd = c->k_id[a]; }
                        if (!wide) {
                            int32_t key = (int32_t)(((uint32_t)fst << 16) ^ (uint32_t)snd);
                            int32_t idx = trove_index(&pd, key);
                            if (idx >= 0) pd.vals[idx]++;
                            else {
                                iv_push(&ffst, fst); iv_push(&fsnd, snd);
                                if ((rc = trove_put(&pd, key, 1))) goto out_p;
                            }
                        } else {
                            if ((rc = wmap_add(&wm, ((uint64_t)(uint32_t)fst << 32) | (uint32_t)snd))) goto out_p;
                        }
                    }
                }
            }
        }
        /* PairData iteration + calcDispatchData (KmerTable.scala:155-187) */
        if (!wide) {
            c->np = (size_t)pd.size;
            c->p_fst = (int32_t *)malloc((c->np + 1) * sizeof(int32_t));
            c->p_snd = (int32_t *)malloc((c->np + 1) * sizeof(int32_t));
            c->p_cnt = (int32_t *)malloc((c->np + 1) * sizeof(int32_t));
            c->pf_fst = ffst.v; c->pf_snd = fsnd.v; ffst.v = fsnd.v = NULL;
            trove_map dd;
            if ((rc = trove_init(&dd))) goto out_p;
            ivec *lists = NULL;
            size_t nl = 0, lcap = 0;
            size_t t = 0;
            for (int32_t i = pd.cap; i-- > 0;) {
                if (pd.states[i] != 1) continue;
                int32_t key = pd.keys[i], cnt = pd.vals[i];
                int32_t a = key >> 16;
                int32_t b = (int32_t)((uint32_t)key << 16) >> 16;
                c->p_fst[t] = a; c->p_snd[t] = b; c->p_cnt[t] = cnt; t++;
                if (s->min_collisions <= cnt && cnt <= s->max_collisions) {
                    int32_t idx = trove_index(&dd, a);
                    int32_t lid;
                    if (idx < 0) {
                        if (nl == lcap) { lcap = lcap ? lcap * 2 : 256; lists = (ivec *)realloc(lists, lcap * sizeof(ivec)); }
                        memset(&lists[nl], 0, sizeof(ivec));
                        lid = (int32_t)nl++;
                        trove_put(&dd, a, lid);
                    } else lid = dd.vals[idx];
                    iv_push(&lists[lid], b);
                }
            }
            /* dispatchCollisionBlocks (KmerTable.scala:246-273) */
            size_t nd = 0;
            for (size_t q = 0; q < nl; q++) nd += lists[q].n;
            c->d_lead = (int32_t *)malloc((nd + 1) * sizeof(int32_t));
            c->d_trail = (int32_t *)malloc((nd + 1) * sizeof(int32_t));
            size_t w = 0;
            for (int32_t i = dd.cap; i-- > 0;) {
                if (dd.states[i] != 1) continue;
                ivec *ls = &lists[dd.vals[i]];
                int32_t lead = dd.keys[i];
                for (size_t q = 0; q < ls->n; q++) {
                    int32_t b = ls->v[q];
                    if (b < 1 || (uint32_t)b > c->n) rc = ORC_E_NPE; /* SequenceData.get(j) == null */
                    c->d_lead[w] = lead; c->d_trail[w] = b; w++;
                }
                if (lead < 1 || (uint32_t)lead > c->n) rc = ORC_E_NPE;
            }
            c->nd = nd;
            for (size_t q = 0; q < nl; q++) free(lists[q].v);
            free(lists);
            trove_free(&dd);
        } else {
            c->np = wm.size;
            int64_t *tmp = (int64_t *)malloc((c->np + 1) * sizeof(int64_t) * 2);
            size_t t = 0;
            for (size_t i = 0; i < wm.cap; i++)
                if (wm.keys[i] != UINT64_MAX) { tmp[2 * t] = (int64_t)wm.keys[i]; tmp[2 * t + 1] = wm.cnt[i]; t++; }
            qsort(tmp, t, 2 * sizeof(int64_t), cmp_wide_pair);
            c->p_fst = (int32_t *)malloc((c->np + 1) * sizeof(int32_t));
            c->p_snd = (int32_t *)malloc((c->np + 1) * sizeof(int32_t));
            c->p_cnt = (int32_t *)malloc((c->np + 1) * sizeof(int32_t));
            size_t nd = 0;
            for (size_t q = 0; q < t; q++) {
                c->p_fst[q] = (int32_t)((uint64_t)tmp[2 * q] >> 32);
                c->p_snd[q] = (int32_t)(uint32_t)tmp[2 * q];
                c->p_cnt[q] = (int32_t)tmp[2 * q + 1];
                if (s->min_collisions <= c->p_cnt[q] && c->p_cnt[q] <= s->max_collisions) nd++;
            }
            /* canonical order: lead descending, trail ascending */
            c->d_lead = (int32_t *)malloc((nd + 1) * sizeof(int32_t));
            c->d_trail = (int32_t *)malloc((nd + 1) * sizeof(int32_t));
            size_t w = 0, q = t;
            while (q > 0) {
                size_t hi = q;
                int32_t lead = c->p_fst[q - 1];
                size_t lo = q;
                while (lo > 0 && c->p_fst[lo - 1] == lead) lo--;
                for (size_t z = lo; z < hi; z++)
                    if (s->min_collisions <= c->p_cnt[z] && c->p_cnt[z] <= s->max_collisions) {
                        c->d_lead[w] = lead; c->d_trail[w] = c->p_snd[z]; w++;
                    }
                q = lo;
            }
            c->nd = nd;
            free(tmp);
        }
    out_p:
        free(st.v); free(md.v); free(en.v); free(ffst.v); free(fsnd.v);
        if (!wide) trove_free(&pd);
        else { free(wm.keys); free(wm.cnt); }
    }
out_b:
    free(border);
    for (size_t q = 0; q < nb; q++) free(buckets[q].v);
    free(buckets);
out_kd:
    trove_free(&kd);
    if (rc) return rc;

    /* genBlockMTAlign (Project4.scala:725-790) + calcOverlaps (:795-825) */
    c->aligns = (orc_align_t *)calloc(c->nd + 1, sizeof(orc_align_t));
    if (skip_align) {
        c->ovl = (char *)calloc(1, 1);
        return ORC_OK;
    }
    size_t ocap = 4096, olen = 0;
    char *ovl = (char *)malloc(ocap);
    dp_buf db = {0};
    for (size_t q = 0; q < c->nd; q++) {
        int32_t a = c->d_lead[q], b = c->d_trail[q];
        const char *A = c->bases + c->off[a - 1];
        const char *B = c->bases + c->off[b - 1];
        int32_t la = (int32_t)(c->off[a] - c->off[a - 1]);
        int32_t lb = (int32_t)(c->off[b] - c->off[b - 1]);
        orc_align_t *o = &c->aligns[q];
        if ((rc = (quadratic ? align_local : align_one)(&db, A, la, B, lb, a, b, s, o))) break;
        judge(o, s);
        if (o->valid && o->ovl_valid) {
            char rec[160];
            int ra = o->is_dud ? 0 : a, rb = o->is_dud ? 0 : b;
            int m = snprintf(rec, sizeof(rec), "{OVL\nadj:N\nrds:%d,%d\nscr:0\nahg:%d\nbhg:%d\n}\n",
                             ra, rb, o->ahg, o->bhg);
            if (olen + (size_t)m + 1 > ocap) { ocap = ocap * 2 + (size_t)m; ovl = (char *)realloc(ovl, ocap); }
            memcpy(ovl + olen, rec, (size_t)m);
            olen += (size_t)m;
        }
    }
    free(db.M); free(db.X); free(db.Y);
    ovl[olen] = 0;
    c->ovl = ovl;
    c->ovl_len = olen;
    return rc;
}

/* ------------------------------------------------------------------------ */
/* all-core variant of the wide-id hash stage (CPU baseline only): the same   */
/* KmerTable semantics as orc_run's wide branch -- generateKmerSet, addKmerSet */
/* grouping, calcPairData's st x md / en x md role pairs with addKmerPair's   */
/* orientation (KmerTable.scala:57-149), the [min, max] filter and the wide   */
/* canonical order (lead descending, trail ascending; KmerTable.scala:155-187)*/
/* -- on OpenMP threads: k-mers per read, buckets grouped by a counting sort  */
/* on the top 16 bits of a mixed hash (each bin then sorted by (hash, g), so  */
/* a bucket lists its occurrences in (read, pos) order as the reference's     */
/* ArrayBuffers do), role pairs counted in thread-local maps over bins, the   */
/* maps merged by lead residue.  The reference's KmerTable itself is single-  */
/* writer (Project4.scala:550-560); this is the all-core restatement SURVEY   */
/* 8(d) asks for beside the single-thread one.                                */
/* ------------------------------------------------------------------------ */
static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return (x > y) - (x < y);
}
static int lead_owner(uint64_t lead, uint32_t n, int nt) { /* ids 1..n in nt ranges */
    return (int)(((lead - 1) * (uint64_t)nt) / ((uint64_t)n + 1));
}
static uint32_t bin_mix(uint32_t h) { /* spreads hashes over the 2^16 bins */
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}

int orc_run_wide_mt(orc_ctx *c, const orc_settings *s, int threads, uint64_t *role_pairs) {
    free_results(c);
    const int nt = threads > 0 ? threads : orc_max_threads();
    const int k = s->kmer_size;
    const float head = s->kmer_edge, tail = 1.0f - s->kmer_edge;
    const float midLead = 0.5f - (s->kmer_center * 0.5f), midTail = 0.5f + (s->kmer_center * 0.5f);
    const uint32_t n = c->n;
    uint64_t *koff = (uint64_t *)malloc(((size_t)n + 1) * sizeof(uint64_t));
    if (!koff) return ORC_E_NOMEM;
    koff[0] = 0;
    for (uint32_t r = 0; r < n; r++) {
        const int64_t L = (int64_t)(c->off[r + 1] - c->off[r]);
        koff[r + 1] = koff[r] + (L - k + 1 > 0 ? (uint64_t)(L - k + 1) : 0);
    }
    const size_t nk = koff[n];
    c->nk = nk;
    c->k_hash = (int32_t *)malloc((nk + 1) * sizeof(int32_t));
    c->k_id = (int32_t *)malloc((nk + 1) * sizeof(int32_t));
    c->k_loc = (float *)malloc((nk + 1) * sizeof(float));
    enum { NBIN = 1 << 16 };
    uint64_t *recs = (uint64_t *)malloc((nk + 1) * sizeof(uint64_t));
    uint64_t *hist = (uint64_t *)calloc((size_t)nt * NBIN + 1, sizeof(uint64_t));
    uint64_t *bstart = (uint64_t *)malloc((NBIN + 1) * sizeof(uint64_t));
    if (!c->k_hash || !c->k_id || !c->k_loc || !recs || !hist || !bstart) {
        free(koff); free(recs); free(hist); free(bstart);
        return ORC_E_NOMEM;
    }
    wmap *loc_maps = (wmap *)calloc((size_t)nt, sizeof(wmap));
    uint64_t rp_total = 0;
    int rc = ORC_OK;
#pragma omp parallel num_threads(nt) reduction(+ : rp_total)
    {
        const int t = omp_get_thread_num();
        /* generateKmerSet (BioLibs.scala:54-61) */
#pragma omp for schedule(dynamic, 256)
        for (uint32_t r = 0; r < n; r++) {
            const int64_t L = (int64_t)(c->off[r + 1] - c->off[r]);
            const char *sq = c->bases + c->off[r];
            const float d = (float)(L - k);
            size_t g = koff[r];
            for (int64_t i = 0; i <= L - k; i++, g++) {
                c->k_hash[g] = seq_hash(sq + i, k);
                c->k_id[g] = (int32_t)(r + 1);
                c->k_loc[g] = (float)i / d;
            }
        }
        /* addKmerSet grouping: counting sort by bin, thread-contiguous chunks (stable) */
        const size_t lo = nk * (size_t)t / (size_t)nt, hi = nk * (size_t)(t + 1) / (size_t)nt;
        uint64_t *h = hist + (size_t)t * NBIN;
        for (size_t g = lo; g < hi; g++) h[bin_mix((uint32_t)c->k_hash[g]) >> 16]++;
#pragma omp barrier
#pragma omp single
        {
            uint64_t acc = 0;
            for (uint32_t b = 0; b < NBIN; b++) {
                bstart[b] = acc;
                for (int q = 0; q < nt; q++) {
                    const uint64_t v = hist[(size_t)q * NBIN + b];
                    hist[(size_t)q * NBIN + b] = acc;
                    acc += v;
                }
            }
            bstart[NBIN] = acc;
        }
        for (size_t g = lo; g < hi; g++) {
            const uint32_t hv = (uint32_t)c->k_hash[g];
            recs[h[bin_mix(hv) >> 16]++] = ((uint64_t)hv << 32) | (uint64_t)g;
        }
#pragma omp barrier
        /* calcPairData (KmerTable.scala:85-149) per bin, thread-local PairData */
        wmap *wm = &loc_maps[t];
        int lrc = wmap_init(wm, 1 << 16);
        ivec st = {0}, md = {0}, en = {0};
        uint64_t rp = 0;
#pragma omp for schedule(dynamic, 64)
        for (uint32_t b = 0; b < NBIN; b++) {
            uint64_t *rb = recs + bstart[b];
            const size_t m = (size_t)(bstart[b + 1] - bstart[b]);
            qsort(rb, m, sizeof(uint64_t), cmp_u64); /* (hash, g): whole buckets, (read, pos) order */
            for (size_t x0 = 0; x0 < m && !lrc;) {
                size_t x1 = x0;
                while (x1 < m && (rb[x1] >> 32) == (rb[x0] >> 32)) x1++;
                st.n = md.n = en.n = 0;
                for (size_t q = x0; q < x1; q++) {
                    const int32_t g = (int32_t)(uint32_t)rb[q];
                    const float l = c->k_loc[g];
                    if (l <= head) iv_push(&st, g);
                    if (midLead <= l && l <= midTail) iv_push(&md, g);
                    if (tail <= l) iv_push(&en, g);
                }
                for (int pass = 0; pass < 2 && !lrc; pass++) {
                    const ivec *ed = pass == 0 ? &st : &en;
                    for (size_t x = 0; x < ed->n && !lrc; x++) {
                        const int32_t a = ed->v[x];
                        for (size_t y = 0; y < md.n; y++) {
                            const int32_t bq = md.v[y];
                            rp++;
                            if (c->k_id[a] == c->k_id[bq]) continue;
                            int32_t fst, snd;
                            if (c->k_loc[a] > c->k_loc[bq]) { fst = c->k_id[a]; snd = c->k_id[bq]; }
                            else { fst = c->k_id[bq]; snd = c->k_id[a]; }
                            if ((lrc = wmap_add(wm, ((uint64_t)(uint32_t)fst << 32) | (uint32_t)snd))) break;
                        }
                    }
                }
                x0 = x1;
            }
        }
        free(st.v); free(md.v); free(en.v);
        rp_total += rp;
        if (lrc) {
#pragma omp critical
            rc = lrc;
        }
    }
    free(koff); free(hist); free(bstart); free(recs);
    if (rc) goto out;
    {
        /* merge: thread t owns the leads of one contiguous id range (counts summed),
         * so the threads' sorted arrays concatenate to the (fst, snd) order */
        wmap *fin = (wmap *)calloc((size_t)nt, sizeof(wmap));
        uint64_t *cnt_t = (uint64_t *)calloc((size_t)nt + 1, sizeof(uint64_t));
        int64_t **arr = (int64_t **)calloc((size_t)nt, sizeof(int64_t *));
#pragma omp parallel num_threads(nt)
        {
            const int t = omp_get_thread_num();
            wmap *f = &fin[t];
            int lrc = wmap_init(f, 1 << 16);
            for (int q = 0; q < nt && !lrc; q++) {
                const wmap *w = &loc_maps[q];
                for (size_t i = 0; i < w->cap && !lrc; i++) {
                    const uint64_t key = w->keys[i];
                    if (key == UINT64_MAX || lead_owner(key >> 32, n, nt) != t) continue;
                    if ((lrc = wmap_add(f, key))) break;
                    /* wmap_add counted 1: add the rest of this map's count */
                    size_t j = mix64(key) & (f->cap - 1);
                    while (f->keys[j] != key) j = (j + 1) & (f->cap - 1);
                    f->cnt[j] += w->cnt[i] - 1;
                }
            }
            int64_t *a = lrc ? NULL : (int64_t *)malloc((f->size + 1) * 2 * sizeof(int64_t));
            size_t z = 0;
            if (a)
                for (size_t i = 0; i < f->cap; i++)
                    if (f->keys[i] != UINT64_MAX) { a[2 * z] = (int64_t)f->keys[i]; a[2 * z + 1] = f->cnt[i]; z++; }
            free(f->keys); free(f->cnt); /* (host memory at configs[4]-shaped sizes) */
            f->keys = NULL; f->cnt = NULL;
            if (a) qsort(a, z, 2 * sizeof(int64_t), cmp_wide_pair);
            arr[t] = a;
            cnt_t[t] = z;
            if (!a) {
#pragma omp critical
                rc = ORC_E_NOMEM;
            }
        }
        if (!rc) {
            /* lead ranges ascend with t: the concatenation is sorted by key */
            size_t np = 0;
            for (int t = 0; t < nt; t++) np += cnt_t[t];
            int64_t *all = (int64_t *)malloc((np + 1) * 2 * sizeof(int64_t));
            size_t z = 0;
            for (int t = 0; t < nt; t++) {
                memcpy(all + 2 * z, arr[t], cnt_t[t] * 2 * sizeof(int64_t));
                z += cnt_t[t];
                free(arr[t]);
                arr[t] = NULL;
            }
            c->np = np;
            c->p_fst = (int32_t *)malloc((np + 1) * sizeof(int32_t));
            c->p_snd = (int32_t *)malloc((np + 1) * sizeof(int32_t));
            c->p_cnt = (int32_t *)malloc((np + 1) * sizeof(int32_t));
            size_t nd = 0;
            for (size_t q = 0; q < np; q++) {
                c->p_fst[q] = (int32_t)((uint64_t)all[2 * q] >> 32);
                c->p_snd[q] = (int32_t)(uint32_t)all[2 * q];
                c->p_cnt[q] = (int32_t)all[2 * q + 1];
                if (s->min_collisions <= c->p_cnt[q] && c->p_cnt[q] <= s->max_collisions) nd++;
            }
            c->d_lead = (int32_t *)malloc((nd + 1) * sizeof(int32_t));
            c->d_trail = (int32_t *)malloc((nd + 1) * sizeof(int32_t));
            size_t w = 0, q = np;
            while (q > 0) { /* lead descending, trail ascending */
                const int32_t lead = c->p_fst[q - 1];
                size_t l0 = q;
                while (l0 > 0 && c->p_fst[l0 - 1] == lead) l0--;
                for (size_t x = l0; x < q; x++)
                    if (s->min_collisions <= c->p_cnt[x] && c->p_cnt[x] <= s->max_collisions) {
                        c->d_lead[w] = lead; c->d_trail[w] = c->p_snd[x]; w++;
                    }
                q = l0;
            }
            c->nd = nd;
            free(all);
        }
        for (int t = 0; t < nt; t++) { free(fin[t].keys); free(fin[t].cnt); free(arr[t]); }
        free(fin); free(cnt_t); free(arr);
    }
out:
    for (int t = 0; t < nt; t++) { free(loc_maps[t].keys); free(loc_maps[t].cnt); }
    free(loc_maps);
    if (role_pairs) *role_pairs = rp_total;
    c->aligns = (orc_align_t *)calloc(c->nd + 1, sizeof(orc_align_t));
    c->ovl = (char *)calloc(1, 1);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* sampled-lead PairData rows: the checker for read sets whose whole PairData  */
/* does not fit host memory (configs[4]'s 6.25M-read slice at k = 12 has      */
/* 1.5e11 distinct pairs).  For every sampled lead r, every PairData entry     */
/* (r, snd, count) of calcPairData (KmerTable.scala:85-149) whose fst is r,   */
/* with addKmerPair's orientation (:57-80: fst = the occurrence with the       */
/* larger loc, tie -> the middle one; same-read pairs skipped; every st x md   */
/* and en x md occurrence pair counts once).  Only the buckets of r's k-mers   */
/* can hold such a pair, so:                                                   */
/*   pass 1  the seqHashes of the sampled leads' k-mers (a bitmap over the     */
/*           2 * min(k, 16)-bit hash space, ObjectStore.scala:48-67)            */
/*   pass 2  every read streamed; occurrences in those buckets kept as          */
/*           (read, pos), grouped by hash (counting sort)                       */
/*   rows    per lead (OpenMP over leads), per occurrence o of r in bucket B:  */
/*           o edge (st / en, once per role) x every middle e of B with         */
/*           loc(o) > loc(e)  -> (r, read(e)); o middle x every edge role of    */
/*           e in B with loc(e) <= loc(o) -> (r, read(e)).  A role pair whose   */
/*           fst is r is exactly one of these (orc_run's loop, :1024-1037).     */
/* Memory is the sampled buckets, not the pairs of the whole read set.         */
/* ------------------------------------------------------------------------ */
static int cmp_i32(const void *a, const void *b) {
    const int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return (x > y) - (x < y);
}
static inline uint32_t hash_code(char ch) { /* Kmer.seqHash codes: A0 C1 T2 G3, others 0 */
    if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
    return ch == 'C' ? 1u : ch == 'T' ? 2u : ch == 'G' ? 3u : 0u;
}

/* seqHash of every k-mer of one read, rolling (== seq_hash(sq + i, k)) */
static void read_hashes(const char *sq, int64_t L, int k, uint32_t *out) {
    const int w = k < 16 ? k : 16;
    const uint32_t mask = w == 16 ? 0xffffffffu : ((1u << (2 * w)) - 1u);
    uint32_t h = 0;
    for (int i = 0; i < w - 1 && i < L; i++) h = (h << 2) | hash_code(sq[i]);
    for (int64_t i = 0; i + k <= L; i++) {
        h = ((h << 2) | hash_code(sq[i + w - 1])) & mask;
        out[i] = h;
    }
}

/* reads as (base + start[r], len[r]) -- reads cut from one genome, the projection's
 * configs[3] / [4] sets without materialising them -- or back to back (off) */
typedef struct { const char *base; const uint64_t *off; const uint64_t *start; const int32_t *len; } rd_src;
static inline const char *rd_seq(const rd_src *R, uint32_t r) { return R->base + (R->start ? R->start[r] : R->off[r]); }
static inline int64_t rd_len(const rd_src *R, uint32_t r) {
    return R->start ? (int64_t)R->len[r] : (int64_t)(R->off[r + 1] - R->off[r]);
}
/* the sharded path's owner rank of a k-mer: the top log_ranks bits of mix32(seqHash)
 * (sa_internal.h mix32, the device's record key) */
static inline uint32_t owner_of_hash(uint32_t h, int log_ranks) {
    if (log_ranks <= 0) return 0;
    h ^= h >> 16; h *= 0x7feb352du;
    h ^= h >> 15; h *= 0x846ca68bu;
    h ^= h >> 16;
    return h >> (32 - log_ranks);
}

/* rows (snd_out / cnt_out non-null): the PairData rows of the sampled leads;
 * stats (st non-null, 4 per lead): distinct partners, role pairs with fst = the
 * lead, partials = distinct (partner, owner rank) of those role pairs when the
 * buckets are owned by 2^log_ranks ranks, dispatched partners ([min, max]) */
static int lead_scan(const rd_src *R, uint32_t n, const orc_settings *s, const int32_t *leads, size_t n_leads,
                     int threads, uint64_t *row_off, int32_t **snd_out, int32_t **cnt_out, int log_ranks,
                     uint64_t *st) {
    if (snd_out) *snd_out = NULL;
    if (cnt_out) *cnt_out = NULL;
    if (log_ranks > 6) return ORC_E_INPUT;  /* owner masks are 64 bits */
    const int nt = threads > 0 ? threads : orc_max_threads();
    const int k = s->kmer_size;
    const int w = k < 16 ? k : 16;
    const float head = s->kmer_edge, tail = 1.0f - s->kmer_edge;
    const float midLead = 0.5f - (s->kmer_center * 0.5f), midTail = 0.5f + (s->kmer_center * 0.5f);
    for (size_t i = 0; i < n_leads; i++)
        if (leads[i] < 1 || (uint32_t)leads[i] > n || (i && leads[i] <= leads[i - 1])) return ORC_E_INPUT;
    const uint64_t nbits = 1ull << (2 * w), nwords = nbits / 64;
    uint64_t *bits = (uint64_t *)calloc(nwords, sizeof(uint64_t));
    uint32_t *rank = (uint32_t *)malloc((nwords + 1) * sizeof(uint32_t));
    int64_t maxL = 0;
    for (uint32_t r = 0; r < n; r++)
        if (rd_len(R, r) > maxL) maxL = rd_len(R, r);
    if (!bits || !rank) { free(bits); free(rank); return ORC_E_NOMEM; }
    /* pass 1: the sampled leads' hashes */
    {
        uint32_t *hs = (uint32_t *)malloc(((size_t)maxL + 1) * sizeof(uint32_t));
        for (size_t i = 0; i < n_leads && hs; i++) {
            const uint32_t r = (uint32_t)leads[i] - 1u;
            const int64_t L = rd_len(R, r);
            read_hashes(rd_seq(R, r), L, k, hs);
            for (int64_t p = 0; p + k <= L; p++) bits[hs[p] >> 6] |= 1ull << (hs[p] & 63);
        }
        if (!hs) { free(bits); free(rank); return ORC_E_NOMEM; }
        free(hs);
    }
    uint64_t m = 0;
    for (uint64_t q = 0; q < nwords; q++) { rank[q] = (uint32_t)m; m += (uint64_t)__builtin_popcountll(bits[q]); }
    rank[nwords] = (uint32_t)m;
    /* pass 2: occurrences in those buckets, counted then placed by hash rank */
    uint64_t *bstart = (uint64_t *)calloc(m + 2, sizeof(uint64_t));
    if (!bstart) { free(bits); free(rank); return ORC_E_NOMEM; }
#define HIT_RANK(h) (rank[(h) >> 6] + (uint32_t)__builtin_popcountll(bits[(h) >> 6] & ((1ull << ((h) & 63)) - 1ull)))
#define IS_HIT(h) ((bits[(h) >> 6] >> ((h) & 63)) & 1ull)
    int rc = ORC_OK;
    for (int phase = 0; phase < 2; phase++) {
        uint64_t *cur = bstart + 1;
        uint32_t *occ = NULL;
        if (phase == 1) {
            for (uint64_t q = 0; q < m; q++) bstart[q + 1] += bstart[q];
            occ = (uint32_t *)malloc((bstart[m] + 1) * 2 * sizeof(uint32_t));
            if (!occ) { rc = ORC_E_NOMEM; break; }
            cur = (uint64_t *)malloc((m + 1) * sizeof(uint64_t));
            if (!cur) { free(occ); rc = ORC_E_NOMEM; break; }
            memcpy(cur, bstart, (m + 1) * sizeof(uint64_t));
        }
#pragma omp parallel num_threads(nt)
        {
            uint32_t *hs = (uint32_t *)malloc(((size_t)maxL + 1) * sizeof(uint32_t));
#pragma omp for schedule(dynamic, 1024)
            for (uint32_t r = 0; r < n; r++) {
                const int64_t L = rd_len(R, r);
                if (!hs || L < k) continue;
                read_hashes(rd_seq(R, r), L, k, hs);
                for (int64_t p = 0; p + k <= L; p++) {
                    const uint32_t h = hs[p];
                    if (!IS_HIT(h)) continue;
                    const uint32_t b = HIT_RANK(h);
                    uint64_t slot;
#pragma omp atomic capture
                    slot = cur[b]++;
                    if (phase == 1) { occ[2 * slot] = r; occ[2 * slot + 1] = (uint32_t)p; }
                }
            }
            if (!hs) {
#pragma omp critical
                rc = ORC_E_NOMEM;
            }
            free(hs);
        }
        if (phase == 0) continue;
        free(cur);
        if (rc) { free(occ); break; }
        /* rows, one lead at a time per thread */
        int32_t **rs = (int32_t **)calloc(n_leads + 1, sizeof(int32_t *));
        int32_t **rcn = (int32_t **)calloc(n_leads + 1, sizeof(int32_t *));
        uint64_t *rn = (uint64_t *)calloc(n_leads + 1, sizeof(uint64_t));
        if (!rs || !rcn || !rn) { free(rs); free(rcn); free(rn); free(occ); rc = ORC_E_NOMEM; break; }
#pragma omp parallel num_threads(nt)
        {
            int32_t *acc = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
            uint64_t *om = st ? (uint64_t *)calloc((size_t)n + 1, sizeof(uint64_t)) : NULL;
            uint32_t *hs = (uint32_t *)malloc(((size_t)maxL + 1) * sizeof(uint32_t));
            ivec touched = {0};
            int lrc = (!acc || !hs || (st && !om)) ? ORC_E_NOMEM : ORC_OK;
#pragma omp for schedule(dynamic, 1)
            for (size_t li = 0; li < n_leads; li++) {
                if (lrc) continue;
                const uint32_t r = (uint32_t)leads[li] - 1u;
                const int64_t L = rd_len(R, r);
                const float dr = (float)(L - k);
                read_hashes(rd_seq(R, r), L, k, hs);
                touched.n = 0;
                uint64_t rp_lead = 0;
                for (int64_t p = 0; p + k <= L; p++) {
                    const float lo = (float)p / dr;
                    const int o_st = lo <= head, o_md = midLead <= lo && lo <= midTail, o_en = tail <= lo;
                    const int o_ed = o_st + o_en;
                    if (!o_ed && !o_md) continue;
                    const uint32_t b = HIT_RANK(hs[p]);
                    const uint64_t obit = st ? 1ull << owner_of_hash(hs[p], log_ranks) : 0ull;
                    for (uint64_t x = bstart[b]; x < bstart[b + 1]; x++) {
                        const uint32_t q = occ[2 * x];
                        if (q == r) continue;
                        const float le = (float)occ[2 * x + 1] / (float)(rd_len(R, q) - k);
                        const int e_md = midLead <= le && le <= midTail;
                        const int e_ed = (le <= head) + (tail <= le);
                        int add = 0;
                        if (o_ed && e_md && lo > le) add += o_ed;    /* o edge, e middle, fst = o */
                        if (o_md && e_ed && !(le > lo)) add += e_ed; /* e edge, o middle, fst = o */
                        if (!add) continue;
                        if (acc[q] == 0 && iv_push(&touched, (int32_t)q)) { lrc = ORC_E_NOMEM; break; }
                        acc[q] += add;
                        rp_lead += (uint64_t)add;
                        if (st) om[q] |= obit;
                    }
                }
                if (st) {  /* per-lead statistics instead of rows */
                    uint64_t parts = 0, nd = 0;
                    for (size_t z = 0; z < touched.n; z++) {
                        const int32_t q = touched.v[z];
                        parts += (uint64_t)__builtin_popcountll(om[q]);
                        nd += s->min_collisions <= acc[q] && acc[q] <= s->max_collisions;
                        acc[q] = 0;
                        om[q] = 0;
                    }
                    st[4 * li] = touched.n;
                    st[4 * li + 1] = rp_lead;
                    st[4 * li + 2] = parts;
                    st[4 * li + 3] = nd;
                    continue;
                }
                int32_t *sv = (int32_t *)malloc((touched.n + 1) * sizeof(int32_t));
                int32_t *cv = (int32_t *)malloc((touched.n + 1) * sizeof(int32_t));
                if (!sv || !cv) { free(sv); free(cv); lrc = ORC_E_NOMEM; continue; }
                /* partners ascending: sort the touched read indices */
                for (size_t z = 0; z < touched.n; z++) sv[z] = touched.v[z];
                qsort(sv, touched.n, sizeof(int32_t), cmp_i32);
                for (size_t z = 0; z < touched.n; z++) { cv[z] = acc[sv[z]]; acc[sv[z]] = 0; sv[z] += 1; }
                rs[li] = sv; rcn[li] = cv; rn[li] = touched.n;
            }
            free(acc); free(om); free(hs); free(touched.v);
            if (lrc) {
#pragma omp critical
                rc = lrc;
            }
        }
        free(occ);
        if (!rc && !st) {
            row_off[0] = 0;
            for (size_t li = 0; li < n_leads; li++) row_off[li + 1] = row_off[li] + rn[li];
            *snd_out = (int32_t *)malloc((row_off[n_leads] + 1) * sizeof(int32_t));
            *cnt_out = (int32_t *)malloc((row_off[n_leads] + 1) * sizeof(int32_t));
            if (!*snd_out || !*cnt_out) rc = ORC_E_NOMEM;
            for (size_t li = 0; li < n_leads && !rc; li++) {
                memcpy(*snd_out + row_off[li], rs[li], rn[li] * sizeof(int32_t));
                memcpy(*cnt_out + row_off[li], rcn[li], rn[li] * sizeof(int32_t));
            }
        }
        for (size_t li = 0; li < n_leads; li++) { free(rs[li]); free(rcn[li]); }
        free(rs); free(rcn); free(rn);
    }
#undef HIT_RANK
#undef IS_HIT
    free(bits); free(rank); free(bstart);
    if (rc && snd_out) { free(*snd_out); free(*cnt_out); *snd_out = *cnt_out = NULL; }
    return rc;
}

int orc_lead_rows(const char *bases, const uint64_t *offsets, uint32_t n, const orc_settings *s,
                  const int32_t *leads, size_t n_leads, int threads, uint64_t *row_off, int32_t **snd_out,
                  int32_t **cnt_out) {
    const rd_src R = {bases, offsets, NULL, NULL};
    return lead_scan(&R, n, s, leads, n_leads, threads, row_off, snd_out, cnt_out, 0, NULL);
}

int orc_lead_stats(const char *genome, const uint64_t *starts, const int32_t *lens, uint32_t n, const orc_settings *s,
                   const int32_t *leads, size_t n_leads, int threads, int log_ranks, uint64_t *stats) {
    const rd_src R = {genome, NULL, starts, lens};
    return lead_scan(&R, n, s, leads, n_leads, threads, NULL, NULL, NULL, log_ranks, stats);
}

/* synth genome base i (bench.synth_workload): z = splitmix64 output i + 1 of `seed`;
 * u = (z >> 11) * 2^-53 < gc ? (z & 1 ? 'G' : 'C') : (z & 1 ? 'T' : 'A') */
void orc_synth_genome(uint64_t seed, uint64_t n, double gc, char *out, int threads) {
    const int nt = threads > 0 ? threads : orc_max_threads();
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
        out[i] = u < gc ? ((z & 1) ? 'G' : 'C') : ((z & 1) ? 'T' : 'A');
    }
}

void orc_free(void *p) { free(p); }

size_t orc_num_kmers(const orc_ctx *c) { return c->nk; }
void orc_kmers(const orc_ctx *c, const int32_t **hash, const int32_t **read_id, const float **loc) {
    *hash = c->k_hash; *read_id = c->k_id; *loc = c->k_loc;
}
size_t orc_num_buckets(const orc_ctx *c) { return c->nb; }
const int32_t *orc_bucket_order(const orc_ctx *c) { return c->bucket_order; }
size_t orc_num_pairs(const orc_ctx *c) { return c->np; }
void orc_pairs(const orc_ctx *c, const int32_t **fst, const int32_t **snd, const int32_t **count) {
    *fst = c->p_fst; *snd = c->p_snd; *count = c->p_cnt;
}
void orc_pairs_first_order(const orc_ctx *c, const int32_t **fst, const int32_t **snd) {
    *fst = c->pf_fst; *snd = c->pf_snd;
}
size_t orc_num_dispatch(const orc_ctx *c) { return c->nd; }
void orc_dispatch(const orc_ctx *c, const int32_t **lead, const int32_t **trail) {
    *lead = c->d_lead; *trail = c->d_trail;
}
const orc_align_t *orc_aligns(const orc_ctx *c) { return c->aligns; }
size_t orc_ovl(const orc_ctx *c, const char **text) { *text = c->ovl; return c->ovl_len; }

int orc_trove_order(const int32_t *keys, size_t n, int32_t *order_out, int32_t *cap_out) {
    trove_map m;
    int rc = trove_init(&m);
    if (rc) return rc;
    for (size_t i = 0; i < n; i++)
        if ((rc = trove_put(&m, keys[i], (int32_t)i))) { trove_free(&m); return rc; }
    size_t t = 0;
    for (int32_t i = m.cap; i-- > 0;)
        if (m.states[i] == 1) order_out[t++] = m.keys[i];
    *cap_out = m.cap;
    trove_free(&m);
    return ORC_OK;
}
