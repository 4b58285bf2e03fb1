/* hash_oracle.c -- CPU restatement of SeqArc 1.6's HASH reference index and
 * its gapless seed alignment (SURVEY.md section 8(f) 3, configs[3]).
 *
 * TEST INFRASTRUCTURE (the checker): only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline may load it; the product path (libseqarc_amd) never
 * does.  Every routine restates the disassembly of SeqArc-1.6 at the cited
 * address.  PARITY UNPINNED: the reference ships no index files and no
 * alignments, and its executable may not be run here, so nothing pins these
 * routines but the disassembly.
 *
 * Scope: the 32-bit index (HashRefIndex32, FASTA files < 5 GiB: every
 * single-genome reference up to human) and the single-read alignment
 * getHashAlignInfo@0x4113c0 that doSEAlign@0x4117b0 and, per mate,
 * doPEAlign@0x4117d0 call.  FASTA lines before the first '>' header are
 * rejected: the reference counts them in one pass but not the other and
 * writes past its position table (buildRefIndex@0x410190).
 */
#define _DEFAULT_SOURCE   /* madvise, posix_memalign */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sys/mman.h>
#include <unistd.h>

#include "hash_oracle.h"

/* base code @0x449fc0: ACGT 0-3 (either case), IUPAC M 5, R 6, Y 7, K 8, S 9,
 * W 10, H 11, B 12, V 13, D 14, anything else 4 (sa_common.h base_code); a
 * byte >= 0x80 indexes the reference's table with a sign-extended offset
 * (movsx) and reads the 128 bytes before it (the tail of the mask table
 * @0x449e80): HO_NEG */
static const uint8_t HO_NEG[128] = {
    255, 255, 255, 255, 255, 255, 0, 0, 255, 255, 255, 255, 255, 255, 3, 0,
    255, 255, 255, 255, 255, 255, 15, 0, 255, 255, 255, 255, 255, 255, 63, 0,
    255, 255, 255, 255, 255, 255, 255, 0, 255, 255, 255, 255, 255, 255, 255, 3,
    255, 255, 255, 255, 255, 255, 255, 15, 255, 255, 255, 255, 255, 255, 255, 63,
    255, 255, 255, 255, 255, 255, 255, 255, 0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
};

static uint8_t ho_code(char c)
{
    const signed char s = (signed char)c;
    if (s < 0) return HO_NEG[128 + s];
    switch (s & 0xdf) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    case 'M': return 5;
    case 'R': return 6;
    case 'Y': return 7;
    case 'K': return 8;
    case 'S': return 9;
    case 'W': return 10;
    case 'H': return 11;
    case 'B': return 12;
    case 'V': return 13;
    case 'D': return 14;
    default: return 4;
    }
}

/* mismatch type @0x44a0c0, [ref * 4 + read] (the read base's rank among the
 * three other bases); a read N/IUPAC base is type 3 */
static const uint8_t HO_MISTYPE[16] = {3, 1, 0, 2, 1, 3, 0, 2, 1, 0, 3, 2, 2, 1, 0, 3};

static uint64_t ho_mask(uint32_t k) { return k >= 32 ? ~0ull : (1ull << (2 * k)) - 1; } /* @0x449e80 */

/* ---- index ------------------------------------------------------------- */
void ho_index_free(ho_index* ix)
{
    free(ix->seq);   /* (ho_alloc: posix_memalign, freed with free) */
    free(ix->num);
    free(ix->ind);
    free(ix->pos);
    memset(ix, 0, sizeof *ix);
}

/* Large tables: 2 MiB-aligned and backed by transparent huge pages where the
 * kernel allows (a genome-scale index does hundreds of millions of random
 * accesses into GB-sized tables; 4 KiB pages make each a TLB miss). */
static void* ho_alloc(uint64_t bytes)
{
    const uint64_t al = 2ull << 20, sz = (bytes + al - 1) / al * al;
    void* p = NULL;
    if (posix_memalign(&p, al, sz ? sz : al)) return NULL;
    if (sz >= al) (void)madvise(p, sz, MADV_HUGEPAGE);
    memset(p, 0, sz ? sz : al);
    return p;
}
static void ho_free(void* p, uint64_t bytes) { (void)bytes; free(p); }

#define HO_SEEDBUF (1u << 24)
#define HO_AHEAD 16
/* The random-access phases run on several threads, each owning a range of
 * K-mers and walking the collected seeds in order: every K-mer's counter and
 * list see exactly the sequential order of updates. */
typedef struct {
    uint32_t *num, *pos, *cur;
    const uint32_t *sk, *sp;
    uint32_t ns, maxcount;
    uint64_t lo, hi;   /* K-mers [lo, hi) */
} ho_job;

/* setSeednum: count the collected seeds in order (saturating at maxcount) */
static void* ho_count_job(void* arg)
{
    const ho_job* j = (const ho_job*)arg;
    for (uint32_t i = 0; i < j->ns; i++) {
        const uint32_t k = j->sk[i];
        if (k < j->lo || k >= j->hi) continue;
        if (j->num[k] < j->maxcount) j->num[k]++;
    }
    return NULL;
}
/* setSeedpos: the collected seeds' positions into their K-mers' lists, in order */
static void* ho_place_job(void* arg)
{
    const ho_job* j = (const ho_job*)arg;
    for (uint32_t i = 0; i < j->ns; i++) {
        const uint32_t k = j->sk[i];
        if (k < j->lo || k >= j->hi) continue;
        const uint32_t c = j->cur[k];
        if (c != UINT32_MAX) {
            j->pos[c] = j->sp[i];
            j->cur[k] = c + 1;
        }
    }
    return NULL;
}

static int ho_threads(void)
{
    long n = sysconf(_SC_NPROCESSORS_ONLN);
    const char* e = getenv("OMP_NUM_THREADS");
    if (e && atoi(e) > 0) n = atoi(e);
    return n < 1 ? 1 : n > 16 ? 16 : (int)n;
}

static uint32_t ho_run_jobs(void* (*fn)(void*), ho_job proto, uint64_t nkmers)
{
    enum { MAXT = 16 };
    const int T = proto.ns < 65536 ? 1 : ho_threads();
    ho_job jobs[MAXT];
    pthread_t th[MAXT];
    int started[MAXT] = {0};
    for (int t = 0; t < T; t++) {
        jobs[t] = proto;
        jobs[t].lo = nkmers * (uint64_t)t / (uint64_t)T;
        jobs[t].hi = nkmers * (uint64_t)(t + 1) / (uint64_t)T;
        if (t > 0) started[t] = pthread_create(&th[t], NULL, fn, &jobs[t]) == 0;
    }
    fn(&jobs[0]);
    for (int t = 1; t < T; t++) {
        if (started[t]) pthread_join(th[t], NULL);
        else fn(&jobs[t]);
    }
    return 0;
}
static uint32_t ho_count_seeds(uint32_t* num, const uint32_t* sk, uint32_t ns, uint32_t maxcount, uint64_t nk)
{
    const ho_job p = {num, NULL, NULL, sk, NULL, ns, maxcount, 0, 0};
    return ho_run_jobs(ho_count_job, p, nk);
}
static uint32_t ho_place_seeds(uint32_t* pos, uint32_t* cur, const uint32_t* sk, const uint32_t* sp, uint32_t ns,
                               uint64_t nk)
{
    const ho_job p = {NULL, pos, cur, sk, sp, ns, 0, 0, 0};
    return ho_run_jobs(ho_place_job, p, nk);
}

/* getdelim('\n') over a buffer: the next line [*at, end) including its '\n' */
static int next_line(const char* fa, uint64_t n, uint64_t* at, const char** line, uint64_t* len)
{
    if (*at >= n) return 0;
    const char* p = fa + *at;
    const char* e = (const char*)memchr(p, '\n', n - *at);
    const uint64_t l = e ? (uint64_t)(e - p) + 1 : n - *at;
    *line = p;
    *len = l;
    *at += l;
    return 1;
}

/* the bases the reference reads from a line: strlen(line) - 1 characters
 * (getdelim keeps the '\n'; strlen stops at a NUL) */
static uint64_t line_bases(const char* line, uint64_t len)
{
    const char* z = (const char*)memchr(line, 0, len);
    const uint64_t sl = z ? (uint64_t)(z - line) : len;
    return sl ? sl - 1 : 0;
}

/* HashAlignment::buildRefIndex@0x410190 with HashRefIndex32's setters
 * (setSeqint@0x41e580, setEndSeqint@0x41e5a0, setSeednum@0x41e5d0,
 * setSeedind@0x41e820, setSeedpos@0x41e5f0); K = param+0x1b64 (14), step =
 * +0x1b70 (2), maxcount = 2^(+0x1b6c) (65536; HashRefIndex32 ctor @0x41f750).
 * Returns 0, -1 on an empty or header-less FASTA. */
int ho_index_build(const char* fa, uint64_t n, uint32_t K, uint32_t step, uint32_t maxcount, ho_index* ix)
{
    memset(ix, 0, sizeof *ix);
    if (K < 1 || K > 16 || step < 1) return -1;
    ix->K = K;
    ix->step = step;
    ix->maxcount = maxcount;
    ix->nkmers = ho_mask(K) + 1;
    const uint64_t mask = ho_mask(K);
    uint8_t code[256], isn[256];   /* ho_code & 3 and the (c & 0xdf) == 'N' test per character */
    for (int c = 0; c < 256; c++) {
        code[c] = ho_code((char)c) & 3;
        isn[c] = (c & 0xdf) == 'N';
    }
    ix->seq = (uint32_t*)ho_alloc((n / 16 + 1) * 4);   /* initMemory@0x41e7e0: file size / 16 + 1 */
    ix->num = (uint32_t*)ho_alloc(ix->nkmers * 4);
    if (!ix->seq || !ix->num) return -1;
    /* pass 1: pack, count sampled seeds.  The seeds of a stretch of input are
     * collected first and counted in order after it (the same increments in
     * the same order), prefetching the counters ahead: genome-scale tables are
     * GBs and each seed is a random access. */
    uint32_t* sk = (uint32_t*)malloc(HO_SEEDBUF * 4);
    uint32_t* sp = (uint32_t*)malloc(HO_SEEDBUF * 4);
    if (!sk || !sp) { free(sk); free(sp); return -1; }
    uint32_t ns = 0;
    uint64_t at = 0, ll, pos = 0, lastword = 0;
    const char* line;
    uint32_t headers = 0, run = 0, kmer = 0;
    while (next_line(fa, n, &at, &line, &ll)) {
        if (line[0] == '>') {
            headers++;
            continue;
        }
        const uint64_t nb = line_bases(line, ll);
        if (!headers) {
            if (nb) { free(sk); free(sp); return -1; }   /* (see the header comment) */
            continue;
        }
        for (uint64_t j = 0; j < nb; j++) {
            const uint8_t ch = (uint8_t)line[j], c = code[ch];
            lastword = pos / 16;
            ix->seq[lastword] = (ix->seq[lastword] << 2) | c;
            kmer = (uint32_t)(((uint64_t)kmer << 2 | c) & mask);
            pos++;
            if (isn[ch]) run = 0;
            else if (run + 1 == K) {
                if (pos % step == 0) {
                    sk[ns++] = kmer;
                    /* (flushed inside the line: an unwrapped chromosome is one line) */
                    if (ns == HO_SEEDBUF) ns = ho_count_seeds(ix->num, sk, ns, maxcount, ix->nkmers);
                }
            } else run++;
        }
    }
    ns = ho_count_seeds(ix->num, sk, ns, maxcount, ix->nkmers);
    if (!headers) { free(sk); free(sp); return -1; }
    if (pos % 16) ix->seq[lastword] <<= 2 * (16 - pos % 16);
    ix->total = (uint32_t)pos;
    ix->nwords = (uint32_t)lastword + 1;
    /* setSeedind: drop seeds at the cap, exclusive scan */
    ix->ind = (uint32_t*)ho_alloc(ix->nkmers * 4);
    if (!ix->ind) { free(sk); free(sp); return -1; }
    uint32_t npos = 0;
    ix->ind[0] = 0;
    for (uint64_t c = 0; c < mask; c++) {
        if (ix->num[c] >= maxcount) ix->num[c] = 0;
        ix->ind[c + 1] = ix->ind[c] + ix->num[c];
        npos += ix->num[c];
    }
    if (ix->num[mask] >= maxcount) ix->num[mask] = 0;
    npos += ix->num[mask];
    ix->npos = npos;
    ix->pos = (uint32_t*)ho_alloc((uint64_t)(npos ? npos : 1) * 4);
    /* the write cursor of each K-mer's list (the reference's ind + running
     * count); dropped K-mers get none */
    uint32_t* cur = (uint32_t*)ho_alloc(ix->nkmers * 4);
    if (!ix->pos || !cur) { free(sk); free(sp); return -1; }
    for (uint64_t c = 0; c <= mask; c++) cur[c] = ix->num[c] ? ix->ind[c] : UINT32_MAX;
    /* pass 2: positions (1-based seed starts), in order */
    at = 0;
    pos = 0;
    run = 0;
    kmer = 0;
    while (next_line(fa, n, &at, &line, &ll)) {
        if (line[0] == '>') continue;
        const uint64_t nb = line_bases(line, ll);
        for (uint64_t j = 0; j < nb; j++) {
            const uint8_t ch = (uint8_t)line[j];
            kmer = (uint32_t)(((uint64_t)kmer << 2 | code[ch]) & mask);
            pos++;
            if (isn[ch]) run = 0;
            else if (run + 1 == K) {
                if (pos % step == 0) {
                    sk[ns] = kmer;
                    sp[ns++] = (uint32_t)(pos - (K - 1));
                    if (ns == HO_SEEDBUF) ns = ho_place_seeds(ix->pos, cur, sk, sp, ns, ix->nkmers);
                }
            } else run++;
        }
    }
    ho_place_seeds(ix->pos, cur, sk, sp, ns, ix->nkmers);
    ho_free(cur, ix->nkmers * 4);
    free(sk);
    free(sp);
    return 0;
}

/* HashRefIndex32::writeIndexFile@0x41ed00 ("%s.hash"): K, total bases, words,
 * positions (u32 each), then seq[words], num[4^K], ind[4^K], pos[positions] */
uint64_t ho_index_bytes(const ho_index* ix) { return 16 + 4ull * (ix->nwords + 2 * ix->nkmers + ix->npos); }

int ho_index_serialize(const ho_index* ix, uint8_t* out, uint64_t cap)
{
    if (cap < ho_index_bytes(ix)) return -1;
    const uint32_t hdr[4] = {ix->K, ix->total, ix->nwords, ix->npos};
    uint8_t* o = out;
    memcpy(o, hdr, 16), o += 16;
    memcpy(o, ix->seq, 4ull * ix->nwords), o += 4ull * ix->nwords;
    memcpy(o, ix->num, 4 * ix->nkmers), o += 4 * ix->nkmers;
    memcpy(o, ix->ind, 4 * ix->nkmers), o += 4 * ix->nkmers;
    memcpy(o, ix->pos, 4ull * ix->npos);
    return 0;
}

/* ---- alignment --------------------------------------------------------- */
/* aligner_args (calloc'd in HashAlignment::loadRefIndex@0x40fdc0): seed length,
 * max mismatches (param+0x1b60 = 7), genome length, the "good enough"
 * threshold (param+0x1b74 = 1) and two flags (0): ho_args, hash_oracle.h;
 * align_info: strand, mismatches (-1: unaligned), read length, 1-based
 * reference position, mismatch offsets and types: ho_align */

static uint32_t mis2(uint32_t x) /* g_mismatch_count@0x65a7c0: differing 2-bit groups */
{
    uint32_t m = 0;
    for (int k = 0; k < 16; k++) m += (x >> (2 * k)) & 3 ? 1 : 0;
    return m;
}

/* getHashSeeds@0x4107f0: the read packed 16 bases a word (codes & 3, the
 * last word left-aligned), every K-mer ending at i >= K - 1; returns the
 * number of N/IUPAC bases */
static int get_seeds(const char* r, int len, uint32_t* packed, uint32_t* seeds, uint32_t K)
{
    const uint64_t mask = ho_mask(K);
    int nn = 0, ns = 0;
    uint32_t kmer = 0;
    for (int w = 0; w <= (len - 1) >> 4; w++) packed[w] = 0;
    for (int i = 0; i < len; i++) {
        const uint8_t c = ho_code(r[i]);
        nn += c >= 4;
        kmer = (uint32_t)(((uint64_t)kmer << 2 | (c & 3)) & mask);
        packed[i >> 4] = (packed[i >> 4] << 2) | (c & 3);
        if (i >= (int)K - 1) seeds[ns++] = kmer;
    }
    if (len & 15) packed[(len - 1) >> 4] <<= 32 - 2 * (len & 15);
    return nn;
}

/* findHashSeeds@0x4108d0: among seeds from, from + 2, ... <= to, the one with
 * the fewest (non-zero, < maxcnt) reference positions; its index -> *out */
static int find_seed(const ho_index* ix, const uint32_t* seeds, int from, int to, int maxcnt, int stop_first,
                     int* out)
{
    uint32_t best = 100000;
    for (int i = from; i <= to; i += 2) {
        const uint32_t c = ix->num[seeds[i]];
        if (c && c < (uint32_t)maxcnt && c < best) {
            best = c;
            *out = i;
            if (stop_first) return 1;
        }
    }
    return best != 100000;
}

/* gaplessHashAlignPositions@0x410990: the read against the reference at
 * 1-based position pos.  A word-wise 2-bit compare first (N reads as A) with
 * an early exit past maxmis; then, unless that count already fails, a
 * base-wise pass listing the mismatches (N counts) up to a limit: *best when
 * the word count beat it, else maxmis + 1.  Success overwrites ai and returns
 * 1 (and lowers *best); failure sets ai->nmis = -1 and returns 0. */
static int align_at(uint64_t pos, const char* r, int len, const ho_args* a, const uint32_t* packed,
                    const ho_index* ix, int rev, ho_align* ai, int* best)
{
    const uint64_t p0 = pos - 1;
    const uint32_t off = (uint32_t)(p0 & 15);
    const int lw = (len - 1) >> 4, nfull = len >> 4;
    int mis = 0;
    if (a->maxmis >= 0) {
        uint64_t w = p0 >> 4;
        for (int j = 0;; j++, w++) {
            uint32_t ref = ix->seq[w];
            if (off) {
                const uint32_t nxt = ix->seq[w + 1];
                ref = (uint32_t)(((nxt >> (32 - 2 * off)) & ho_mask(off)) | (((uint64_t)ref << (2 * off)) & ~ho_mask(off)));
            }
            uint64_t x = ref ^ packed[j];
            if (j >= nfull) x &= ~ho_mask(16 - (len & 15));
            mis += (int)mis2((uint32_t)x);
            if (mis > a->maxmis || j + 1 > lw) break;
        }
    }
    int limit;
    if (*best > mis) limit = *best;
    else if (a->maxmis >= mis) limit = a->maxmis + 1;
    else {
        ai->nmis = -1;
        return 0;
    }
    int n = 0;
    if (len > 0) {
        if (p0 >= a->glen) n = a->maxmis + 1;
        else {
            uint64_t q = p0;
            for (int i = 0;; i++) {
                const uint32_t rb = (ix->seq[q >> 4] >> (30 - 2 * (q & 15))) & 3;
                const uint32_t rc = ho_code(r[i]);
                if (rb != rc) {
                    if (n == a->maxmis) {
                        n++;
                        break;
                    }
                    ai->mispos[n] = i;
                    ai->mistype[n] = rc > 3 ? 3 : HO_MISTYPE[rc + rb * 4];
                    n++;
                }
                if (i == len - 1) break;
                q++;
                if (q >= a->glen) {
                    n = a->maxmis + 1;
                    break;
                }
            }
        }
    }
    if (limit <= n) {
        ai->nmis = -1;
        return 0;
    }
    ai->pos = pos;
    ai->rev = (uint8_t)rev;
    ai->len = len;
    ai->nmis = n;
    if (n < *best) *best = n;
    return 1;
}

/* gaplessSEHashAlign@0x410d80: the reference positions of seed `so` (kmer)
 * as alignment starts, until one aligns within maxmis, *best reaches the
 * threshold, or more than 300 candidates were tried (cnt over the read).
 * (mode != 0, the mate-constrained variant, is not reached from doSEAlign /
 * doPEAlign.) */
static int try_seed(int so, const char* r, int len, const ho_args* a, uint32_t kmer, const uint32_t* packed,
                    const ho_index* ix, int rev, ho_align* ai, uint32_t* cnt, int* best, int thr)
{
    const uint32_t n = ix->num[kmer];
    int acc = 0;
    for (uint32_t j = 0; j < n; j++) {
        const uint64_t p = ix->pos[ix->ind[kmer] + j];
        if (p <= (uint64_t)(int64_t)so) continue;
        if (p >= (uint64_t)(int64_t)so + a->glen - (uint64_t)(int64_t)len) continue;
        (*cnt)++;
        const int got = align_at(p - (uint64_t)(int64_t)so, r, len, a, packed, ix, rev, ai, best);
        if (thr >= *best) return acc;
        if (ai->nmis >= 0 && ai->nmis <= a->maxmis) return acc;
        acc += got;
        if (*cnt > 300) return acc;
    }
    return acc;
}

/* hashAligner@0x410f50: the rarest even-offset seed, then the rarest odd one */
static void aligner(const char* r, int len, const ho_args* a, int* sidx, const uint32_t* packed,
                    const uint32_t* seeds, const ho_index* ix, ho_align* ai, uint32_t* cnt, int rev, int* best, int thr)
{
    for (int par = 0; par < 2; par++) {
        if (find_seed(ix, seeds, par, len - (int)a->K, 100000, 0, &sidx[par]))
            try_seed(sidx[par], r, len, a, seeds[sidx[par]], packed, ix, rev, ai, cnt, best, thr);
        if (thr >= *best || *cnt > 300) return;
        if (ai->nmis >= 0 && ai->nmis <= a->maxmis) return;
    }
}

/* hashAlignerShortPart@0x411070: the read in 2, 3 or 4 parts (len <= 44,
 * 45..75, > 75); the rarest seed (< 620 positions) of each part and parity
 * that differs from hashAligner's; if the last search found nothing, the
 * parts again, from `ovl` past each part's start to 8 before its end, first
 * qualifying seed */
static void aligner_parts(const char* r, int len, const ho_args* a, int* sidx, const uint32_t* packed,
                          const uint32_t* seeds, const ho_index* ix, ho_align* ai, uint32_t* cnt, int rev,
                          int* best, int thr)
{
    const int np = len > 75 ? 4 : len >= 45 ? 3 : 2;
    const int K = (int)a->K;
    const int ovl = len > np * K ? len / np - K : 0;
    int found = 0, b = 0;
    for (int p = 0; p < np; p++) {
        const int e = (len + b) / np, s = b / np;
        b += len;
        for (int par = 0; par < 2; par++) {
            found = find_seed(ix, seeds, s + par, e - K, 620, 0, &sidx[par + 2]);
            if (found && sidx[par + 2] != sidx[par]) {
                try_seed(sidx[par + 2], r, len, a, seeds[sidx[par + 2]], packed, ix, rev, ai, cnt, best, thr);
                if (thr >= *best || *cnt > 300) return;
                if (ai->nmis >= 0 && ai->nmis <= a->maxmis) return;
            }
        }
    }
    if (found) return;
    b = 0;
    for (int p = 0; p < np; p++) {
        const int e8 = (len + b) / np - 8, s = b / np + ovl;
        b += len;
        for (int par = 0; par < 2; par++) {
            const int to = e8 < len - K ? e8 : len - K;
            if (find_seed(ix, seeds, s + par, to, 620, 1, &sidx[par + 2]) && sidx[par + 2] != sidx[par]) {
                try_seed(sidx[par + 2], r, len, a, seeds[sidx[par + 2]], packed, ix, rev, ai, cnt, best, thr);
                if (thr >= *best || *cnt > 300) return;
                if (ai->nmis >= 0 && ai->nmis <= a->maxmis) return;
            }
        }
    }
}

/* rev@0x40d9a0: complement of an ACGT/acgt base (upper case), others unchanged */
static char ho_comp(char c)
{
    switch (c) {
    case 'A': case 'a': return 'T';
    case 'C': case 'c': return 'G';
    case 'G': case 'g': return 'C';
    case 'T': case 't': return 'A';
    default: return c;
    }
}

/* getHashAlignInfo@0x4113c0 (mode 0): forward then reverse-complement
 * hashAligner, then the same with hashAlignerShortPart, stopping at the first
 * alignment within maxmis or when more than 299 candidates were tried.  One
 * seed-index array serves all four calls (as the reference's stack array;
 * its unset slots start at -1 here, uninitialised there).  Returns the
 * mismatch count, or -1 (ai->nmis = -1) when the read does not align. */
/* ai is the caller's align_info and keeps its state between reads: the
 * reference's AlignEncode{SE,PE}Job::doAlign (@0x411910) passes the same
 * AlignParam member for every read of a block and nothing resets ai.nmis, so
 * hashAligner's "aligned already?" test (ai.nmis in [0, maxmis]) sees the
 * previous read's outcome until this read's first candidate is verified: when
 * the even-offset seed search finds nothing, an aligned predecessor ends the
 * strand's search before the odd offsets are tried. */
int ho_align_read(const ho_index* ix, const ho_args* a, const char* r, int len, ho_align* ai)
{
    if (len <= 0 || a->maxmis > HO_MAXMIS || a->K != ix->K) return -2;
    const int nw = ((len - 1) >> 4) + 1;
    uint32_t* pk = (uint32_t*)calloc((size_t)nw, 4);
    uint32_t* sd = (uint32_t*)calloc((size_t)len, 4);
    uint32_t* pk2 = (uint32_t*)calloc((size_t)nw, 4);
    uint32_t* sd2 = (uint32_t*)calloc((size_t)len, 4);
    char* rc = (char*)calloc((size_t)len + 1, 1);
    int sidx[4] = {-1, -1, -1, -1};
    int best = -1, ret;
    uint32_t cnt = 0;
    ai->rev = 0;
    const int nn = get_seeds(r, len, pk, sd, a->K);
    int thr = a->maxmis;
    if (!a->f15) thr = a->good < a->maxmis ? a->good : a->maxmis;
    if (nn > a->maxmis) {
        ai->nmis = -1;
        ret = best;
        goto done;
    }
    best = a->maxmis + 1;
    aligner(r, len, a, sidx, pk, sd, ix, ai, &cnt, 0, &best, thr);
    if (a->maxmis >= best) goto ok;
    if (cnt > 299) goto miss;
    for (int i = 0; i < len; i++) rc[i] = ho_comp(r[len - 1 - i]);
    ai->rev = 1;
    get_seeds(rc, len, pk2, sd2, a->K);
    aligner(rc, len, a, sidx, pk2, sd2, ix, ai, &cnt, 1, &best, thr);
    if (a->f14) goto end;
    if (a->maxmis >= best) goto ok;
    if (cnt > 299) goto miss;
    aligner_parts(r, len, a, sidx, pk, sd, ix, ai, &cnt, 0, &best, thr);
    if (a->maxmis >= best) goto ok;
    if (cnt > 299) goto miss;
    aligner_parts(rc, len, a, sidx, pk2, sd2, ix, ai, &cnt, 1, &best, thr);
end:
    if (best > a->maxmis) goto miss;
ok:
    ret = best;
    goto done;
miss:
    ai->nmis = -1;
    ret = -1;
done:
    free(pk);
    free(sd);
    free(pk2);
    free(sd2);
    free(rc);
    return ret;
}

/* ---- flat C entry points for the tests (ctypes) -------------------------- */
static ho_index g_ix;

/* builds the index of a FASTA buffer (keeps it for ho_align_reads); returns
 * the serialized .hash size, or -1 */
int64_t ho_build(const char* fa, uint64_t n, uint32_t K, uint32_t step, uint32_t maxcount)
{
    ho_index_free(&g_ix);
    if (ho_index_build(fa, n, K, step, maxcount, &g_ix)) {
        ho_index_free(&g_ix);
        return -1;
    }
    return (int64_t)ho_index_bytes(&g_ix);
}

int ho_serialize(uint8_t* out, uint64_t cap) { return ho_index_serialize(&g_ix, out, cap); }

uint32_t ho_genome_length(void) { return g_ix.total; }

const ho_index *ho_current_index(void) { return &g_ix; }

/* aligns n reads (seq + offsets / lengths), in order, against the last built
 * index; *ai_nmis: the carried align_info state (in: before the first read;
 * out: after the last).  Per read: ret (mismatches or -1), rev, pos and up to
 * maxmis mismatch offsets / types (row stride maxmis + 1) */
int ho_align_reads(const char* seq, const uint64_t* off, const int32_t* lens, int64_t n, int32_t maxmis,
                   int32_t good, int32_t* ai_nmis, int32_t* ret, uint8_t* rev, uint64_t* pos, int32_t* mispos,
                   int32_t* mistype)
{
    ho_args a = {g_ix.K, maxmis, g_ix.total, good, 0, 0};
    ho_align ai;
    memset(&ai, 0, sizeof ai);
    ai.nmis = *ai_nmis;   /* the align_info's state before the first read */
    for (int64_t i = 0; i < n; i++) {
        const int r = ho_align_read(&g_ix, &a, seq + off[i], lens[i], &ai);
        if (r == -2) return -1;
        ret[i] = r;
        rev[i] = r >= 0 ? ai.rev : 0;
        pos[i] = r >= 0 ? ai.pos : 0;
        for (int k = 0; k <= maxmis; k++) {
            mispos[i * (maxmis + 1) + k] = r >= 0 && k < ai.nmis ? ai.mispos[k] : -1;
            mistype[i * (maxmis + 1) + k] = r >= 0 && k < ai.nmis ? ai.mistype[k] : -1;
        }
    }
    *ai_nmis = ai.nmis;
    return 0;
}
