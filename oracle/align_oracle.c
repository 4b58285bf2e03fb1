/* align_oracle.c -- CPU restatement of SeqArc 1.6's reference (HASH index)
 * block path: the per-block alignment driver and the bookkeeping that turns
 * alignments into the SeqArcMemBuf arrays doAlignEncode@0x42d4c0 codes.
 *
 * TEST INFRASTRUCTURE ONLY (see fqz_oracle.h): only tests/ and bench.py's
 * cpu_baseline leg load it.  Restated from static disassembly of
 * /root/reference/SeqArc-1.6 (never executed).  PARITY UNPINNED: the reference
 * ships no index, no aligned archive and no fixture of this path; the one
 * undetermined input is the align_info state the encode thread starts with
 * (AlignParam@0x405b00 leaves nmis uninitialised in a fresh operator-new
 * chunk): callers pass it (0, i.e. "aligned", for a fresh heap).
 *
 * Routines:
 *   getbitnum@0x40d470, int2bit@0x40dcd0, decomposeAlignInfo@0x433860,
 *   AlignEncodeSEJob::AlignInfoProcess@0x4118b0 / doAlign@0x411910,
 *   AlignEncodePEJob::AlignInfoProcessPE@0x412290 / doAlign@0x413580 /
 *   CaclInsertSize@0x413270, HashAlignment::loadRefIndex@0x40fdc0 (shift and
 *   mask of the position split, param+0x1858 / +0x1860).
 */
#include <stdlib.h>
#include <string.h>

#include "fqz_oracle.h"
#include "hash_oracle.h"

typedef struct {
    uint8_t *v;
    uint32_t n, cap;
} bv8;

static int push(bv8 *a, uint8_t x)
{
    if (a->n == a->cap) {
        uint32_t nc = a->cap ? a->cap * 2 : 4096;
        uint8_t *nv = (uint8_t *)realloc(a->v, nc);
        if (!nv) return -1;
        a->v = nv;
        a->cap = nc;
    }
    a->v[a->n++] = x;
    return 0;
}

/* getbitnum@0x40d470: bits of v (0 for 0) */
static int getbitnum(uint64_t v)
{
    int n = 0;
    while (v) { n++; v >>= 1; }
    return n;
}

/* int2bit@0x40dcd0: v as exactly nbits bits, least significant first; the
 * reference asserts nbits >= the bits v needs (-1 here) */
static int int2bit(uint64_t v, int nbits, bv8 *a)
{
    int cnt = 0;
    for (; v; v >>= 1, cnt++)
        if (push(a, (uint8_t)(v & 1))) return -1;
    if (nbits < cnt) return -1;
    for (; cnt < nbits; cnt++)
        if (push(a, 0)) return -1;
    return 0;
}

typedef struct {
    bv8 order, pos, cigal, mis, rev, cigav, perel;
    uint32_t align_count;
    int shift;          /* param+0x1858 = getbitnum(glen) - 2 */
    uint64_t mask;      /* param+0x1860 = 2^shift - 1          */
    uint64_t glen;      /* param+0x1868                        */
    int err;
} astate;

/* decomposeAlignInfo@0x433860: mismatch offsets as gaps (bits sized by the
 * rest of the read), their types, the count, the strand; one aligned read */
static void decompose(astate *s, const ho_align *ai)
{
    int prev = 0, rem = ai->len;
    for (int k = 0; k < ai->nmis; k++) {
        s->err |= int2bit((uint64_t)(int64_t)(ai->mispos[k] - prev), getbitnum((uint64_t)(int64_t)rem), &s->cigal);
        prev = ai->mispos[k];
        rem = ai->len - prev;
        s->err |= push(&s->cigav, (uint8_t)ai->mistype[k]);
    }
    s->err |= push(&s->mis, (uint8_t)ai->nmis);
    s->err |= push(&s->rev, ai->rev);
    s->align_count++;
}

/* AlignEncodeSEJob::AlignInfoProcess@0x4118b0: low position bits, then the
 * mismatches; returns pos >> shift (the order byte is that + 1) */
static uint64_t info_se(astate *s, const ho_align *ai)
{
    s->err |= int2bit(ai->pos & s->mask, s->shift, &s->pos);
    decompose(s, ai);
    return ai->pos >> s->shift;
}

/* AlignEncodePEJob::AlignInfoProcessPE@0x412290 */
static void info_pe(astate *s, const ho_align *a1, const ho_align *a2, uint32_t win, int ibits)
{
    if (a1->nmis < 0) {
        if (a2->nmis < 0) {
            s->err |= push(&s->order, 0);
            s->err |= push(&s->order, 0);
        } else {
            s->err |= int2bit(a2->pos & s->mask, s->shift, &s->pos);
            decompose(s, a2);
            s->err |= push(&s->order, 0);
            s->err |= push(&s->order, (uint8_t)((a2->pos >> s->shift) + 1));
        }
        return;
    }
    if (a2->nmis < 0) {
        s->err |= int2bit(a1->pos & s->mask, s->shift, &s->pos);
        decompose(s, a1);
        s->err |= push(&s->order, (uint8_t)((a1->pos >> s->shift) + 1));
        s->err |= push(&s->order, 0);
        return;
    }
    s->err |= int2bit(a1->pos & s->mask, s->shift, &s->pos);
    const uint64_t o = a1->pos >> s->shift;
    decompose(s, a1);
    const int64_t sd = (int64_t)a1->pos - (int64_t)a2->pos;
    const uint64_t d = (uint64_t)(sd < 0 ? -sd : sd);
    if (d < (uint64_t)win) {           /* the mate within the insert window */
        s->err |= push(&s->perel, a1->pos < a2->pos ? 1 : 0);
        s->err |= int2bit(d, ibits, &s->pos);
    } else if (a1->pos < a2->pos) {    /* further right: the distance */
        s->err |= push(&s->perel, 3);
        s->err |= int2bit(d, getbitnum(s->glen - a1->pos), &s->pos);
    } else {                           /* further left: the position itself */
        s->err |= push(&s->perel, 2);
        s->err |= int2bit(a2->pos, getbitnum(a1->pos), &s->pos);
    }
    decompose(s, a2);
    s->err |= push(&s->order, (uint8_t)(o + 1));
    s->err |= push(&s->order, (uint8_t)(o + 1));
}

static int cmp_int(const void *x, const void *y)
{
    const int a = *(const int *)x, b = *(const int *)y;
    return a < b ? -1 : a > b;
}

/* AlignEncodePEJob::CaclInsertSize@0x413270 (over the distances of the first
 * pairs of a block that both aligned within 20000): the median, then the
 * smallest window med +- 2^e (e = 2, 3, ...) holding more than 90 % of them;
 * win = 2^(e + 1), bits = e + 1, and membuf+0x28 = bits.  No distances:
 * win 512, bits 9. */
static void calc_insert(int *v, size_t n, uint32_t *win, int *bits)
{
    if (n == 0) {
        *win = 0x200;
        *bits = 9;
        return;
    }
    qsort(v, n, sizeof(int), cmp_int);
    const int N = (int)n;
    int med, lo, hi;
    if (N & 1) {
        lo = hi = (N - 1) / 2;
        med = v[lo];
    } else {
        lo = (N - 2) / 2;
        hi = lo + 1;
        med = (v[lo] + v[lo + 1]) / 2;
    }
    const int thr = (int)(0.9 * (double)N);   /* @0x44a2b8 */
    for (int e = 2;; e++) {
        const int w = (int)(1u << e);
        const int a = med - w, b = med + w;
        while (lo >= 0 && v[lo] > a) lo--;
        while (hi < N && v[hi] < b) hi++;
        if (thr < hi - lo) {
            *win = (uint32_t)(b - a);
            *bits = e + 1;
            return;
        }
    }
}

/* DegeInfoProcess@0x433a10's return: the read's bases outside ACGT/acgt */
static int n_dege(const uint8_t *s, int len)
{
    int n = 0;
    for (int i = 0; i < len; i++) {
        switch (s[i]) {
        case 'A': case 'C': case 'G': case 'T': case 'a': case 'c': case 'g': case 't': break;
        default: n++;
        }
    }
    return n;
}

/* getHashAlignInfo@0x4113c0 on the carried align_info (a zero-length read does
 * not align) */
static void align_one(const ho_index *ix, const ho_args *a, const uint8_t *r, int len, ho_align *ai)
{
    if (len <= 0 || ho_align_read(ix, a, (const char *)r, len, ai) < 0) ai->nmis = -1;
}

static void st_free(astate *s)
{
    free(s->order.v); free(s->pos.v); free(s->cigal.v); free(s->mis.v);
    free(s->rev.v); free(s->cigav.v); free(s->perel.v);
}

int64_t orc_encode_block_hash(const orc_block *b, const orc_cfg *cfg, int paired, int maxmis, int good,
                              uint32_t insert_size, int32_t carry[2], uint8_t *out, size_t cap)
{
    const ho_index *ix = ho_current_index();
    if (!ix->seq || maxmis < 0 || maxmis > HO_MAXMIS || ix->total < 4) return -1;
    if (paired && (b->nreads & 1)) return -1;
    const ho_args args = {ix->K, maxmis, ix->total, good, 0, 0};
    astate s;
    memset(&s, 0, sizeof s);
    s.glen = ix->total;
    s.shift = getbitnum(s.glen) - 2;                 /* loadRefIndex@0x40fe9b */
    s.mask = (1ull << s.shift) - 1;
    /* per-read offsets */
    uint64_t *off = (uint64_t *)malloc(((size_t)b->nreads + 1) * 8);
    if (!off) return -1;
    off[0] = 0;
    for (uint32_t r = 0; r < b->nreads; r++) off[r + 1] = off[r] + (uint64_t)(b->seq_lens[r] > 0 ? b->seq_lens[r] : 0);
    const int limit = (int)((double)(int)b->nreads * 0.05);   /* @0x44a218 */
    uint32_t insert_bits = 0;
    int64_t ret = -1;
    if (!paired) {
        /* AlignEncodeSEJob::doAlign@0x411910 */
        ho_align ai;
        memset(&ai, 0, sizeof ai);
        ai.nmis = carry[0];
        int checking = 1;
        for (uint32_t i = 0; i < b->nreads;) {
            const int len = b->seq_lens[i] > 0 ? b->seq_lens[i] : 0;
            const uint8_t *rd = b->seq + off[i];
            uint8_t ord = 0;
            if (n_dege(rd, len) <= maxmis) {   /* else the aligner is not called */
                align_one(ix, &args, rd, len, &ai);
                if (ai.nmis >= 0) ord = (uint8_t)(info_se(&s, &ai) + 1);
            }
            s.err |= push(&s.order, ord);
            i++;
            if ((uint32_t)limit < i && checking) {
                if ((double)i * 0.5 > (double)s.align_count) break;   /* bail out: the rest unaligned */
                checking = 0;
            }
        }
        carry[0] = ai.nmis;
    } else {
        /* AlignEncodePEJob::doAlign@0x413580 */
        ho_align a1, a2;
        memset(&a1, 0, sizeof a1);
        memset(&a2, 0, sizeof a2);
        a1.nmis = carry[0];
        a2.nmis = carry[1];
        uint32_t win = insert_size;
        int ibits = insert_size ? getbitnum(insert_size) : 0;   /* job ctor @0x412ec2 */
        ho_align *def = (ho_align *)malloc(sizeof(ho_align) * ((size_t)b->nreads + 2));
        int *ins = (int *)malloc(sizeof(int) * ((size_t)b->nreads / 2 + 1));
        size_t ndef = 0, nins = 0;
        if (!def || !ins) s.err = 1;
        int checking = 1;
        for (uint32_t r = 0; r < b->nreads && !s.err;) {
            const int l1 = b->seq_lens[r] > 0 ? b->seq_lens[r] : 0, l2 = b->seq_lens[r + 1] > 0 ? b->seq_lens[r + 1] : 0;
            align_one(ix, &args, b->seq + off[r], l1, &a1);
            align_one(ix, &args, b->seq + off[r + 1], l2, &a2);
            if (win) info_pe(&s, &a1, &a2, win, ibits);
            else {
                if (a1.nmis >= 0 && a2.nmis >= 0) {
                    const int64_t sd = (int64_t)a1.pos - (int64_t)a2.pos;
                    const int64_t d = sd < 0 ? -sd : sd;
                    if (d <= 0x4e1f) ins[nins++] = (int)d;
                }
                def[ndef++] = a1;
                def[ndef++] = a2;
            }
            r += 2;
            if ((int)r > limit && checking) {
                if (!insert_size) calc_insert(ins, nins, &win, &ibits), insert_bits = (uint32_t)ibits;
                for (size_t k = 0; k < ndef; k += 2) info_pe(&s, &def[k], &def[k + 1], win, ibits);
                ndef = 0;
                if ((double)(int)r * 0.5 > (double)s.align_count) break;
                checking = 0;
            }
        }
        free(def);
        free(ins);
        carry[0] = a1.nmis;
        carry[1] = a2.nmis;
    }
    free(off);
    if (!s.err) {
        orc_align_streams as;
        memset(&as, 0, sizeof as);
        as.paired = paired;
        as.maxmis = maxmis;
        as.order_count = s.order.n;
        as.align_count = s.align_count;
        as.insert_bits = insert_bits;
        as.order = s.order.v;
        as.pos = s.pos.v, as.npos = s.pos.n;
        as.cigal = s.cigal.v, as.ncigal = s.cigal.n;
        as.mis = s.mis.v, as.nmis = s.mis.n;
        as.rev = s.rev.v, as.nrev = s.rev.n;
        as.cigav = s.cigav.v, as.ncigav = s.cigav.n;
        as.perel = s.perel.v, as.nperel = s.perel.n;
        ret = orc_encode_block_aligned(b, cfg, &as, out, cap);
    }
    st_free(&s);
    return ret;
}
