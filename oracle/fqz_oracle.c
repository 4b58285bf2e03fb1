/*
 * fqz_oracle.c -- CPU restatement of the SeqArc-1.6 no-reference block encoder.
 *
 * TEST INFRASTRUCTURE ONLY (see fqz_oracle.h).  The product never links this.
 *
 * Every routine cites the address in /root/reference/SeqArc-1.6 of the routine
 * whose behaviour it restates (static disassembly; the binary is never run).
 * The entropy core is fqzcomp-4.x (J. Bonfield), vendored and inlined in the
 * reference; the restatement follows the binary, not upstream fqzcomp.
 */
#include "fqz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Range coder: inlined everywhere, e.g. encode_seq@0x422010-0x422085,       */
/* finish = 8 x (low>>56) @0x424a1c.                                         */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint64_t low;
    uint32_t range;
    uint8_t *out;
    uint8_t *end;
    int      err;
} rc_t;

static void rc_init(rc_t *rc, uint8_t *out, uint8_t *end)
{
    rc->low = 0;
    rc->range = 0xffffffffu;
    rc->out = out;
    rc->end = end;
    rc->err = 0;
}

static void rc_put(rc_t *rc, uint8_t b)
{
    if (rc->out < rc->end) *rc->out++ = b;
    else rc->err = 1;
}

static void rc_encode(rc_t *rc, uint32_t cum, uint32_t freq, uint32_t tot)
{
    uint32_t r = rc->range / tot;
    rc->low += (uint32_t)(cum * r);
    rc->range = r * freq;
    if (cum + freq > tot) { rc->err = 1; return; }   /* reference: abort() */
    while (rc->range < (1u << 24)) {
        if ((rc->low ^ (rc->low + rc->range)) >> 56)
            rc->range = ((uint32_t)rc->low | 0xffffffu) - (uint32_t)rc->low;
        rc_put(rc, (uint8_t)(rc->low >> 56));
        rc->range <<= 8;
        rc->low <<= 8;
    }
}

static void rc_finish(rc_t *rc)
{
    for (int i = 0; i < 8; i++) {
        rc_put(rc, (uint8_t)(rc->low >> 56));
        rc->low <<= 8;
    }
}

int64_t orc_rc_encode(const uint16_t *cum, const uint16_t *freq, const uint16_t *tot, size_t n,
                      uint8_t *out, size_t cap)
{
    rc_t rc;
    rc_init(&rc, out, out + cap);
    for (size_t i = 0; i < n && !rc.err; i++) rc_encode(&rc, cum[i], freq[i], tot[i]);
    rc_finish(&rc);
    return rc.err ? -1 : (int64_t)(rc.out - out);
}

/* ------------------------------------------------------------------------ */
/* SIMPLE_MODEL<N>: layout {u32 TotFreq, u32 BubCnt, sentinel, F[N+1]}.      */
/* Clearest inlined instance: kModelEncode@0x42ccb0; init @0x426f30.         */
/* ------------------------------------------------------------------------ */
typedef struct { uint16_t sym, freq; } sf_t;
typedef struct {
    uint32_t tot, bub;
    sf_t     sentinel;
    sf_t     F[257];
} smodel;

static void sm_init(smodel *m, int n)
{
    m->tot = (uint32_t)n;
    m->bub = 0;
    m->sentinel.sym = 0;
    m->sentinel.freq = 0xffe0;
    for (int i = 0; i < n; i++) { m->F[i].sym = (uint16_t)i; m->F[i].freq = 1; }
    m->F[n].sym = 0;
    m->F[n].freq = 0;
}

static void sm_encode(smodel *m, rc_t *rc, uint16_t sym)
{
    sf_t *s = m->F;
    uint32_t acc = 0;
    while (s->sym != sym) {
        if (s->freq == 0) { rc->err = 1; return; }   /* symbol outside model */
        acc += s->freq;
        s++;
    }
    rc_encode(rc, acc, s->freq, m->tot);
    s->freq += 8;
    m->tot += 8;
    if (m->tot > 0xffe0) {
        m->tot = 0;
        for (sf_t *p = m->F; p->freq; p++) {
            p->freq -= p->freq >> 1;
            m->tot += p->freq;
        }
    }
    if (((++m->bub) & 15) == 0 && s[0].freq > s[-1].freq) {
        sf_t t = s[0];
        s[0] = s[-1];
        s[-1] = t;
    }
}

/* ------------------------------------------------------------------------ */
/* Encap (EBML-style VINTs): setID@0x420720, setSize@0x420780.               */
/* ------------------------------------------------------------------------ */
static int encap_set_id(uint64_t v, uint8_t *out)
{
    int n = 1;
    for (; n < 9; n++) {
        /* 32-bit shift in the binary: (1 << (7n mod 32)) - 2 */
        int64_t lim = (int64_t)(int32_t)((1u << ((7 * n) & 31)) - 2u);
        if ((uint64_t)lim >= v) { v |= (uint64_t)(lim + 2); break; }
    }
    for (int i = n - 1; i >= 0; i--) *out++ = (uint8_t)(v >> (8 * i));
    return n;
}

static void encap_set_size(uint64_t v, int width, uint8_t *out)
{
    v |= (uint64_t)1 << (7 * width);
    for (int i = width - 1; i >= 0; i--) *out++ = (uint8_t)(v >> (8 * i));
}

static void put_u32le(uint8_t *p, uint32_t v)  /* IntTo4Ch@0x40dae0 */
{
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

/* ------------------------------------------------------------------------ */
/* MD5: RFC 1321 (vendored RSA reference; MDString@0x4058f0).                */
/* ------------------------------------------------------------------------ */
#define ROL(x, c) (((x) << (c)) | ((x) >> (32 - (c))))
static const uint32_t md5_K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const int md5_S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static void md5_block(uint32_t h[4], const uint8_t *p)
{
    uint32_t M[16];
    for (int i = 0; i < 16; i++)
        M[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) |
               ((uint32_t)p[4 * i + 2] << 16) | ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        uint32_t t = d;
        d = c;
        c = b;
        b = b + ROL(a + f + md5_K[i] + M[g], md5_S[i]);
        a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}

void orc_md5(const uint8_t *data, size_t len, uint8_t digest[16])
{
    uint32_t h[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
    size_t i = 0;
    for (; i + 64 <= len; i += 64) md5_block(h, data + i);
    uint8_t tail[128];
    size_t rem = len - i;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, data + i, rem);
    tail[rem] = 0x80;
    size_t tl = (rem < 56) ? 64 : 128;
    /* the RSA MDString takes an unsigned int length: bit count mod 2^64 of (u32)len */
    uint64_t bits = (uint64_t)(uint32_t)len << 3;
    for (int k = 0; k < 8; k++) tail[tl - 8 + k] = (uint8_t)(bits >> (8 * k));
    md5_block(h, tail);
    if (tl == 128) md5_block(h, tail + 64);
    for (int k = 0; k < 4; k++) put_u32le(digest + 4 * k, h[k]);
}

/* ------------------------------------------------------------------------ */
/* Base code table seq_val_table@0x44b800 (same values at 0x44bd00):         */
/* A/a=0 C/c=1 G/g=2 T/t=3, IUPAC M R Y K S W H B V D = 5..14, other ASCII 4. */
/* Bytes >= 0x80 index memory before the table in the reference (undefined); */
/* the restatement maps them to 4 and the product rejects such input.        */
/* ------------------------------------------------------------------------ */
static uint8_t base_code(uint8_t c)
{
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    case 'M': case 'm': return 5;
    case 'R': case 'r': return 6;
    case 'Y': case 'y': return 7;
    case 'K': case 'k': return 8;
    case 'S': case 's': return 9;
    case 'W': case 'w': return 10;
    case 'H': case 'h': return 11;
    case 'B': case 'b': return 12;
    case 'V': case 'v': return 13;
    case 'D': case 'd': return 14;
    default: return 4;
    }
}

/* ------------------------------------------------------------------------ */
/* Sequence stream: compressSeq@0x4248a0 + encode_seq@0x421f30.              */
/* BASE_MODEL<u8>: 4 u8 counts per context, init 3 (reset per block at       */
/* 0x424934); halve (c -= c>>1) when sum > 253; code; c[b]++.                */
/* k = Slevel + 7 (ctor 0x42f63e); NS = 1u << ((2k) & 31) (x86 shl masks).   */
/* ------------------------------------------------------------------------ */
/* skip / nskip: the reference path's compressSeq (@0x424976-0x4249d5) codes
 * only the reads r < nskip with skip[r] == 0 (order byte 0: not aligned) and
 * every read from nskip on; NULL: every read (no reference) */
static int64_t seq_payload_sel(const orc_block *b, int k, const uint8_t *skip, uint32_t nskip, uint8_t *out,
                               uint8_t *end);
static int64_t seq_payload(const orc_block *b, int k, uint8_t *out, uint8_t *end)
{
    return seq_payload_sel(b, k, NULL, 0, out, end);
}

static int64_t seq_payload_sel(const orc_block *b, int k, const uint8_t *skip, uint32_t nskip, uint8_t *out,
                               uint8_t *end)
{
    uint32_t ns = 1u << ((2 * k) & 31);
    uint32_t mask = ns - 1;
    uint8_t *tab = (uint8_t *)malloc((size_t)ns * 4);
    if (!tab) return -1;
    memset(tab, 3, (size_t)ns * 4);
    rc_t rc;
    rc_init(&rc, out, end);
    const uint8_t *p = b->seq;
    for (uint32_t r = 0; r < b->nreads; r++) {
        int32_t len = b->seq_lens[r];
        uint32_t ctx = 0x7616c7u & mask;
        if (skip && r < nskip && skip[r]) {
            if (len > 0) p += len;
            continue;
        }
        for (int32_t i = 0; i < len; i++) {
            uint8_t c = base_code(p[i]);
            if (c > 3) continue;
            uint8_t *m = tab + (size_t)ctx * 4;
            uint32_t tot = (uint32_t)m[0] + m[1] + m[2] + m[3];
            if (tot > 253) {
                for (int j = 0; j < 4; j++) m[j] = (uint8_t)(m[j] - (m[j] >> 1));
                tot = (uint32_t)m[0] + m[1] + m[2] + m[3];
            }
            uint32_t cum = 0;
            for (int j = 0; j < c; j++) cum += m[j];
            rc_encode(&rc, cum, m[c], tot);
            m[c]++;
            ctx = ((ctx << 2) + c) & mask;
        }
        if (len > 0) p += len;
    }
    rc_finish(&rc);
    free(tab);
    return rc.err ? -1 : (int64_t)(rc.out - out);
}

int64_t orc_seq_payload(const orc_block *b, int k, uint8_t *out, size_t cap)
{
    return seq_payload(b, k, out, out + cap);
}

static uint64_t total_seq(const orc_block *b)
{
    uint64_t t = 0;
    for (uint32_t r = 0; r < b->nreads; r++) t += (uint64_t)(int64_t)b->seq_lens[r];
    return t;
}

static uint64_t total_names(const orc_block *b)
{
    uint64_t t = 0;
    for (uint32_t r = 0; r < b->nreads; r++) t += b->name_lens[r];
    return t;
}

/* encap = setID(id) + 4-byte size + [md5] + payload */
int64_t orc_encap_seq(const orc_block *b, const orc_cfg *cfg, uint8_t *out, size_t cap)
{
    if (cap < 32) return -1;
    int n = encap_set_id(6, out);
    uint8_t *p = out + n + 4;
    int hdr = 0;
    if (cfg->md5) {
        orc_md5(b->seq, (size_t)total_seq(b), p);
        p += 16;
        hdr = 16;
    }
    int64_t pl = seq_payload(b, cfg->slevel + 7, p, out + cap);
    if (pl < 0) return -1;
    encap_set_size((uint64_t)(hdr + pl), 4, out + n);
    return n + 4 + hdr + pl;
}

/* ------------------------------------------------------------------------ */
/* Quality stream: compressQual@0x426e80 + encode_qual@0x422180.             */
/* 65536 (Qlevel<=2) or 0x100000 SIMPLE_MODEL<95>, reset per block @0x426f10. */
/* ------------------------------------------------------------------------ */
static int64_t qual_payload(const orc_block *b, int qlevel, uint8_t *out, uint8_t *end)
{
    uint32_t nm = qlevel > 2 ? 0x100000u : 0x10000u;
    smodel *models = (smodel *)malloc((size_t)nm * sizeof(smodel));
    if (!models) return -1;
    for (uint32_t i = 0; i < nm; i++) sm_init(&models[i], 95);
    rc_t rc;
    rc_init(&rc, out, end);
    const uint8_t *q = b->qual;
    for (uint32_t r = 0; r < b->nreads && !rc.err; r++) {
        int32_t len = b->seq_lens[r];
        if (len <= 0) continue;
        int32_t n = len;
        while (n > 0 && q[n - 1] == '#') n--;       /* strip trailing '#' */
        uint32_t last = 0;
        int q1 = 0, q2 = 0, delta = 5;
        for (int32_t i = 0; i < n; i++) {
            int sym = (uint8_t)(q[i] - 33);
            if (sym > 93) { rc.err = 1; break; }       /* outside the 95-symbol model */
            sm_encode(&models[last], &rc, (uint16_t)sym);
            uint32_t ctx = ((uint32_t)((q1 > q2 ? q1 : q2) << 6) + (uint32_t)sym) & 0xfffu;
            if (qlevel > 1) {
                ctx += (q1 == q2) ? 0x1000u : 0u;
                delta += (q1 > sym) ? (q1 - sym) : 0;
                ctx += (uint32_t)(((delta <= 56 ? delta : 56) & 0xf8) << 10);
                if (qlevel > 2)
                    ctx += (i <= 0x6f) ? (uint32_t)(((i + 15) & 0x78) << 13) : 0xf0000u;
            }
            q2 = q1;
            q1 = sym;
            last = ctx;
        }
        if (n != len) sm_encode(&models[last], &rc, 94);
        q += len;
    }
    rc_finish(&rc);
    free(models);
    return rc.err ? -1 : (int64_t)(rc.out - out);
}

int64_t orc_qual_payload(const orc_block *b, int qlevel, uint8_t *out, size_t cap)
{
    return qual_payload(b, qlevel, out, out + cap);
}

/* EncapFqzComp::rblock@0x426c10, restated from the disassembly.  One greedy
 * pass over the block's whole quality buffer (runs cross read boundaries; the
 * reference stops at the '\n' after the last quality).  A run keeps its min and
 * max; a new character c inside [min, max] extends it; c > max extends it iff
 * R > g/min and R > c/g with g = round(sqrt(c*min)) (@0x426cc0); c < min iff
 * R > g/c and R > max/g with g = round(sqrt(c*max)) (@0x426d48); otherwise the
 * run [start, i) is overwritten with round(sqrt(min*max)) (@0x426c6d) and a new
 * run starts at i.  The last run is flushed at the terminator (@0x426dd0). */
void orc_rblock(uint8_t *q, size_t n, double ratio)
{
    if (n == 0) return;
    uint32_t start = 0;
    uint32_t mx = q[0], mn = q[0];    /* r13d, edx */
    for (uint32_t i = 1; i < (uint32_t)n; i++) {
        const uint32_t c = q[i];
        int ext;
        if (mx >= c) {
            if (mn <= c) continue;                       /* inside [min, max] */
            uint32_t g = (uint32_t)(int64_t)round(sqrt((double)(uint64_t)(c * mx)));
            ext = ratio > (double)g / (double)c && ratio > (double)mx / (double)g;
            if (ext) { mn = c; continue; }
        } else {
            uint32_t g = (uint32_t)(int64_t)round(sqrt((double)(uint64_t)(c * mn)));
            ext = ratio > (double)g / (double)mn && ratio > (double)c / (double)g;
            if (ext) { mx = c; continue; }
        }
        const uint8_t g = (uint8_t)(int64_t)round(sqrt((double)(uint64_t)(mx * mn)));
        for (uint32_t j = start; j < i; j++) q[j] = g;
        mx = mn = c;
        start = i;
    }
    const uint8_t g = (uint8_t)(int64_t)round(sqrt((double)(uint64_t)(mx * mn)));
    for (uint32_t j = start; j < (uint32_t)n; j++) q[j] = g;
}

/* compressQual@0x426e80: the MD5 is written only when param+0x1880 is set and
 * the lossy flag param+0x1870 is clear (@0x426eca-0x426ee4); with -l the block's
 * quality buffer goes through rblock before encode_qual (@0x427142).  The
 * N/IUPAC side streams keep the original qualities (DegeInfoProcess@0x433a10
 * runs in doTask@0x433dd0 before doFqzEncode). */
int64_t orc_encap_qual(const orc_block *b, const orc_cfg *cfg, uint8_t *out, size_t cap)
{
    if (cap < 32) return -1;
    int n = encap_set_id(7, out);
    uint8_t *p = out + n + 4;
    int hdr = 0;
    const int lossy = cfg->lossy > 0.0;
    if (cfg->md5 && !lossy) {
        orc_md5(b->qual, (size_t)total_seq(b), p);
        p += 16;
        hdr = 16;
    }
    int64_t pl;
    if (lossy) {
        const size_t nq = (size_t)total_seq(b);
        uint8_t *lq = (uint8_t *)malloc(nq ? nq : 1);
        if (!lq) return -1;
        memcpy(lq, b->qual, nq);
        orc_rblock(lq, nq, cfg->lossy);
        orc_block lb = *b;
        lb.qual = lq;
        pl = qual_payload(&lb, cfg->qlevel, p, out + cap);
        free(lq);
    } else {
        pl = qual_payload(b, cfg->qlevel, p, out + cap);
    }
    if (pl < 0) return -1;
    encap_set_size((uint64_t)(hdr + pl), 4, out + n);
    return n + 4 + hdr + pl;
}

/* ------------------------------------------------------------------------ */
/* Length stream: compressLen@0x424120 -> compressLen_short@0x423f50 ->      */
/* encode_len_short@0x4239a0.  same_len SIMPLE_MODEL<2>, lo/hi <256>.        */
/* last_len (+0x1060) is compared but never updated: always 0.               */
/* ------------------------------------------------------------------------ */
/* compressLen@0x424120 picks compressLen_long@0x423710 when the block's
 * long-read flag (SeqArcMemBuf+0x2) is set: getBlockRead@0x411d2a (and the PE
 * parse @0x412a76/0x412bb3) sets it for any read longer than 0xffff; it is
 * cleared per block (clearCommonBuf@0x414b18).  encode_len_long@0x422e70 codes
 * same_len, then all four length bytes, each with its own SIMPLE_MODEL<256>
 * (+0x8, +0x418 -- the short path's lo/hi -- then +0x828, +0xc38). */
int64_t orc_encap_len(const orc_block *b, uint8_t *out, size_t cap)
{
    if (cap < 16) return -1;
    int lng = 0;
    for (uint32_t r = 0; r < b->nreads; r++)
        if (b->seq_lens[r] > 0xffff) lng = 1;
    int n = encap_set_id(4, out);
    uint8_t *p = out + n + 4;
    smodel *m = (smodel *)malloc(5 * sizeof(smodel));
    if (!m) return -1;
    smodel *same = &m[0], *by = &m[1];
    sm_init(same, 2);
    for (int k = 0; k < 4; k++) sm_init(&by[k], 256);
    rc_t rc;
    rc_init(&rc, p, out + cap);
    const int32_t last_len = 0;
    for (uint32_t r = 0; r < b->nreads; r++) {
        int32_t len = b->seq_lens[r];
        if (len == last_len) {
            sm_encode(same, &rc, 1);
        } else {
            sm_encode(same, &rc, 0);
            for (int k = 0; k < (lng ? 4 : 2); k++)
                sm_encode(&by[k], &rc, (uint16_t)(((uint32_t)len >> (8 * k)) & 0xff));
        }
    }
    rc_finish(&rc);
    free(m);
    if (rc.err) return -1;
    int64_t pl = rc.out - p;
    encap_set_size((uint64_t)pl, 4, out + n);
    return n + 4 + pl;
}

/* ------------------------------------------------------------------------ */
/* Name stream: compressName@0x4241a0 + encode_name@0x421070.                */
/* ------------------------------------------------------------------------ */
typedef struct {
    smodel  *prefix;     /* 256 x SIMPLE_MODEL<256> @+0x1068 */
    smodel  *suffix;     /* 256 x SIMPLE_MODEL<256> @+0x1070 */
    smodel  *lenm;       /* 256 x SIMPLE_MODEL<256> @+0x1078 */
    smodel  *mid;        /* 8192 x SIMPLE_MODEL<128> @+0x1080 */
    uint8_t  lastbuf[1 + 1024];  /* lastbuf[0] models last[-1] (0x00) */
    int      last_len, last_p, last_s;
} name_state;

static int encode_name(name_state *st, rc_t *rc, const uint8_t *name, int len)
{
    uint8_t *last = st->lastbuf + 1;
    int ll = st->last_len;
    int p = 0, s = 0;
    if (len <= 0 || ll <= 0) {
        p = 0; s = 0;
        if (len - s - p < 0) s = len - p;
    } else {
        if (name[0] == last[0]) {
            int i = 1;
            while (i < len && i < ll && name[i] == last[i]) i++;
            p = i;
        }
        if (name[len - 1] == last[ll - 1]) {
            int i = len - 1, j = ll - 1;
            for (;;) {
                i--; j--;
                if (j < 0 || i < 0) break;
                if (name[i] != last[j]) break;
            }
            s = len - 1 - i;
            if (len - s - p < 0) s = len - p;
        } else {
            s = 0;
        }
    }
    if (p > 255 || s > 255 || len > 255 || s < 0) return -1;
    sm_encode(&st->prefix[st->last_p], rc, (uint16_t)p);
    sm_encode(&st->suffix[st->last_s], rc, (uint16_t)s);
    sm_encode(&st->lenm[ll], rc, (uint16_t)len);
    st->last_p = p;
    st->last_s = s;

    int len2 = len - s;
    int lc = p != 0;
    int k = 0, j = p;
    for (int i = p; i < len2; i++) {
        if (j > 1023) return -1;
        int ctx = (k * 64 + lc + 2 * ((int)(int8_t)last[j] - 32)) % 8192;
        if (ctx < 0) return -1;            /* reference indexes out of bounds */
        sm_encode(&st->mid[ctx], rc, (uint16_t)(name[i] & 0x7f));
        uint8_t c = name[i];
        int reset = 0;
        if (c == ' ') {
            if (last[j] != ' ' && last[j + 1] != ':') j = j + 1;
            k = (k + 3) & ~3;
            if (j < 0) reset = 1;
        } else {
            uint8_t d = last[j];
            if (d == ' ') { j--; d = last[j]; }
            if (c == ':') {
                j += (d != ':');
                k = (k + 3) & ~3;
                if (j < 0) reset = 1;
            } else {
                j -= (d == ':');
                if (j < 0) reset = 1;
            }
        }
        if (reset) {
            j = 0; lc = 0; k++;
        } else {
            lc = (c == last[j]);
            j++; k++;
        }
    }
    memcpy(last, name, (size_t)len);
    st->last_len = len;
    return 0;
}

static int64_t name_payload(const orc_block *b, uint8_t *out, uint8_t *end)
{
    name_state st;
    st.prefix = (smodel *)malloc(768 * sizeof(smodel));
    st.mid = (smodel *)malloc(8192 * sizeof(smodel));
    if (!st.prefix || !st.mid) { free(st.prefix); free(st.mid); return -1; }
    st.suffix = st.prefix + 256;
    st.lenm = st.prefix + 512;
    for (int i = 0; i < 768; i++) sm_init(&st.prefix[i], 256);
    for (int i = 0; i < 8192; i++) sm_init(&st.mid[i], 128);
    memset(st.lastbuf + 1, ' ', 1024);
    st.lastbuf[0] = 0;
    st.last_len = st.last_p = st.last_s = 0;
    rc_t rc;
    rc_init(&rc, out, end);
    const uint8_t *nm = b->names;
    int bad = 0;
    for (uint32_t r = 0; r < b->nreads && !bad; r++) {
        if (encode_name(&st, &rc, nm, b->name_lens[r])) bad = 1;
        nm += b->name_lens[r];
    }
    rc_finish(&rc);
    free(st.prefix);
    free(st.mid);
    return (rc.err || bad) ? -1 : (int64_t)(rc.out - out);
}

/* compressID@0x4247c0: [md5(names)] + encodeIDS@0x430040 (bin) or names. */
int64_t orc_encap_id(const orc_block *b, const orc_cfg *cfg, uint8_t *out, size_t cap)
{
    if (cap < 64) return -1;
    int n = encap_set_id(5, out);
    uint8_t *p = out + n + 4;
    int hdr = 0;
    if (cfg->md5) {
        orc_md5(b->names, (size_t)total_names(b), p);
        p += 16;
        hdr = 16;
    }
    int64_t pl;
    if (cfg->bin_mode) {
        uint16_t l0 = b->nreads ? b->name_lens[0] : 0;   /* reference reads lens[0] */
        if ((size_t)(p - out) + 2 + l0 > cap) return -1;
        p[0] = (uint8_t)l0;                                /* IntTo2Ch@0x40db00 */
        p[1] = (uint8_t)(l0 >> 8);
        memcpy(p + 2, b->names, l0);
        pl = 2 + l0;
    } else {
        pl = name_payload(b, p, out + cap);
        if (pl < 0) return -1;
    }
    encap_set_size((uint64_t)(hdr + pl), 4, out + n);
    return n + 4 + hdr + pl;
}

/* ------------------------------------------------------------------------ */
/* Degenerate-base side streams.                                             */
/* DegeInfoProcess@0x433a10 per read, then compressDegeTip@0x424dd0 (23),     */
/* compressDegeCh@0x425080 (14), compressDegeMaxQual@0x425310 (24),           */
/* kModelInit@0x42cbe0 / kModelEncode@0x42ccb0 via compressNDegeCnt@0x42d010  */
/* (25) and compressNDegePos@0x42d170 (26).                                   */
/* ------------------------------------------------------------------------ */
typedef struct { uint8_t *v; size_t n, cap; } vec8;
typedef struct { uint32_t *v; size_t n, cap; } vec32;

static int v8_push(vec8 *a, uint8_t x)
{
    if (a->n == a->cap) {
        size_t nc = a->cap ? a->cap * 2 : 1024;
        uint8_t *nv = (uint8_t *)realloc(a->v, nc);
        if (!nv) return -1;
        a->v = nv; a->cap = nc;
    }
    a->v[a->n++] = x;
    return 0;
}

static int v32_push(vec32 *a, uint32_t x)
{
    if (a->n == a->cap) {
        size_t nc = a->cap ? a->cap * 2 : 1024;
        uint32_t *nv = (uint32_t *)realloc(a->v, nc * 4);
        if (!nv) return -1;
        a->v = nv; a->cap = nc;
    }
    a->v[a->n++] = x;
    return 0;
}

typedef struct { vec8 tip, ch, maxq; vec32 cnt, pos; } dege_t;

static int dege_read(dege_t *d, const uint8_t *seq, const uint8_t *qual, int len)
{
    int count = 0;
    uint8_t maxq = 0;
    for (int i = 0; i < len; i++) {
        if (base_code(seq[i]) > 3) {
            if (v8_push(&d->ch, seq[i])) return -1;
            count++;
            if ((int)(int8_t)qual[i] > (int)maxq) maxq = qual[i];
        }
    }
    if (count == 0) return v8_push(&d->tip, 0);
    if (v8_push(&d->tip, 1) || v8_push(&d->maxq, maxq)) return -1;
    uint32_t gap = 0, exc = 0;
    for (int i = 0; i < len; i++) {
        if ((int)maxq < (int)(int8_t)qual[i]) continue;
        if (base_code(seq[i]) > 3) {
            gap++;
        } else {
            exc++;
            if (v32_push(&d->pos, gap)) return -1;
            gap = 0;
        }
    }
    return v32_push(&d->cnt, exc);
}

/* encap = ID + size4 + u32 count + rc bytes; omitted (0 bytes) when count==0 */
static int64_t dege_sm_stream(int id, int nsym, const uint8_t *vals, size_t n, int sub,
                              uint8_t *out, uint8_t *end)
{
    if (n == 0) return 0;
    int idn = encap_set_id((uint64_t)id, out);
    uint8_t *p = out + idn + 4;
    if (p + 4 > end) return -1;
    put_u32le(p, (uint32_t)n);
    p += 4;
    smodel *m = (smodel *)malloc(sizeof(smodel));
    if (!m) return -1;
    sm_init(m, nsym);
    rc_t rc;
    rc_init(&rc, p, end);
    for (size_t i = 0; i < n; i++) {
        int s;
        if (sub == 0) s = vals[i];
        else if (sub == 1) s = base_code(vals[i]) - 4;
        else s = (uint8_t)(vals[i] - 33);
        if (s < 0 || s >= nsym) { rc.err = 1; break; }
        sm_encode(m, &rc, (uint16_t)s);
    }
    rc_finish(&rc);
    free(m);
    if (rc.err) return -1;
    int64_t pl = rc.out - p;
    encap_set_size((uint64_t)(pl + 4), 4, out + idn);
    return idn + 4 + 4 + pl;
}

typedef struct { smodel nbits; smodel bits[64]; } kmodel;

static void kmodel_init(kmodel *k)
{
    sm_init(&k->nbits, 64);
    for (int i = 0; i < 64; i++) sm_init(&k->bits[i], 2);
}

static void kmodel_encode(kmodel *k, rc_t *rc, uint64_t v)
{
    uint8_t bits[64];
    int nb = 0;
    while (v) { bits[nb++] = (uint8_t)(v & 1); v >>= 1; }
    sm_encode(&k->nbits, rc, (uint16_t)nb);
    for (int i = 0; i < nb; i++) sm_encode(&k->bits[i], rc, bits[i]);
}

static int64_t dege_k_stream(int id, kmodel *km, const uint32_t *vals, size_t n,
                             uint8_t *out, uint8_t *end)
{
    if (n == 0) return 0;
    int idn = encap_set_id((uint64_t)id, out);
    uint8_t *p = out + idn + 4;
    if (p + 4 > end) return -1;
    put_u32le(p, (uint32_t)n);
    p += 4;
    rc_t rc;
    rc_init(&rc, p, end);
    for (size_t i = 0; i < n; i++) kmodel_encode(km, &rc, vals[i]);
    rc_finish(&rc);
    if (rc.err) return -1;
    int64_t pl = rc.out - p;
    encap_set_size((uint64_t)(pl + 4), 4, out + idn);
    return idn + 4 + 4 + pl;
}

/* ------------------------------------------------------------------------ */
/* Block assembly: doFqzEncode@0x42d2d0.                                     */
/* 81 size4 | count(1) | len(4) | ID(5) | qual(7) | tip(23) | ch(14) |       */
/* maxq(24) | ncnt(25) | npos(26) | seq(6)                                  */
/* ------------------------------------------------------------------------ */
int64_t orc_encode_block(const orc_block *b, const orc_cfg *cfg, uint8_t *out, size_t cap)
{
    uint8_t *end = out + cap;
    if (cap < 16) return -1;
    int idn = encap_set_id(1, out);
    uint8_t *p = out + idn + 4;

    /* compressCount@0x422a00: ID 1, size byte 0x84, u32 LE */
    p += encap_set_id(1, p);
    encap_set_size(4, 1, p);
    p += 1;
    put_u32le(p, b->nreads);
    p += 4;

    int64_t r;
    if ((r = orc_encap_len(b, p, (size_t)(end - p))) < 0) return -1;
    p += r;
    if ((r = orc_encap_id(b, cfg, p, (size_t)(end - p))) < 0) return -1;
    p += r;
    if ((r = orc_encap_qual(b, cfg, p, (size_t)(end - p))) < 0) return -1;
    p += r;

    dege_t d;
    memset(&d, 0, sizeof d);
    const uint8_t *s = b->seq, *q = b->qual;
    int bad = 0;
    for (uint32_t i = 0; i < b->nreads && !bad; i++) {
        int32_t len = b->seq_lens[i];
        if (dege_read(&d, s, q, len > 0 ? len : 0)) bad = 1;
        s += len;
        q += len;
    }
    kmodel *km = (kmodel *)malloc(sizeof(kmodel));
    if (!km) bad = 1;
    else kmodel_init(km);
    if (!bad && (r = dege_sm_stream(23, 2, d.tip.v, d.tip.n, 0, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    if (!bad && (r = dege_sm_stream(14, 11, d.ch.v, d.ch.n, 1, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    if (!bad && (r = dege_sm_stream(24, 95, d.maxq.v, d.maxq.n, 2, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    if (!bad && (r = dege_k_stream(25, km, d.cnt.v, d.cnt.n, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    if (!bad && (r = dege_k_stream(26, km, d.pos.v, d.pos.n, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    free(km);
    free(d.tip.v); free(d.ch.v); free(d.maxq.v); free(d.cnt.v); free(d.pos.v);
    if (bad) return -1;

    if ((r = orc_encap_seq(b, cfg, p, (size_t)(end - p))) < 0) return -1;
    p += r;
    int64_t total = p - (out + idn + 4);
    encap_set_size((uint64_t)total, 4, out + idn);
    return p - out;
}

/* ------------------------------------------------------------------------ */
/* Reference (HASH index) path: EncapFqzComp::doAlignEncode@0x42d4c0.         */
/* 81 size4 | count(1) | len(4) | count(0x1b) | order(8) | ID(5) | qual(7) | */
/* count(0x11..0x14) | [PE: count(0x15) count(0x16) perel(9)] | pos(0xb) |    */
/* mis(0xf) | rev(0xa) | cigal(0xc) | cigav(0xd) | dege 23 14 24 25 26 |      */
/* seq(6) -- the seq stream codes only the reads that did not align.          */
/* ------------------------------------------------------------------------ */

/* compressCount@0x422a00: setID(id), 1-byte size 0x84, u32 LE */
static int64_t count_encap(uint32_t id, uint32_t v, uint8_t *out, uint8_t *end)
{
    if (end - out < 16) return -1;
    int n = encap_set_id(id, out);
    encap_set_size(4, 1, out + n);
    put_u32le(out + n + 1, v);
    return n + 5;
}

/* One SIMPLE_MODEL<nsym> over a byte array, own range coder: the template of
 * compressOrder@0x424b70 (8, <5>), compressPERelation@0x422be0 (9, <4>),
 * compressAlignInfo_Pos@0x425d70 (0xb, <2>), _Rev@0x426480 (0xa, <2>),
 * _CigaL@0x426700 (0xc, <2>), _CigaV@0x426980 (0xd, <4>) and _Mis@0x425ff0
 * (0xf, <8> for maxmis 1..7, <9> for 8, no symbols otherwise).  setID + size4
 * + the coded bytes; no count, always written (8 flush bytes when empty). */
static int64_t sm_stream_encap(uint32_t id, int nsym, const uint8_t *vals, uint32_t n, uint8_t *out, uint8_t *end)
{
    if (end - out < 16) return -1;
    int idn = encap_set_id(id, out);
    uint8_t *p = out + idn + 4;
    smodel *m = (smodel *)malloc(sizeof(smodel));
    if (!m) return -1;
    rc_t rc;
    rc_init(&rc, p, end);
    if (nsym > 0) {
        sm_init(m, nsym);
        for (uint32_t i = 0; i < n && !rc.err; i++) {
            if (vals[i] >= nsym) { rc.err = 1; break; }
            sm_encode(m, &rc, vals[i]);
        }
    }
    rc_finish(&rc);
    free(m);
    if (rc.err) return -1;
    int64_t pl = rc.out - p;
    encap_set_size((uint64_t)pl, 4, out + idn);
    return idn + 4 + pl;
}

int64_t orc_encode_block_aligned(const orc_block *b, const orc_cfg *cfg, const orc_align_streams *a,
                                 uint8_t *out, size_t cap)
{
    uint8_t *end = out + cap;
    if (cap < 16 || a->order_count > b->nreads) return -1;
    int idn = encap_set_id(1, out);
    uint8_t *p = out + idn + 4;
    int64_t r;
#define PUT(expr) do { if ((r = (expr)) < 0) return -1; p += r; } while (0)
    PUT(count_encap(1, b->nreads, p, end));
    PUT(orc_encap_len(b, p, (size_t)(end - p)));
    PUT(count_encap(0x1b, a->order_count, p, end));
    PUT(sm_stream_encap(8, 5, a->order, a->order_count, p, end));
    PUT(orc_encap_id(b, cfg, p, (size_t)(end - p)));
    PUT(orc_encap_qual(b, cfg, p, (size_t)(end - p)));
    PUT(count_encap(0x11, a->align_count, p, end));
    PUT(count_encap(0x12, a->npos, p, end));
    PUT(count_encap(0x13, a->ncigal, p, end));
    PUT(count_encap(0x14, a->ncigav, p, end));
    if (a->paired) {   /* param+0x1b38 == 0 (-2 given) */
        PUT(count_encap(0x15, a->insert_bits, p, end));
        PUT(count_encap(0x16, a->nperel, p, end));
        PUT(sm_stream_encap(9, 4, a->perel, a->nperel, p, end));
    }
    PUT(sm_stream_encap(0xb, 2, a->pos, a->npos, p, end));
    PUT(sm_stream_encap(0xf, a->maxmis >= 1 && a->maxmis <= 7 ? 8 : a->maxmis == 8 ? 9 : 0, a->mis, a->nmis, p, end));
    PUT(sm_stream_encap(0xa, 2, a->rev, a->nrev, p, end));
    PUT(sm_stream_encap(0xc, 2, a->cigal, a->ncigal, p, end));
    PUT(sm_stream_encap(0xd, 4, a->cigav, a->ncigav, p, end));
#undef PUT
    dege_t d;
    memset(&d, 0, sizeof d);
    const uint8_t *s = b->seq, *q = b->qual;
    int bad = 0;
    for (uint32_t i = 0; i < b->nreads && !bad; i++) {
        int32_t len = b->seq_lens[i];
        if (dege_read(&d, s, q, len > 0 ? len : 0)) bad = 1;
        s += len;
        q += len;
    }
    kmodel *km = (kmodel *)malloc(sizeof(kmodel));
    if (!km) bad = 1;
    else kmodel_init(km);
    if (!bad && (r = dege_sm_stream(23, 2, d.tip.v, d.tip.n, 0, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    if (!bad && (r = dege_sm_stream(14, 11, d.ch.v, d.ch.n, 1, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    if (!bad && (r = dege_sm_stream(24, 95, d.maxq.v, d.maxq.n, 2, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    if (!bad && (r = dege_k_stream(25, km, d.cnt.v, d.cnt.n, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    if (!bad && (r = dege_k_stream(26, km, d.pos.v, d.pos.n, p, end)) < 0) bad = 1;
    if (!bad) p += r;
    free(km);
    free(d.tip.v); free(d.ch.v); free(d.maxq.v); free(d.cnt.v); free(d.pos.v);
    if (bad) return -1;
    /* sequence: compressSeq@0x4248a0, aligned reads skipped */
    {
        if (end - p < 32) return -1;
        int n = encap_set_id(6, p);
        uint8_t *q6 = p + n + 4;
        int hdr = 0;
        if (cfg->md5) {
            orc_md5(b->seq, (size_t)total_seq(b), q6);
            q6 += 16;
            hdr = 16;
        }
        int64_t pl = seq_payload_sel(b, cfg->slevel + 7, a->order, a->order_count, q6, end);
        if (pl < 0) return -1;
        encap_set_size((uint64_t)(hdr + pl), 4, p + n);
        p += n + 4 + hdr + pl;
    }
    int64_t total = p - (out + idn + 4);
    encap_set_size((uint64_t)total, 4, out + idn);
    return p - out;
}

/* ------------------------------------------------------------------------ */
/* ID template analysis: IDProcess::analysisIDBinType@0x4310a0,             */
/* analysisPEType@0x430f50, strSplit@0x40e0d0 with delimiters               */
/* " !\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~" (.rodata 0x44b9e8).                 */
/* ------------------------------------------------------------------------ */
typedef struct { const uint8_t *s; int n; } tok_t;

static int is_delim(uint8_t c)
{
    return c == ' ' || (c >= '!' && c <= '/') || (c >= ':' && c <= '@') ||
           (c >= '[' && c <= '`') || (c >= '{' && c <= '~');
}

static int split(const uint8_t *s, int n, tok_t *toks, int maxt)
{
    int nt = 0, i = 0;
    for (;;) {
        while (i < n && is_delim(s[i])) i++;
        if (i >= n) break;
        int j = i;
        while (j < n && !is_delim(s[j])) j++;
        if (nt >= maxt) return -1;
        toks[nt].s = s + i;
        toks[nt].n = j - i;
        nt++;
        i = j;
    }
    return nt;
}

static int ieq(const tok_t *t, const char *w)
{
    size_t wl = strlen(w);
    if ((size_t)t->n != wl) return 0;
    for (size_t i = 0; i < wl; i++) {
        uint8_t a = t->s[i], b = (uint8_t)w[i];
        if (a >= 'A' && a <= 'Z') a = (uint8_t)(a + 32);
        if (a != b) return 0;
    }
    return 1;
}

static int all_digits(const tok_t *t)
{
    for (int i = 0; i < t->n; i++)
        if (t->s[i] < '0' || t->s[i] > '9') return 0;
    return 1;
}

/* std::stoul on a digit-only token (empty -> invalid_argument) */
static int tok_ul(const tok_t *t, uint64_t *v)
{
    if (t->n == 0) return -1;
    uint64_t x = 0;
    for (int i = 0; i < t->n; i++) {
        uint64_t nx = x * 10 + (uint64_t)(t->s[i] - '0');
        if (nx / 10 != x) return -1;   /* out_of_range */
        x = nx;
    }
    *v = x;
    return 0;
}

/* std::stoi-like strtol on the token's text (leading part) */
static int tok_l(const tok_t *t, int64_t *v)
{
    int i = 0, neg = 0;
    /* strtol reads from the token start; the token has no whitespace */
    if (i < t->n && (t->s[i] == '+' || t->s[i] == '-')) { neg = t->s[i] == '-'; i++; }
    if (i >= t->n || t->s[i] < '0' || t->s[i] > '9') return -1;
    int64_t x = 0;
    for (; i < t->n && t->s[i] >= '0' && t->s[i] <= '9'; i++) {
        x = x * 10 + (t->s[i] - '0');
        if (x > 0x7fffffffLL + 1) return -1;
    }
    x = neg ? -x : x;
    if (x > 0x7fffffffLL || x < -0x80000000LL) return -1;
    *v = x;
    return 0;
}

static int pe_type(const uint8_t *a, int la, const uint8_t *b, int lb)
{
    if (la == lb && memcmp(a, b, (size_t)la) == 0) return 1;
    if (la > 0 && lb > 0 && a[la - 1] == '1' && b[lb - 1] == '2' &&
        memcmp(a, b, (size_t)(la - 1)) == 0)
        return 2;
    for (int i = 0; i + 6 <= la; i++)
        if (memcmp(a + i, "length", 6) == 0) return memcmp(a, b, (size_t)i) == 0 ? 3 : 0;
    return 0;
}

#define MAXTOK 256
int orc_analyze_idbin(const orc_block *first, int se, uint8_t T[512])
{
    if (first->nreads == 0) return 0;
    tok_t *A = (tok_t *)malloc(sizeof(tok_t) * MAXTOK), *B = (tok_t *)malloc(sizeof(tok_t) * MAXTOK);
    if (!A || !B) { free(A); free(B); return -1; }
    int rc = 0;
    int na = split(first->names, first->name_lens[0], A, MAXTOK);
    int lenIdx = -1;
    if (na < 0) { rc = -1; goto done; }
    for (int i = 1; i <= na && na > 0; i++) {
        if (lenIdx < 0) {
            if (ieq(&A[i - 1], "length") || ieq(&A[i - 1], "len")) {
                if (i >= na) { rc = -1; goto done; }   /* reference reads past the vector */
                int64_t v;
                if (tok_l(&A[i], &v)) { rc = -1; goto done; }
                if (v == (int64_t)first->seq_lens[0]) {
                    lenIdx = i;
                    if (i + 1 < 512) T[i + 1] = 0;
                }
            }
        } else if (lenIdx == i - 1) {
            if (i + 1 < 512) T[i + 1] = 3;
        }
    }
    {
        int petypes[4] = {0, 0, 0, 0};
        const uint8_t *ptr = first->names;
        uint32_t idx = 0;
        while (idx < first->nreads) {
            const uint8_t *s = ptr;
            int ls = first->name_lens[idx];
            ptr += ls;
            idx++;
            if (!se) {
                if (idx >= first->nreads) { rc = -1; goto done; }
                int l2 = first->name_lens[idx];
                petypes[pe_type(s, ls, ptr, l2)] = 1;
                ptr += l2;
                idx++;
            }
            int nb = split(s, ls, B, MAXTOK);
            if (nb < 0) { rc = -1; goto done; }
            if (nb != na) { T[0] = 0; goto done; }
            for (int k = 0; k < nb; k++) {
                if ((k != 0 && k - 1 == lenIdx) || k == lenIdx) continue;
                if (B[k].n == A[k].n && memcmp(B[k].s, A[k].s, (size_t)A[k].n) == 0) {
                    if (k + 2 < 512) T[k + 2] = 0;
                    continue;
                }
                if (!all_digits(&A[k]) || !all_digits(&B[k])) { T[0] = 0; goto done; }
                uint64_t va, vb;
                if (tok_ul(&A[k], &va) || tok_ul(&B[k], &vb)) { rc = -1; goto done; }
                if (vb - va != 1) { T[0] = 0; goto done; }
                if (k + 2 < 512) T[k + 2] = 1;
            }
            tok_t *t = A; A = B; B = t;
        }
        if (se) {
            T[0] = 1;
        } else {
            int any = petypes[0] || petypes[1] || petypes[2] || petypes[3];
            if (!any) { T[0] = 1; T[1] = 0; }
            else if (petypes[0]) { T[0] = 0; T[1] = 0; }
            else { T[0] = 1; T[1] = petypes[3] ? 3 : petypes[2] ? 2 : 1; }
        }
    }
done:
    free(A);
    free(B);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* FASTQ parsing: getBlockRead@0x411b60 (SE), getBlockReadPE@0x412920 (PE).  */
/* ------------------------------------------------------------------------ */
int64_t orc_parse_se(const uint8_t *t, size_t len, uint8_t *names, uint16_t *nl,
                     uint8_t *seq, int32_t *sl, uint8_t *qual)
{
    size_t start = 1;
    int state = 1;
    int64_t n = 0, nseq = 0;
    int32_t lastlen = 0;
    for (size_t i = 0; i < len; i++) {
        if (t[i] != '\n') continue;
        switch (state) {
        case 1: {
            size_t l = i - start;
            if (l > 0xffff) return -1;
            memcpy(names, t + start, l);
            names += l;
            nl[n++] = (uint16_t)l;
            state = 2;
            start = i + 1;
            break;
        }
        case 2: {
            int32_t l = (int32_t)(i - start);
            memcpy(seq, t + start, (size_t)l);
            seq += l;
            sl[nseq++] = l;
            lastlen = l;
            state = 3;
            start = i + 1;
            break;
        }
        case 3:
            start = i + 1;
            state = 4;
            break;
        case 4:
            if (start + (size_t)lastlen > len) return -1;
            memcpy(qual, t + start, (size_t)lastlen);
            qual += lastlen;
            start = i + 2;
            state = 1;
            break;
        }
    }
    if (state != 1 || n != nseq) return -1;   /* truncated record: not restated */
    return n;
}

static size_t count_nl(const uint8_t *t, size_t len, size_t *pos, size_t maxn)
{
    size_t n = 0;
    for (size_t i = 0; i < len; i++)
        if (t[i] == '\n') {
            if (n < maxn) pos[n] = i;
            n++;
        }
    return n;
}

int64_t orc_parse_pe(const uint8_t *t1, size_t len1, const uint8_t *t2, size_t len2,
                     uint8_t *names, uint16_t *nlens, uint8_t *seq, int32_t *slens, uint8_t *qual)
{
    size_t c1 = count_nl(t1, len1, NULL, 0), c2 = count_nl(t2, len2, NULL, 0);
    size_t *a = (size_t *)malloc((c1 + 1) * sizeof(size_t)), *b = (size_t *)malloc((c2 + 1) * sizeof(size_t));
    if (!a || !b) { free(a); free(b); return -1; }
    count_nl(t1, len1, a, c1);
    count_nl(t2, len2, b, c2);
    size_t k = c1 < c2 ? c1 : c2;
    if (k % 4) { free(a); free(b); return -1; }
    size_t s1 = 1, s2 = 1;
    int64_t n = 0;
    for (size_t o = 0; o < k; o += 4) {
        size_t l;
        l = a[o] - s1;
        if (l > 0xffff) goto bad;
        memcpy(names, t1 + s1, l); names += l; nlens[n] = (uint16_t)l;
        l = a[o + 1] - (a[o] + 1);
        memcpy(seq, t1 + a[o] + 1, l); seq += l; slens[n] = (int32_t)l;
        l = a[o + 3] - (a[o + 2] + 1);
        memcpy(qual, t1 + a[o + 2] + 1, l); qual += l;
        if ((int32_t)l != slens[n]) goto bad;
        s1 = a[o + 3] + 2;
        n++;
        l = b[o] - s2;
        if (l > 0xffff) goto bad;
        memcpy(names, t2 + s2, l); names += l; nlens[n] = (uint16_t)l;
        l = b[o + 1] - (b[o] + 1);
        memcpy(seq, t2 + b[o] + 1, l); seq += l; slens[n] = (int32_t)l;
        l = b[o + 3] - (b[o + 2] + 1);
        memcpy(qual, t2 + b[o + 2] + 1, l); qual += l;
        if ((int32_t)l != slens[n]) goto bad;
        s2 = b[o + 3] + 2;
        n++;
    }
    free(a);
    free(b);
    return n;
bad:
    free(a);
    free(b);
    return -1;
}

/* ------------------------------------------------------------------------ */
/* Block cutting.  getEndPos@0x4320c0: scan back from n for "\n@" followed   */
/* by >5 consecutive matches against the file's first line; the match run   */
/* counter is not reset between candidate positions (reproduced).            */
/* ------------------------------------------------------------------------ */
static int64_t get_end_pos(const uint8_t *data, size_t avail, int64_t n,
                           const uint8_t *first, size_t flen)
{
    if (n <= 0) return 0;
    int run = 0;
    for (int64_t pos = n; pos > 0; pos--) {
        if (data[pos] != '\n' || (size_t)(pos + 1) >= avail + 1 || data[pos + 1] != '@' || flen == 0)
            continue;
        for (size_t k = 0; k < flen; k++) {
            size_t at = (size_t)pos + 1 + k;
            /* the reference may read one byte past the filled region; treat as mismatch */
            if (at < avail && data[at] == first[k]) {
                if (++run > 5) return pos;
            } else {
                run = 0;
            }
        }
    }
    return 0;
}

static size_t first_line_len(const uint8_t *t, size_t len)
{
    size_t i = 0;
    while (i < len && t[i] != '\n') i++;
    return i + 1 <= len ? i + 1 : len;   /* getFirstLine keeps the '\n' */
}

int64_t orc_cut_se(const uint8_t *text, size_t len, size_t bs, size_t *ends, size_t maxb)
{
    size_t flen = first_line_len(text, len);
    const uint8_t *first = text;
    size_t off = 0, nb = 0;
    while (off < len) {
        size_t avail = len - off;
        if (nb >= maxb) return -1;
        if (avail < bs) {                 /* short read: last block of the file */
            ends[nb++] = len;
            break;
        }
        const uint8_t *d = text + off;
        int64_t e = get_end_pos(d, bs, (int64_t)bs - (int64_t)flen, first, flen);
        if (e <= 0) return -1;            /* reference prints an error and emits garbage */
        ends[nb++] = off + (size_t)e + 1;
        off += (size_t)e + 1;
    }
    return (int64_t)nb;
}

int64_t orc_cut_pe(const uint8_t *t1, size_t len1, const uint8_t *t2, size_t len2,
                   size_t bs, size_t *e1, size_t *e2, size_t maxb)
{
    size_t half = (size_t)((uint32_t)bs >> 1);
    size_t flen = first_line_len(t1, len1);
    size_t o1 = 0, o2 = 0, nb = 0;
    size_t *nl1 = (size_t *)malloc((half + 1) * sizeof(size_t));
    size_t *nl2 = (size_t *)malloc((half + 1) * sizeof(size_t));
    if (!nl1 || !nl2) { free(nl1); free(nl2); return -1; }
    for (;;) {
        if (nb >= maxb) { nb = (size_t)-1; break; }
        size_t a1 = len1 - o1 < half ? len1 - o1 : half;
        size_t a2 = len2 - o2 < half ? len2 - o2 : half;
        int more = (a1 >= half) || (a2 >= half);
        size_t c1 = count_nl(t1 + o1, a1, nl1, half + 1);
        size_t c2 = count_nl(t2 + o2, a2, nl2, half + 1);
        size_t k = c1 < c2 ? c1 : c2;
        if (!more) {
            e1[nb] = len1;
            e2[nb] = len2;
            nb++;
            break;
        }
        if (k < 2) { nb = (size_t)-1; break; }
        int64_t j = (int64_t)k - 2;
        int64_t pos = get_end_pos(t1 + o1, a1, (int64_t)nl1[j], t1, flen);
        while (j >= 0 && (int64_t)nl1[j] != pos) j--;
        if (j < 0) { nb = (size_t)-1; break; }   /* the reference loops forever here */
        o1 += nl1[j] + 1;
        o2 += nl2[j] + 1;
        e1[nb] = o1;
        e2[nb] = o2;
        nb++;
        if (o1 >= len1 && o2 >= len2) break;
    }
    free(nl1);
    free(nl2);
    return (int64_t)nb;
}
