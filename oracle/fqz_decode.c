/*
 * fqz_decode.c -- CPU decoder of a SeqArc-1.6 no-reference block.
 *
 * TEST INFRASTRUCTURE ONLY (see fqz_oracle.h): the round-trip checker for the
 * GPU encoder.  It is the exact inverse of the encoder restated in
 * fqz_oracle.c (range coder, SIMPLE_MODEL / BASE_MODEL updates, stream layout
 * of doFqzEncode@0x42d2d0); the reference's own decoder is doFqzDecode@0x42c680
 * (decode_seq@0x4296b0, decode_qual@0x42a750, decode_name@0x428380), whose
 * model updates mirror the encoder's.  A block encoded from bases other than
 * ACGT / IUPAC decodes them as 'N' and lowercase as uppercase (the encoder
 * keeps only base codes: seq_val_table@0x44b800), so the MD5 check then fails
 * exactly as it would for the reference.
 */
#include "fqz_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ---- carry-less range decoder (inverse of rc_encode / rc_finish) -------- */
typedef struct {
    const uint8_t *p, *end;
    uint64_t low, code;
    uint32_t range;
    int err;
} rd_t;

static uint8_t rd_byte(rd_t *d)
{
    if (d->p < d->end) return *d->p++;
    d->err = 1;
    return 0;
}

static void rd_init(rd_t *d, const uint8_t *p, const uint8_t *end)
{
    d->p = p;
    d->end = end;
    d->low = 0;
    d->code = 0;
    d->range = 0xffffffffu;
    d->err = 0;
    for (int i = 0; i < 8; i++) d->code = (d->code << 8) | rd_byte(d);
}

/* the symbol slot in [0, tot) and the scale r = range / tot */
static uint32_t rd_slot(rd_t *d, uint32_t tot, uint32_t *r)
{
    *r = d->range / tot;
    uint64_t v = (d->code - d->low) / *r;
    if (v >= tot) {
        d->err = 1;
        v = tot - 1;
    }
    return (uint32_t)v;
}

static void rd_take(rd_t *d, uint32_t r, uint32_t cum, uint32_t freq)
{
    d->low += (uint32_t)(cum * r);
    d->range = r * freq;
    while (d->range < (1u << 24)) {
        if ((d->low ^ (d->low + d->range)) >> 56)
            d->range = ((uint32_t)d->low | 0xffffffu) - (uint32_t)d->low;
        d->code = (d->code << 8) | rd_byte(d);
        d->range <<= 8;
        d->low <<= 8;
    }
}

/* ---- SIMPLE_MODEL<N> decode (inverse of sm_encode) ---------------------- */
typedef struct { uint16_t sym, freq; } dsf_t;
typedef struct {
    uint32_t tot, bub;
    dsf_t    sentinel;
    dsf_t    F[257];
} dmodel;

static void dm_init(dmodel *m, int n)
{
    m->tot = (uint32_t)n;
    m->bub = 0;
    m->sentinel.sym = 0;
    m->sentinel.freq = 0xffe0;
    for (int i = 0; i < n; i++) { m->F[i].sym = (uint16_t)i; m->F[i].freq = 1; }
    m->F[n].sym = 0;
    m->F[n].freq = 0;
}

static int dm_decode(dmodel *m, rd_t *d)
{
    uint32_t r;
    const uint32_t v = rd_slot(d, m->tot, &r);
    dsf_t *s = m->F;
    uint32_t acc = 0;
    while (acc + s->freq <= v) {
        if (s->freq == 0) { d->err = 1; return 0; }
        acc += s->freq;
        s++;
    }
    if (s->freq == 0) { d->err = 1; return 0; }
    const int sym = s->sym;
    rd_take(d, r, acc, s->freq);
    s->freq += 8;
    m->tot += 8;
    if (m->tot > 0xffe0) {
        m->tot = 0;
        for (dsf_t *p = m->F; p->freq; p++) {
            p->freq -= p->freq >> 1;
            m->tot += p->freq;
        }
    }
    if (((++m->bub) & 15) == 0 && s[0].freq > s[-1].freq) {
        dsf_t t = s[0];
        s[0] = s[-1];
        s[-1] = t;
    }
    return sym;
}

typedef struct { dmodel nbits; dmodel bits[64]; } dkmodel;

static void dk_init(dkmodel *k)
{
    dm_init(&k->nbits, 64);
    for (int i = 0; i < 64; i++) dm_init(&k->bits[i], 2);
}

static uint64_t dk_decode(dkmodel *k, rd_t *d)
{
    const int nb = dm_decode(&k->nbits, d);
    uint64_t v = 0;
    for (int i = 0; i < nb && i < 64; i++) v |= (uint64_t)dm_decode(&k->bits[i], d) << i;
    return v;
}

/* ---- encap parsing (setID@0x420720 / setSize@0x420780 as written) ------- */
typedef struct {
    const uint8_t *p, *end;
    int err;
} cur_t;

static int take_id(cur_t *c, int id)   /* the one-byte IDs of this layout */
{
    if (c->p >= c->end || *c->p != (uint8_t)(0x80 | id)) return 0;
    c->p++;
    return 1;
}

static uint32_t take_size4(cur_t *c)
{
    if (c->end - c->p < 4) { c->err = 1; return 0; }
    const uint32_t v = ((uint32_t)c->p[0] << 24) | ((uint32_t)c->p[1] << 16) | ((uint32_t)c->p[2] << 8) | c->p[3];
    c->p += 4;
    return v & 0x0fffffffu;
}

static uint32_t get_u32le(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static const char IUPAC[] = "NMRYKSWHBVD";   /* base codes 4..14 */

/* ---- names (inverse of encode_name) ------------------------------------ */
typedef struct {
    dmodel *prefix, *suffix, *lenm, *mid;
    uint8_t lastbuf[1 + 1024];
    int last_len, last_p, last_s;
} dname_t;

static int decode_name(dname_t *st, rd_t *d, uint8_t *name, int cap)
{
    uint8_t *last = st->lastbuf + 1;
    const int ll = st->last_len;
    const int p = dm_decode(&st->prefix[st->last_p], d);
    const int s = dm_decode(&st->suffix[st->last_s], d);
    const int len = dm_decode(&st->lenm[ll], d);
    if (d->err || len > cap || p + s > len || p > ll || s > ll) return -1;
    st->last_p = p;
    st->last_s = s;
    memcpy(name, last, (size_t)p);
    const int len2 = len - s;
    int lc = p != 0, k = 0, j = p;
    for (int i = p; i < len2; i++) {
        if (j > 1023) return -1;
        const int ctx = (k * 64 + lc + 2 * ((int)(int8_t)last[j] - 32)) % 8192;
        if (ctx < 0) return -1;
        const uint8_t c = (uint8_t)dm_decode(&st->mid[ctx], d);
        name[i] = c;
        int reset = 0;
        if (c == ' ') {
            if (last[j] != ' ' && last[j + 1] != ':') j = j + 1;
            k = (k + 3) & ~3;
            if (j < 0) reset = 1;
        } else {
            uint8_t dd = last[j];
            if (dd == ' ') { j--; dd = last[j]; }
            if (c == ':') {
                j += (dd != ':');
                k = (k + 3) & ~3;
                if (j < 0) reset = 1;
            } else {
                j -= (dd == ':');
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
    memcpy(name + len2, last + ll - s, (size_t)s);
    memcpy(last, name, (size_t)len);
    st->last_len = len;
    return d->err ? -1 : len;
}

/* ---- block -------------------------------------------------------------- */
int64_t orc_decode_block(const uint8_t *in, size_t in_len, const orc_cfg *cfg, orc_decoded *o)
{
    cur_t c = {in, in + in_len, 0};
    o->md5_ok = 1;
    if (!take_id(&c, 1)) return -1;
    const uint32_t bsize = take_size4(&c);
    if (c.err || (size_t)(c.end - c.p) < bsize) return -1;
    c.end = c.p + bsize;
    /* count (compressCount@0x422a00) */
    if (!take_id(&c, 1) || c.end - c.p < 5 || c.p[0] != 0x84) return -1;
    const uint32_t n = get_u32le(c.p + 1);
    c.p += 5;
    if (n > o->max_reads) return -1;
    o->nreads = n;
    int64_t ret = -1;
    uint32_t *len = (uint32_t *)calloc((size_t)n + 1, 4);
    dmodel *qm = NULL;
    uint8_t *tab = NULL;
    uint8_t *tip = NULL, *isn = NULL;
    if (!len) return -1;

    /* lengths (compressLen_short@0x423f50): same / lo / hi, last_len stays 0 */
    {
        if (!take_id(&c, 4)) goto out;
        const uint32_t sz = take_size4(&c);
        if (c.err || (size_t)(c.end - c.p) < sz) goto out;
        dmodel *m = (dmodel *)malloc(3 * sizeof(dmodel));
        if (!m) goto out;
        dm_init(&m[0], 2); dm_init(&m[1], 256); dm_init(&m[2], 256);
        rd_t d;
        rd_init(&d, c.p, c.p + sz);
        for (uint32_t r = 0; r < n; r++) {
            if (dm_decode(&m[0], &d)) {
                len[r] = 0;
            } else {
                const uint32_t lo = (uint32_t)dm_decode(&m[1], &d);
                len[r] = lo | ((uint32_t)dm_decode(&m[2], &d) << 8);
            }
        }
        free(m);
        if (d.err) goto out;
        c.p += sz;
    }
    uint64_t total = 0;
    for (uint32_t r = 0; r < n; r++) {
        o->seq_lens[r] = (int32_t)len[r];
        total += len[r];
    }
    if (total > o->seq_cap) goto out;

    /* IDs (compressID@0x4247c0) */
    uint64_t name_total = 0;
    uint8_t md5_id[16], md5_qual[16], md5_seq[16];
    {
        if (!take_id(&c, 5)) goto out;
        const uint32_t sz = take_size4(&c);
        if (c.err || (size_t)(c.end - c.p) < sz) goto out;
        const uint8_t *q = c.p;
        if (cfg->md5) { memcpy(md5_id, q, 16); q += 16; }
        if (cfg->bin_mode) { ret = -2; goto out; }   /* encodeIDS@0x430040: not inverted here */
        dname_t *st = (dname_t *)malloc(sizeof(dname_t));
        dmodel *ms = (dmodel *)malloc((768 + 8192) * sizeof(dmodel));
        if (!st || !ms) { free(st); free(ms); goto out; }
        st->prefix = ms; st->suffix = ms + 256; st->lenm = ms + 512; st->mid = ms + 768;
        for (int i = 0; i < 768; i++) dm_init(&ms[i], 256);
        for (int i = 0; i < 8192; i++) dm_init(&st->mid[i], 128);
        memset(st->lastbuf + 1, ' ', 1024);
        st->lastbuf[0] = 0;
        st->last_len = st->last_p = st->last_s = 0;
        rd_t d;
        rd_init(&d, q, c.p + sz);
        int bad = 0;
        for (uint32_t r = 0; r < n && !bad; r++) {
            const int64_t room = (int64_t)o->name_cap - (int64_t)name_total;
            const int l = decode_name(st, &d, o->names + name_total, room > 255 ? 255 : (int)room);
            if (l < 0) bad = 1;
            else { o->name_lens[r] = (uint16_t)l; name_total += (uint64_t)l; }
        }
        free(st);
        free(ms);
        if (bad || d.err) goto out;
        c.p += sz;
    }

    /* qualities (compressQual@0x426e80 / encode_qual@0x422180) */
    {
        if (!take_id(&c, 7)) goto out;
        const uint32_t sz = take_size4(&c);
        if (c.err || (size_t)(c.end - c.p) < sz) goto out;
        const uint8_t *q = c.p;
        if (cfg->md5 && !(cfg->lossy > 0.0)) { memcpy(md5_qual, q, 16); q += 16; }
        const uint32_t nm = cfg->qlevel > 2 ? 0x100000u : 0x10000u;
        qm = (dmodel *)malloc((size_t)nm * sizeof(dmodel));
        if (!qm) goto out;
        for (uint32_t i = 0; i < nm; i++) dm_init(&qm[i], 95);
        rd_t d;
        rd_init(&d, q, c.p + sz);
        uint8_t *Q = o->qual;
        for (uint32_t r = 0; r < n && !d.err; r++) {
            const uint32_t L = len[r];
            uint32_t last = 0;
            int q1 = 0, q2 = 0, delta = 5;
            for (uint32_t i = 0; i < L; i++) {
                const int sym = dm_decode(&qm[last], &d);
                if (sym == 94) {   /* the trailing '#' run */
                    memset(Q + i, '#', L - i);
                    break;
                }
                Q[i] = (uint8_t)(sym + 33);
                uint32_t ctx = ((uint32_t)((q1 > q2 ? q1 : q2) << 6) + (uint32_t)sym) & 0xfffu;
                if (cfg->qlevel > 1) {
                    ctx += (q1 == q2) ? 0x1000u : 0u;
                    delta += (q1 > sym) ? (q1 - sym) : 0;
                    ctx += (uint32_t)(((delta <= 56 ? delta : 56) & 0xf8) << 10);
                    if (cfg->qlevel > 2) ctx += (i <= 0x6f) ? (uint32_t)(((i + 15) & 0x78) << 13) : 0xf0000u;
                }
                q2 = q1;
                q1 = sym;
                last = ctx;
            }
            Q += L;
        }
        free(qm);
        qm = NULL;
        if (d.err) goto out;
        c.p += sz;
    }

    /* N / IUPAC side streams (DegeInfoProcess@0x433a10; 23, 14, 24, 25, 26) */
    tip = (uint8_t *)calloc((size_t)n + 1, 1);
    isn = (uint8_t *)calloc((size_t)total + 1, 1);   /* per base: 0 = ACGT, else its character */
    if (!tip || !isn) goto out;
    {
        uint32_t ntip = 0;
        dkmodel *km = (dkmodel *)malloc(sizeof(dkmodel));
        uint8_t *chs = NULL, *maxq = NULL;
        uint32_t *exc = NULL, *gaps = NULL;
        uint32_t nch = 0, nmax = 0, nexc = 0, ngap = 0;
        int bad = !km;
        if (!bad) dk_init(km);
        const int ids[5] = {23, 14, 24, 25, 26};
        for (int s = 0; s < 5 && !bad; s++) {
            if (!take_id(&c, ids[s])) continue;   /* omitted when empty */
            const uint32_t sz = take_size4(&c);
            if (c.err || (size_t)(c.end - c.p) < sz || sz < 4) { bad = 1; break; }
            const uint32_t cnt = get_u32le(c.p);
            rd_t d;
            rd_init(&d, c.p + 4, c.p + sz);
            if (ids[s] == 23) {
                dmodel m;
                dm_init(&m, 2);
                for (uint32_t i = 0; i < cnt && i < n; i++) { tip[i] = (uint8_t)dm_decode(&m, &d); ntip += tip[i]; }
            } else if (ids[s] == 14 || ids[s] == 24) {
                dmodel *m = (dmodel *)malloc(sizeof(dmodel));
                uint8_t *v = (uint8_t *)malloc((size_t)cnt + 1);
                if (!m || !v) { free(m); free(v); bad = 1; break; }
                dm_init(m, ids[s] == 14 ? 11 : 95);
                for (uint32_t i = 0; i < cnt; i++) v[i] = (uint8_t)dm_decode(m, &d);
                free(m);
                if (ids[s] == 14) { chs = v; nch = cnt; } else { maxq = v; nmax = cnt; }
            } else {
                uint32_t *v = (uint32_t *)malloc(4 * ((size_t)cnt + 1));
                if (!v) { bad = 1; break; }
                for (uint32_t i = 0; i < cnt; i++) v[i] = (uint32_t)dk_decode(km, &d);   /* km shared by 25 and 26 */
                if (ids[s] == 25) { exc = v; nexc = cnt; } else { gaps = v; ngap = cnt; }
            }
            if (d.err) bad = 1;
            c.p += sz;
        }
        /* place the N / IUPAC bases: a tip-1 read's candidates (qual <= maxq)
         * are N^g1 B N^g2 B ... N^gE B N..., B = the E "exc" ACGT bases */
        uint32_t it = 0, ig = 0, ic = 0;
        uint64_t at = 0;
        const uint8_t *Q = o->qual;
        if (!bad && (nmax != ntip || nexc != ntip)) bad = 1;
        for (uint32_t r = 0; r < n && !bad; r++) {
            const uint32_t L = len[r];
            if (tip[r]) {
                const int mq = (int)maxq[it] + 33;
                const uint32_t E = exc[it];
                it++;
                uint32_t e = 0;
                uint64_t rem = E ? (ig < ngap ? gaps[ig] : (bad = 1, 0)) : ~0ull;
                for (uint32_t i = 0; i < L && !bad; i++) {
                    if ((int)(int8_t)Q[i] > mq) continue;
                    if (e < E && rem == 0) {
                        e++;
                        ig++;
                        rem = e < E ? (ig < ngap ? gaps[ig] : (bad = 1, 0)) : ~0ull;
                    } else {
                        if (ic >= nch) { bad = 1; break; }
                        const uint8_t sc = chs[ic++];
                        isn[at + i] = (uint8_t)IUPAC[sc < 11 ? sc : 0];
                        rem--;
                    }
                }
            }
            Q += L;
            at += L;
        }
        if (!bad && ic != nch) bad = 1;
        free(km); free(chs); free(maxq); free(exc); free(gaps);
        if (bad) goto out;
    }

    /* bases (compressSeq@0x4248a0 / encode_seq@0x421f30) */
    {
        if (!take_id(&c, 6)) goto out;
        const uint32_t sz = take_size4(&c);
        if (c.err || (size_t)(c.end - c.p) < sz) goto out;
        const uint8_t *q = c.p;
        if (cfg->md5) { memcpy(md5_seq, q, 16); q += 16; }
        const int k = cfg->slevel + 7;
        const uint32_t ns = 1u << ((2 * k) & 31), mask = ns - 1;
        tab = (uint8_t *)malloc((size_t)ns * 4);
        if (!tab) goto out;
        memset(tab, 3, (size_t)ns * 4);
        rd_t d;
        rd_init(&d, q, c.p + sz);
        uint8_t *S = o->seq;
        uint64_t at = 0;
        for (uint32_t r = 0; r < n && !d.err; r++) {
            const uint32_t L = len[r];
            uint32_t ctx = 0x7616c7u & mask;
            for (uint32_t i = 0; i < L; i++) {
                if (isn[at + i]) { S[i] = isn[at + i]; continue; }
                uint8_t *m = tab + (size_t)ctx * 4;
                uint32_t tot = (uint32_t)m[0] + m[1] + m[2] + m[3];
                if (tot > 253) {
                    for (int j = 0; j < 4; j++) m[j] = (uint8_t)(m[j] - (m[j] >> 1));
                    tot = (uint32_t)m[0] + m[1] + m[2] + m[3];
                }
                uint32_t r2;
                const uint32_t v = rd_slot(&d, tot, &r2);
                uint32_t cum = 0, b = 0;
                while (b < 3 && cum + m[b] <= v) { cum += m[b]; b++; }
                rd_take(&d, r2, cum, m[b]);
                m[b]++;
                S[i] = (uint8_t)"ACGT"[b];
                ctx = ((ctx << 2) + b) & mask;
            }
            S += L;
            at += L;
        }
        if (d.err) goto out;
        c.p += sz;
    }
    if (c.p != c.end) goto out;
    if (cfg->md5) {
        uint8_t dg[16];
        orc_md5(o->names, (size_t)name_total, dg);
        if (memcmp(dg, md5_id, 16)) o->md5_ok = 0;
        if (!(cfg->lossy > 0.0)) {   /* compressQual@0x426eca: no qual MD5 with -l */
            orc_md5(o->qual, (size_t)total, dg);
            if (memcmp(dg, md5_qual, 16)) o->md5_ok = 0;
        }
        orc_md5(o->seq, (size_t)total, dg);
        if (memcmp(dg, md5_seq, 16)) o->md5_ok = 0;
    }
    ret = (int64_t)n;
out:
    free(len);
    free(qm);
    free(tab);
    free(tip);
    free(isn);
    return ret;
}
