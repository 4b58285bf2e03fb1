// sa_logic.h -- per-thread logic of the encoder kernels, written once as
// host+device functions.  sa_kernels.hip wraps each in a kernel; the CPU
// decomposition test (tests/cpu_emu) drives the same functions sequentially to
// check the decomposition against the oracle before it runs on the GPU.
#pragma once
#include "sa_common.h"
#include "sa_device.h"

namespace sa {

// ---- per-read counts (k_prep) ----------------------------------------------
// The columns of a read's SEQ / QUAL / N-IUPAC side streams (and their input
// checks) from its seq_stat and trimmed quality length.
// seq_skip: an aligned read of the reference path, whose bases the SEQ stream
// leaves out (compressSeq@0x4249b3: order byte != 0).
SA_HD uint32_t prep_sq_cols(uint32_t* c, uint32_t len, uint32_t nq, const SeqStat& st, bool qual_bad,
                            bool seq_skip = false)
{
    uint32_t e = st.err;
    c[C_SEQ] = seq_skip ? 0u : st.valid;
    c[C_QUAL] = nq + (nq != len ? 1 : 0);
    if (qual_bad) e |= E_QUALRANGE;
    c[C_CH] = st.nch;
    const uint32_t has = st.nch ? 1 : 0;
    c[C_MAXQ] = has;
    if (has && (st.maxq < 33 || st.maxq > 127)) e |= E_QUALRANGE;
    c[C_NCNT] = has ? 1 + (uint32_t)nbits_u32(st.exc) : 0;
    c[C_NPOS] = has ? st.npos_syms : 0;
    c[C_NPOSV] = has ? st.exc : 0;
    return e;
}

// Every column of read r; bulk = false leaves out the SEQ / QUAL / N-IUPAC
// columns (k_prep_sq computes those one wave per read).
SA_HD uint32_t prep_read(const BatchView& bv, uint32_t r, uint32_t* counts, int16_t* name_p, int16_t* name_s,
                         bool bulk)
{
    const uint32_t b = bv.read_block[r];
    const DevBlock& blk = bv.blocks[b];
    const uint32_t lr = r - blk.read0;
    const uint8_t* s = bv.seq + blk.seq_base + bv.seq_off[r];
    const uint8_t* q = bv.qual + blk.seq_base + bv.seq_off[r];
    const uint32_t len = bv.seq_len[r];
    uint32_t e = 0;

    uint32_t* c = counts + (size_t)r * NCOL;
    if (bulk) {
        const SeqStat st = seq_stat(s, q, len);   // N/IUPAC side info: original qualities
        const uint8_t* qq = bv.qual_q + blk.seq_base + bv.seq_off[r];
        const uint32_t n = qual_nonhash(qq, len);
        bool qbad = false;
        for (uint32_t i = 0; i < n; i++)
            if (qq[i] < 33 || qq[i] > 126) { qbad = true; break; }
        e |= prep_sq_cols(c, len, n, st, qbad, bv.seq_skip && bv.seq_skip[r]);
    }
    c[C_LEN] = len == 0 ? 1 : (blk.len_long ? 5 : 3);
    c[C_TIP] = 1;

    if (bv.bin_mode) {
        c[C_NAME] = 0;
    } else {
        const uint8_t* nm = bv.names + blk.name_base + bv.name_off[r];
        const int nl = bv.name_len[r];
        int p = 0, sfx = 0;
        if (lr > 0) {
            const uint8_t* pv = bv.names + blk.name_base + bv.name_off[r - 1];
            name_prefix_suffix(nm, nl, pv, bv.name_len[r - 1], p, sfx);
        } else {
            name_prefix_suffix(nm, nl, nm, 0, p, sfx);
        }
        if (nl > 255) e |= E_NAME;
        name_p[r] = (int16_t)p;
        name_s[r] = (int16_t)sfx;
        int mid = nl - sfx - p;
        c[C_NAME] = 3 + (mid > 0 ? (uint32_t)mid : 0);
    }
    return e;
}

// ---- symbol emission (k_emit) ----------------------------------------------
struct AuxEmit {
    uint32_t* key;
    uint32_t* val;
    uint32_t pos;
    SA_HD void operator()(uint32_t model, uint32_t s)
    {
        key[pos] = (model << AUX_SYM_BITS) | s;
        if (val) val[pos] = pos;   // (the device leaves the AUX values out: they are the index)
        pos++;
    }
};

SA_HD void emit_kmodel(AuxEmit& em, uint32_t v)
{
    int nb = nbits_u32(v);
    em(M_KBITS, (uint32_t)nb);
    for (int i = 0; i < nb; i++) em(M_KBIT0 + (uint32_t)i, (v >> i) & 1);
}

// Symbols of column `col` of read r: the difference of the exclusive offsets
// k_scan_reads left in `counts` (the block total after its last read).
SA_HD uint32_t read_col_count(const BatchView& bv, const uint32_t* counts, const uint32_t* totals, uint32_t r,
                              int col)
{
    const uint32_t b = bv.read_block[r];
    const DevBlock& blk = bv.blocks[b];
    const uint32_t next = r + 1 < blk.read0 + blk.nreads ? counts[(size_t)(r + 1) * NCOL + col]
                                                          : totals[(size_t)b * NCOL + col];
    return next - counts[(size_t)r * NCOL + col];
}

// Every symbol of read r.  bulk = false leaves out the SEQ and QUAL symbols
// (k_emit_sq writes those one wave per read).
SA_HD uint32_t emit_read(const BatchView& bv, uint32_t r, const uint32_t* counts, const uint32_t* totals,
                         const int16_t* name_p, const int16_t* name_s, const uint16_t* name_maxlen,
                         uint32_t* seq_key, uint32_t* seq_val, uint32_t* aux_key, uint32_t* aux_val, bool bulk,
                         const uint8_t* dege_maxq = nullptr)
{
    uint32_t e = 0;
    const uint32_t b = bv.read_block[r];
    const DevBlock& blk = bv.blocks[b];
    const uint32_t lr = r - blk.read0;
    const uint8_t* s = bv.seq + blk.seq_base + bv.seq_off[r];
    const uint8_t* q = bv.qual + blk.seq_base + bv.seq_off[r];
    const uint32_t len = bv.seq_len[r];
    const uint32_t* off = counts + (size_t)r * NCOL;

    // sequence: BASE_MODEL contexts (encode_seq@0x421f30)
    if (bulk && !(bv.seq_skip && bv.seq_skip[r])) {
        uint32_t* K = seq_key + blk.seq_sym_base;
        uint32_t* V = seq_val + blk.seq_sym_base;
        uint32_t d = off[C_SEQ];
        const uint32_t mask = bv.seq_mask;
        uint32_t ctx = 0x7616c7u & mask;
        for (uint32_t i = 0; i < len; i++) {
            uint32_t cd = base_code(s[i]);
            if (cd > 3) continue;
            K[d] = ctx;
            V[d] = (d << 2) | cd;
            d++;
            ctx = ((ctx << 2) + cd) & mask;
        }
    }
    AuxEmit em{aux_key + blk.aux_sym_base, aux_val ? aux_val + blk.aux_sym_base : nullptr, 0};
    // lengths (encode_len_short@0x4239a0; last_len stays 0)
    em.pos = blk.sbase[ST_LEN] + off[C_LEN];
    if (len == 0) {
        em(M_LEN_SAME, 1);
    } else {
        em(M_LEN_SAME, 0);
        em(M_LEN_LO, len & 0xff);
        em(M_LEN_HI, (len >> 8) & 0xff);
        if (blk.len_long) {   // encode_len_long@0x422e70: bytes 2 and 3 as well
            em(M_LEN_B2, (len >> 16) & 0xff);
            em(M_LEN_B3, len >> 24);
        }
    }
    // names (encode_name@0x421070)
    if (!bv.bin_mode) {
        em.pos = blk.sbase[ST_NAME] + off[C_NAME];
        const uint8_t* nm = bv.names + blk.name_base + bv.name_off[r];
        const int nl = bv.name_len[r];
        const int ll = lr ? bv.name_len[r - 1] : 0;
        const int lp = lr ? name_p[r - 1] : 0;
        const int ls = lr ? name_s[r - 1] : 0;
        const int p = name_p[r], sf = name_s[r];
        em(M_NAME_PRE + (uint32_t)lp, (uint32_t)p);
        em(M_NAME_SUF + (uint32_t)ls, (uint32_t)sf);
        em(M_NAME_LEN + (uint32_t)ll, (uint32_t)nl);
        // the reference's last-name buffer: each byte j holds the latest earlier
        // name of the block longer than j, or ' ' (reset per block @0x42452c)
        const uint32_t maxlen = name_maxlen[r];
        const uint32_t rb = blk.read0;
        auto last = [&](int j) -> uint8_t {
            if (j < 0) return 0;
            if ((uint32_t)j >= maxlen) return ' ';
            for (uint32_t m = r; m > rb; m--) {
                if ((uint32_t)bv.name_len[m - 1] > (uint32_t)j)
                    return bv.names[blk.name_base + bv.name_off[m - 1] + (uint32_t)j];
            }
            return ' ';
        };
        auto emid = [&](uint32_t ctx, uint32_t sym) { em(M_NAME_MID + ctx, sym); };
        if (!name_mid(nm, nl, p, sf, last, emid)) e |= E_NAME;
    }
    // qualities (encode_qual@0x422180)
    if (bulk) {
        em.pos = blk.sbase[ST_QUAL] + off[C_QUAL];
        const uint8_t* qq = bv.qual_q + blk.seq_base + bv.seq_off[r];
        const uint32_t n = qual_nonhash(qq, len);
        QualCtx qc{0, 0, 5};
        uint32_t last = 0;
        for (uint32_t i = 0; i < n; i++) {
            int sym = (uint8_t)(qq[i] - 33);
            em(M_QUAL + last, (uint32_t)sym);
            last = qual_next_ctx(qc, sym, i, bv.qlevel);
        }
        if (n != len) em(M_QUAL + last, 94);
    }
    // degenerate-base side streams (DegeInfoProcess@0x433a10)
    {
        em.pos = blk.sbase[ST_TIP] + off[C_TIP];
        const uint32_t nch = read_col_count(bv, counts, totals, r, C_CH);   // from k_prep
        em(M_TIP, nch ? 1u : 0u);
        if (nch && dege_maxq) {   // device: k_prep_sq16 kept maxq; the CH / NPOS streams are k_emit_sq's
            em.pos = blk.sbase[ST_MAXQ] + off[C_MAXQ];
            em(M_MAXQ, (uint8_t)(dege_maxq[r] - 33));
            em.pos = blk.sbase[ST_NCNT] + off[C_NCNT];
            emit_kmodel(em, read_col_count(bv, counts, totals, r, C_NPOSV));
        } else if (nch) {
            const SeqStat st = seq_stat(s, q, len);
            em.pos = blk.sbase[ST_CH] + off[C_CH];
            for (uint32_t i = 0; i < len; i++) {
                uint32_t cd = base_code(s[i]);
                if (cd > 3) em(M_CH, cd - 4);
            }
            em.pos = blk.sbase[ST_MAXQ] + off[C_MAXQ];
            em(M_MAXQ, (uint8_t)(st.maxq - 33));
            em.pos = blk.sbase[ST_NCNT] + off[C_NCNT];
            emit_kmodel(em, st.exc);
            em.pos = blk.sbase[ST_NPOS] + off[C_NPOS];
            uint32_t gap = 0;
            for (uint32_t i = 0; i < len; i++) {
                if ((int)st.maxq < (int)(int8_t)q[i]) continue;
                if (base_code(s[i]) > 3) {
                    gap++;
                } else {
                    emit_kmodel(em, gap);
                    gap = 0;
                }
            }
        }
    }
    return e;
}

// ---- reference (HASH index) path: the alignment streams of one read ---------
// What AlignEncodeSEJob::AlignInfoProcess@0x4118b0 / AlignEncodePEJob::
// AlignInfoProcessPE@0x412290 and decomposeAlignInfo@0x433860 push for a read
// (int2bit@0x40dcd0: values as bit strings, least significant bit first), as
// em(column, model, symbol) calls in stream order.  A read of the block's first
// order_count reads is aligned iff av.ret >= 0 (the host chose its variant of
// the carried align_info state and cut the block at the bail-out); PE pairs are
// reads (2j, 2j+1) of the block: mate 1 carries the pair's relation (the
// position of mate 2 from the insert window, further right as a distance,
// further left absolutely) and, with both mates aligned, both carry mate 1's
// order byte.
SA_HD uint32_t aln_bits(uint64_t v)   // getbitnum@0x40d470
{
    uint32_t n = 0;
    while (v) { n++; v >>= 1; }
    return n;
}

template <class Em>
SA_HD void align_read_syms(const BatchView& bv, const AlignView& av, uint32_t r, Em em)
{
    const DevBlock& blk = bv.blocks[bv.read_block[r]];
    const uint32_t i = r - blk.read0;
    if (i >= blk.order_count) return;
    const bool al = av.ret[r] >= 0;
    auto bits = [&](uint64_t v, uint32_t nb) {
        for (uint32_t k = 0; k < nb; k++) em(A_POS, M_POS, (uint32_t)((v >> k) & 1u));
    };
    uint64_t ord = 0;
    if (!av.paired) {
        if (al) {
            const uint64_t p = av.pos[r];
            bits(p & av.mask, av.shift);
            ord = (p >> av.shift) + 1;
        }
    } else {
        const bool mate2 = (i & 1u) != 0;
        const uint32_t r1 = mate2 ? r - 1 : r, r2 = r1 + 1;
        const bool a1 = av.ret[r1] >= 0, a2 = av.ret[r2] >= 0;
        const uint64_t p1 = av.pos[r1], p2 = av.pos[r2];
        if (!mate2) {
            if (a1) {
                bits(p1 & av.mask, av.shift);
                ord = (p1 >> av.shift) + 1;
                if (a2) {
                    const uint64_t d = p1 > p2 ? p1 - p2 : p2 - p1;
                    if (d < (uint64_t)blk.win) {
                        em(A_PEREL, M_PEREL, p1 < p2 ? 1u : 0u);
                        bits(d, blk.ibits);
                    } else if (p1 < p2) {
                        em(A_PEREL, M_PEREL, 3u);
                        bits(d, aln_bits(av.glen - p1));
                    } else {
                        em(A_PEREL, M_PEREL, 2u);
                        bits(p2, aln_bits(p1));
                    }
                }
            }
        } else if (a2) {
            if (a1) {
                ord = (p1 >> av.shift) + 1;
            } else {
                bits(p2 & av.mask, av.shift);
                ord = (p2 >> av.shift) + 1;
            }
        }
    }
    em(A_ORD, M_ORD, (uint32_t)(ord & 0xffu));
    if (!al) return;
    // decomposeAlignInfo@0x433860: each mismatch offset as the gap from the
    // previous one in bits(len - previous) bits, its type; the count, the strand
    const int nm = av.ret[r];
    const int32_t* mp = av.mispos + (size_t)r * av.stride;
    const int32_t* mt = av.mistype + (size_t)r * av.stride;
    const int len = (int)bv.seq_len[r];
    int prev = 0;
    for (int k = 0; k < nm; k++) {
        const uint32_t v = (uint32_t)(mp[k] - prev), nb = aln_bits((uint64_t)(int64_t)(len - prev));
        for (uint32_t j = 0; j < nb; j++) em(A_CIGL, M_CIGL, (v >> j) & 1u);
        prev = mp[k];
        em(A_CIGV, M_CIGV, (uint32_t)mt[k]);
    }
    em(A_MIS, av.mis_model, (uint32_t)nm);
    em(A_REV, M_REV, (uint32_t)av.rev[r]);
}

// The count columns of read r (and whether its bases leave the SEQ stream).
SA_HD bool align_read_counts(const BatchView& bv, const AlignView& av, uint32_t r, uint32_t* c)
{
    for (int k = 0; k < NACOL; k++) c[k] = 0;
    align_read_syms(bv, av, r, [&](int col, uint32_t, uint32_t) { c[col]++; });
    const DevBlock& blk = bv.blocks[bv.read_block[r]];
    return r - blk.read0 < blk.order_count && av.ret[r] >= 0;
}

// The keys of read r's alignment symbols; off = its exclusive column offsets.
// (The Mis symbols are counted for align_count but written only when the
// maxmis in force has a Mis model.)
SA_HD void align_read_emit(const BatchView& bv, const AlignView& av, uint32_t r, const uint32_t* off, uint32_t* aux_key,
                           uint32_t* aux_val)
{
    const DevBlock& blk = bv.blocks[bv.read_block[r]];
    uint32_t at[NACOL];   // (column k is stream ST_ORD + k)
    for (int k = 0; k < NACOL; k++) at[k] = blk.sbase[ST_ORD + k] + off[k];
    uint32_t* K = aux_key + blk.aux_sym_base;
    uint32_t* V = aux_val ? aux_val + blk.aux_sym_base : nullptr;
    align_read_syms(bv, av, r, [&](int col, uint32_t model, uint32_t sym) {
        if (col == A_MIS && !model) return;
        const uint32_t p = at[col]++;
        K[p] = (model << AUX_SYM_BITS) | sym;
        if (V) V[p] = p;
    });
}

// ---- coder records written by the model replays ---------------------------
// Per coded symbol, in stream order: the Pass-R record {ceil(2^32/tot),
// tot | freq << 16} and cum (< 2^16: every model total is <= 0xffe0).
struct SymSink {
    PRec* prs;
    uint16_t* cum;
};
SA_HD void sink_put(const SymSink& o, uint32_t pos, uint32_t cum, uint32_t f, uint32_t t);

// ---- BASE_MODEL replay of one context run (k_replay_seq) -------------------
// keys/vals: the block's sorted SEQ symbols (val = stream position << 2 | base);
// the run of `key` starts at i.  rec: the block's SEQ records.  Keys and
// values are read 8 ahead so the loads overlap the serial model update.
constexpr int RP_CHUNK = 8;

SA_HD void replay_seq_run(const uint32_t* keys, const uint32_t* vals, size_t i, size_t end, uint32_t key,
                          const SymSink& rec)
{
    uint32_t st = 0x03030303u;
    uint32_t kk[RP_CHUNK], vv[RP_CHUNK];
    for (int c = 0; c < RP_CHUNK; c++) { kk[c] = keys[i + c]; vv[c] = vals[i + c]; }
    for (size_t j = i;; j += RP_CHUNK) {
        uint32_t kn[RP_CHUNK], vn[RP_CHUNK];
        for (int c = 0; c < RP_CHUNK; c++) { kn[c] = keys[j + RP_CHUNK + c]; vn[c] = vals[j + RP_CHUNK + c]; }
        for (int c = 0; c < RP_CHUNK; c++) {
            if (j + c >= end || kk[c] != key) return;
            const uint32_t b = vv[c] & 3, pos = vv[c] >> 2;
            uint32_t tot = (st & 0xff) + ((st >> 8) & 0xff) + ((st >> 16) & 0xff) + (st >> 24);
            if (tot > 253) {
                st -= (st >> 1) & 0x7f7f7f7fu;
                tot = (st & 0xff) + ((st >> 8) & 0xff) + ((st >> 16) & 0xff) + (st >> 24);
            }
            const uint32_t below = b ? (st & (0xffffffffu >> (32 - 8 * b))) : 0u;
            const uint32_t cum = (below & 0xff) + ((below >> 8) & 0xff) + ((below >> 16) & 0xff);
            const uint32_t f = (st >> (8 * b)) & 0xff;
            sink_put(rec, pos, cum, f, tot);
            st += 1u << (8 * b);
        }
        for (int c = 0; c < RP_CHUNK; c++) { kk[c] = kn[c]; vv[c] = vn[c]; }
    }
}

// ---- SIMPLE_MODEL<N> (kModelEncode@0x42ccb0 and every inlined copy) --------
// Model = {TotFreq, BubCnt, sentinel, F[0..N-1] of {symbol, freq}}.  The first
// RP_REG entries live in registers (the hot symbols bubble there); the rest in
// F (LDS), indexed from RP_REG.  Entry = sym << 16 | freq; an unused register
// slot (N < RP_REG) has sym 0xffff and freq 0.
constexpr int RP_REG = 4;

struct SModel {
    uint32_t R[RP_REG];
    uint32_t N, tot, bub;
};

SA_HD void sm_init(SModel& m, uint32_t N, uint32_t* F, uint32_t first, uint32_t step)
{
    for (int k = 0; k < RP_REG; k++) m.R[k] = (uint32_t)k < N ? (((uint32_t)k << 16) | 1u) : 0xffff0000u;
    for (uint32_t k = RP_REG + first; k < N; k += step) F[k - RP_REG] = (k << 16) | 1u;
    m.N = N;
    m.tot = N;
    m.bub = 0;
}

// Codes one symbol: cf = cum | freq << 16 and t = TotFreq before the update,
// then applies the update (freq += 8, TotFreq += 8, halve when > 0xffe0, and
// every 16th update bubble the symbol one place forward).  false if `sym` is
// not in the model (the reference would run off the array).
SA_HD bool sm_code(SModel& m, uint32_t* F, uint32_t sym, uint32_t& cf, uint32_t& t)
{
    // register slots first, as an early-exit chain (the hot symbol is R[0])
    uint32_t cum = 0, f = 0, idx = RP_REG;
#pragma unroll
    for (int k = 0; k < RP_REG; k++) {
        if ((m.R[k] >> 16) == sym) {
            idx = (uint32_t)k;
            f = m.R[k] & 0xffff;
            m.R[k] += 8;
            break;
        }
        cum += m.R[k] & 0xffff;
    }
    if (idx == RP_REG) {
        uint32_t k = RP_REG;
        for (;; k++) {
            if (k >= m.N) return false;
            const uint32_t e = F[k - RP_REG];
            if ((e >> 16) == sym) { f = e & 0xffff; break; }
            cum += e & 0xffff;
        }
        idx = k;
        F[idx - RP_REG] += 8;
    }
    cf = cum | (f << 16);
    t = m.tot;
    m.tot += 8;
    if (m.tot > 0xffe0) {
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < RP_REG; k++) {
            const uint32_t fr = m.R[k] & 0xffff, h = fr - (fr >> 1);
            m.R[k] = (m.R[k] & 0xffff0000u) | h;
            tot += h;
        }
        for (uint32_t k = RP_REG; k < m.N; k++) {
            const uint32_t x = F[k - RP_REG], fr = x & 0xffff, h = fr - (fr >> 1);
            F[k - RP_REG] = (x & 0xffff0000u) | h;
            tot += h;
        }
        m.tot = tot;
    }
    if (((++m.bub) & 15) == 0 && idx > 0) {
        if (idx < RP_REG) {
#pragma unroll
            for (int k = 1; k < RP_REG; k++) {
                if (idx == (uint32_t)k && (m.R[k] & 0xffff) > (m.R[k - 1] & 0xffff)) {
                    const uint32_t x = m.R[k];
                    m.R[k] = m.R[k - 1];
                    m.R[k - 1] = x;
                }
            }
        } else if (idx == RP_REG) {
            const uint32_t cur = F[0];
            if ((cur & 0xffff) > (m.R[RP_REG - 1] & 0xffff)) {
                F[0] = m.R[RP_REG - 1];
                m.R[RP_REG - 1] = cur;
            }
        } else {
            const uint32_t cur = F[idx - RP_REG], prv = F[idx - RP_REG - 1];
            if ((cur & 0xffff) > (prv & 0xffff)) {
                F[idx - RP_REG] = prv;
                F[idx - RP_REG - 1] = cur;
            }
        }
    }
    return true;
}

// Per-lane replay of one model run (short runs; k_replay_aux_short).
SA_HD uint32_t replay_simple_run(const uint32_t* keys, const uint32_t* vals, size_t i, size_t end, uint32_t model,
                                 const SymSink& rec, uint32_t* F)
{
    SModel m;
    sm_init(m, model_nsym(model), F, 0, 1);
    for (size_t j = i; j < end; j++) {
        const uint32_t key = keys[j];
        if ((key >> AUX_SYM_BITS) != model) break;
        uint32_t cf, t;
        if (!sm_code(m, F, key & 0xff, cf, t)) return E_CODER;
        sink_put(rec, vals[j], cf & 0xffff, cf >> 16, t);
    }
    return 0;
}

// ---- decomposed range coder ------------------------------------------------
// The carry-less coder of encode_seq@0x422010-0x422085 has two state words:
// range (u32) and low (u64).  Apart from the rare "squeeze" (range forced to
// the distance to the next 2^24 boundary when low and low+range straddle a
// top-byte boundary, probability ~2^-32 per normalisation), range evolves
// independently of low:
//     q = range / tot;  rr = q * f;  n = clz(rr) / 8;  range = rr << 8n
// and low evolves as an affine map of its previous value per symbol:
//     low = (low + cum * q) << 8n    (mod 2^64; the shifted-out bytes are output)
// So the coder is split into
//   R  (serial, one wave per stream): the range chain only, on the scalar unit,
//      keeping one range checkpoint per SEG_SYMS symbols;
//   L1 (parallel, one lane per segment): re-run the segment's range chain from
//      its checkpoint and reduce its effect on low to an affine map
//      low -> (low << 8N) + D  plus its byte count N;
//   L2 (per stream): exclusive scan of those maps -> low and output offset at
//      every segment start;
//   L3 (parallel, one lane per segment): the exact reference coder over the
//      segment from (range, low), writing its bytes at the segment's offset and
//      checking the squeeze condition exactly.  A squeeze voids the checkpoints
//      after it: the stream restarts R/L1/L2/L3 after that segment from the exact
//      state L3 computed (the host loops until no stream squeezes).

// ceil(2^32 / t) for 2 <= t < 2^32 (t = 2^32 = a t + b: b > 0 -> a + 1; b = 0 -> a)
SA_HD uint32_t recip32(uint32_t t) { return 0xffffffffu / t + 1u; }
// ... and 0 for t = 0 (a record not written yet: sends the range to 0)
SA_HD uint32_t recip32z(uint32_t t) { return t ? recip32(t) : 0u; }

// Two record formats.  Wide (AUX, SIMPLE_MODEL totals up to 0xffe0):
// tf = t | f << 16, cum in its own array.  Packed (SEQ, BASE_MODEL: t <= 253):
// tf = t | cum << 8 | f << 16 and no cum array (SymSink::cum == nullptr), one
// scattered store per symbol instead of two.
SA_HD void sink_put(const SymSink& o, uint32_t pos, uint32_t cum, uint32_t f, uint32_t t)
{
    if (!o.cum) {
        o.prs[pos] = PRec{t | (cum << 8) | (f << 16)};
    } else {
        o.prs[pos] = PRec{t | (f << 16)};
        o.cum[pos] = (uint16_t)cum;
    }
}

SA_HD uint32_t rec_tmask(const uint16_t* cum) { return cum ? 0xffffu : 0xffu; }

SA_HD uint32_t clz32(uint32_t v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_clz(v);
#else
    return v ? (uint32_t)__builtin_clz(v) : 32u;
#endif
}

SA_HD uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

// one symbol of the range chain (m = recip32z(t)); returns q, updates r, sets
// n (bytes shifted)
SA_HD uint32_t range_step(uint32_t& r, const PRec p, uint32_t m, uint32_t tmask, uint32_t& n)
{
    const uint32_t t = p.tf & tmask, f = p.tf >> 16;
    uint32_t q = mulhi32(r, m);
    q -= (r < q * t) ? 1u : 0u;
    const uint32_t rr = q * f;
    const uint32_t sh = clz32(rr) & 24u;
    n = sh >> 3;
    r = rr << sh;
    return q;
}

SA_HD uint64_t shl64(uint64_t x, uint32_t s) { return s >= 64 ? 0ull : x << s; }

// apply a then b
SA_HD LowMap lowmap_compose(const LowMap& a, const LowMap& b)
{
    LowMap c;
    c.B = shl64(a.B, b.s) + b.B;
    c.s = a.s + b.s >= 64 ? 64u : a.s + b.s;
    c.nbytes = a.nbytes + b.nbytes;
    return c;
}

// L1: a segment's map from its range checkpoint.
// The records of a segment, RC_CHUNK at a time: a chunk's loads are issued
// back to back before it is coded (on the GPU one lane walks one segment, so
// its cache lines must not be evicted between dependent steps).  The last
// chunk re-reads record n - 1 instead of reading past the segment.  32
// records are one 128-byte line: with 16, a lane's second half-line was often
// evicted before it came back for it (L1 / L3 read 1.5 / 2.1 x the records' bytes,
// round 4 r4c PMC); the reciprocals are derived as the records are coded (off
// the chain), so the 32 records cost no more registers than 16 with their
// reciprocals did (88 VGPRs).
constexpr uint32_t RC_CHUNK = 32;
template <bool PACKED, uint32_t CH = RC_CHUNK, class Fn>
SA_HD void seg_for_each(const PRec* P, const uint16_t* cum, uint32_t n, Fn&& fn)
{
    const uint32_t tmask = PACKED ? 0xffu : 0xffffu;
    if (n == SEG_SYMS) {   // (round 6) a full segment -- all but a stream's last: no per-symbol bound test
#pragma unroll 1
        for (uint32_t b = 0; b < SEG_SYMS; b += CH) {
            PRec p[CH];
            uint32_t c[PACKED ? 1 : CH];
#pragma unroll
            for (uint32_t k = 0; k < CH; k++) {
                p[k] = P[b + k];
                if constexpr (!PACKED) c[k] = cum[b + k];
            }
#pragma unroll
            for (uint32_t k = 0; k < CH; k++)
                fn(p[k], recip32z(p[k].tf & tmask), PACKED ? (p[k].tf >> 8) & 0xffu : c[PACKED ? 0 : k]);
        }
        return;
    }
    for (uint32_t b = 0; b < n; b += CH) {
        PRec p[CH];
        uint32_t c[PACKED ? 1 : CH];
#pragma unroll
        for (uint32_t k = 0; k < CH; k++) {
            const uint32_t i = b + k < n ? b + k : n - 1;
            p[k] = P[i];
            if constexpr (!PACKED) c[k] = cum[i];
        }
#pragma unroll
        for (uint32_t k = 0; k < CH; k++)
            if (b + k < n) fn(p[k], recip32z(p[k].tf & tmask), PACKED ? (p[k].tf >> 8) & 0xffu : c[PACKED ? 0 : k]);
    }
}

// L1's per-symbol step: the affine map of low over the symbols so far
struct LowMapAcc {
    uint64_t low = 0;
    uint32_t sbits = 0, nbytes = 0;
    SA_HD void step(uint32_t& r, const PRec pr, uint32_t pm, uint32_t c, uint32_t tmask)
    {
        uint32_t nb;
        const uint32_t q = range_step(r, pr, pm, tmask, nb);
        low = shl64(low + (uint64_t)c * q, 8 * nb);
        sbits += 8 * nb;
        nbytes += nb;
    }
    SA_HD LowMap map() const { return LowMap{low, sbits >= 64 ? 64u : sbits, nbytes}; }
};

template <bool PACKED, uint32_t CH = RC_CHUNK>
SA_HD LowMap seg_lowmap_t(const PRec* P, const uint16_t* cum, uint32_t r, uint32_t n)
{
    LowMapAcc a;
    const uint32_t tmask = PACKED ? 0xffu : 0xffffu;
    seg_for_each<PACKED, CH>(P, cum, n, [&](const PRec pr, uint32_t pm, uint32_t c) { a.step(r, pr, pm, c, tmask); });
    return a.map();
}

// L3: the exact coder over one segment from (r, low).  Writes the bytes to
// o[0..) (bytes at or beyond cap are dropped) and returns how many it produced;
// `squeezed` is set if the carry-less squeeze fired.  If `finish`, the 8 flush
// bytes of low follow (rc finish @0x424a1c).
struct SegEnd {
    uint64_t low;
    uint32_t r;
    uint32_t nbytes;
    uint32_t squeezed;
};

SA_HD uint32_t seg_count(uint32_t n, uint32_t seg) { return n - seg * SEG_SYMS < SEG_SYMS ? n - seg * SEG_SYMS : SEG_SYMS; }

// L3's per-symbol step: the exact coder from (r, low), its bytes to o[0..cap)
struct SegCoder {
    uint32_t r;
    uint64_t low;
    uint8_t* o;
    uint64_t cap;
    uint32_t op = 0, squeezed = 0;
    SA_HD void step(const PRec pr, uint32_t pm, uint32_t c, uint32_t tmask)
    {
        const uint32_t t = pr.tf & tmask, f = pr.tf >> 16;
        uint32_t q = mulhi32(r, pm);
        q -= (r < q * t) ? 1u : 0u;
        low += (uint64_t)c * q;
        r = q * f;
        while (r < (1u << 24)) {
            if ((low ^ (low + r)) >> 56) {
                r = ((uint32_t)low | 0xffffffu) - (uint32_t)low;
                squeezed = 1;
            }
            if (op < cap) o[op] = (uint8_t)(low >> 56);
            op++;
            r <<= 8;
            low <<= 8;
        }
    }
    SA_HD SegEnd end(bool finish)
    {
        if (finish) {
            for (int k = 0; k < 8; k++) {
                if (op < cap) o[op] = (uint8_t)(low >> 56);
                op++;
                low <<= 8;
            }
        }
        return SegEnd{low, r, op, squeezed};
    }
};

template <bool PACKED, uint32_t CH = RC_CHUNK>
SA_HD SegEnd seg_code_t(const PRec* P, const uint16_t* cum, uint32_t r, uint64_t low, uint32_t n, uint8_t* o,
                        uint64_t cap, bool finish)
{
    SegCoder sc{r, low, o, cap};
    const uint32_t tmask = PACKED ? 0xffu : 0xffffu;
    seg_for_each<PACKED, CH>(P, cum, n, [&](const PRec pr, uint32_t pm, uint32_t c) { sc.step(pr, pm, c, tmask); });
    return sc.end(finish);
}

// cum == nullptr: packed (SEQ) records
template <uint32_t CH = RC_CHUNK>
SA_HD LowMap seg_lowmap(const PRec* P, const uint16_t* cum, uint32_t r, uint32_t n)
{
    return cum ? seg_lowmap_t<false, CH>(P, cum, r, n) : seg_lowmap_t<true, CH>(P, cum, r, n);
}
template <uint32_t CH = RC_CHUNK>
SA_HD SegEnd seg_code(const PRec* P, const uint16_t* cum, uint32_t r, uint64_t low, uint32_t n, uint8_t* o,
                      uint64_t cap, bool finish)
{
    return cum ? seg_code_t<false, CH>(P, cum, r, low, n, o, cap, finish)
               : seg_code_t<true, CH>(P, cum, r, low, n, o, cap, finish);
}

// ---- block assembly plan (k_assemble; doFqzEncode@0x42d2d0) ----------------
SA_HD uint32_t put_id(uint8_t* o, uint32_t id) { o[0] = (uint8_t)(0x80 | id); return 1; }
SA_HD void put_size4(uint8_t* o, uint32_t v)
{
    v |= 1u << 28;
    o[0] = (uint8_t)(v >> 24); o[1] = (uint8_t)(v >> 16); o[2] = (uint8_t)(v >> 8); o[3] = (uint8_t)v;
}
SA_HD void put_u32le(uint8_t* o, uint32_t v)
{
    o[0] = (uint8_t)v; o[1] = (uint8_t)(v >> 8); o[2] = (uint8_t)(v >> 16); o[3] = (uint8_t)(v >> 24);
}

// ---------------------------------------------------------------------------
// R-Block lossy pre-pass, EncapFqzComp::rblock@0x426c10 (-l R).  One greedy
// pass over a block's whole quality buffer: a run keeps its min and max; a new
// character c in [min, max] extends it; c > max extends it iff R > g/min and
// R > c/g, g = round(sqrt(c*min)) (@0x426cc0); c < min iff R > g/c and
// R > max/g, g = round(sqrt(c*max)) (@0x426d48); otherwise the run is
// overwritten with round(sqrt(min*max)) (@0x426c6d) and a new run opens at c.
// The divisions are IEEE double as in the reference; round(sqrt(n)) of an
// integer n is exact in integers (sqrt(n) is never within 2^-20 of k + 1/2).
//
// Parallel form: every chunk runs the greedy pass speculatively from a fresh
// run at its first byte and records where its runs open (rb_spec); one lane
// per block carries the true open run across the chunks, re-running a chunk
// only until the true pass closes a run where the speculative one opened one
// (from there both agree), else to the chunk's end (rb_fix); every chunk then
// replays from its true entry run and writes the runs that close inside it
// (rb_apply), so each byte is written exactly once.
// ---------------------------------------------------------------------------
SA_HD uint32_t rb_round_sqrt(uint32_t n)
{
    uint32_t g = 0;
    for (uint32_t b = 1u << 15; b; b >>= 1)   // floor(sqrt(n)), n < 2^30
        if ((g + b) * (g + b) <= n) g += b;
    return n > g * g + g ? g + 1 : g;
}

// The two decisions of a character outside the open run depend on two
// bytes each, so they are tables of 256 x 256 bits per R (round 5; built once
// per batch on the host with the reference's double arithmetic, staged in LDS
// by the kernels): lo[c][mx] -- c below the run extends it (R > g/c and
// R > mx/g, g = round(sqrt(c*mx)), @0x426d48), hi[c][mn] -- c above it does
// (R > g/mn and R > c/g, g = round(sqrt(c*mn)), @0x426cc0).  The per-byte
// step is then two compares and one bit test instead of an integer square root
// and two double divisions in divergent lanes.
constexpr uint32_t RB_TAB_WORDS = 256 * 256 / 32;
struct RbTab {
    const uint32_t* lo;
    const uint32_t* hi;
};

SA_HD bool rb_tab_bit(const uint32_t* t, uint32_t c, uint32_t v)
{
    const uint32_t i = (c << 8) | (v & 0xffu);
    return (t[i >> 5] >> (i & 31)) & 1u;
}

// lo / hi: RB_TAB_WORDS words each
SA_HD void rb_tab_build(double R, uint32_t* lo, uint32_t* hi)
{
    for (uint32_t w = 0; w < RB_TAB_WORDS; w++) lo[w] = hi[w] = 0;
    for (uint32_t c = 0; c < 256; c++)
        for (uint32_t v = 0; v < 256; v++) {
            const uint32_t i = (c << 8) | v;
            uint32_t g = rb_round_sqrt(c * v);   // v = mx
            if (R > (double)g / (double)c && R > (double)v / (double)g) lo[i >> 5] |= 1u << (i & 31);
            g = rb_round_sqrt(c * v);            // v = mn
            if (R > (double)g / (double)v && R > (double)c / (double)g) hi[i >> 5] |= 1u << (i & 31);
        }
}

// One character c of the open run; false: the run closes before c.
SA_HD bool rb_extend(RbRun& s, uint32_t c, const RbTab& t)
{
    if (s.mx >= c) {
        if (s.mn <= c) return true;
        if (rb_tab_bit(t.lo, c, s.mx)) { s.mn = c; return true; }
    } else {
        if (rb_tab_bit(t.hi, c, s.mn)) { s.mx = c; return true; }
    }
    return false;
}

constexpr uint32_t RB_CHUNK = 8192;   // the longest chunk (SA_RB_CHUNK)
constexpr uint32_t RB_WORDS = RB_CHUNK / 32;
constexpr uint32_t RB_CHUNK_DEFAULT = 7904;   // (247 words: see sa_ctx::rb_chunk)

// The bytes [from, len) of the chunk starting at q + base, in order, to
// f(i, c) until it returns false.  16 bytes per load (a lane walks its own
// chunk: byte loads left it at one load latency per byte, 39 / 64 ms for
// k_rb_spec / k_rb_apply per ONT batch, r3t); chunk bases are 16-byte aligned
// (blocks start on 16 bytes, chunks every RB_CHUNK bytes of a block).
template <class F>
SA_HD void rb_for_bytes(const uint8_t* q, uint64_t base, uint32_t from, uint32_t len, F f)
{
    for (uint32_t i0 = from & ~15u; i0 < len; i0 += 16) {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        const uint8_t* p = q + base + i0;
        if (i0 + 16 <= len && ((base + i0) & 15) == 0) {
            __builtin_memcpy(w, __builtin_assume_aligned(p, 16), 16);
        } else {
            for (uint32_t j = 0; j < 16 && i0 + j < len; j++) w[j >> 2] |= (uint32_t)p[j] << (8 * (j & 3));
        }
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            uint32_t x = w[k];
            for (uint32_t j = 0; j < 4; j++, x >>= 8) {
                const uint32_t i = i0 + 4 * k + j;
                if (i < from) continue;
                if (i >= len) return;
                if (!f(i, x & 0xffu)) return;
            }
        }
    }
}

// Speculative pass over one chunk: bit i of opens = a run opens at byte i
// (nwords: the chunk stride's words of opens, all written).
SA_HD RbRun rb_spec(const uint8_t* q, const RbChunk& ck, const RbTab& R, uint32_t* opens, uint32_t nwords = RB_WORDS)
{
    RbRun s{ck.base, q[ck.base], q[ck.base]};
    uint32_t w = 1u;   // a run opens at the chunk's first byte
    rb_for_bytes(q, ck.base, 1, ck.len, [&](uint32_t i, uint32_t c) {
        if (!rb_extend(s, c, R)) {
            s = RbRun{ck.base + i, c, c};
            w |= 1u << (i & 31);
        }
        if ((i & 31) == 31) { opens[i >> 5] = w; w = 0; }
        return true;
    });
    if ((ck.len & 31) != 0) opens[(ck.len - 1) >> 5] = w;
    for (uint32_t k = (ck.len + 31) >> 5; k < nwords; k++) opens[k] = 0;
    return s;
}

// The true open run after chunk ck, given the true run open before it.
SA_HD RbRun rb_carry(const uint8_t* q, const RbChunk& ck, RbRun s, const RbTab& R, const uint32_t* opens,
                     const RbRun& spec_exit)
{
    bool conv = false;
    rb_for_bytes(q, ck.base, 0, ck.len, [&](uint32_t i, uint32_t c) {
        if (!rb_extend(s, c, R)) {
            if ((opens[i >> 5] >> (i & 31)) & 1u) {   // converged
                conv = true;
                return false;
            }
            s = RbRun{ck.base + i, c, c};
        }
        return true;
    });
    return conv ? spec_exit : s;
}

// Writes every run that closes inside chunk ck (and, in the block's last
// chunk, the final run); entry = the true run open before the chunk.
SA_HD void rb_apply(const uint8_t* q, uint8_t* out, const RbChunk& ck, RbRun s, const RbTab& R)
{
    uint32_t from = 0;
    if (ck.flags & RB_FIRST) {
        s = RbRun{ck.base, q[ck.base], q[ck.base]};
        from = 1;
    }
    rb_for_bytes(q, ck.base, from, ck.len, [&](uint32_t i, uint32_t c) {
        if (!rb_extend(s, c, R)) {
            const uint8_t g = (uint8_t)rb_round_sqrt(s.mn * s.mx);
            for (uint64_t j = s.start; j < ck.base + i; j++) out[j] = g;
            s = RbRun{ck.base + i, c, c};
        }
        return true;
    });
    if (ck.flags & RB_LAST) {
        const uint8_t g = (uint8_t)rb_round_sqrt(s.mn * s.mx);
        for (uint64_t j = s.start; j < ck.base + ck.len; j++) out[j] = g;
    }
}

// ---- R-Block output without a second full walk (round 5) ------------------
// rb_apply walked every chunk a second time from its true entry and wrote each
// closed run byte by byte (a divergent loop per close in lanes that close at
// different bytes).  Instead: the speculative pass also records the value of
// every run that closes inside the chunk at the run's start (vals, one byte
// per chunk byte); rb_true re-walks a chunk from its true entry only until it
// converges with the speculative pass, fixing the open bits and values of that
// prefix; rb_fill_word then writes every byte from the open bits (the run a
// byte belongs to starts at the last open at or before it) and the values --
// 32 bytes per thread, no walk.  Per chunk (RbInfo): the value of the run
// entering it if that run closes inside it (known), and where the run open at
// its end starts (RB_OPEN_NONE in a block's last chunk, where the final run
// closes; RB_OPEN_ENTRY if the entering run spans the chunk).  A run open at a
// chunk's end takes its value from the chunks after it (rb_chase).
constexpr uint32_t RB_OPEN_NONE = 0xffffffffu, RB_OPEN_ENTRY = 0xfffffffeu;
struct RbInfo {
    uint32_t entry_val;    // value of the run entering the chunk | known << 8
    uint32_t last_start;   // start (chunk offset) of the run open at the chunk's end
};

// round(sqrt(n)) for n <= 255 * 255 without a loop: the float root (n and
// its root are exact in a float's mantissa; v_sqrt_f32 may be off by an ulp)
// corrected in integers -- equal to rb_round_sqrt (tests/cpu_emu checks every n)
SA_HD uint32_t rb_round_sqrt_fast(uint32_t n)
{
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t g = (uint32_t)__builtin_amdgcn_sqrtf((float)n);   // (v_sqrt_f32 alone: n is no denormal)
#else
    uint32_t g = (uint32_t)__builtin_sqrtf((float)n);
#endif
    g -= g * g > n ? 1u : 0u;
    g += (g + 1) * (g + 1) <= n ? 1u : 0u;
    return n > g * g + g ? g + 1 : g;
}

// rb_extend with selects instead of branches: true if c extends the open run
// (its min / max updated), false if the run closes before c (then s holds the
// run of c alone, start left to the caller)
SA_HD bool rb_extend_sel(RbRun& s, uint32_t c, const RbTab& t)
{
    const uint32_t mn = s.mn, mx = s.mx;
    const bool bl = rb_tab_bit(t.lo, c, mx), bh = rb_tab_bit(t.hi, c, mn);
    const bool ext = c > mx ? bh : (c >= mn || bl);
    s.mn = ext && c > mn ? mn : c;
    s.mx = ext && c < mx ? mx : c;
    return ext;
}

// Speculative pass (rb_spec) recording run values: vals = the chunk's
// RB_CHUNK bytes, vals[s] = the value of the run starting at s if it closes in
// the chunk.  The speculative pass opens a run at byte 0, so no run enters.
// (Round 6: every lane of a wave walks RB_CHUNK bytes in step, 16 per load --
// past its chunk's end a lane's state stays as it is -- and each byte is one
// straight sequence of selects: the round-5 walk branched per byte on the run
// decision and looped rb_round_sqrt's 16 steps at every close, in divergent
// lanes, and k_rb_spec took most of the ONT front.)
SA_HD RbRun rb_spec_vals(const uint8_t* q, const RbChunk& ck, const RbTab& R, uint32_t* opens, uint8_t* vals,
                         RbInfo& info, uint32_t span = RB_CHUNK)
{
    RbRun s{ck.base, q[ck.base], q[ck.base]};
    uint32_t w = 1u;   // a run opens at the chunk's first byte
    const uint32_t len = ck.len;
    for (uint32_t i0 = 0; i0 < span; i0 += 16) {   // (span: the chunk length, >= len)
        uint32_t x[4];
        // (a lane past its chunk's end reads its chunk's first line again: in bounds)
        const uint8_t* p = q + ck.base + (i0 < len ? i0 : 0u);
        if (((ck.base + i0) & 15) == 0 && i0 + 16 <= len) {
            __builtin_memcpy(x, __builtin_assume_aligned(p, 16), 16);
        } else {
            for (uint32_t j = 0; j < 4; j++) x[j] = 0;
            for (uint32_t j = 0; j < 16; j++)
                if (i0 + j < len) x[j >> 2] |= (uint32_t)p[j] << (8 * (j & 3));
        }
#pragma unroll
        for (uint32_t j = 0; j < 16; j++) {
            const uint32_t i = i0 + j;
            const uint32_t c = (x[j >> 2] >> (8 * (j & 3))) & 0xffu;
            const bool live = i >= 1 && i < len;
            const uint32_t v = rb_round_sqrt_fast(s.mn * s.mx);   // (the open run's value, were it to close at i)
            RbRun t = s;
            const bool ext = rb_extend_sel(t, c, R) || !live;
            if (!ext) vals[s.start - ck.base] = (uint8_t)v;
            s.mn = live ? t.mn : s.mn;
            s.mx = live ? t.mx : s.mx;
            s.start = ext ? s.start : ck.base + i;
            w |= (ext ? 0u : 1u) << (i & 31);
            if ((i & 31) == 31) {
                opens[i >> 5] = w;
                w = 0;
            }
        }
    }
    info.entry_val = 0;
    if (ck.flags & RB_LAST) {   // the final run closes at the block's end
        vals[s.start - ck.base] = (uint8_t)rb_round_sqrt(s.mn * s.mx);
        info.last_start = RB_OPEN_NONE;
    } else {
        info.last_start = (uint32_t)(s.start - ck.base);
    }
    return s;
}

// The true pass over chunk ck from its true entry run s (not the block's first
// chunk: there the speculative pass is the true one), until it closes a run
// where the speculative pass opened one -- from there both agree -- or to the
// chunk's end.  Rewrites the open bits of that prefix, records the values of
// the runs closing in it (the entering run's in info.entry_val) and, without
// convergence, where the run open at the chunk's end starts.
SA_HD void rb_true(const uint8_t* q, const RbChunk& ck, RbRun s, const RbTab& R, uint32_t* opens, uint8_t* vals,
                   RbInfo& info)
{
    uint32_t w = 0;            // true open bits of the current word
    uint32_t conv = ck.len;    // first byte from which both passes agree
    bool entry_open = true;    // the run entering the chunk has not closed
    info.entry_val = 0;
    rb_for_bytes(q, ck.base, 0, ck.len, [&](uint32_t i, uint32_t c) {
        if (!rb_extend(s, c, R)) {
            const uint8_t g = (uint8_t)rb_round_sqrt(s.mn * s.mx);
            if (entry_open) {
                info.entry_val = (uint32_t)g | 0x100u;
                entry_open = false;
            } else {
                vals[s.start - ck.base] = g;
            }
            if ((opens[i >> 5] >> (i & 31)) & 1u) {   // converged at i
                conv = i;
                return false;
            }
            s = RbRun{ck.base + i, c, c};
            w |= 1u << (i & 31);
        }
        if ((i & 31) == 31) { opens[i >> 5] = w; w = 0; }
        return true;
    });
    if (conv < ck.len) {   // the word holding conv: true bits below it, the speculative ones from it
        const uint32_t k = conv >> 5, lo = (conv & 31) ? (1u << (conv & 31)) - 1u : 0u;
        opens[k] = (w & lo) | (opens[k] & ~lo);
        return;            // (info.last_start: the speculative pass's)
    }
    if ((ck.len & 31) != 0) opens[(ck.len - 1) >> 5] = w;
    const uint8_t g = (uint8_t)rb_round_sqrt(s.mn * s.mx);
    if (ck.flags & RB_LAST) {   // the final run closes at the block's end
        if (entry_open) info.entry_val = (uint32_t)g | 0x100u;
        else vals[s.start - ck.base] = g;
        info.last_start = RB_OPEN_NONE;
    } else {
        info.last_start = entry_open ? RB_OPEN_ENTRY : (uint32_t)(s.start - ck.base);
    }
}

// The value of the run open at the end of chunk c: the run entering c + 1,
// which closes in c + 1 or, spanning it, later (a block's last chunk closes it).
SA_HD uint32_t rb_chase(const RbInfo* info, const RbChunk* ck, uint32_t c)
{
    if (ck[c].flags & RB_LAST) return 0;   // (no run is open at a block's end)
    for (uint32_t k = c + 1;; k++) {
        if (info[k].entry_val & 0x100u) return info[k].entry_val & 0xffu;
        if (ck[k].flags & RB_LAST) return 0;   // (unreachable: the last chunk closes it)
    }
}

// Bytes [32 t, 32 t + 32) of chunk ck into out, t < RB_WORDS: prev = the last
// open before the word (chunk offset, or -1: none), entry / tail = the values
// of the entering run and of the run open at the chunk's end.
SA_HD void rb_fill_word(uint8_t* out, const RbChunk& ck, uint32_t t, uint32_t word, int32_t prev, const uint8_t* vals,
                        const RbInfo& info, uint32_t entry, uint32_t tail)
{
    uint32_t o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int32_t cur = prev;
    for (uint32_t i = 0; i < 32; i++) {
        if ((word >> i) & 1u) cur = (int32_t)(32 * t + i);
        uint32_t v;
        if (cur < 0) v = info.last_start == RB_OPEN_ENTRY ? tail : entry;
        else if ((uint32_t)cur == info.last_start) v = tail;
        else v = vals[cur];
        o[i >> 2] |= v << (8 * (i & 3));
    }
    const uint32_t at = 32 * t;
    if (at + 32 <= ck.len) {
        __builtin_memcpy(out + ck.base + at, o, 32);
    } else {
        for (uint32_t i = 0; at + i < ck.len; i++) out[ck.base + at + i] = (uint8_t)(o[i >> 2] >> (8 * (i & 3)));
    }
}

// Writes every header, MD5 and the ID-bin payload of block b into o, and lists
// the coder payloads still to copy (destination offset, coder task, length).
// Returns the block's total length.
SA_HD uint32_t assemble_plan(const BatchView& bv, uint32_t b, const AsmBlock& ab, const uint32_t* out_len,
                             const uint32_t* digests, uint8_t* o, uint32_t* seg_dst, uint32_t* seg_src_task,
                             uint32_t* seg_len, uint32_t& nseg)
{
    const DevBlock& blk = bv.blocks[b];
    uint32_t p = 5;   // 0x81 + size4
    uint32_t ns = 0;
    // compressCount@0x422a00: setID(id), size byte 0x84, u32 LE
    auto count = [&](uint32_t id, uint32_t v) {
        p += put_id(o + p, id);
        o[p++] = 0x84;
        put_u32le(o + p, v);
        p += 4;
    };
    // a stream's encap: setID(id), size4, the coded bytes
    auto stream = [&](uint32_t id, int st) {
        const uint32_t L = out_len[ab.task[st]];
        p += put_id(o + p, id);
        put_size4(o + p, L);
        p += 4;
        seg_dst[ns] = p; seg_src_task[ns] = ab.task[st]; seg_len[ns] = L; ns++; p += L;
    };
    count(1, blk.nreads);
    const int md5 = bv.md5;
    stream(4, ST_LEN);
    if (bv.aligned) {   // doAlignEncode@0x42d4c0: order count and order bytes
        count(0x1b, blk.order_count);
        stream(8, ST_ORD);
    }
    // ID (compressID@0x4247c0)
    {
        p += put_id(o + p, 5);
        uint32_t szp = p; p += 4;
        uint32_t h = 0;
        if (md5) {
            for (int k = 0; k < 4; k++) put_u32le(o + p + 4 * k, digests[(size_t)ab.md5_task[0] * 4 + k]);
            p += 16; h = 16;
        }
        uint32_t L;
        if (bv.bin_mode) {   // IDProcess::encodeIDS@0x430040: u16 len + first ID
            const uint32_t l0 = blk.nreads ? bv.name_len[blk.read0] : 0;
            o[p] = (uint8_t)l0; o[p + 1] = (uint8_t)(l0 >> 8);
            const uint8_t* nm = bv.names + blk.name_base;
            for (uint32_t k = 0; k < l0; k++) o[p + 2 + k] = nm[k];
            L = 2 + l0; p += L;
        } else {
            L = out_len[ab.task[ST_NAME]];
            seg_dst[ns] = p; seg_src_task[ns] = ab.task[ST_NAME]; seg_len[ns] = L; ns++; p += L;
        }
        put_size4(o + szp, h + L);
    }
    // quality
    {
        p += put_id(o + p, 7);
        uint32_t szp = p; p += 4;
        uint32_t h = 0;
        if (md5 && !bv.lossy) {   // compressQual@0x426eca: no quality MD5 with -l
            for (int k = 0; k < 4; k++) put_u32le(o + p + 4 * k, digests[(size_t)ab.md5_task[2] * 4 + k]);
            p += 16; h = 16;
        }
        uint32_t L = out_len[ab.task[ST_QUAL]];
        seg_dst[ns] = p; seg_src_task[ns] = ab.task[ST_QUAL]; seg_len[ns] = L; ns++; p += L;
        put_size4(o + szp, h + L);
    }
    if (bv.aligned) {   // the alignment streams (@0x42d5bd-0x42d6bb, 0x42d830)
        count(0x11, blk.align_count);
        count(0x12, blk.scount[ST_POS]);
        count(0x13, blk.scount[ST_CIGL]);
        count(0x14, blk.scount[ST_CIGV]);
        if (bv.paired) {
            count(0x15, blk.insert_bits);
            count(0x16, blk.scount[ST_PEREL]);
            stream(9, ST_PEREL);
        }
        stream(0xb, ST_POS);
        stream(0xf, ST_MIS);
        stream(0xa, ST_REV);
        stream(0xc, ST_CIGL);
        stream(0xd, ST_CIGV);
    }
    // degenerate-base streams: encap omitted when its value count is 0
    const uint32_t ids[5] = {23, 14, 24, 25, 26};
    for (int k = 0; k < 5; k++) {
        const int st = ST_TIP + k;
        const uint32_t cnt = blk.vcount[st];
        if (!cnt) continue;
        uint32_t L = out_len[ab.task[st]];
        p += put_id(o + p, ids[k]);
        put_size4(o + p, L + 4); p += 4;
        put_u32le(o + p, cnt); p += 4;
        seg_dst[ns] = p; seg_src_task[ns] = ab.task[st]; seg_len[ns] = L; ns++; p += L;
    }
    // sequence
    {
        p += put_id(o + p, 6);
        uint32_t szp = p; p += 4;
        uint32_t h = 0;
        if (md5) {
            for (int k = 0; k < 4; k++) put_u32le(o + p + 4 * k, digests[(size_t)ab.md5_task[1] * 4 + k]);
            p += 16; h = 16;
        }
        uint32_t L = out_len[ab.task[ST_SEQ]];
        seg_dst[ns] = p; seg_src_task[ns] = ab.task[ST_SEQ]; seg_len[ns] = L; ns++; p += L;
        put_size4(o + szp, h + L);
    }
    o[0] = 0x81;
    put_size4(o + 1, p - 5);
    nseg = ns;
    return p;
}

}  // namespace sa
