// sa_common.h -- data layout and per-read symbol extraction shared by the HIP
// kernels (sa_kernels.hip) and the CPU decomposition check (tests/cpu_emu).
//
// The reference encodes each stream of a block with adaptive models and one
// serial range coder (EncapFqzComp::doFqzEncode@0x42d2d0).  On MI355X the block
// is decomposed into
//   1. per-read symbol extraction:  every coded symbol becomes (model id, symbol,
//      position in its stream), computed independently per read;
//   2. a stable per-block sort of the symbols by model id;
//   3. model replay: each model's symbols are replayed in stream order by one
//      lane, producing (cum, freq, 2^64/tot) per symbol;
//   4. one range-coder lane per (block, stream).
// This header holds step 1 plus the layout constants.  All functions are
// plain integer code that compiles for gfx950 and for the host test harness.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SA_HD __host__ __device__ inline
#else
#define SA_HD inline
#endif

namespace sa {

// ---- stream ids in block output order (doFqzEncode@0x42d2d0) -------------
enum Stream : int {
    ST_LEN = 0,    // encap 4   compressLen_short@0x423f50
    ST_NAME = 1,   // encap 5   compressName@0x4241a0 (tokenizer mode)
    ST_QUAL = 2,   // encap 7   compressQual@0x426e80
    ST_TIP = 3,    // encap 23  compressDegeTip@0x424dd0
    ST_CH = 4,     // encap 14  compressDegeCh@0x425080
    ST_MAXQ = 5,   // encap 24  compressDegeMaxQual@0x425310
    ST_NCNT = 6,   // encap 25  compressNDegeCnt@0x42d010
    ST_NPOS = 7,   // encap 26  compressNDegePos@0x42d170
    ST_SEQ = 8,    // encap 6   compressSeq@0x4248a0 (own symbol space)
    // reference (HASH index) path only, doAlignEncode@0x42d4c0:
    ST_ORD = 9,    // encap 8   compressOrder@0x424b70
    ST_PEREL = 10, // encap 9   compressPERelation@0x422be0 (PE)
    ST_POS = 11,   // encap 0xb compressAlignInfo_Pos@0x425d70
    ST_MIS = 12,   // encap 0xf compressAlignInfo_Mis@0x425ff0
    ST_REV = 13,   // encap 0xa compressAlignInfo_Rev@0x426480
    ST_CIGL = 14,  // encap 0xc compressAlignInfo_CigaL@0x426700
    ST_CIGV = 15,  // encap 0xd compressAlignInfo_CigaV@0x426980
    NSTREAM = 16,
    NAUX = 8,      // AUX streams with a per-read count column (ST_LEN .. ST_NPOS)
    NALN = 7       // alignment streams (ST_ORD .. ST_CIGV)
};

// ---- per-read count columns of the alignment streams (reference path) -------
enum ACol : int {
    A_ORD = 0,    // 1 per read with an order byte (block reads < order count)
    A_PEREL = 1,  // 1 per PE pair with both mates aligned (on mate 1)
    A_POS = 2,    // position bits
    A_MIS = 3,    // 1 per aligned read
    A_REV = 4,    // 1 per aligned read
    A_CIGL = 5,   // mismatch-offset bits
    A_CIGV = 6,   // mismatches
    NACOL = 7
};
static_assert(ST_ORD + A_CIGV == ST_CIGV, "alignment column k is stream ST_ORD + k");

// ---- per-read count columns (exclusive-scanned per block) -----------------
enum Col : int {
    C_SEQ = 0,    // valid (ACGT) bases               -> SEQ symbols
    C_LEN = 1,    // 1 or 3                          -> LEN symbols
    C_NAME = 2,   // 3 + mid chars (0 in bin mode)   -> NAME symbols
    C_QUAL = 3,   // non-trailing-# quals + terminator -> QUAL symbols
    C_TIP = 4,    // 1
    C_CH = 5,     // non-ACGT bases
    C_MAXQ = 6,   // 1 if the read has non-ACGT bases
    C_NCNT = 7,   // kModel symbols of the exception count
    C_NPOS = 8,   // kModel symbols of all gaps
    C_NPOSV = 9,  // number of gap values (exceptions)
    NCOL = 10
};

// ---- model ids of the shared AUX symbol space ------------------------------
// Every adaptive SIMPLE_MODEL<N> instance of the non-sequence streams gets a
// global id; the stable sort groups symbols by id and one lane replays each.
constexpr uint32_t M_LEN_SAME = 0;        // SIMPLE_MODEL<2>   @+0x1048
constexpr uint32_t M_LEN_LO = 1;          // SIMPLE_MODEL<256> @+0x8
constexpr uint32_t M_LEN_HI = 2;          // SIMPLE_MODEL<256> @+0x418
constexpr uint32_t M_TIP = 3;             // SIMPLE_MODEL<2>  (stack, per block)
constexpr uint32_t M_CH = 4;              // SIMPLE_MODEL<11>
constexpr uint32_t M_MAXQ = 5;            // SIMPLE_MODEL<95>
constexpr uint32_t M_KBITS = 6;           // kModel SIMPLE_MODEL<64> @+0x15c0
constexpr uint32_t M_KBIT0 = 7;           // 64 x SIMPLE_MODEL<2> (vector @+0x15a8)
constexpr uint32_t M_LEN_B2 = 71;         // SIMPLE_MODEL<256> @+0x828 (compressLen_long@0x423710)
constexpr uint32_t M_LEN_B3 = 72;         // SIMPLE_MODEL<256> @+0xc38
// one model per alignment stream (each compressX keeps its model on the stack)
constexpr uint32_t M_ORD = 73;            // SIMPLE_MODEL<5>  compressOrder@0x424b70
constexpr uint32_t M_PEREL = 74;          // SIMPLE_MODEL<4>  compressPERelation@0x422be0
constexpr uint32_t M_POS = 75;            // SIMPLE_MODEL<2>  compressAlignInfo_Pos@0x425d70
constexpr uint32_t M_MIS8 = 76;           // SIMPLE_MODEL<8>  compressAlignInfo_Mis@0x425ff0 (maxmis 1..7)
constexpr uint32_t M_REV = 77;            // SIMPLE_MODEL<2>  compressAlignInfo_Rev@0x426480
constexpr uint32_t M_CIGL = 78;           // SIMPLE_MODEL<2>  compressAlignInfo_CigaL@0x426700
constexpr uint32_t M_CIGV = 79;           // SIMPLE_MODEL<4>  compressAlignInfo_CigaV@0x426980
constexpr uint32_t M_MIS9 = 80;           // SIMPLE_MODEL<9>  compressAlignInfo_Mis (maxmis 8)
constexpr uint32_t M_NAME_PRE = 128;      // 256 x SIMPLE_MODEL<256> @+0x1068
constexpr uint32_t M_NAME_SUF = 384;      // 256 x SIMPLE_MODEL<256> @+0x1070
constexpr uint32_t M_NAME_LEN = 640;      // 256 x SIMPLE_MODEL<256> @+0x1078
constexpr uint32_t M_NAME_MID = 1024;     // 8192 x SIMPLE_MODEL<128> @+0x1080
constexpr uint32_t M_QUAL = 16384;        // 65536 (or 2^20) x SIMPLE_MODEL<95> @+0x1500

SA_HD uint32_t model_nsym(uint32_t id)
{
    if (id >= M_QUAL) return 95;
    if (id >= M_NAME_MID) return 128;
    if (id >= M_NAME_PRE) return 256;
    if (id == M_LEN_B2 || id == M_LEN_B3) return 256;
    switch (id) {
    case M_ORD: return 5;
    case M_PEREL: return 4;
    case M_MIS8: return 8;
    case M_CIGV: return 4;
    case M_MIS9: return 9;
    default: break;
    }
    if (id >= M_KBIT0) return 2;   // (also M_POS, M_REV, M_CIGL)
    switch (id) {
    case M_LEN_SAME: return 2;
    case M_LEN_LO: return 256;
    case M_LEN_HI: return 256;
    case M_TIP: return 2;
    case M_CH: return 11;
    case M_MAXQ: return 95;
    default: return 64;   // M_KBITS
    }
}

// ---- error bits reported by the device --------------------------------------
enum Err : uint32_t {
    E_NONASCII = 1u,     // sequence byte >= 0x80 (reference behaviour undefined)
    E_QUALRANGE = 2u,    // quality byte outside '!'..'~' (outside SIMPLE_MODEL<95>)
    E_NAME = 4u,         // name > 255 bytes or out-of-range model index
    E_LONGREAD = 8u,     // (unused: reads > 65535 bp take compressLen_long@0x423710)
    E_OVERFLOW = 16u,    // a range coder output overflowed its buffer
    E_CODER = 32u,       // cum + freq > tot (reference: abort())
};

// seq_val_table@0x44b800: A/a C/c G/g T/t -> 0..3, the IUPAC letters M R Y K
// S W H B V D (either case) -> 5..14, every other byte -> 4.  Branch-free (a
// switch became a compare-and-branch tree per byte in the per-read kernels):
// only bytes 0x40..0x7f can be letters; `(c | 0x20) - 0x60` indexes a table
// of 32 nibbles held in two 64-bit constants.
SA_HD uint32_t base_code(uint8_t c)
{
    constexpr uint64_t LO = 0x4454844b244e1c04ull;   // nibbles of '`' a b c ... o
    constexpr uint64_t HI = 0x44444474ad439644ull;   // p q r s ... z { | } ~ DEL
    const uint32_t idx = ((uint32_t)c | 0x20u) - 0x60u;
    const uint64_t v = (idx & 16u) ? HI : LO;
    const uint32_t code = (uint32_t)(v >> (4u * (idx & 15u))) & 15u;
    return ((uint32_t)c & 0xc0u) == 0x40u ? code : 4u;
}
// `c | 0x20` folds case but also maps some non-letters onto letters
// (e.g. 'A'-0x20 = '!' stays '!'); only letters can reach the cases above
// because `c|0x20` equals a lowercase letter iff c is that letter in either case.

SA_HD int nbits_u32(uint32_t v)   // bits of v (0 for 0)
{
    return v ? 32 - __builtin_clz(v) : 0;
}

// ---- per-read statistics (pass 1) ------------------------------------------
struct SeqStat {
    uint32_t valid;      // ACGT bases
    uint32_t nch;        // non-ACGT bases
    uint32_t maxq;       // max quality over non-ACGT bases (DegeInfoProcess@0x433a10)
    uint32_t exc;        // ACGT bases with qual <= maxq
    uint32_t npos_syms;  // kModel symbols of the gap values
    uint32_t err;
};

SA_HD SeqStat seq_stat(const uint8_t* s, const uint8_t* q, uint32_t len)
{
    SeqStat st{0, 0, 0, 0, 0, 0};
    uint32_t maxq = 0;
    for (uint32_t i = 0; i < len; i++) {
        uint8_t c = s[i];
        if (c >= 0x80) st.err |= E_NONASCII;
        if (base_code(c) > 3) {
            st.nch++;
            int qi = (int)(int8_t)q[i];
            if (qi > (int)maxq) maxq = (uint32_t)qi & 0xff;
        } else {
            st.valid++;
        }
    }
    st.maxq = maxq;
    if (st.nch) {
        uint32_t gap = 0;
        for (uint32_t i = 0; i < len; i++) {
            if ((int)maxq < (int)(int8_t)q[i]) continue;
            if (base_code(s[i]) > 3) {
                gap++;
            } else {
                st.exc++;
                st.npos_syms += 1 + (uint32_t)nbits_u32(gap);
                gap = 0;
            }
        }
    }
    return st;
}

// quality: number of coded symbols (encode_qual@0x422180 strips trailing '#'
// and appends symbol 94 when it stripped any)
SA_HD uint32_t qual_nonhash(const uint8_t* q, uint32_t len)
{
    uint32_t n = len;
    while (n > 0 && q[n - 1] == '#') n--;
    return n;
}

// qual model index transition (encode_qual@0x422474..0x422505)
struct QualCtx {
    int q1, q2, delta;
};
SA_HD uint32_t qual_next_ctx(QualCtx& c, int sym, uint32_t i, int qlevel)
{
    uint32_t ctx = ((uint32_t)((c.q1 > c.q2 ? c.q1 : c.q2) << 6) + (uint32_t)sym) & 0xfffu;
    if (qlevel > 1) {
        ctx += (c.q1 == c.q2) ? 0x1000u : 0u;
        c.delta += (c.q1 > sym) ? (c.q1 - sym) : 0;
        ctx += (uint32_t)(((c.delta <= 56 ? c.delta : 56) & 0xf8) << 10);
        if (qlevel > 2) ctx += (i <= 0x6f) ? (uint32_t)(((i + 15) & 0x78) << 13) : 0xf0000u;
    }
    c.q2 = c.q1;
    c.q1 = sym;
    return ctx;
}

// ---- name tokenizer (encode_name@0x421070) ----------------------------------
// prefix / suffix match lengths of `name` against the previous name.
SA_HD void name_prefix_suffix(const uint8_t* name, int len, const uint8_t* prev, int ll,
                              int& p, int& s)
{
    p = 0;
    s = 0;
    if (len <= 0 || ll <= 0) {
        if (len - s - p < 0) s = len - p;
        return;
    }
    if (name[0] == prev[0]) {
        int i = 1;
        while (i < len && i < ll && name[i] == prev[i]) i++;
        p = i;
    }
    if (name[len - 1] == prev[ll - 1]) {
        int i = len - 1, j = ll - 1;
        for (;;) {
            i--;
            j--;
            if (j < 0 || i < 0) break;
            if (name[i] != prev[j]) break;
        }
        s = len - 1 - i;
        if (len - s - p < 0) s = len - p;
    }
}

// Middle-character loop of encode_name@0x421070 (0x421578..0x42173f).
// `last(j)` returns byte j of the reference's 1024-byte last-name buffer as it
// stands before this name (j == -1 models the byte in front of the buffer,
// which is the top byte of a heap pointer: 0).  emit(ctx, sym) is called per
// middle character.  Returns false on an out-of-range model index.
template <class Last, class Emit>
SA_HD bool name_mid(const uint8_t* name, int len, int p, int s, Last last, Emit emit)
{
    int len2 = len - s;
    int lc = p != 0;
    int k = 0, j = p;
    for (int i = p; i < len2; i++) {
        if (j > 1022) return false;
        int ctx = (k * 64 + lc + 2 * ((int)(int8_t)last(j) - 32)) % 8192;
        if (ctx < 0) return false;
        emit((uint32_t)ctx, (uint32_t)(name[i] & 0x7f));
        uint8_t c = name[i];
        bool reset = false;
        if (c == ' ') {
            if (last(j) != ' ' && last(j + 1) != ':') j = j + 1;
            k = (k + 3) & ~3;
            if (j < 0) reset = true;
        } else {
            uint8_t d = last(j);
            if (d == ' ') {
                j--;
                d = last(j);
            }
            if (c == ':') {
                j += (d != ':');
                k = (k + 3) & ~3;
                if (j < 0) reset = true;
            } else {
                j -= (d == ':');
                if (j < 0) reset = true;
            }
        }
        if (reset) {
            j = 0;
            lc = 0;
            k++;
        } else {
            lc = (c == last(j));
            j++;
            k++;
        }
    }
    return true;
}

// ---- range coder records ----------------------------------------------------
// Coder record of one coded symbol: tf = tot | freq << 16 (AUX; cum in its own
// array) or tot | cum << 8 | freq << 16 (SEQ, tot <= 253).  The readers derive
// the reciprocal m = ceil(2^32 / tot) themselves (recip32z, off the range
// chain): q0 = mulhi(range, m) is q or q + 1 and q0 * tot never wraps
// (DESIGN.md "Coder"), so one borrow corrects it.  4 bytes per symbol.
struct PRec {
    uint32_t tf;
};

// Coder segment: symbols per range checkpoint (DESIGN.md "Coder").
constexpr uint32_t SEG_SYMS = 64;

// Affine effect of a run of symbols on the coder's low word:
// low -> (low << s) + B  (s in bits, saturated at 64 meaning "all shifted out"),
// plus the number of bytes the run emits.
struct LowMap {
    uint64_t B;
    uint32_t s;
    uint32_t nbytes;
};

// AUX sort keys carry the symbol in the low 8 bits (not sorted on):
// key = model << 8 | symbol; the radix sort orders by bits [8, 8 + model bits).
constexpr uint32_t AUX_SYM_BITS = 8;

}  // namespace sa
