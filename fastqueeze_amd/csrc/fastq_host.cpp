// fastq_host.cpp -- host-side block plumbing of the drop-in encoder (C++):
// FASTQ block cutting and parsing and the ID template analysis, mirroring the
// reference's reader thread and pre-processing so the GPU receives exactly the
// blocks SeqArc-1.6 would encode.
#include <emmintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <future>
#include <string>
#include <vector>

#include "../../include/seqarc_amd.h"

namespace {

// getFirstLine@0x431eb0 keeps the first line of file 1 including its '\n'.
size_t first_line_len(const uint8_t* t, uint64_t len)
{
    const void* nl = std::memchr(t, '\n', (size_t)len);
    return nl ? (size_t)((const uint8_t*)nl - t) + 1 : (size_t)len;
}

// getEndPos@0x4320c0: walk back from n to the last "\n@" whose header matches
// more than five consecutive bytes of the file's first line.  The consecutive
// match counter is carried from one candidate to the next, as in the binary.
int64_t end_pos(const uint8_t* data, uint64_t avail, int64_t n, const uint8_t* first, size_t flen)
{
    if (n <= 0 || flen == 0) return 0;
    int run = 0;
    for (int64_t pos = n; pos > 0; --pos) {
        if ((uint64_t)pos + 1 >= avail || data[pos] != '\n' || data[pos + 1] != '@') continue;
        for (size_t k = 0; k < flen; k++) {
            const uint64_t at = (uint64_t)pos + 1 + k;
            if (at < avail && data[at] == first[k]) {
                if (++run > 5) return pos;
            } else {
                run = 0;
            }
        }
    }
    return 0;
}

void newline_positions(const uint8_t* t, uint64_t len, std::vector<uint64_t>& out)
{
    out.clear();
    const uint8_t* p = t;
    const uint8_t* e = t + len;
    while (p < e) {
        const void* nl = std::memchr(p, '\n', (size_t)(e - p));
        if (!nl) break;
        out.push_back((uint64_t)((const uint8_t*)nl - t));
        p = (const uint8_t*)nl + 1;
    }
}

// Newlines in t[0, len): 64 bytes per step, compare + movemask + popcount.
uint64_t count_nl(const uint8_t* t, uint64_t len)
{
    uint64_t n = 0, i = 0;
    const __m128i nl = _mm_set1_epi8('\n');
    for (; i + 64 <= len; i += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i*)(t + i));
        const __m128i b = _mm_loadu_si128((const __m128i*)(t + i + 16));
        const __m128i c = _mm_loadu_si128((const __m128i*)(t + i + 32));
        const __m128i d = _mm_loadu_si128((const __m128i*)(t + i + 48));
        const uint64_t m = (uint64_t)(uint16_t)_mm_movemask_epi8(_mm_cmpeq_epi8(a, nl)) |
                           (uint64_t)(uint16_t)_mm_movemask_epi8(_mm_cmpeq_epi8(b, nl)) << 16 |
                           (uint64_t)(uint16_t)_mm_movemask_epi8(_mm_cmpeq_epi8(c, nl)) << 32 |
                           (uint64_t)(uint16_t)_mm_movemask_epi8(_mm_cmpeq_epi8(d, nl)) << 48;
        n += (uint64_t)__builtin_popcountll(m);
    }
    for (; i < len; i++) n += t[i] == '\n';
    return n;
}

// count_nl over `parts` concurrent slices
uint64_t count_nl_par(const uint8_t* t, uint64_t len, int parts)
{
    if (parts <= 1 || len < (4u << 20)) return count_nl(t, len);
    const uint64_t sl = (len + (uint64_t)parts - 1) / (uint64_t)parts;
    std::vector<std::future<uint64_t>> fs;
    for (int i = 1; i < parts; i++) {
        const uint64_t a = std::min(len, (uint64_t)i * sl), b = std::min(len, a + sl);
        fs.push_back(std::async(std::launch::async, [t, a, b]() { return count_nl(t + a, b - a); }));
    }
    uint64_t n = count_nl(t, std::min(len, sl));
    for (auto& f : fs) n += f.get();
    return n;
}

// Position of the newline `back` places before the last one in t[0, len)
// (back = 0: the last newline), or -1.
int64_t nl_from_end(const uint8_t* t, uint64_t len, uint64_t back)
{
    uint64_t e = len;
    for (;;) {
        const void* p = memrchr(t, '\n', (size_t)e);
        if (!p) return -1;
        const uint64_t at = (uint64_t)((const uint8_t*)p - t);
        if (back == 0) return (int64_t)at;
        --back;
        e = at;
    }
}

}  // namespace

extern "C" {

int64_t sa_cut_se(const uint8_t* text, uint64_t len, uint64_t bs, uint64_t* ends, uint64_t max_blocks)
{
    if (!text || !ends || bs == 0) return -1;
    const size_t flen = first_line_len(text, len);
    uint64_t off = 0, nb = 0;
    while (off < len) {
        if (nb >= max_blocks) return -1;
        const uint64_t avail = len - off;
        if (avail < bs) {   // the short read of the last buffer of the file
            ends[nb++] = len;
            break;
        }
        const int64_t e = end_pos(text + off, bs, (int64_t)(bs - flen), text, flen);
        if (e <= 0) return -1;
        off += (uint64_t)e + 1;
        ends[nb++] = off;
    }
    return (int64_t)nb;
}

int64_t sa_cut_pe(const uint8_t* t1, uint64_t len1, const uint8_t* t2, uint64_t len2, uint64_t bs,
                  uint64_t* e1, uint64_t* e2, uint64_t max_blocks)
{
    if (!t1 || !t2 || !e1 || !e2 || bs < 2) return -1;
    const uint64_t half = (uint64_t)((uint32_t)bs >> 1);
    const size_t flen = first_line_len(t1, len1);
    uint64_t o1 = 0, o2 = 0, nb = 0;
    std::vector<uint64_t> nl1, nl2;
    for (;;) {
        if (nb >= max_blocks) return -1;
        const uint64_t a1 = std::min<uint64_t>(len1 - o1, half), a2 = std::min<uint64_t>(len2 - o2, half);
        if (a1 < half && a2 < half) {   // both reads short: last block takes the rest
            e1[nb] = len1;
            e2[nb] = len2;
            return (int64_t)(nb + 1);
        }
        newline_positions(t1 + o1, a1, nl1);
        newline_positions(t2 + o2, a2, nl2);
        const size_t k = std::min(nl1.size(), nl2.size());
        if (k < 2) return -1;
        int64_t j = (int64_t)k - 2;
        const int64_t pos = end_pos(t1 + o1, a1, (int64_t)nl1[(size_t)j], t1, flen);
        while (j >= 0 && (int64_t)nl1[(size_t)j] != pos) --j;
        if (j < 0) return -1;   // the reference spins forever here (defect i)
        o1 += nl1[(size_t)j] + 1;
        o2 += nl2[(size_t)j] + 1;
        e1[nb] = o1;
        e2[nb] = o2;
        ++nb;
        if (o1 >= len1 && o2 >= len2) return (int64_t)nb;
    }
}

// Streaming forms of the two cuts: the next block of a window of the input.
int64_t sa_cut_next_se(const uint8_t* win, uint64_t avail, int eof, uint64_t bs, const uint8_t* first,
                       uint64_t flen)
{
    if (!win || bs == 0 || !first || flen == 0) return -1;
    if (avail < bs) return eof ? (int64_t)avail : -1;   // the short read of the file's last buffer
    const int64_t e = end_pos(win, bs, (int64_t)(bs - flen), first, (size_t)flen);
    return e <= 0 ? -1 : e + 1;
}

int sa_cut_next_pe(const uint8_t* w1, uint64_t avail1, int eof1, const uint8_t* w2, uint64_t avail2, int eof2,
                   uint64_t bs, const uint8_t* first, uint64_t flen, uint64_t* end1, uint64_t* end2)
{
    if (!w1 || !w2 || !end1 || !end2 || bs < 2 || !first || flen == 0) return -1;
    const uint64_t half = (uint64_t)((uint32_t)bs >> 1);
    if ((avail1 < half && !eof1) || (avail2 < half && !eof2)) return -1;   // the caller reads more first
    const uint64_t a1 = std::min<uint64_t>(avail1, half), a2 = std::min<uint64_t>(avail2, half);
    if (a1 < half && a2 < half) {   // both reads short: the last block takes the rest
        *end1 = avail1;
        *end2 = avail2;
        return 0;
    }
    // The same cut as sa_cut_pe (cultPEbuf@0x432180 over the newline arrays of
    // both windows) without materialising the arrays: the newline counts of
    // both windows (counted concurrently), then short walks back from their ends.
    std::future<uint64_t> f2 = std::async(std::launch::async, [&]() { return count_nl_par(w2, a2, 2); });
    const uint64_t k1 = count_nl_par(w1, a1, 2);
    const uint64_t k2 = f2.get();
    return sa_cut_next_pe_nl(w1, avail1, eof1, k1, w2, avail2, eof2, k2, bs, first, flen, end1, end2);
}

// sa_cut_next_pe with the windows' newline counts given (k1 / k2: newlines in
// the first min(avail, bs / 2) bytes of each window), e.g. counted by the
// threads that read the input
int sa_cut_next_pe_nl(const uint8_t* w1, uint64_t avail1, int eof1, uint64_t k1, const uint8_t* w2, uint64_t avail2,
                      int eof2, uint64_t k2, uint64_t bs, const uint8_t* first, uint64_t flen, uint64_t* end1,
                      uint64_t* end2)
{
    if (!w1 || !w2 || !end1 || !end2 || bs < 2 || !first || flen == 0) return -1;
    const uint64_t half = (uint64_t)((uint32_t)bs >> 1);
    if ((avail1 < half && !eof1) || (avail2 < half && !eof2)) return -1;
    const uint64_t a1 = std::min<uint64_t>(avail1, half), a2 = std::min<uint64_t>(avail2, half);
    if (a1 < half && a2 < half) {
        *end1 = avail1;
        *end2 = avail2;
        return 0;
    }
    const uint64_t k = std::min(k1, k2);
    if (k < 2) return -1;
    int64_t j = (int64_t)k - 2;
    const int64_t pj = nl_from_end(w1, a1, k1 - 1 - (uint64_t)j);
    if (pj < 0) return -1;
    const int64_t pos = end_pos(w1, a1, pj, first, (size_t)flen);
    // index of the newline at pos: walk back from newline j
    int64_t at = pj;
    while (j >= 0 && at != pos) {
        if (at < pos) return -1;   // pos is not a newline (the reference spins forever, SURVEY 5 i)
        --j;
        if (j < 0) break;
        const void* p = memrchr(w1, '\n', (size_t)at);
        if (!p) return -1;
        at = (int64_t)((const uint8_t*)p - w1);
    }
    if (j < 0) return -1;
    const int64_t q = nl_from_end(w2, a2, k2 - 1 - (uint64_t)j);
    if (q < 0) return -1;
    *end1 = (uint64_t)pos + 1;
    *end2 = (uint64_t)q + 1;
    return 0;
}

int64_t sa_parse_se(const uint8_t* t, uint64_t len, uint8_t* names, uint16_t* nlens, uint8_t* seq,
                    int32_t* slens, uint8_t* qual)
{
    // getBlockRead@0x411b60: state machine over '\n'; the header starts after
    // '@' (skipped by position), the quality copy uses the sequence length.
    uint64_t start = 1;
    int state = 0;
    int64_t n = 0;
    int32_t seqlen = 0;
    uint8_t *pn = names, *ps = seq, *pq = qual;
    for (uint64_t i = 0; i < len; i++) {
        if (t[i] != '\n') continue;
        switch (state) {
        case 0: {
            const uint64_t l = i - start;
            if (l > 0xffff) return -1;
            std::memcpy(pn, t + start, (size_t)l);
            pn += l;
            nlens[n] = (uint16_t)l;
            start = i + 1;
            state = 1;
            break;
        }
        case 1:
            seqlen = (int32_t)(i - start);
            std::memcpy(ps, t + start, (size_t)seqlen);
            ps += seqlen;
            slens[n] = seqlen;
            start = i + 1;
            state = 2;
            break;
        case 2:
            start = i + 1;
            state = 3;
            break;
        default:
            if (start + (uint64_t)seqlen > len) return -1;
            std::memcpy(pq, t + start, (size_t)seqlen);
            pq += seqlen;
            ++n;
            start = i + 2;
            state = 0;
            break;
        }
    }
    return state == 0 ? n : -1;
}

int64_t sa_parse_pe(const uint8_t* t1, uint64_t len1, const uint8_t* t2, uint64_t len2, uint8_t* names,
                    uint16_t* nlens, uint8_t* seq, int32_t* slens, uint8_t* qual)
{
    // getBlockReadPE@0x412920: records located through the newline arrays of
    // both files; reads interleaved r1, r2; the quality copy uses its own line.
    std::vector<uint64_t> a, b;
    newline_positions(t1, len1, a);
    newline_positions(t2, len2, b);
    const size_t k = std::min(a.size(), b.size());
    if (k % 4) return -1;
    uint64_t s1 = 1, s2 = 1;
    int64_t n = 0;
    uint8_t *pn = names, *ps = seq, *pq = qual;
    for (size_t o = 0; o < k; o += 4) {
        for (int mate = 0; mate < 2; mate++) {
            const uint8_t* t = mate ? t2 : t1;
            const std::vector<uint64_t>& nl = mate ? b : a;
            uint64_t& s = mate ? s2 : s1;
            const uint64_t ln = nl[o] - s;
            if (ln > 0xffff) return -1;
            std::memcpy(pn, t + s, (size_t)ln);
            pn += ln;
            nlens[n] = (uint16_t)ln;
            const uint64_t ls = nl[o + 1] - (nl[o] + 1);
            std::memcpy(ps, t + nl[o] + 1, (size_t)ls);
            ps += ls;
            slens[n] = (int32_t)ls;
            const uint64_t lq = nl[o + 3] - (nl[o + 2] + 1);
            if (lq != ls) return -1;   // the reference then misaligns the quality buffer
            std::memcpy(pq, t + nl[o + 2] + 1, (size_t)lq);
            pq += lq;
            s = nl[o + 3] + 2;
            ++n;
        }
    }
    return n;
}

// ---- IDProcess::analysisIDBinType@0x4310a0 ---------------------------------
namespace {

struct Tok {
    const uint8_t* s;
    size_t n;
    bool operator==(const Tok& o) const { return n == o.n && std::memcmp(s, o.s, n) == 0; }
};

// strSplit@0x40e0d0 with the delimiter set at .rodata 0x44b9e8: space and all
// ASCII punctuation; tokens are maximal runs of other bytes.
bool delim(uint8_t c)
{
    static const char* D = " !\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~";
    return c && std::strchr(D, c) != nullptr;
}

void tokenize(const uint8_t* s, size_t n, std::vector<Tok>& out)
{
    out.clear();
    size_t i = 0;
    while (i < n) {
        while (i < n && delim(s[i])) ++i;
        if (i >= n) break;
        size_t j = i;
        while (j < n && !delim(s[j])) ++j;
        out.push_back(Tok{s + i, j - i});
        i = j;
    }
}

bool word_ieq(const Tok& t, const char* w)
{
    const size_t wl = std::strlen(w);
    if (t.n != wl) return false;
    for (size_t i = 0; i < wl; i++) {
        uint8_t c = t.s[i];
        if (c >= 'A' && c <= 'Z') c = (uint8_t)(c + 32);
        if (c != (uint8_t)w[i]) return false;
    }
    return true;
}

bool digits_only(const Tok& t)
{
    for (size_t i = 0; i < t.n; i++)
        if (t.s[i] < '0' || t.s[i] > '9') return false;
    return true;
}

// std::stoi/strtol semantics on the token text; false where the binary throws
bool parse_int(const Tok& t, int64_t& v)
{
    size_t i = 0;
    bool neg = false;
    if (i < t.n && (t.s[i] == '+' || t.s[i] == '-')) neg = t.s[i++] == '-';
    if (i >= t.n || t.s[i] < '0' || t.s[i] > '9') return false;
    int64_t x = 0;
    for (; i < t.n && t.s[i] >= '0' && t.s[i] <= '9'; i++) {
        x = x * 10 + (t.s[i] - '0');
        if (x > (1ll << 31)) return false;
    }
    v = neg ? -x : x;
    return v >= -(1ll << 31) && v < (1ll << 31);
}

bool parse_ul(const Tok& t, uint64_t& v)
{
    if (t.n == 0) return false;
    uint64_t x = 0;
    for (size_t i = 0; i < t.n; i++) {
        const uint64_t nx = x * 10 + (uint64_t)(t.s[i] - '0');
        if (nx / 10 != x) return false;
        x = nx;
    }
    v = x;
    return true;
}

// analysisPEType@0x430f50
int mate_type(const uint8_t* a, size_t la, const uint8_t* b, size_t lb)
{
    if (la == lb && std::memcmp(a, b, la) == 0) return 1;
    if (la && lb && a[la - 1] == '1' && b[lb - 1] == '2' && std::memcmp(a, b, la - 1) == 0) return 2;
    const std::string sa((const char*)a, la);
    const size_t at = sa.find("length");
    if (at == std::string::npos) return 0;
    return std::memcmp(a, b, at) == 0 ? 3 : 0;
}

}  // namespace

int sa_analyze_ids(const sa_block* first, int single_end, uint8_t T[512])
{
    if (!first || !T) return -1;
    if (first->nreads == 0) return 0;
    std::vector<Tok> prev, cur;
    tokenize(first->names, first->name_lens[0], prev);
    const int na = (int)prev.size();
    int len_idx = -1;
    for (int i = 1; i <= na; i++) {
        if (len_idx < 0) {
            if (word_ieq(prev[(size_t)i - 1], "length") || word_ieq(prev[(size_t)i - 1], "len")) {
                int64_t v;
                if (i >= na || !parse_int(prev[(size_t)i], v)) return -1;
                if (v == first->seq_lens[0]) {
                    len_idx = i;
                    if (i + 1 < 512) T[i + 1] = 0;
                }
            }
        } else if (len_idx == i - 1 && i + 1 < 512) {
            T[i + 1] = 3;
        }
    }
    bool mates[4] = {false, false, false, false};
    const uint8_t* p = first->names;
    uint32_t idx = 0;
    while (idx < first->nreads) {
        const uint8_t* s = p;
        const size_t ls = first->name_lens[idx];
        p += ls;
        ++idx;
        if (!single_end) {
            if (idx >= first->nreads) return -1;
            const size_t l2 = first->name_lens[idx];
            mates[mate_type(s, ls, p, l2)] = true;
            p += l2;
            ++idx;
        }
        tokenize(s, ls, cur);
        if ((int)cur.size() != na) {
            T[0] = 0;
            return 0;
        }
        for (int k = 0; k < na; k++) {
            if ((k != 0 && k - 1 == len_idx) || k == len_idx) continue;
            if (cur[(size_t)k] == prev[(size_t)k]) {
                if (k + 2 < 512) T[k + 2] = 0;
                continue;
            }
            if (!digits_only(prev[(size_t)k]) || !digits_only(cur[(size_t)k])) {
                T[0] = 0;
                return 0;
            }
            uint64_t va, vb;
            if (!parse_ul(prev[(size_t)k], va) || !parse_ul(cur[(size_t)k], vb)) return -1;
            if (vb - va != 1) {
                T[0] = 0;
                return 0;
            }
            if (k + 2 < 512) T[k + 2] = 1;
        }
        prev.swap(cur);
    }
    if (single_end) {
        T[0] = 1;
    } else if (!(mates[0] || mates[1] || mates[2] || mates[3])) {
        T[0] = 1;
        T[1] = 0;
    } else if (mates[0]) {
        T[0] = 0;
        T[1] = 0;
    } else {
        T[0] = 1;
        T[1] = mates[3] ? 3 : mates[2] ? 2 : 1;
    }
    return 0;
}

}  // extern "C"
