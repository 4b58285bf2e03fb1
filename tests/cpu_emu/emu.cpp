// emu.cpp -- CPU check of the GPU decomposition (test infrastructure only).
//
// Runs the encoder's per-thread logic (fastqueeze_amd/csrc/sa_logic.h) and the
// batch plan (sa_plan.h) sequentially on the host, with std::stable_sort in
// place of the radix sort and the oracle's MD5, then compares every block with
// the CPU restatement (oracle/fqz_oracle.c).  This validates the
// extract -> sort -> replay -> code decomposition before it runs on MI355X;
// the GPU parity tests (tests/test_gpu_parity.py) check the kernels themselves.
//
//   emu [-b block_bytes] [-s slevel] [-q qlevel] [-r ref.fa [-I insert]] in1.fq [in2.fq]
//
// -r: the reference (HASH index) path: the oracle's index and aligner give
// every read's alignment under both carried align_info states (what the GPU
// pass computes), the engine's host bookkeeping (sa_align_host.h) chooses and
// plans the blocks, sa_logic.h emits the alignment streams, and each block is
// compared with the oracle's doAlign + doAlignEncode restatement.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../fastqueeze_amd/csrc/sa_align_host.h"
#include "../../fastqueeze_amd/csrc/sa_logic.h"
#include "../../fastqueeze_amd/csrc/sa_plan.h"
#include "../../include/seqarc_amd.h"
#include "../../oracle/fqz_oracle.h"
#include "../../oracle/hash_oracle.h"

using namespace sa;

static std::vector<uint8_t> slurp(const char* p)
{
    std::vector<uint8_t> v;
    FILE* f = std::fopen(p, "rb");
    if (!f) return v;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    v.resize((size_t)n);
    if (std::fread(v.data(), 1, (size_t)n, f) != (size_t)n) v.clear();
    std::fclose(f);
    return v;
}

// The GPU coder decomposition (pass R, L1, L2, L3, restart after a squeeze)
// run sequentially; returns the stream's byte count.
static uint32_t code_decomposed(const PRec* P, const uint16_t* C, uint32_t n, uint8_t* o, uint32_t cap, int& restarts)
{
    const uint32_t nseg = n ? (n + SEG_SYMS - 1) / SEG_SYMS : 1;
    std::vector<uint32_t> ck(nseg), offat(nseg);
    std::vector<LowMap> mp(nseg);
    std::vector<uint64_t> lowat(nseg);
    uint32_t start = 0, r0 = 0xffffffffu, off0 = 0, out_len = 0;
    uint64_t low0 = 0;
    for (;;) {
        uint32_t r = r0;
        for (uint32_t g = start; g < nseg; g++) {
            ck[g] = r;
            if (g + 1 < nseg)
                for (uint32_t i = 0; i < SEG_SYMS; i++) {
                    uint32_t nb;
                    range_step(r, P[g * SEG_SYMS + i], recip32z(P[g * SEG_SYMS + i].tf & rec_tmask(C)), rec_tmask(C), nb);
                }
        }
        for (uint32_t g = start; g < nseg; g++)
            mp[g] = seg_lowmap(P + g * SEG_SYMS, C ? C + g * SEG_SYMS : nullptr, ck[g], seg_count(n, g));
        uint64_t low = low0;
        uint32_t off = off0;
        for (uint32_t g = start; g < nseg; g++) {
            lowat[g] = low;
            offat[g] = off;
            low = shl64(low, mp[g].s) + mp[g].B;
            off += mp[g].nbytes;
        }
        int64_t sq = -1;
        SegEnd sqe{};
        for (uint32_t g = start; g < nseg; g++) {
            const uint64_t room = cap > offat[g] ? cap - offat[g] : 0;
            SegEnd e = seg_code(P + g * SEG_SYMS, C ? C + g * SEG_SYMS : nullptr, ck[g], lowat[g], seg_count(n, g),
                                o + offat[g], room,
                                g + 1 == nseg);
            if (g + 1 == nseg) out_len = offat[g] + e.nbytes;
            if (e.squeezed && sq < 0) { sq = g; sqe = e; }
        }
        if (sq < 0 || sq + 1 == (int64_t)nseg) return out_len;
        restarts++;
        start = (uint32_t)sq + 1;
        r0 = sqe.r;
        low0 = sqe.low;
        off0 = offat[(size_t)sq] + sqe.nbytes;
    }
}

// Coder-only check on synthetic record streams, including streams built to hit
// the carry-less squeeze (the same symbol at probability 1/2 drives low towards
// all-ones): decomposed == serial, and the restart path is exercised.
static int coder_selftest()
{
    uint32_t x = 99;
    auto rnd = [&]() { x = x * 1664525u + 1013904223u; return x >> 8; };
    int restarts = 0, fails = 0;
    for (int tc = 0; tc < 400; tc++) {
        const uint32_t n = tc < 8 ? (uint32_t)tc : 1 + rnd() % 20000;
        std::vector<PRec> P(n + 1);
        std::vector<uint16_t> C(n + 1);
        const int kind = tc % 4;
        for (uint32_t i = 0; i < n; i++) {
            uint32_t t, f, c;
            if (kind == 0) { t = 2; f = 1; c = 1; }                                  // squeeze generator
            else if (kind == 1) { t = 2 + rnd() % 0xffdf; f = 1 + rnd() % t; if (f > t) f = t; c = rnd() % (t - f + 1); }
            else if (kind == 2) { t = 0xffe0; f = (rnd() & 1) ? 0xffd0 : 1; c = f == 1 ? 0xffdf : 0; }
            else { t = 12 + rnd() % 240; f = 1 + rnd() % (t - 1); c = rnd() % (t - f + 1); }
            P[i] = PRec{t | (f << 16)};
            C[i] = (uint16_t)c;
        }
        const uint32_t cap = 2 * n + 64;
        std::vector<uint8_t> a(cap), b(cap);
        uint32_t la = code_decomposed(P.data(), C.data(), n, a.data(), cap, restarts);
        SegEnd e = seg_code(P.data(), C.data(), 0xffffffffu, 0, n, b.data(), cap, true);
        if (la != e.nbytes || std::memcmp(a.data(), b.data(), la)) fails++;
    }
    std::printf("%s coder self-test: %d fails, %d restarts\n", fails || !restarts ? "FAIL" : "OK", fails, restarts);
    return fails || !restarts ? 1 : 0;
}

struct HostBlock {
    std::vector<uint8_t> names, seq, qual;
    std::vector<uint16_t> nl;
    std::vector<int32_t> sl;
    uint32_t nreads = 0;
};

int main(int argc, char** argv)
{
    uint64_t bs = 50ull << 20;
    int slevel = 3, qlevel = 2;
    double lossy = 0.0;
    const char* ref = nullptr;
    uint32_t insert_size = 0;
    int maxmis = 7;
    const int good = 1;
    std::vector<const char*> in;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "-r") && i + 1 < argc) { ref = argv[++i]; continue; }
        if (!std::strcmp(argv[i], "-I") && i + 1 < argc) { insert_size = (uint32_t)std::atoi(argv[++i]); continue; }
        if (!std::strcmp(argv[i], "-m") && i + 1 < argc) { maxmis = std::atoi(argv[++i]); continue; }
        if (!std::strcmp(argv[i], "-b") && i + 1 < argc) bs = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "-s") && i + 1 < argc) slevel = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "-q") && i + 1 < argc) qlevel = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "-l") && i + 1 < argc) lossy = std::atof(argv[++i]);
        else in.push_back(argv[i]);
    }
    if (in.size() == 1 && !std::strcmp(in[0], "--coder")) return coder_selftest();
    if (in.empty()) return 2;
    std::vector<uint8_t> t1 = slurp(in[0]), t2 = in.size() > 1 ? slurp(in[1]) : std::vector<uint8_t>();
    const bool pe = in.size() > 1;
    std::vector<uint64_t> e1(4096), e2(4096);
    int64_t nb = pe ? sa_cut_pe(t1.data(), t1.size(), t2.data(), t2.size(), bs, e1.data(), e2.data(), 4096)
                    : sa_cut_se(t1.data(), t1.size(), bs, e1.data(), 4096);
    if (nb <= 0) { std::printf("FAIL cut\n"); return 1; }
    // the oracle's cut must agree
    {
        std::vector<size_t> o1(4096), o2(4096);
        int64_t onb = pe ? orc_cut_pe(t1.data(), t1.size(), t2.data(), t2.size(), bs, o1.data(), o2.data(), 4096)
                         : orc_cut_se(t1.data(), t1.size(), bs, o1.data(), 4096);
        if (onb != nb) { std::printf("FAIL cut count %lld vs oracle %lld\n", (long long)nb, (long long)onb); return 1; }
        for (int64_t b = 0; b < nb; b++)
            if (o1[b] != e1[b] || (pe && o2[b] != e2[b])) { std::printf("FAIL cut boundary %lld\n", (long long)b); return 1; }
    }
    std::vector<HostBlock> hb((size_t)nb);
    uint64_t p1 = 0, p2 = 0;
    for (int64_t b = 0; b < nb; b++) {
        HostBlock& h = hb[(size_t)b];
        uint64_t l1 = e1[b] - p1, l2 = pe ? e2[b] - p2 : 0;
        h.names.resize(l1 + l2 + 16); h.seq.resize(l1 + l2 + 16); h.qual.resize(l1 + l2 + 16);
        h.nl.resize((l1 + l2) / 4 + 8); h.sl.resize((l1 + l2) / 4 + 8);
        int64_t nr = pe ? sa_parse_pe(t1.data() + p1, l1, t2.data() + p2, l2, h.names.data(), h.nl.data(), h.seq.data(), h.sl.data(), h.qual.data())
                        : sa_parse_se(t1.data() + p1, l1, h.names.data(), h.nl.data(), h.seq.data(), h.sl.data(), h.qual.data());
        if (nr < 0) { std::printf("FAIL parse block %lld\n", (long long)b); return 1; }
        h.nreads = (uint32_t)nr;
        p1 = e1[b];
        if (pe) p2 = e2[b];
    }
    uint8_t T[512] = {0}, To[512] = {0};
    sa_block first{hb[0].names.data(), hb[0].nl.data(), hb[0].seq.data(), hb[0].sl.data(), hb[0].qual.data(), hb[0].nreads};
    if (sa_analyze_ids(&first, !pe, T)) { std::printf("FAIL id analysis\n"); return 1; }
    orc_block ofirst{hb[0].names.data(), hb[0].nl.data(), hb[0].seq.data(), hb[0].sl.data(), hb[0].qual.data(), hb[0].nreads};
    orc_analyze_idbin(&ofirst, !pe, To);
    if (std::memcmp(T, To, 512)) { std::printf("FAIL id template differs from oracle\n"); return 1; }

    // ---- host BatchView (what sa_stage uploads) ----
    std::vector<DevBlock> blocks((size_t)nb);
    std::vector<uint8_t> names, seq, qual;
    std::vector<uint32_t> read_block, name_off, seq_off, seq_len;
    std::vector<uint16_t> name_len;
    uint32_t nr = 0;
    for (int64_t b = 0; b < nb; b++) {
        HostBlock& h = hb[(size_t)b];
        DevBlock& d = blocks[(size_t)b];
        d.nreads = h.nreads;
        d.read0 = nr;
        uint64_t ln = 0, ls = 0;
        for (uint32_t r = 0; r < h.nreads; r++) {
            ln += h.nl[r];
            ls += (uint64_t)h.sl[r];
            if (h.sl[r] > 0xffff) d.len_long = 1;
        }
        d.name_base = names.size();
        d.seq_base = seq.size();
        d.name_bytes = ln;
        d.seq_bytes = ls;
        names.insert(names.end(), h.names.begin(), h.names.begin() + (long)ln);
        seq.insert(seq.end(), h.seq.begin(), h.seq.begin() + (long)ls);
        qual.insert(qual.end(), h.qual.begin(), h.qual.begin() + (long)ls);
        names.resize(align_up(names.size(), 16));
        seq.resize(align_up(seq.size(), 16));
        qual.resize(align_up(qual.size(), 16));
        uint32_t no = 0, so = 0;
        for (uint32_t r = 0; r < h.nreads; r++) {
            read_block.push_back((uint32_t)b);
            name_off.push_back(no);
            name_len.push_back(h.nl[r]);
            seq_off.push_back(so);
            seq_len.push_back((uint32_t)h.sl[r]);
            no += h.nl[r];
            so += (uint32_t)h.sl[r];
        }
        nr += h.nreads;
    }
    const int k = slevel + 7;
    const uint32_t ns = 1u << ((2 * k) & 31);
    BatchView bv{};
    bv.blocks = blocks.data();
    bv.nblocks = (uint32_t)nb;
    bv.nreads_total = nr;
    bv.read_block = read_block.data();
    bv.names = names.data();
    bv.seq = seq.data();
    bv.qual = qual.data();
    bv.name_off = name_off.data();
    bv.name_len = name_len.data();
    bv.seq_off = seq_off.data();
    bv.seq_len = seq_len.data();
    bv.seq_mask = ns - 1;
    bv.qlevel = qlevel;
    bv.bin_mode = T[0];
    bv.md5 = 1;
    bv.qual_q = qual.data();
    bv.lossy = lossy > 0.0;
    // ---- -r: alignments (both carried states), the host plan, the variant choice ----
    std::vector<int32_t> a_ret(nr, -1), a_mp((size_t)nr * (maxmis + 1), -1), a_mt((size_t)nr * (maxmis + 1), 0);
    std::vector<uint8_t> a_rev(nr, 0), seq_skip(nr, 0);
    std::vector<uint32_t> a_pos(nr, 0);
    AlignView av{};
    if (ref) {
        std::vector<uint8_t> fa = slurp(ref);
        if (fa.empty() || ho_build((const char*)fa.data(), fa.size(), 14, 2, 1u << 16) < 0) {
            std::printf("FAIL index\n");
            return 1;
        }
        const ho_index* ix = ho_current_index();
        const ho_args args{ix->K, maxmis, ix->total, good, 0, 0};
        std::vector<ho_align> v0(nr), v1(nr);
        std::vector<uint8_t> st(nr, 0);
        std::vector<uint32_t> p0(nr, 0), p1(nr, 0);
        for (uint32_t r = 0; r < nr; r++) {
            const DevBlock& d = blocks[read_block[r]];
            const char* rd = (const char*)seq.data() + d.seq_base + seq_off[r];
            const int len = (int)seq_len[r];
            int nn = 0;
            for (int i = 0; i < len; i++) nn += base_code((uint8_t)rd[i]) > 3;
            std::memset(&v0[r], 0, sizeof(ho_align));
            std::memset(&v1[r], 0, sizeof(ho_align));
            v0[r].nmis = -1;
            v1[r].nmis = 0;
            const int r0 = len > 0 ? ho_align_read(ix, &args, rd, len, &v0[r]) : -1;
            const int r1 = len > 0 ? ho_align_read(ix, &args, rd, len, &v1[r]) : -1;
            if (r0 < 0) v0[r].nmis = -1;
            if (r1 < 0) v1[r].nmis = -1;
            bool differ = r0 != r1;
            if (!differ && r0 >= 0)
                differ = v0[r].pos != v1[r].pos || v0[r].rev != v1[r].rev ||
                         std::memcmp(v0[r].mispos, v1[r].mispos, sizeof(int32_t) * (size_t)r0) ||
                         std::memcmp(v0[r].mistype, v1[r].mistype, sizeof(int32_t) * (size_t)r0);
            st[r] = (uint8_t)((r0 >= 0 ? AL_OK0 : 0) | (differ ? AL_CONS : 0) | (!pe && nn > maxmis ? AL_NSKIP : 0) |
                              (r1 >= 0 ? AL_OK1 : 0));
            p0[r] = (uint32_t)v0[r].pos;
            p1[r] = (uint32_t)v1[r].pos;
        }
        AlignChainState ch;   // fresh align_info: nmis 0 ("aligned")
        for (int64_t b = 0; b < nb; b++) {
            DevBlock& d = blocks[(size_t)b];
            std::vector<uint32_t> sel;
            const AlignBlockPlan bp = align_plan_block(pe, d.nreads, &st[d.read0], &p0[d.read0], &p1[d.read0], insert_size,
                                                       ch, sel);
            d.order_count = bp.order_count;
            d.win = bp.win;
            d.ibits = bp.ibits;
            d.insert_bits = bp.insert_bits;
            std::vector<uint8_t> use1(d.nreads, 0);
            for (uint32_t i : sel) use1[i] = 1;
            if (std::getenv("EMU_ALN"))   // what the case exercised
                std::printf("block %lld: reads %u order %u aligned %u variant-1 %zu win %u ibits %u\n", (long long)b,
                            d.nreads, bp.order_count, bp.aligned, sel.size(), bp.win, bp.ibits);
            for (uint32_t i = 0; i < d.nreads; i++) {
                const uint32_t r = d.read0 + i;
                const ho_align& a = use1[i] ? v1[r] : v0[r];
                a_ret[r] = a.nmis;
                a_rev[r] = a.rev;
                a_pos[r] = (uint32_t)a.pos;
                for (int k2 = 0; k2 < a.nmis && k2 <= maxmis; k2++) {
                    a_mp[(size_t)r * (maxmis + 1) + k2] = a.mispos[k2];
                    a_mt[(size_t)r * (maxmis + 1) + k2] = a.mistype[k2];
                }
            }
        }
        const uint32_t shift = host_bits(ix->total) - 2;
        av = AlignView{a_ret.data(), a_rev.data(), a_pos.data(), a_mp.data(), a_mt.data(), (uint32_t)maxmis + 1, shift,
                       (1ull << shift) - 1, ix->total, pe ? 1 : 0,
                       maxmis >= 1 && maxmis <= 7 ? M_MIS8 : maxmis == 8 ? M_MIS9 : 0u};
        for (uint32_t r = 0; r < nr; r++) {
            uint32_t c[NACOL];
            seq_skip[r] = align_read_counts(bv, av, r, c) ? 1 : 0;
        }
        bv.aligned = 1;
        bv.paired = pe ? 1 : 0;
        bv.seq_skip = seq_skip.data();
    }
    // -l: the chunked rblock (what k_rb_spec / k_rb_fix / k_rb_apply compute),
    // checked against the oracle's serial restatement block by block
    std::vector<uint8_t> qual_q;
    if (lossy > 0.0) {
        for (uint32_t n = 0; n <= 255u * 255u; n++)   // (the walks' loop-free root, round 6)
            if (rb_round_sqrt_fast(n) != rb_round_sqrt(n)) {
                std::printf("FAIL rb_round_sqrt_fast(%u)\n", n);
                return 1;
            }
        qual_q.assign(qual.size(), 0);
        std::vector<uint32_t> tabw(2 * RB_TAB_WORDS);   // (the R decision tables the kernels stage in LDS)
        rb_tab_build(lossy, tabw.data(), tabw.data() + RB_TAB_WORDS);
        const RbTab tab{tabw.data(), tabw.data() + RB_TAB_WORDS};
        for (int64_t b = 0; b < nb; b++) {
            const DevBlock& d = blocks[(size_t)b];
            std::vector<RbChunk> ck;
            // (SA_RB_CHUNK: the engine's chunk length, also the arrays' stride)
            const char* rce = std::getenv("SA_RB_CHUNK");
            const uint64_t rc = rce && std::atoi(rce) >= 32 && (uint32_t)std::atoi(rce) <= RB_CHUNK &&
                                        std::atoi(rce) % 32 == 0
                                    ? (uint64_t)std::atoi(rce)
                                    : RB_CHUNK_DEFAULT;
            const uint64_t rw = rc / 32;
            for (uint64_t o = 0; o < d.seq_bytes; o += rc) {
                const uint32_t len = (uint32_t)std::min<uint64_t>(rc, d.seq_bytes - o);
                ck.push_back(RbChunk{d.seq_base + o, len, (o == 0 ? RB_FIRST : 0u) | (o + len == d.seq_bytes ? RB_LAST : 0u)});
            }
            if (ck.empty()) continue;
            std::vector<uint32_t> opens(ck.size() * rw);
            std::vector<RbRun> spec(ck.size()), entry(ck.size());
            std::vector<uint8_t> vals(ck.size() * rc);
            std::vector<RbInfo> info(ck.size());
            // k_rb_spec (with the run values, round 5), k_rb_fix's carry,
            // then k_rb_true + k_rb_fill -- or (SA_RB_APPLY=1) the round-4 k_rb_apply
            const bool walk = std::getenv("SA_RB_APPLY") != nullptr;
            for (size_t c = 0; c < ck.size(); c++)
                spec[c] = walk ? rb_spec(qual.data(), ck[c], tab, &opens[c * rw], (uint32_t)rw)
                               : rb_spec_vals(qual.data(), ck[c], tab, &opens[c * rw], &vals[c * rc], info[c],
                                              (uint32_t)rc);
            RbRun cur = spec[0];
            for (size_t c = 1; c < ck.size(); c++) {
                entry[c] = cur;
                cur = rb_carry(qual.data(), ck[c], cur, tab, &opens[c * rw], spec[c]);
            }
            if (walk) {
                for (size_t c = ck.size(); c-- > 0;) rb_apply(qual.data(), qual_q.data(), ck[c], entry[c], tab);
            } else {
                for (size_t c = 1; c < ck.size(); c++)
                    rb_true(qual.data(), ck[c], entry[c], tab, &opens[c * rw], &vals[c * rc], info[c]);
                for (size_t c = 0; c < ck.size(); c++) {
                    const uint32_t ev = info[c].entry_val & 0xffu, tv = rb_chase(info.data(), ck.data(), (uint32_t)c);
                    int32_t prev = -1;
                    for (uint32_t t = 0; t < rw && 32 * t < ck[c].len; t++) {
                        const uint32_t w = opens[c * rw + t];
                        rb_fill_word(qual_q.data(), ck[c], t, w, prev, &vals[c * rc], info[c], ev, tv);
                        if (w) prev = (int32_t)(32 * t + 31 - (uint32_t)__builtin_clz(w));
                    }
                }
            }
            std::vector<uint8_t> ref(qual.begin() + (long)d.seq_base, qual.begin() + (long)(d.seq_base + d.seq_bytes));
            orc_rblock(ref.data(), ref.size(), lossy);
            if (std::memcmp(ref.data(), qual_q.data() + d.seq_base, ref.size())) {
                std::printf("FAIL chunked rblock differs from the oracle (block %lld)\n", (long long)b);
                return 1;
            }
        }
        bv.qual_q = qual_q.data();
    }

    // ---- prep + scan ----
    std::vector<uint32_t> counts((size_t)nr * NCOL);
    std::vector<int16_t> name_p(nr), name_s(nr);
    std::vector<uint16_t> maxlen(nr);
    uint32_t err = 0;
    for (uint32_t r = 0; r < nr; r++) err |= prep_read(bv, r, counts.data(), name_p.data(), name_s.data(), true);
    if (err) { std::printf("FAIL prep error bits %x\n", err); return 1; }
    std::vector<uint32_t> totals((size_t)nb * NCOL);
    for (int64_t b = 0; b < nb; b++) {
        const DevBlock& d = blocks[(size_t)b];
        uint32_t carry[NCOL] = {0};
        uint32_t m = 0;
        for (uint32_t i = 0; i < d.nreads; i++) {
            uint32_t* c = &counts[(size_t)(d.read0 + i) * NCOL];
            for (int col = 0; col < NCOL; col++) { uint32_t v = c[col]; c[col] = carry[col]; carry[col] += v; }
            maxlen[d.read0 + i] = (uint16_t)m;
            m = std::max<uint32_t>(m, name_len[d.read0 + i]);
        }
        for (int col = 0; col < NCOL; col++) totals[(size_t)b * NCOL + col] = carry[col];
    }
    // alignment columns: per read, exclusive per block
    std::vector<uint32_t> acounts((size_t)nr * NACOL, 0), atot((size_t)nb * NACOL, 0);
    if (ref) {
        for (int64_t b = 0; b < nb; b++) {
            const DevBlock& d = blocks[(size_t)b];
            uint32_t carry[NACOL] = {0};
            for (uint32_t i = 0; i < d.nreads; i++) {
                uint32_t* c = &acounts[(size_t)(d.read0 + i) * NACOL];
                align_read_counts(bv, av, d.read0 + i, c);
                for (int col = 0; col < NACOL; col++) { uint32_t v = c[col]; c[col] = carry[col]; carry[col] += v; }
            }
            for (int col = 0; col < NACOL; col++) atot[(size_t)b * NACOL + col] = carry[col];
        }
    }
    BatchPlan bp;
    if (!plan_batch(blocks, totals, bp, ref ? &atot : nullptr, av.mis_model)) { std::printf("FAIL plan\n"); return 1; }

    // ---- emit ----
    const size_t stot = bp.seq.total + 64, atot_sz = bp.aux.total + 64;   // slack as the engine
    std::vector<uint32_t> sk(stot, SORT_PAD), sv(stot), ak(atot_sz, SORT_PAD), av_(atot_sz);
    for (uint32_t r = 0; r < nr; r++)
        err |= emit_read(bv, r, counts.data(), totals.data(), name_p.data(), name_s.data(), maxlen.data(), sk.data(),
                         sv.data(), ak.data(), av_.data(), true);
    if (err) { std::printf("FAIL emit error bits %x\n", err); return 1; }
    if (ref)
        for (uint32_t r = 0; r < nr; r++) align_read_emit(bv, av, r, &acounts[(size_t)r * NACOL], ak.data(), av_.data());

    // ---- stable sort per segment (what k_sort_* computes) ----
    auto sort_space = [](std::vector<uint32_t>& K, std::vector<uint32_t>& V, const SortPlan& p, int lo) {
        for (const SortSeg& g : p.segs) {
            const size_t n = (size_t)g.ntiles * SORT_TILE;
            std::vector<uint32_t> idx(n);
            std::iota(idx.begin(), idx.end(), 0u);
            std::stable_sort(idx.begin(), idx.end(),
                             [&](uint32_t a, uint32_t b) { return (K[g.base + a] >> lo) < (K[g.base + b] >> lo); });
            std::vector<uint32_t> k2(n), v2(n);
            for (size_t i = 0; i < n; i++) { k2[i] = K[g.base + idx[i]]; v2[i] = V[g.base + idx[i]]; }
            std::copy(k2.begin(), k2.end(), K.begin() + (long)g.base);
            std::copy(v2.begin(), v2.end(), V.begin() + (long)g.base);
        }
    };
    sort_space(sk, sv, bp.seq, 0);
    sort_space(ak, av_, bp.aux, AUX_SYM_BITS);

    // EMU_RUNS=1: the longest model runs per space (what bounds the replay kernels)
    if (std::getenv("EMU_RUNS")) {
        auto runs = [](const std::vector<uint32_t>& K, const SortPlan& p, int lo, const char* name) {
            std::vector<std::pair<size_t, uint32_t>> r;
            for (const SortSeg& g : p.segs)
                for (size_t i = g.base, s = g.base; i <= g.base + g.count; i++)
                    if (i == g.base + g.count || (K[i] >> lo) != (K[s] >> lo)) {
                        r.push_back({i - s, K[s] >> lo});
                        s = i;
                    }
            std::sort(r.begin(), r.end(), std::greater<>());
            size_t n512 = 0, tot = 0;
            for (auto& x : r) { if (x.first >= 512) { n512++; tot += x.first; } }
            std::printf("%s: %zu runs, %zu >= 512 holding %zu symbols; longest:", name, r.size(), n512, tot);
            for (size_t i = 0; i < r.size() && i < 12; i++) std::printf(" %zu(m%x)", r[i].first, r[i].second);
            std::printf("\n");
        };
        runs(sk, bp.seq, 0, "seq");
        runs(ak, bp.aux, AUX_SYM_BITS, "aux");
    }
    // ---- replays ----
    std::vector<PRec> ps(stot), pa(atot_sz);
    std::vector<uint16_t> cs(stot), ca(atot_sz);
    std::vector<uint32_t> F(256);
    for (const SortSeg& g : bp.seq.segs) {
        const SymSink sink{ps.data() + g.base, nullptr};   // packed SEQ records
        for (size_t i = g.base; i < g.base + g.count; i++)
            if (i == g.base || sk[i - 1] != sk[i]) replay_seq_run(sk.data(), sv.data(), i, g.base + g.count, sk[i], sink);
    }
    for (const SortSeg& g : bp.aux.segs) {
        const SymSink sink{pa.data() + g.base, ca.data() + g.base};
        for (size_t i = g.base; i < g.base + g.count; i++)
            if (i == g.base || (ak[i - 1] >> AUX_SYM_BITS) != (ak[i] >> AUX_SYM_BITS))
                err |= replay_simple_run(ak.data(), av_.data(), i, g.base + g.count, ak[i] >> AUX_SYM_BITS, sink, F.data());
    }
    if (err) { std::printf("FAIL replay error bits %x\n", err); return 1; }

    // ---- coders: the decomposed coder, checked against the serial one ----
    std::vector<uint8_t> payload(bp.payload_bytes + 16);
    std::vector<uint32_t> out_len(bp.tasks.size());
    int restarts = 0;
    for (size_t t = 0; t < bp.tasks.size(); t++) {
        const CoderTask& tk = bp.tasks[t];
        const PRec* P = (tk.space ? pa.data() : ps.data()) + tk.rec_base;
        const uint16_t* C = tk.space ? ca.data() + tk.rec_base : nullptr;   // SEQ: packed records
        uint8_t* o = payload.data() + tk.out_base;
        out_len[t] = code_decomposed(P, C, tk.n, o, tk.out_cap, restarts);
        std::vector<uint8_t> ser(tk.out_cap);
        SegEnd e = seg_code(P, C, 0xffffffffu, 0, tk.n, ser.data(), tk.out_cap, true);
        if (e.nbytes != out_len[t] || std::memcmp(ser.data(), o, e.nbytes)) {
            std::printf("FAIL decomposed coder differs from the serial coder (task %zu)\n", t);
            return 1;
        }
    }
    std::vector<uint32_t> digests((size_t)nb * 12);
    for (int64_t b = 0; b < nb; b++) {
        const DevBlock& d = blocks[(size_t)b];
        uint8_t dg[16];
        const uint8_t* src[3] = {names.data() + d.name_base, seq.data() + d.seq_base, qual.data() + d.seq_base};
        const uint64_t ln[3] = {d.name_bytes, d.seq_bytes, d.seq_bytes};
        for (int f = 0; f < 3; f++) {
            orc_md5(src[f], ln[f], dg);
            std::memcpy(&digests[((size_t)b * 3 + f) * 4], dg, 16);
        }
    }
    int fails = 0;
    uint64_t total_out = 0;
    int32_t ocarry[2] = {0, 0};   // the oracle's own align_info chain (fresh: nmis 0)
    for (int64_t b = 0; b < nb; b++) {
        std::vector<uint8_t> o(bp.final_bytes + 64);
        uint32_t dst[ASM_MAX_COPIES], tsk[ASM_MAX_COPIES], len[ASM_MAX_COPIES], nseg = 0;
        uint32_t L = assemble_plan(bv, (uint32_t)b, bp.asmb[(size_t)b], out_len.data(), digests.data(), o.data(), dst, tsk,
                                   len, nseg);
        for (uint32_t s = 0; s < nseg; s++) std::memcpy(o.data() + dst[s], payload.data() + bp.task_out_base[tsk[s]], len[s]);
        HostBlock& h = hb[(size_t)b];
        orc_block ob{h.names.data(), h.nl.data(), h.seq.data(), h.sl.data(), h.qual.data(), h.nreads};
        orc_cfg oc{slevel, qlevel, 1, T[0], lossy};
        std::vector<uint8_t> want(3 * (h.seq.size() + h.names.size()) + 64 * h.nreads + 8192);
        int64_t rl = ref ? orc_encode_block_hash(&ob, &oc, pe ? 1 : 0, maxmis, good, insert_size, ocarry, want.data(),
                                                 want.size())
                         : orc_encode_block(&ob, &oc, want.data(), want.size());
        bool ok = rl == (int64_t)L && std::memcmp(want.data(), o.data(), L) == 0;
        if (!ok) {
            size_t at = 0;
            while (at < L && at < (size_t)rl && want[at] == o[at]) at++;
            std::printf("block %lld MISMATCH emu %u oracle %lld first diff at %zu\n", (long long)b, L, (long long)rl, at);
            fails++;
        }
        total_out += L;
    }
    std::printf("%s blocks %lld reads %u out %llu bin_mode %d coder restarts %d\n", fails ? "FAIL" : "OK", (long long)nb,
                nr, (unsigned long long)total_out, T[0], restarts);
    return fails ? 1 : 0;
}
