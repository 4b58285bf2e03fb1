// seqarc_amd -- the SeqArc -c command line over libseqarc_amd (host C++).
//
//   seqarc_amd -c -1 A.fq[.gz] [-2 B.fq[.gz]] -o PREFIX [-l R] [-n] [-t N]
//              [--slevel K] [--qlevel Q] [--device D] [--devices N] [--batch BLOCKS]
//   seqarc_amd -d [-t N] ARCHIVE.arc PREFIX
//
// --devices N: batches of blocks are dealt to N gfx950 devices (one host
// thread and sa_ctx each; blocks are independent, so there is no device-to-
// device exchange) and gathered back in input order (--share-device: N
// contexts on one device, for testing the scatter/gather on one GPU).
//
// Mirrors the reference's encode path (SeqArc-1.6 main@0x41fd40 ->
// SeqArcContext::doReadAndEncode@0x41a4e0): the reader cuts 50 MiB blocks
// (SeqArcRead::doReadJob@0x432a80 / doReadPEJob@0x432d10), the first block
// decides the ID template (IDProcess::analysisIDBinType@0x4310a0), every block
// is encoded (here on one gfx950 device, a batch of blocks per launch) and the
// blocks are written after a 16-byte header in input order, followed by the
// trailer (SeqArcFile::writeFileInfo@0x4171b0).  Output: PREFIX.arc.
// -t is accepted for command-line compatibility (the GPU encodes a batch of
// blocks concurrently); Slevel / Qlevel are the reference's developer options
// (./seqarc.config), given here as --slevel / --qlevel.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/seqarc_amd.h"

namespace {

bool slurp(const char* path, std::vector<uint8_t>& out, bool& gz)
{
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    unsigned char m[2] = {0, 0};
    gz = fread(m, 1, 2, f) == 2 && m[0] == 0x1f && m[1] == 0x8b;   // getFileType@0x40d9f0
    fclose(f);
    gzFile g = gzopen(path, "rb");
    if (!g) return false;
    gzbuffer(g, 1 << 18);
    out.clear();
    std::vector<uint8_t> buf(1 << 22);
    for (;;) {
        const int n = gzread(g, buf.data(), (unsigned)buf.size());
        if (n < 0) { gzclose(g); return false; }
        if (n == 0) break;
        out.insert(out.end(), buf.begin(), buf.begin() + n);
    }
    gzclose(g);
    return true;
}

// getFirstLine@0x431eb0: the '+' line of the first record is bare ("+\n")
int bare_plus(const std::vector<uint8_t>& t)
{
    size_t nl[3] = {0, 0, 0};
    int k = 0;
    for (size_t i = 0; i < t.size() && k < 3; i++)
        if (t[i] == '\n') nl[k++] = i + 1;
    if (k < 3) return 1;
    return nl[2] - nl[1] > 2 ? 0 : 1;
}

struct Parsed {
    std::vector<uint8_t> names, seq, qual;
    std::vector<uint16_t> nl;
    std::vector<int32_t> sl;
    uint32_t nreads = 0;
    uint64_t text1 = 0, text2 = 0;
    sa_block view() const { return sa_block{names.data(), nl.data(), seq.data(), sl.data(), qual.data(), nreads}; }
};

int usage()
{
    fprintf(stderr,
            "usage: seqarc_amd -c -1 A.fq[.gz] [-2 B.fq[.gz]] -o PREFIX [-l R] [-n] [-t N]\n"
            "                  [--slevel K] [--qlevel Q] [--device D] [--devices N] [--batch BLOCKS]\n"
            "                  [--block-size MiB]\n"
            "       seqarc_amd -d [-t N] [--slevel K] [--qlevel Q] ARCHIVE.arc PREFIX\n");
    return 2;
}

uint64_t be(const uint8_t* p, int n)
{
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | p[i];
    return v;
}

// EBML VINT (Encap::getValue@0x420680): value and width
uint64_t vint(const uint8_t* p, const uint8_t* end, int& w)
{
    w = 1;
    if (p >= end) { w = 0; return 0; }
    while (w <= 8 && !(p[0] & (0x80 >> (w - 1)))) w++;
    if (w > 8 || end - p < w) { w = 0; return 0; }
    uint64_t v = p[0] & ((0x80u >> (w - 1)) - 1);
    for (int i = 1; i < w; i++) v = (v << 8) | p[i];
    return v;
}

// SeqArc -d: SeqArcFile::readFileInfo@0x419660 (header, trailer params, block
// table), one block per host thread (ISeqArcDecodeThread::doJob@0x435580),
// FASTQ written in block order as PREFIX_1.fastq / PREFIX_2.fastq (PE,
// .rodata +0x7b2) or PREFIX.fastq (SE).
int decode_archive(const char* path, const char* prefix, sa_cfg cfg, int threads)
{
    std::vector<uint8_t> a;
    {
        FILE* f = fopen(path, "rb");
        if (!f) { fprintf(stderr, "seqarc_amd: cannot read %s\n", path); return 1; }
        fseek(f, 0, SEEK_END);
        a.resize((size_t)ftell(f));
        fseek(f, 0, SEEK_SET);
        if (fread(a.data(), 1, a.size(), f) != a.size()) { fclose(f); return 1; }
        fclose(f);
    }
    if (a.size() < 16 || memcmp(a.data(), ".arc", 4) || a[7] != 0x82) {
        fprintf(stderr, "seqarc_amd: %s is not a SeqArc 1.6 archive\n", path);
        return 1;
    }
    const uint64_t region = be(a.data() + 8, 8) & ((1ull << 56) - 1);
    if (16 + region > a.size()) return 1;
    const uint8_t *t = a.data() + 16 + region, *end = a.data() + a.size();
    int w;
    if (vint(t, end, w) != 3 || !w) return 1;
    t += w + 4;
    // params encap (ID 1, 2-byte size): fields 1-18
    if (vint(t, end, w) != 1 || !w) return 1;
    t += w;
    const uint64_t psz = be(t, 2) & 0x3fff;
    t += 2;
    const uint8_t* pend = t + psz;
    uint8_t tmpl[512] = {0};
    int bare = 1, paired = 0, lossy = 0, md5 = 1;
    uint32_t nblocks = 0;
    while (t < pend) {
        const uint64_t id = vint(t, pend, w);
        if (!w) return 1;
        t += w;
        const int sw = id == 15 ? 2 : 1;
        const uint64_t ln = be(t, sw) & ((1ull << (7 * sw)) - 1);
        t += sw;
        if (t + ln > pend) return 1;
        if (id == 2) bare = t[0];
        else if (id == 11 && ln >= 4) nblocks = (uint32_t)(t[0] | t[1] << 8 | t[2] << 16 | (uint32_t)t[3] << 24);
        else if (id == 14 && ln) paired = 1;
        else if (id == 15 && ln == 512) memcpy(tmpl, t, 512);
        else if (id == 16) lossy = t[0];
        else if (id == 17) md5 = t[0];
        t += ln;
    }
    if (vint(t, end, w) != 7 || !w) return 1;
    t += w;
    const uint64_t bt = be(t, 4) & 0x0fffffff;
    t += 4;
    const uint32_t rec = paired ? 40 : 32;
    if (bt != (uint64_t)rec * nblocks || t + bt > end) return 1;
    struct Blk { uint64_t off, size, text; uint32_t lng; };
    std::vector<Blk> blks(nblocks);
    for (uint32_t b = 0; b < nblocks; b++) {
        const uint8_t* r = t + (size_t)rec * b;
        const uint32_t s2 = r[0] | r[1] << 8 | r[2] << 16 | (uint32_t)r[3] << 24;
        uint64_t off = 0;
        for (int k = 7; k >= 0; k--) off = (off << 8) | r[0x10 + k];
        const uint64_t text = paired ? (uint64_t)(r[4] | r[5] << 8 | r[6] << 16 | (uint32_t)r[7] << 24) +
                                           (uint64_t)(r[8] | r[9] << 8 | r[10] << 16 | (uint32_t)r[11] << 24)
                                     : (uint64_t)(r[8] | r[9] << 8 | r[10] << 16 | (uint32_t)r[11] << 24);
        blks[b] = Blk{off, s2 >> 1, text, s2 & 1u};
        if (off + blks[b].size > 16 + region) return 1;
    }
    cfg.md5 = md5;
    cfg.lossy = lossy ? 1.0 : 0.0;
    cfg.bin_mode = tmpl[0];
    const std::string p1 = std::string(prefix) + (paired ? "_1.fastq" : ".fastq"), p2 = std::string(prefix) + "_2.fastq";
    FILE* o1 = fopen(p1.c_str(), "wb");
    FILE* o2 = paired ? fopen(p2.c_str(), "wb") : nullptr;
    if (!o1 || (paired && !o2)) { fprintf(stderr, "seqarc_amd: cannot write %s\n", p1.c_str()); return 1; }
    struct Dec {
        std::vector<uint8_t> names, seq, qual;
        std::vector<uint16_t> nl;
        std::vector<int32_t> sl;
        sa_decoded d{};
        int64_t rc = -1;
    };
    int rc = 0, bad_md5 = 0;
    const uint32_t nt = (uint32_t)std::max(1, threads);
    for (uint32_t b0 = 0; b0 < nblocks && !rc; b0 += nt) {
        const uint32_t n = std::min(nt, nblocks - b0);
        std::vector<Dec> ds(n);
        std::vector<std::thread> th;
        for (uint32_t i = 0; i < n; i++)
            th.emplace_back([&, i]() {
                const Blk& bk = blks[b0 + i];
                Dec& d = ds[i];
                const uint64_t cap = bk.text + 64;   // names, bases, qualities each fit the FASTQ text
                d.names.resize(cap); d.seq.resize(cap); d.qual.resize(cap);
                d.nl.resize(cap / 4 + 8); d.sl.resize(cap / 4 + 8);
                d.d = sa_decoded{d.names.data(), d.nl.data(), d.seq.data(), d.sl.data(), d.qual.data(), cap, cap,
                                 (uint32_t)(cap / 4 + 8), 0, 0};
                d.rc = sa_decode_block(a.data() + bk.off, bk.size, &cfg, tmpl, (int32_t)bk.lng, &d.d);
            });
        for (auto& x : th) x.join();
        for (uint32_t i = 0; i < n && !rc; i++) {
            Dec& d = ds[i];
            if (d.rc < 0) { fprintf(stderr, "seqarc_amd: block %u does not decode\n", b0 + i); rc = 1; break; }
            bad_md5 |= !d.d.md5_ok;
            const uint8_t *nm = d.names.data(), *sq = d.seq.data(), *ql = d.qual.data();
            for (uint32_t r = 0; r < d.d.nreads; r++) {
                FILE* f = paired && (r & 1) ? o2 : o1;
                const size_t L = (size_t)d.sl[r], N = d.nl[r];
                fputc('@', f); fwrite(nm, 1, N, f); fputc('\n', f);
                fwrite(sq, 1, L, f);
                fputs("\n+", f);
                if (!bare) fwrite(nm, 1, N, f);
                fputc('\n', f);
                fwrite(ql, 1, L, f); fputc('\n', f);
                nm += N; sq += L; ql += L;
            }
        }
    }
    fclose(o1);
    if (o2) fclose(o2);
    if (bad_md5) {   // blockMd5Verify@0x414e00: "Name/Seq/Qual md5 unequal"
        fprintf(stderr, "seqarc_amd: Name/Seq/Qual md5 unequal\n");
        rc = rc ? rc : 3;
    }
    return rc;
}

}  // namespace

int main(int argc, char** argv)
{
    const char *f1 = nullptr, *f2 = nullptr, *outp = nullptr;
    bool compress = false, decompress = false;
    const char* arc = nullptr;
    int threads = 1;
    sa_cfg cfg{3, 2, 1, 0, 0.0};
    int device = 0, batch = 16, devices = 1, block_mib = 50;
    bool share_device = false;
    for (int i = 1; i < argc; i++) {
        const char* a = argv[i];
        auto val = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
        if (!strcmp(a, "-c")) compress = true;
        else if (!strcmp(a, "-1")) f1 = val();
        else if (!strcmp(a, "-2")) f2 = val();
        else if (!strcmp(a, "-o")) outp = val();
        else if (!strcmp(a, "-n")) cfg.md5 = 0;
        else if (!strcmp(a, "-l")) { const char* v = val(); if (!v) return usage(); cfg.lossy = atof(v); }
        else if (!strcmp(a, "-t")) { const char* v = val(); if (!v) return usage(); threads = atoi(v) > 0 ? atoi(v) : 1; }
        else if (!strcmp(a, "--slevel")) { const char* v = val(); if (!v) return usage(); cfg.slevel = atoi(v); }
        else if (!strcmp(a, "--qlevel")) { const char* v = val(); if (!v) return usage(); cfg.qlevel = atoi(v); }
        else if (!strcmp(a, "--device")) { const char* v = val(); if (!v) return usage(); device = atoi(v); }
        else if (!strcmp(a, "--devices")) { const char* v = val(); if (!v) return usage(); devices = atoi(v) > 0 ? atoi(v) : 1; }
        else if (!strcmp(a, "--share-device")) share_device = true;
        else if (!strcmp(a, "--block-size")) { const char* v = val(); if (!v) return usage(); block_mib = atoi(v) > 0 ? atoi(v) : 50; }
        else if (!strcmp(a, "--batch")) { const char* v = val(); if (!v) return usage(); batch = atoi(v) > 0 ? atoi(v) : 1; }
        else if (!strcmp(a, "-d")) decompress = true;
        else if (a[0] != '-' && decompress && !arc) arc = a;
        else if (a[0] != '-' && decompress && !outp) outp = a;
        else return usage();
    }
    if (decompress) {
        if (!arc || !outp) return usage();
        return decode_archive(arc, outp, cfg, threads);
    }
    if (!compress || !f1 || !outp) return usage();
    const bool pe = f2 && *f2;

    std::vector<uint8_t> t1, t2;
    bool gz1 = false, gz2 = false;
    if (!slurp(f1, t1, gz1) || (pe && !slurp(f2, t2, gz2))) {
        fprintf(stderr, "seqarc_amd: cannot read input\n");
        return 1;
    }
    const uint64_t bs = (uint64_t)block_mib << 20;   // BlockSize(M), default 50 (param+0x1b78)
    const uint64_t maxb = (t1.size() + t2.size()) / 1024 + 16;
    std::vector<uint64_t> e1(maxb), e2(maxb);
    const int64_t nb = pe ? sa_cut_pe(t1.data(), t1.size(), t2.data(), t2.size(), bs, e1.data(), e2.data(), maxb)
                          : sa_cut_se(t1.data(), t1.size(), bs, e1.data(), maxb);
    if (nb < 0) {
        fprintf(stderr, "seqarc_amd: block cut failed\n");
        return 1;
    }
    auto parse = [&](int64_t b, Parsed& p) -> bool {
        const uint64_t s1 = b ? e1[b - 1] : 0, s2 = (pe && b) ? e2[b - 1] : 0;
        const uint64_t l1 = e1[b] - s1, l2 = pe ? e2[b] - s2 : 0;
        const uint64_t cap = l1 + l2 + 16;
        p.names.resize(cap); p.seq.resize(cap); p.qual.resize(cap);
        p.nl.resize(cap / 4 + 8); p.sl.resize(cap / 4 + 8);
        const int64_t n = pe ? sa_parse_pe(t1.data() + s1, l1, t2.data() + s2, l2, p.names.data(), p.nl.data(),
                                           p.seq.data(), p.sl.data(), p.qual.data())
                             : sa_parse_se(t1.data() + s1, l1, p.names.data(), p.nl.data(), p.seq.data(), p.sl.data(),
                                           p.qual.data());
        if (n < 0) return false;
        p.nreads = (uint32_t)n;
        p.text1 = l1;
        p.text2 = l2;
        return true;
    };

    uint8_t tmpl[512] = {0};
    if (nb > 0) {
        Parsed first;
        if (!parse(0, first)) { fprintf(stderr, "seqarc_amd: parse failed\n"); return 1; }
        const sa_block fb = first.view();
        if (sa_analyze_ids(&fb, pe ? 0 : 1, tmpl) != 0) {
            fprintf(stderr, "seqarc_amd: ID analysis failed\n");
            return 1;
        }
    }
    cfg.bin_mode = tmpl[0];

    // one encoder context (and host thread) per device: batches of blocks are
    // dealt to the devices in order, encoded independently (blocks share no
    // model state), and gathered back in input order by this thread
    std::vector<sa_ctx*> ctxs;
    for (int d = 0; d < devices; d++) {
        sa_ctx* c = sa_create(device + (share_device ? 0 : d));
        if (!c) {
            if (ctxs.empty()) { fprintf(stderr, "seqarc_amd: no usable gfx950 device %d\n", device); return 1; }
            break;   // fewer devices than asked for: use those present
        }
        ctxs.push_back(c);
    }
    const std::string path = std::string(outp) + ".arc";
    FILE* fo = fopen(path.c_str(), "wb");
    if (!fo) {
        fprintf(stderr, "seqarc_amd: cannot write %s\n", path.c_str());
        for (sa_ctx* c : ctxs) sa_destroy(c);
        return 1;
    }
    uint8_t hdr[16] = {0};
    fwrite(hdr, 1, 16, fo);   // patched at the end (createOutFile@0x417480 / writeFileInfo@0x4171b0)
    std::vector<sa_arc_block> info;
    uint64_t total = 0;
    int rc = 0;
    struct Batch {
        std::vector<Parsed> ps;
        std::vector<std::vector<uint8_t>> bufs;
        std::vector<sa_out> outs;
        int status = 0;   // 0 pending, 1 done, -1 failed
        std::string err;
    };
    const int64_t nbatch = (nb + batch - 1) / batch;
    std::vector<Batch> bt((size_t)nbatch);
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<int64_t> next{0};
    std::atomic<bool> stop{false};
    const size_t max_ahead = 2 * ctxs.size();   // batches held in memory beyond the writer
    int64_t written = 0;
    auto worker = [&](sa_ctx* ctx) {
        for (;;) {
            int64_t k;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || next.load() < written + (int64_t)max_ahead || next.load() >= nbatch; });
                if (stop || next.load() >= nbatch) return;
                k = next++;
            }
            Batch& B = bt[(size_t)k];
            const int64_t b0 = k * batch, n = std::min<int64_t>(batch, nb - b0);
            B.ps.resize((size_t)n);
            B.bufs.resize((size_t)n);
            B.outs.resize((size_t)n);
            std::vector<sa_block> in((size_t)n);
            int st = 1;
            for (int64_t i = 0; i < n; i++) {
                if (!parse(b0 + i, B.ps[(size_t)i])) { st = -1; B.err = "parse failed"; break; }
                in[(size_t)i] = B.ps[(size_t)i].view();
                B.bufs[(size_t)i].resize(sa_output_bound(&in[(size_t)i]));
                B.outs[(size_t)i] = sa_out{B.bufs[(size_t)i].data(), B.bufs[(size_t)i].size(), 0};
            }
            if (st > 0 && sa_encode_blocks(ctx, in.data(), (int)n, &cfg, B.outs.data()) != 0) {
                st = -1;
                B.err = std::string("encode failed: ") + sa_last_error(ctx);
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                B.status = st;
            }
            cv.notify_all();
        }
    };
    std::vector<std::thread> th;
    for (sa_ctx* c : ctxs) th.emplace_back(worker, c);
    for (int64_t k = 0; k < nbatch && !rc; k++) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return bt[(size_t)k].status != 0; });
        }
        Batch& B = bt[(size_t)k];
        if (B.status < 0) { fprintf(stderr, "seqarc_amd: %s\n", B.err.c_str()); rc = 1; break; }
        for (size_t i = 0; i < B.ps.size(); i++) {
            const Parsed& p = B.ps[i];
            uint32_t lng = 0;
            for (uint32_t r = 0; r < p.nreads; r++) lng |= p.sl[r] > 0xffff;
            fwrite(B.outs[i].data, 1, B.outs[i].size, fo);
            info.push_back(sa_arc_block{(uint32_t)B.outs[i].size, lng, p.text1, p.text2});
            total += B.outs[i].size;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            B = Batch{};
            B.status = 1;
            written = k + 1;
        }
        cv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        stop = true;
    }
    cv.notify_all();
    for (auto& x : th) x.join();
    for (sa_ctx* c : ctxs) sa_destroy(c);
    if (!rc) {
        sa_arc_info ai{f1, pe ? f2 : nullptr, pe ? 1 : 0, gz1 ? 1 : 0, bare_plus(pe ? t2 : t1), cfg.md5,
                       cfg.lossy > 0.0 ? 1 : 0, tmpl};
        std::vector<uint8_t> tr(4096 + 40 * info.size());
        const int64_t tl = sa_arc_trailer(&ai, info.data(), (uint32_t)info.size(), tr.data(), tr.size());
        if (tl < 0) { fprintf(stderr, "seqarc_amd: trailer failed\n"); rc = 1; }
        else {
            fwrite(tr.data(), 1, (size_t)tl, fo);
            sa_arc_header(total, hdr);
            fseek(fo, 0, SEEK_SET);
            fwrite(hdr, 1, 16, fo);
            fprintf(stderr, "seqarc_amd: %lld block(s), %llu -> %llu bytes (%.2fx)\n", (long long)nb,
                    (unsigned long long)(t1.size() + t2.size()), (unsigned long long)(16 + total + tl),
                    (double)(t1.size() + t2.size()) / (double)(16 + total + tl));
        }
    }
    fclose(fo);
    return rc;
}
