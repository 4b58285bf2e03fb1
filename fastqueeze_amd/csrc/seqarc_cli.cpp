// seqarc_amd -- the SeqArc command line over libseqarc_amd (host C++).
//
//   seqarc_amd -i ref.fa                                                   -> ref.fa.hash, ref.fa.md5
//   seqarc_amd -c [options] [ref.fa] -1 A.fq[.gz] [-2 B.fq[.gz]] (-o OUT | OUT)  -> OUT.arc
//   seqarc_amd -d [options] [ref.fa] ARCHIVE.arc [PREFIX] [-o PREFIX]
//
//   ref.fa     the HASH index path (SeqArcContext::doBuildIndex@0x419db0 /
//              HashAlignment::buildRefIndex@0x410190 for -i; with -c the blocks
//              take EncapFqzComp::doAlignEncode@0x42d4c0, aligned on the GPU;
//              the index is read from ref.fa.hash, or built on the GPU if absent)
//   -I N       max insert size of PE alignment (param+0x28), --maxmis M (param+0x1b60, 7)
//   -t N       host threads that parse (-c) or decode (-d) blocks
//   -l R       R-Block lossy qualities (rblock@0x426c10)      -n  no per-block MD5
//   -f         overwrite existing outputs ("%s has exist!" otherwise, .rodata +0x877)
//   -p         outputs in the directory of the input (README.md "-p")
//   -P 1|2|3   decode to stdout: SE or PE1 reads / PE2 reads / each pair in order
//              (DecodePipeOutJob@0x42f930)
//   --slevel K --qlevel Q   the reference's developer options (./seqarc.config)
//   --devices N   GPUs (default 1), --contexts K   encoder contexts per GPU
//   --batch B     blocks per encode, --block-size MiB (default 50)
//   --share-device   all contexts on one GPU (tests of the multi-GPU gather)
//   --host-only      read, cut and parse only (no device; measures the host pipeline)
//   --host-parse     parse the blocks on host threads (default: on the device, sa_stage_text)
//   --read-threads N plain-file reader threads (default 16; 0: the per-block window reader)
//   --writers N      archive writer threads (default 8: page maps at the blocks' offsets; 1: write(2))
//   --ingest-only    the reader and block cut alone, batches dealt to devices x contexts
//                    consumers (no device); --ingest-crc: the consumers CRC the texts
//
// Compression mirrors SeqArc-1.6 main@0x41fd40 -> SeqArcContext::doReadAndEncode
// @0x41a4e0 as a stream: one reader thread cuts 50 MiB blocks as the input
// arrives (doReadJob@0x432a80 / doReadPEJob@0x432d10, plain or gzip), -t parser
// threads turn them into the SoA blocks (getBlockRead[PE]), the first block
// decides the ID template (IDProcess::analysisIDBinType@0x4310a0), encoder
// threads -- K contexts per GPU sharing one front scratch, batches dealt round
// robin -- encode batches of blocks, and this thread writes them in input order
// (the reference's -t 1 order; the copies on --writers threads) after a 16-byte header, then the trailer
// (SeqArcFile::writeFileInfo@0x4171b0).  The blocks in flight are bounded
// (ReadBufPool@0x4341e0 plays that role in the reference).
#include <dlfcn.h>
#include <emmintrin.h>
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/seqarc_amd.h"

namespace {

int usage()
{
    fprintf(stderr,
            "usage: seqarc_amd -c [-t N] [-l R] [-n] [-f] [-p] -1 A.fq[.gz] [-2 B.fq[.gz]] (-o OUT | OUT)\n"
            "                  [--slevel K] [--qlevel Q] [--devices N] [--contexts K] [--batch BLOCKS]\n"
            "                  [--block-size MiB] [--device D] [--share-device] [--ramp] [--release]\n"
            "                  [--stage-ahead] [--writers N] [--read-threads N]\n"
            "       seqarc_amd -d [-t N] [-f] [-p] [-P 1|2|3] [ref.fa] ARCHIVE.arc [PREFIX] [-o PREFIX]\n"
            "       seqarc_amd -i ref.fa            (HASH index: ref.fa.hash + ref.fa.md5)\n"
            "       (-s with -i / -c / -d and ref.fa: the index image in /dev/shm/<ref file name>)\n"
            "       (-c / -d with ref.fa: the reference path; -I N insert size, --maxmis M)\n");
    return 2;
}

bool slurp(const std::string& path, std::vector<uint8_t>& out)
{
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    const bool ok = n >= 0 && fread(out.data(), 1, out.size(), f) == out.size();
    fclose(f);
    return ok;
}

bool spill(const std::string& path, const uint8_t* p, size_t n)
{
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = fwrite(p, 1, n, f) == n;
    return fclose(f) == 0 && ok;
}

bool is_fasta_name(const std::string& s)
{
    for (const char* e : {".fa", ".fasta", ".fna"}) {
        const size_t l = strlen(e);
        if (s.size() > l && s.compare(s.size() - l, l, e) == 0) return true;
    }
    return false;
}

// The genome the index packs (k_hash_pack, buildRefIndex@0x410190: every
// line not starting with '>', up to strlen - 1 characters), 16 bases a word,
// 2 bits a base (code & 3: N reads as A), the last word left-aligned
bool pack_fasta(const std::vector<uint8_t>& fa, std::vector<uint32_t>& words, uint64_t& bases)
{
    words.clear();
    bases = 0;
    uint32_t w = 0;
    bool header = false;
    for (size_t at = 0; at < fa.size();) {
        const uint8_t* p = fa.data() + at;
        const uint8_t* e = (const uint8_t*)memchr(p, '\n', fa.size() - at);
        const size_t len = e ? (size_t)(e - p) + 1 : fa.size() - at;
        at += len;
        if (p[0] == '>') { header = true; continue; }
        const uint8_t* z = (const uint8_t*)memchr(p, 0, len);
        const size_t sl = z ? (size_t)(z - p) : len;
        if (sl <= 1) continue;
        if (!header) return false;
        for (size_t i = 0; i + 1 < sl; i++) {
            uint32_t c;
            switch (p[i] | 0x20) {
            case 'c': c = 1; break;
            case 'g': c = 2; break;
            case 't': c = 3; break;
            case 'm': c = 1; break;   // IUPAC codes 5..14, & 3
            case 'r': c = 2; break;
            case 'y': c = 3; break;
            case 'k': c = 0; break;
            case 's': c = 1; break;
            case 'w': c = 2; break;
            case 'h': c = 3; break;
            case 'b': c = 0; break;
            case 'v': c = 1; break;
            case 'd': c = 2; break;
            default: c = 0;   // A, N and anything else
            }
            w = (w << 2) | c;
            if (++bases % 16 == 0) { words.push_back(w); w = 0; }
        }
    }
    if (bases % 16) words.push_back(w << (2 * (16 - bases % 16)));
    if (words.empty()) words.push_back(0);
    return header;
}

std::string dir_of(const std::string& p)
{
    const size_t s = p.rfind('/');
    return s == std::string::npos ? std::string() : p.substr(0, s + 1);
}


// isFileExist@0x40cc50 + getFileSize@0x40cc10: an existing non-empty output
// stops the run unless -f (SeqArcParam::parseOptFromMem@0x407210)
bool may_write(const std::string& path, bool force)
{
    struct stat sb;
    if (!force && stat(path.c_str(), &sb) == 0 && sb.st_size > 0) {
        fprintf(stderr, "seqarc_amd: %s has exist!\n", path.c_str());
        return false;
    }
    return true;
}

// An uninitialised growable array (std::vector would zero-fill the tens of MB
// of every block's buffers, which costs more than parsing them).  `pinned`
// (set while empty): page-locked storage (sa_host_alloc), so that staging the
// text to the device is a DMA.
template <class T>
struct Buf {
    T* d = nullptr;
    size_t n = 0, cap = 0;
    bool pinned = false;
    bool external = false;   // d belongs to an arena (TextPool): never freed here
    bool huge = false;       // (set while empty) 2 MiB-aligned with the huge-page hint (OutPool)
    // how d was allocated (its allocator frees it, whatever the flags above ask
    // of the next allocation)
    enum Kind : uint8_t { K_NEW, K_ALIGNED, K_PINNED } kind = K_NEW;
    Buf() = default;
    Buf(const Buf&) = delete;
    Buf& operator=(const Buf&) = delete;
    Buf(Buf&& o) noexcept { take(o); }
    Buf& operator=(Buf&& o) noexcept
    {
        if (this != &o) {
            release();
            take(o);
        }
        return *this;
    }
    ~Buf() { release(); }
    void take(Buf& o)
    {
        d = o.d;
        n = o.n;
        cap = o.cap;
        pinned = o.pinned;
        external = o.external;
        huge = o.huge;
        kind = o.kind;
        o.d = nullptr;
        o.n = o.cap = 0;
        o.external = false;
    }
    void reserve(size_t c)
    {
        if (c <= cap) return;
        T* nd = pinned ? static_cast<T*>(sa_host_alloc(c * sizeof(T))) : nullptr;
        Kind nk = K_PINNED;
        if (!nd && huge) {
            void* q = nullptr;
            if (posix_memalign(&q, 2u << 20, c * sizeof(T)) == 0) {
                (void)madvise(q, c * sizeof(T), MADV_HUGEPAGE);
                nd = static_cast<T*>(q);
                nk = K_ALIGNED;
            }
        }
        if (!nd) {   // (pageable when page-locked memory runs out: staging is then a slower copy)
            nd = new T[c];
            nk = K_NEW;
        }
        if (n) memcpy(nd, d, n * sizeof(T));
        free_(d);   // (with the old buffer's own allocator)
        d = nd;
        kind = nk;
        cap = c;
        external = false;
        pinned = nk == K_PINNED;
    }
    void resize(size_t c)
    {
        reserve(c);
        n = c;
    }
    void free_(T* p)
    {
        if (!p || external) return;
        if (kind == K_PINNED) sa_host_free(p);
        else if (kind == K_ALIGNED) free(p);
        else delete[] p;
    }
    void release()
    {
        free_(d);
        d = nullptr;
        n = cap = 0;
        external = false;
    }
    T& operator[](size_t i) { return d[i]; }
    const T& operator[](size_t i) const { return d[i]; }
    T* data() { return d; }
    const T* data() const { return d; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
};

// byte buffers that resize without zero-filling (filled right after)
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept
    {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a)
    {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
using Bytes = std::vector<uint8_t, NoInitAlloc<uint8_t>>;

// ---- gzip input -------------------------------------------------------------
// The reference inflates with gzread on its reader thread.  Here a producer
// thread per input inflates ahead of the block cut into a bounded queue of
// chunks.  BGZF files (bgzip: gzip members of <= 64 KiB with the 'BC' extra
// field giving each member's size) are inflated in parallel: the producer reads
// a slab of members, `workers` threads inflate them into their places (each
// member's ISIZE gives its output size) and check their CRCs.  Other gzip files
// (one member, or several concatenated) inflate on the producer thread.
// BGZF members are whole raw-deflate streams of known output size: the
// system's libdeflate (whole-buffer decompression, PCLMUL CRC-32) inflates them
// at several times zlib 1.2.11's rate.  It is loaded at run time; without it
// the members go through zlib as before.  (Declared here: the image has the
// library but no header; these four entry points are libdeflate's stable API.)
struct LibDeflate {
    void* (*alloc)() = nullptr;
    int (*decompress)(void*, const void*, size_t, void*, size_t, size_t*) = nullptr;
    void (*release)(void*) = nullptr;
    uint32_t (*crc32)(uint32_t, const void*, size_t) = nullptr;
    LibDeflate()
    {
        if (std::getenv("SA_NO_LIBDEFLATE")) return;   // (A/B)
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = reinterpret_cast<void* (*)()>(dlsym(h, "libdeflate_alloc_decompressor"));
        decompress = reinterpret_cast<int (*)(void*, const void*, size_t, void*, size_t, size_t*)>(
            dlsym(h, "libdeflate_deflate_decompress"));
        release = reinterpret_cast<void (*)(void*)>(dlsym(h, "libdeflate_free_decompressor"));
        crc32 = reinterpret_cast<uint32_t (*)(uint32_t, const void*, size_t)>(dlsym(h, "libdeflate_crc32"));
        if (!alloc || !decompress || !release || !crc32) alloc = nullptr;
    }
    bool ok() const { return alloc != nullptr; }
};
const LibDeflate& libdeflate()
{
    static const LibDeflate d;
    return d;
}

// Inflate threads run at a lower priority than the encoder threads: those
// sleep on their streams and wake for a few host steps per batch, and with
// every core inflating they woke late (BGZF short leg, r4i: encode busy 14.3 s
// against 7.1 s on plain input).
void lower_priority()
{
    (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), 5);
}

struct GzStream {
    int fd = -1;
    int workers = 1;
    bool bgzf = false;
    std::thread prod;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Bytes> q;
    size_t q_bytes = 0;
    bool done = false, failed = false, stop = false;
    Bytes cur;
    size_t cur_at = 0;
    static constexpr size_t kMaxQueued = 512u << 20;

    bool start(int f, int w)
    {
        fd = f;
        workers = std::max(1, w);
        uint8_t h[18];
        const ssize_t r = ::pread(fd, h, sizeof h, 0);
        bgzf = r == 18 && h[0] == 0x1f && h[1] == 0x8b && h[2] == 8 && (h[3] & 4) && h[10] == 6 && h[11] == 0 &&
               h[12] == 'B' && h[13] == 'C' && h[14] == 2 && h[15] == 0;
        prod = std::thread([this]() {
            lower_priority();
            const bool ok = bgzf ? run_bgzf() : run_plain();
            std::lock_guard<std::mutex> g(mu);
            failed = !ok;
            done = true;
            cv.notify_all();
        });
        return true;
    }
    bool push(Bytes&& v)   // false: the reader went away
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || q_bytes < kMaxQueued; });
        if (stop) return false;
        q_bytes += v.size();
        q.push_back(std::move(v));
        cv.notify_all();
        return true;
    }
    long readn(uint8_t* dst, size_t n, uint64_t& at)
    {
        size_t got = 0;
        while (got < n) {
            const ssize_t r = ::pread(fd, dst + got, n - got, (off_t)(at + got));
            if (r < 0 && errno == EINTR) continue;
            if (r < 0) return -1;
            if (r == 0) break;
            got += (size_t)r;
        }
        at += got;
        return (long)got;
    }
    // one member or several concatenated (gzread's reading of them)
    bool run_plain()
    {
        z_stream z{};
        if (inflateInit2(&z, 15 + 16) != Z_OK) return false;
        std::vector<uint8_t> in(4u << 20);
        uint64_t at = 0;
        bool eof = false, member_end = false;
        Bytes out(8u << 20);
        size_t have = 0;
        for (;;) {
            if (z.avail_in == 0 && !eof) {
                const long r = readn(in.data(), in.size(), at);
                if (r < 0) { inflateEnd(&z); return false; }
                if (r == 0) eof = true;
                z.next_in = in.data();
                z.avail_in = (uInt)r;
            }
            if (z.avail_in == 0 && eof) break;
            if (member_end) {   // the next member, if it is one (trailing bytes otherwise end the stream)
                if (z.avail_in < 2 && !eof) {
                    // (rare: a member boundary at the end of a read slab) keep the byte, read more
                    memmove(in.data(), z.next_in, z.avail_in);
                    const long r = readn(in.data() + z.avail_in, in.size() - z.avail_in, at);
                    if (r < 0) { inflateEnd(&z); return false; }
                    if (r == 0) eof = true;
                    z.next_in = in.data();
                    z.avail_in += (uInt)r;
                }
                if (z.avail_in < 2 || z.next_in[0] != 0x1f || z.next_in[1] != 0x8b) break;
                inflateReset(&z);
                member_end = false;
            }
            z.next_out = out.data() + have;
            z.avail_out = (uInt)(out.size() - have);
            const int rc = inflate(&z, Z_NO_FLUSH);
            have = out.size() - z.avail_out;
            if (rc == Z_STREAM_END) member_end = true;
            else if (rc != Z_OK && rc != Z_BUF_ERROR) { inflateEnd(&z); return false; }
            else if (rc == Z_BUF_ERROR && z.avail_in == 0 && eof) { inflateEnd(&z); return false; }   // truncated
            if (have == out.size() || (member_end && have > (6u << 20))) {
                out.resize(have);
                if (!push(std::move(out))) { inflateEnd(&z); return true; }
                out = Bytes();
                out.resize(8u << 20);
                have = 0;
            }
        }
        inflateEnd(&z);
        if (!member_end && at > 0) return false;   // ended inside a member
        out.resize(have);
        if (have && !push(std::move(out))) return true;
        return true;
    }
    // BGZF: slabs of whole members; a pool of `workers` threads inflates the
    // members of up to kInFlight slabs (each member into its place, by its
    // ISIZE; CRC checked), while this thread reads and parses the next slab;
    // finished slabs leave in order.  (Round 3 started the workers per slab
    // and joined them before the next one: every slab waited for its slowest
    // member and the threads' start-up; the outputs were zero-filled first.)
    bool run_bgzf()
    {
        const size_t kSlab = 32u << 20;
        const size_t kInFlight = 4;
        struct Mem { size_t off, len; uint64_t out; uint32_t crc, isize; };
        struct Slab {
            std::vector<uint8_t> in;
            std::vector<Mem> ms;
            Bytes out;
            size_t next = 0, done = 0;
            bool bad = false;
        };
        std::mutex pm;
        std::condition_variable pcv;
        std::deque<std::unique_ptr<Slab>> jobs;   // in file order
        bool quit = false;
        auto work = [&]() {
            lower_priority();
            const LibDeflate& ld = libdeflate();
            void* dd = ld.ok() ? ld.alloc() : nullptr;
            z_stream z{};
            const bool ok = dd ? true : inflateInit2(&z, -15) == Z_OK;
            std::unique_lock<std::mutex> lk(pm);
            for (;;) {
                Slab* s = nullptr;
                pcv.wait(lk, [&] {
                    if (quit) return true;
                    for (auto& j : jobs)
                        if (j->next < j->ms.size()) return true;
                    return false;
                });
                if (quit) break;
                for (auto& j : jobs)
                    if (j->next < j->ms.size()) { s = j.get(); break; }
                const size_t i = s->next++;
                lk.unlock();
                const Mem& m = s->ms[i];
                bool bad = !ok;
                if (ok && m.isize == 0) {   // (the BGZF end-of-file marker: an empty member)
                    bad = m.crc != 0;
                } else if (dd) {
                    size_t got = 0;
                    const int rc = ld.decompress(dd, s->in.data() + m.off, m.len, s->out.data() + m.out, m.isize, &got);
                    bad = rc != 0 || got != m.isize || ld.crc32(0, s->out.data() + m.out, m.isize) != m.crc;
                } else if (ok) {
                    inflateReset(&z);
                    z.next_in = s->in.data() + m.off;
                    z.avail_in = (uInt)m.len;
                    z.next_out = s->out.data() + m.out;
                    z.avail_out = (uInt)m.isize;
                    const int rc = inflate(&z, Z_FINISH);
                    bad = rc != Z_STREAM_END || z.avail_out != 0 ||
                          crc32(0L, s->out.data() + m.out, (uInt)m.isize) != m.crc;
                }
                lk.lock();
                s->bad |= bad;
                if (++s->done == s->ms.size()) pcv.notify_all();
            }
            if (dd) ld.release(dd);
            else if (ok) inflateEnd(&z);
        };
        std::vector<std::thread> pool;
        for (int k = 0; k < workers; k++) pool.emplace_back(work);
        auto finish = [&](bool rc) {
            {
                std::lock_guard<std::mutex> g(pm);
                quit = true;
            }
            pcv.notify_all();
            for (auto& t : pool) t.join();
            return rc;
        };
        // the oldest slab, once inflated, to the reader (false: failed or the reader went away)
        auto retire = [&](bool& stopped) -> bool {
            std::unique_ptr<Slab> s;
            {
                std::unique_lock<std::mutex> lk(pm);
                pcv.wait(lk, [&] { return jobs.front()->done == jobs.front()->ms.size(); });
                s = std::move(jobs.front());
                jobs.pop_front();
            }
            if (s->bad) return false;
            if (!s->out.empty() && !push(std::move(s->out))) stopped = true;
            return true;
        };
        std::vector<uint8_t> carry_buf;   // a member cut by the end of the previous slab
        uint64_t at = 0;
        bool eof = false, stopped = false;
        while (!eof || !carry_buf.empty()) {
            std::unique_ptr<Slab> s(new Slab());
            s->in.resize(kSlab);
            const size_t c0 = carry_buf.size();
            if (c0) memcpy(s->in.data(), carry_buf.data(), c0);
            carry_buf.clear();
            const long r = eof ? 0 : readn(s->in.data() + c0, kSlab - c0, at);
            if (r < 0) return finish(false);
            if ((size_t)r < kSlab - c0) eof = true;
            const size_t have = c0 + (size_t)r;
            size_t p = 0;
            uint64_t total = 0;
            while (p + 18 <= have) {
                const uint8_t* h = s->in.data() + p;
                if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return finish(false);
                const size_t xlen = h[10] | (size_t)h[11] << 8;
                size_t bsize = 0;
                for (size_t x = 12; x + 4 <= 12 + xlen && p + x + 4 <= have;) {   // the 'BC' subfield
                    const size_t sl = h[x + 2] | (size_t)h[x + 3] << 8;
                    if (h[x] == 'B' && h[x + 1] == 'C' && sl == 2) bsize = (h[x + 4] | (size_t)h[x + 5] << 8) + 1;
                    x += 4 + sl;
                }
                if (!bsize || bsize < 12 + xlen + 8) return finish(false);   // not BGZF after all
                if (p + bsize > have) break;                                // the member continues in the next slab
                const uint8_t* t = h + bsize - 8;
                const Mem m{p + 12 + xlen, bsize - 12 - xlen - 8, total,
                            (uint32_t)(t[0] | t[1] << 8 | t[2] << 16 | (uint32_t)t[3] << 24),
                            (uint32_t)(t[4] | t[5] << 8 | t[6] << 16 | (uint32_t)t[7] << 24)};
                total += m.isize;
                s->ms.push_back(m);
                p += bsize;
            }
            if (s->ms.empty()) {
                if (eof && have == 0) break;
                return finish(false);   // a truncated or oversized member, or trailing bytes that are no member
            }
            carry_buf.assign(s->in.begin() + (std::ptrdiff_t)p, s->in.begin() + (std::ptrdiff_t)have);
            if (eof && !carry_buf.empty() && carry_buf.size() < 18) return finish(false);
            s->out.resize(total);   // (default-initialised: no zero fill)
            {
                std::lock_guard<std::mutex> g(pm);
                jobs.push_back(std::move(s));
            }
            pcv.notify_all();
            size_t n;
            {
                std::lock_guard<std::mutex> g(pm);
                n = jobs.size();
            }
            if (n >= kInFlight && !retire(stopped)) return finish(false);
            if (stopped) return finish(true);
        }
        for (;;) {
            {
                std::lock_guard<std::mutex> g(pm);
                if (jobs.empty()) break;
            }
            if (!retire(stopped)) return finish(false);
            if (stopped) return finish(true);
        }
        return finish(true);
    }
    // up to n bytes into dst; 0 at the end; -1 on a gzip error
    long read(uint8_t* dst, size_t n)
    {
        size_t got = 0;
        while (got < n) {
            if (cur_at == cur.size()) {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !q.empty() || done; });
                if (q.empty()) {
                    if (failed) return -1;
                    break;
                }
                cur = std::move(q.front());
                q.pop_front();
                q_bytes -= cur.size();
                cur_at = 0;
                cv.notify_all();
            }
            const size_t k = std::min(n - got, cur.size() - cur_at);
            memcpy(dst + got, cur.data() + cur_at, k);
            cur_at += k;
            got += k;
        }
        return (long)got;
    }
    ~GzStream()
    {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
            cv.notify_all();
        }
        if (prod.joinable()) prod.join();
    }
};

// ---- input ---------------------------------------------------------------
// getFileType@0x40d9f0 (gzip magic); plain files are read with read(2) /
// parallel pread slices, gzip through a GzStream (inflated ahead, BGZF in
// parallel).
int g_gz_workers = 8;   // inflate threads per BGZF input (-t / 2 for PE)

struct Input {
    int fd = -1;
    std::unique_ptr<GzStream> gz;
    bool is_gz = false, eof = false, seekable = true;
    uint64_t off = 0;   // file offset of the next byte (plain files)
    bool open(const char* path)
    {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) return false;
        unsigned char m[2] = {0, 0};
        is_gz = ::pread(fd, m, 2, 0) == 2 && m[0] == 0x1f && m[1] == 0x8b;
        if (is_gz) {
            gz.reset(new GzStream());
            gz->start(fd, g_gz_workers);
        }
        return true;
    }
    // A plain file is read in slices by several threads at once (pread): one
    // thread copies ~4 GB/s out of the page cache, below the device's rate.
    long pread_all(uint8_t* dst, size_t n, uint64_t at)
    {
        size_t got = 0;
        while (got < n) {
            const ssize_t r = ::pread(fd, dst + got, n - got, (off_t)(at + got));
            if (r < 0 && errno == EINTR) continue;
            if (r < 0) return -1;
            if (r == 0) break;
            got += (size_t)r;
        }
        return (long)got;
    }
    // appends up to n bytes to b; false on a read error
    bool fill(Buf<uint8_t>& b, size_t n)
    {
        size_t have = b.size();
        b.resize(have + n);
        const size_t kSlice = 8u << 20;
        if (!is_gz && seekable && !eof && n >= 2 * kSlice) {
            // (four slices: the box's CPU share is a cgroup quota -- more copy
            // threads throttle the whole process, encoder threads included)
            const size_t ns = std::min<size_t>(4, n / kSlice), part = (n + ns - 1) / ns;
            std::vector<std::future<long>> fs;
            for (size_t i = 1; i < ns; i++) {
                const size_t s0 = i * part, len = std::min(n, s0 + part) - s0;
                fs.push_back(std::async(std::launch::async,
                                        [this, &b, have, s0, len]() { return pread_all(b.data() + have + s0, len, off + s0); }));
            }
            const long r0 = pread_all(b.data() + have, std::min(n, part), off);
            std::vector<long> rs{r0};
            for (auto& f : fs) rs.push_back(f.get());
            if (r0 >= 0 || errno != ESPIPE) {
                size_t got = 0;
                for (size_t i = 0; i < rs.size(); i++) {
                    if (rs[i] < 0) { b.resize(have); return false; }
                    const size_t want = std::min(n, i * part + part) - i * part;
                    got += (size_t)rs[i];
                    if ((size_t)rs[i] < want) {   // end of file inside slice i
                        eof = true;
                        break;
                    }
                }
                off += got;
                b.resize(have + got);
                return true;
            }
            seekable = false;   // a pipe: sequential reads below
        }
        size_t got = 0;
        while (got < n && !eof) {
            long r;
            if (is_gz) {
                r = gz->read(b.data() + have + got, n - got);
            } else {
                r = (long)::read(fd, b.data() + have + got, n - got);
                if (r < 0 && errno == EINTR) continue;
                if (r > 0) off += (uint64_t)r;
            }
            if (r < 0) { b.resize(have + got); return false; }
            if (r == 0) eof = true;
            got += (size_t)r;
        }
        b.resize(have + got);
        return true;
    }
    ~Input()
    {
        gz.reset();
        if (fd >= 0) ::close(fd);
    }
};

// Newlines in t[0, len): 64 bytes a step (compare, movemask, popcount).
uint64_t count_newlines(const uint8_t* t, uint64_t len)
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

// ---- plain files: read ahead in segments (round 5) -------------------------
// The input files are read in segments of S bytes plus an overlap of W bytes
// (one block window: bs / 2 + 64 KiB for PE, bs + 64 KiB for SE), so that every
// window that starts inside a segment lies inside it, into a ring of R
// page-locked buffers per file.  A pool of fill threads copies 4 MiB slices out
// of the page cache (pread: one thread copies ~7 GB/s, eight ~58 GB/s on the
// GPU box, profiles/round5_r5a_ingest_probe.txt) and counts the newlines of
// every 256 KiB chunk of the slice while it is in cache.  The cut then reads a
// window's newline count off the chunk counts (cultPEbuf@0x432180 counts both
// windows' newlines: sa_cut_next_pe_nl) and walks back from the window's end as
// before, and a block is a view into its segment -- no per-block window, no
// carry copy.  A segment's slot is refilled once the cut has moved past it and
// every block in it was staged (its text copied to the device) or parsed.
struct SegReader {
    static constexpr uint64_t kSlice = 4ull << 20, kChunk = 256ull << 10;
    struct Seg {
        uint8_t* p = nullptr;
        uint64_t cap = 0;           // bytes of p
        int64_t idx = -1;           // segment number held (-1: none yet)
        uint64_t base = 0, len = 0;
        uint32_t nslices = 0, next_slice = 0, done = 0;
        int refs = 0;               // blocks (and the cut) still reading it
        bool ready = false;         // p is allocated for this segment
        bool filled = false;
    };
    struct File {
        int fd = -1;
        uint64_t size = 0;
        int64_t nseg = 0;
        int64_t next_start = 0;     // next segment number to start filling
        int64_t low = 0;            // the cut's segment (the lower ones are free once their refs are 0)
        std::vector<uint32_t> nl;   // newlines per kChunk of the file (the segments' primary parts)
        std::vector<Seg> ring;
    };
    File f[2];
    int nf = 1;
    uint64_t S = 0, W = 0;
    bool pinned = false, failed = false, stop = false;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::thread> workers;
    std::atomic<uint64_t> alloc_bytes{0};
    double fill_s = 0;   // fill threads' busy time (under mu)

    // fds: open plain regular files; W: the cut's window
    bool start(const int* fds, const uint64_t* sizes, int n, uint64_t window, int64_t ahead_bytes, int threads,
               bool pin, uint64_t batch_blocks = 1)
    {
        nf = n;
        W = window;
        pinned = pin;
        uint64_t mx = 0;
        for (int i = 0; i < n; i++) mx = std::max(mx, sizes[i]);
        // segments of 512 MiB (a small input: one segment; SA_CLI_SEG_SLICES=n: n slices, for the tests)
        // (round 5: 256 MiB, SA_CLI_SEG_MIB to change: the ring is unmapped at the
        // end, ~25 GB/s of page-locked memory, and while device work runs the
        // unmapping stalls it -- a smaller ring costs less of both, r5x)
        const char* sm = std::getenv("SA_CLI_SEG_MIB");
        const uint64_t smax = (uint64_t)(sm ? std::max(4, std::atoi(sm)) : 256) << 20;
        S = std::max<uint64_t>(kSlice, std::min<uint64_t>(smax, (mx + kSlice - 1) / kSlice * kSlice));
        if (const char* e = std::getenv("SA_CLI_SEG_SLICES")) S = kSlice * std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
        int R = (int)std::max<int64_t>(3, (ahead_bytes + (int64_t)S - 1) / (int64_t)S + 3);
        // (A/B) SA_CLI_RING_SEGS=n: n segments per file.  The ring is page-locked
        // once, at ~12 GB/s for the whole process (hipHostRegister does not scale
        // with threads, profiles/round5_r5a_ingest_probe.txt): a smaller ring
        // costs less of it before the first pass over it completes
        if (const char* e = std::getenv("SA_CLI_RING_SEGS")) R = std::max(3, std::atoi(e));
        // (at least a batch of windows and two segments of slack: the blocks of
        // a batch keep their segments until the batch is staged; r5i: a ring of
        // four 512 MiB segments deadlocked a 69-block batch)
        R = std::max<int>(R, (int)(((uint64_t)batch_blocks * window + S - 1) / S) + 2);
        for (int i = 0; i < n; i++) {
            File& F = f[i];
            F.fd = fds[i];
            F.size = sizes[i];
            F.nseg = (int64_t)((F.size + S - 1) / S);
            F.nl.assign((size_t)(F.size / kChunk + 1), 0);
            F.ring.resize((size_t)std::max<int64_t>(1, std::min<int64_t>(R, F.nseg)));
        }
        for (int t = 0; t < std::max(1, threads); t++) workers.emplace_back([this]() { work(); });
        return true;
    }
    ~SegReader() { free_all(); }
    // the fill threads stopped, the segments' page-locked memory released (once
    // every block was staged: off the exit, where unpinning ~10 GB took ~0.5 s)
    void free_all()
    {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
            cv.notify_all();
        }
        for (auto& t : workers) t.join();
        workers.clear();
        // (on up to SA_CLI_FREE_THREADS threads, default 8: releasing ~10 GB of
        // page-locked segments one by one took ~0.47 s past the last encode, r5m)
        std::vector<Seg*> all;
        for (int i = 0; i < nf; i++)
            for (Seg& s : f[i].ring) all.push_back(&s);
        const char* e = std::getenv("SA_CLI_FREE_THREADS");
        const size_t nt = std::min<size_t>(all.size(), e ? (size_t)std::max(1, std::atoi(e)) : 8);
        std::vector<std::thread> th;
        for (size_t t = 1; t < nt; t++)
            th.emplace_back([&, t]() {
                for (size_t k = t; k < all.size(); k += nt) free_buf(*all[k]);
            });
        for (size_t k = 0; k < all.size(); k += std::max<size_t>(nt, 1)) free_buf(*all[k]);
        for (auto& t : th) t.join();
    }
    void free_buf(Seg& s)
    {
        if (!s.p) return;
        if (pinned) sa_host_free(s.p);
        else free(s.p);
        s.p = nullptr;
        s.cap = 0;
    }
    // under mu: a slice to fill (file, segment slot, slice), starting a segment when its slot is free
    bool pick(int& fi, Seg*& sg, uint32_t& sl, bool& must_alloc)
    {
        int best = -1;
        uint64_t best_off = ~0ull;
        for (int i = 0; i < nf; i++) {
            File& F = f[i];
            // the lowest segment with slices left, else the next one to start
            Seg* cand = nullptr;
            for (int64_t k = std::max<int64_t>(0, F.next_start - (int64_t)F.ring.size()); k < F.next_start; k++) {
                Seg& s = F.ring[(size_t)(k % (int64_t)F.ring.size())];
                if (s.idx == k && s.ready && s.next_slice < s.nslices) {
                    cand = &s;
                    break;
                }
            }
            uint64_t off;
            if (cand) {
                off = cand->base + (uint64_t)cand->next_slice * kSlice;
            } else {
                if (F.next_start >= F.nseg) continue;
                Seg& s = F.ring[(size_t)(F.next_start % (int64_t)F.ring.size())];
                const bool free_slot = s.idx < 0 || (s.refs == 0 && s.idx < F.low && s.filled);
                if (!free_slot) continue;
                off = (uint64_t)F.next_start * S;
            }
            if (off < best_off) {
                best_off = off;
                best = i;
                sg = cand;
            }
        }
        if (best < 0) return false;
        fi = best;
        File& F = f[best];
        must_alloc = false;
        if (!sg) {   // start segment next_start in its slot
            Seg& s = F.ring[(size_t)(F.next_start % (int64_t)F.ring.size())];
            s.idx = F.next_start++;
            s.base = (uint64_t)s.idx * S;
            s.len = std::min<uint64_t>(S + W, F.size - s.base);
            s.nslices = (uint32_t)((s.len + kSlice - 1) / kSlice);
            s.next_slice = s.done = 0;
            s.filled = false;
            s.ready = s.cap >= s.len;
            must_alloc = !s.ready;
            sg = &s;
        }
        sl = sg->next_slice++;
        return true;
    }
    void work()
    {
        for (;;) {
            int fi = 0;
            Seg* sg = nullptr;
            uint32_t sl = 0;
            bool must_alloc = false;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || failed || pick(fi, sg, sl, must_alloc); });
                if (stop || failed) return;
            }
            const auto t0 = std::chrono::steady_clock::now();
            if (must_alloc) {   // (one worker per segment; the others wait for `ready`)
                free_buf(*sg);
                const uint64_t want = std::max<uint64_t>(sg->len, std::min<uint64_t>(S + W, f[fi].size));
                void* p = pinned ? sa_host_alloc(want) : nullptr;
                if (!p) {   // (no device: pageable, on huge pages where the kernel has them)
                    if (posix_memalign(&p, 2u << 20, want) != 0) p = nullptr;
                    else (void)madvise(p, want, MADV_HUGEPAGE);
                }
                std::lock_guard<std::mutex> g(mu);
                if (!p) {
                    failed = true;
                    cv.notify_all();
                    return;
                }
                alloc_bytes += want;
                sg->p = static_cast<uint8_t*>(p);
                sg->cap = want;
                sg->ready = true;
                cv.notify_all();
            }
            const uint64_t a = (uint64_t)sl * kSlice, n = std::min<uint64_t>(kSlice, sg->len - a);
            uint64_t got = 0;
            while (got < n) {
                const ssize_t r = ::pread(f[fi].fd, sg->p + a + got, n - got, (off_t)(sg->base + a + got));
                if (r < 0 && errno == EINTR) continue;
                if (r <= 0) break;
                got += (uint64_t)r;
            }
            // newlines of the slice's whole chunks in the segment's primary part
            const uint64_t fa = sg->base + a, fe = std::min(sg->base + a + got, std::min(sg->base + S, f[fi].size));
            for (uint64_t c = fa / kChunk; (c + 1) * kChunk <= fe && c * kChunk >= fa; c++)
                f[fi].nl[(size_t)c] = (uint32_t)count_newlines(sg->p + (c * kChunk - sg->base), kChunk);
            std::lock_guard<std::mutex> g(mu);
            fill_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (got < n) {
                failed = true;   // (the file shrank under us)
            } else if (++sg->done == sg->nslices) {
                sg->filled = true;
            }
            cv.notify_all();
        }
    }
    // the cut's window at file offset off: waits for its segment, takes a
    // reference for the block (release(fi, seg)), returns the bytes available
    // from off within the segment; nullptr on a read failure
    const uint8_t* window(int fi, uint64_t off, uint64_t& avail, int64_t& seg)
    {
        File& F = f[fi];
        const int64_t k = std::min<int64_t>((int64_t)(off / S), std::max<int64_t>(F.nseg - 1, 0));
        std::unique_lock<std::mutex> lk(mu);
        F.low = k;
        cv.notify_all();
        Seg& s = F.ring[(size_t)(k % (int64_t)F.ring.size())];
        cv.wait(lk, [&] { return failed || (s.idx == k && s.filled); });
        if (failed) return nullptr;
        s.refs++;
        seg = k;
        avail = s.base + s.len - off;
        return s.p + (off - s.base);
    }
    void release(int fi, int64_t seg)
    {
        if (seg < 0) return;
        std::lock_guard<std::mutex> g(mu);
        Seg& s = f[fi].ring[(size_t)(seg % (int64_t)f[fi].ring.size())];
        if (s.idx == seg && s.refs > 0) s.refs--;
        cv.notify_all();
    }
    // the cut has passed every segment (the end of the input)
    void finish()
    {
        std::lock_guard<std::mutex> g(mu);
        for (int i = 0; i < nf; i++) f[i].low = f[i].nseg;
        cv.notify_all();
    }
    // newlines in [off, off + len) of file fi, inside the segment that holds off
    // (filled): whole chunks of its primary part from the chunk counts, the rest counted
    uint64_t newlines(int fi, uint64_t off, uint64_t len, const uint8_t* at_off)
    {
        const uint64_t seg_base = off / S * S, prim_end = seg_base + S, e = off + len;
        const uint64_t e1 = std::min(e, prim_end);
        uint64_t n = 0;
        const uint64_t ca = (off + kChunk - 1) / kChunk, cb = e1 / kChunk;
        if (ca >= cb) {
            n += count_newlines(at_off, e1 - off);
        } else {
            n += count_newlines(at_off, ca * kChunk - off);
            for (uint64_t c = ca; c < cb; c++) n += f[fi].nl[(size_t)c];
            n += count_newlines(at_off + (cb * kChunk - off), e1 - cb * kChunk);
        }
        if (e > prim_end) n += count_newlines(at_off + (prim_end - off), e - prim_end);
        return n;
    }
};

struct Parsed {
    // (not page-locked: hipHostRegister from the parser threads serialised in
    // the driver -- 129 s of parser time for 14 GB, r2p; pageable staging from
    // five contexts reaches ~19 GB/s, scripts/probe_h2d.py)
    Buf<uint8_t> names, seq, qual;
    Buf<uint16_t> nl;
    Buf<int32_t> sl;
    uint32_t nreads = 0;
    uint64_t text1 = 0, text2 = 0;
    sa_block view() const { return sa_block{names.data(), nl.data(), seq.data(), sl.data(), qual.data(), nreads}; }
};

// Parsed blocks are recycled: a later block reuses their buffers instead of
// faulting in fresh pages (~150 MB per block).
struct ParsedPool {
    std::mutex mu;
    std::vector<std::unique_ptr<Parsed>> free;
    std::unique_ptr<Parsed> get()
    {
        std::lock_guard<std::mutex> g(mu);
        if (free.empty()) return std::unique_ptr<Parsed>(new Parsed());
        std::unique_ptr<Parsed> p = std::move(free.back());
        free.pop_back();
        return p;
    }
    void put(std::unique_ptr<Parsed> p)
    {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu);
        free.push_back(std::move(p));
    }
};

// Text windows are recycled too: a fresh 25-50 MiB allocation per block is
// mapped anew and faults in every page on the first read into it.
//
// Device parse: the windows are page-locked, carved from arena chunks of
// kChunk windows each -- one sa_host_alloc per chunk, not per window (the
// runtime serialises host allocations against the encoder threads' calls).
struct TextPool {
    static constexpr size_t kChunk = 16;
    std::mutex mu;
    std::vector<Buf<uint8_t>> free;
    std::vector<void*> chunks;
    bool pinned = false;   // new windows in page-locked memory (device parse)
    size_t win = 0;        // window bytes of the arena (set before the first get)
    // (-v) chunks pinned on demand by the reader, and when the last one was
    std::atomic<uint32_t> on_demand{0};
    std::atomic<double> last_on_demand{0.0};
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~TextPool()
    {
        free.clear();
        for (void* c : chunks) sa_host_free(c);
    }
    void add_locked(uint8_t* c)
    {
        chunks.push_back(c);
        for (size_t k = 0; k < kChunk; k++) {
            Buf<uint8_t> b;
            b.pinned = true;
            b.external = true;
            b.d = c + k * win;
            b.cap = win;
            free.push_back(std::move(b));
        }
    }
    // one more chunk of windows, pinned outside the lock (the prefill thread:
    // pinning runs beside the contexts' creation and the reader's first reads)
    bool grow()
    {
        if (!pinned || !win) return false;
        uint8_t* c = static_cast<uint8_t*>(sa_host_alloc(kChunk * win));
        if (!c) return false;
        std::lock_guard<std::mutex> g(mu);
        add_locked(c);
        return true;
    }
    Buf<uint8_t> get()
    {
        std::lock_guard<std::mutex> g(mu);
        if (free.empty() && pinned && win)
            if (uint8_t* c = static_cast<uint8_t*>(sa_host_alloc(kChunk * win))) {
                add_locked(c);
                on_demand++;
                last_on_demand = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            }
        if (free.empty()) {
            Buf<uint8_t> b;
            b.pinned = pinned;
            return b;
        }
        Buf<uint8_t> b = std::move(free.back());
        free.pop_back();
        b.n = 0;
        return b;
    }
    void put(Buf<uint8_t>& b)
    {
        if (!b.cap) return;
        std::lock_guard<std::mutex> g(mu);
        free.push_back(std::move(b));
        b.n = b.cap = 0;
    }
};

// The encoded blocks' host buffers, recycled (round 5): a fresh buffer per
// block is a fresh mapping that the runtime's device-to-host copy faults in
// (and may page-lock) and that is unmapped again once the block is written,
// every batch.  The pool keeps them for the next batch's blocks; the virtual
// size is the output bound (~2x the block's symbols), only the written bytes
// are ever touched.  SA_CLI_OUT_POOL=0: a fresh buffer per block (A/B).
struct OutPool {
    std::mutex mu;
    std::vector<Buf<uint8_t>> free;
    const bool on = !(std::getenv("SA_CLI_OUT_POOL") && std::atoi(std::getenv("SA_CLI_OUT_POOL")) == 0);
    void take(Buf<uint8_t>& b, size_t n)
    {
        if (on && !b.cap) {
            std::lock_guard<std::mutex> g(mu);
            if (!free.empty()) {
                b = std::move(free.back());
                free.pop_back();
            }
        }
        if (on && !b.cap) b.huge = true;   // (huge pages: the copies' page-locking is undone 2x faster at the exit, pin_probe)
        if (on && b.cap < n) b.reserve(n + n / 8);   // (slack: the next block's bound may be a little larger)
        b.resize(n);
    }
    void give(Buf<uint8_t>& b)
    {
        if (!on || !b.cap) return;
        std::lock_guard<std::mutex> g(mu);
        free.push_back(std::move(b));
    }
};

struct Job {                     // one block between the reader and the writer
    Buf<uint8_t> t1, t2;          // its FASTQ text (recycled once parsed / staged; a view into a SegReader segment)
    SegReader* segr = nullptr;    // (views: the segments' references, released with the text)
    int64_t seg[2] = {-1, -1};
    uint64_t text1 = 0, text2 = 0;   // its text bytes in input 1 / 2
    uint32_t nreads = 0, len_long = 0;
    std::unique_ptr<Parsed> p;     // host parse (--host-parse; block 0 for the ID template)
    Buf<uint8_t> out;             // the encoded block
    int state = 0;                // 0 read, 1 parsed, 2 encoded
    uint32_t crc = 0;             // --ingest-only: CRC-32 of t1 then t2 (the writer folds them in order)
};

// The archive file, written by several threads (round 5).  A block's place
// is known once the blocks before it are (the writer hands them over in input
// order with their offsets); a pool of threads copies each block into a map
// of its page range, and a fallocate thread allocates the file's pages ahead
// of the copies.  One stream of fwrite ran at 1.2 GB/s into tmpfs and the last
// batch's ~450 MB held the run's end 0.39 s after its encode (r5j); the maps
// on 8 threads over allocated pages take 2 GB at ~10 GB/s (2 GB without the
// allocation ahead: 4 GB/s; with MAP_POPULATE: 1 GB/s).  Not a regular file
// (a pipe, a device): one thread, write(2) in order.
class ArcWriter {
public:
    using Done = std::function<void(std::unique_ptr<Job>)>;
    bool open(const std::string& path, int threads, Done done)
    {
        done_ = std::move(done);
        fd_ = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
        if (fd_ < 0) return false;
        struct stat st;
        mapped_ = fstat(fd_, &st) == 0 && S_ISREG(st.st_mode) && threads > 1;
        const int n = mapped_ ? threads : 1;
        for (int i = 0; i < n; i++) pool_.emplace_back([this] { work(); });
        if (mapped_) fa_ = std::thread([this] { allocate(); });
        return true;
    }
    // block j (its encoded bytes j->out) at byte off; the blocks come in order
    void put(std::unique_ptr<Job> j, uint64_t off)
    {
        const uint64_t end = off + j->out.size();
        std::lock_guard<std::mutex> g(mu_);
        if (mapped_ && end > size_) {   // (grown a GiB at a time; cut to the archive's size in finish)
            const uint64_t s = std::max<uint64_t>(end, size_ + (1ull << 30));
            if (ftruncate(fd_, (off_t)s) == 0) size_ = s;   // (else the copies past size_ use pwrite: no map past EOF)
            else bad_ = true;
        }
        end_ = end;
        q_.emplace_back(std::move(j), off);
        cv_.notify_all();
    }
    bool bad() const { return bad_.load(); }
    // every block written; the archive cut to tail_off, the trailer written there, the header at 0
    bool finish(const uint8_t* tail, size_t tn, uint64_t tail_off, const uint8_t* hdr, size_t hn)
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
            cv_.notify_all();
        }
        for (auto& t : pool_) t.join();
        if (fa_.joinable()) fa_.join();
        pool_.clear();
        if (fd_ < 0) return false;
        bool ok = !bad_;
        if (mapped_ && ftruncate(fd_, (off_t)tail_off) != 0) ok = false;
        if (tail && !put_at(tail, tn, tail_off)) ok = false;
        if (hdr && pwrite(fd_, hdr, hn, 0) != (ssize_t)hn) ok = false;   // (a pipe: ESPIPE, as fseek was)
        if (::close(fd_) != 0) ok = false;
        fd_ = -1;
        return ok && hdr;
    }
    // the reserved header bytes at 0 (before the first block)
    bool lead(const uint8_t* p, size_t n) { return put_at(p, n, 0); }
    ~ArcWriter()
    {
        if (fd_ >= 0) finish(nullptr, 0, 0, nullptr, 0);
    }

private:
    static constexpr uint64_t kAhead = 768ull << 20, kStep = 64ull << 20;
    bool put_at(const uint8_t* p, size_t n, uint64_t off)
    {
        if (!mapped_) {   // (in order: lead, the blocks, then the trailer)
            while (n) {
                const ssize_t w = ::write(fd_, p, n);
                if (w <= 0) return false;
                p += w;
                n -= (size_t)w;
            }
            return true;
        }
        while (n) {
            const ssize_t w = pwrite(fd_, p, n, (off_t)off);
            if (w <= 0) return false;
            p += w;
            n -= (size_t)w;
            off += (uint64_t)w;
        }
        return true;
    }
    // A block is copied into a map of its pages only where fallocate has
    // allocated them (alloc_upto_ <= size_): a store to a page the file system
    // cannot back (disk full, quota) raises SIGBUS and would kill the process
    // with a partial archive; everywhere else pwrite, whose errors are reported.
    bool copy(const uint8_t* p, size_t n, uint64_t off)
    {
        if (!n) return true;
        if (!mapped_ || off + n > alloc_upto_.load()) return put_at(p, n, off);
        static const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE);
        const uint64_t a = off & ~(pg - 1), len = off + n - a;
        void* m = mmap(nullptr, len, PROT_WRITE, MAP_SHARED, fd_, (off_t)a);
        if (m == MAP_FAILED) return put_at(p, n, off);
        memcpy(static_cast<uint8_t*>(m) + (off - a), p, n);
        munmap(m, len);
        return true;
    }
    void work()
    {
        for (;;) {
            std::unique_ptr<Job> j;
            uint64_t off = 0;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                j = std::move(q_.front().first);
                off = q_.front().second;
                q_.pop_front();
                cv_.notify_all();   // (the allocation ahead follows the queue's head)
            }
            if (!copy(j->out.data(), j->out.size(), off)) bad_ = true;
            done_(std::move(j));
        }
    }
    void allocate()   // the file's pages, kAhead beyond the last block handed over
    {
        uint64_t at = 0;
        for (;;) {
            uint64_t to;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || std::min(end_ + kAhead, size_) > at; });
                if (stop_) return;
                to = std::min(std::min(end_ + kAhead, size_), at + kStep);
            }
            // (a failure -- no space, a quota, unsupported -- ends the allocation:
            // the copies past alloc_upto_ then write with pwrite and report errors)
            if (fallocate(fd_, FALLOC_FL_KEEP_SIZE, (off_t)at, (off_t)(to - at)) != 0) return;
            at = to;
            alloc_upto_ = at;
        }
    }
    int fd_ = -1;
    bool mapped_ = false;
    Done done_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::pair<std::unique_ptr<Job>, uint64_t>> q_;
    uint64_t size_ = 0, end_ = 0;
    std::atomic<uint64_t> alloc_upto_{0};   // bytes of the file fallocate has allocated (from 0)
    bool stop_ = false;
    std::atomic<bool> bad_{false};
    std::vector<std::thread> pool_;
    std::thread fa_;
};

// getFirstLine@0x431eb0: the '+' line of the first record carries no ID
int bare_plus(const uint8_t* t, size_t n)
{
    size_t nl[3] = {0, 0, 0};
    int k = 0;
    for (size_t i = 0; i < n && k < 3; i++)
        if (t[i] == '\n') nl[k++] = i + 1;
    if (k < 3) return 1;
    return nl[2] - nl[1] > 2 ? 0 : 1;
}

// a block's text back to the reader: its windows recycled, its segment references dropped
void give_back(Job& j, TextPool& texts)
{
    texts.put(j.t1);
    texts.put(j.t2);
    if (j.segr) {
        j.segr->release(0, j.seg[0]);
        j.segr->release(1, j.seg[1]);
    }
    j.seg[0] = j.seg[1] = -1;
}

bool parse_job(Job& j, bool pe, ParsedPool& pool, TextPool& texts, bool keep_text)
{
    const uint64_t cap = j.t1.size() + j.t2.size() + 16;
    j.p = pool.get();
    Parsed& p = *j.p;
    p.names.resize(cap);
    p.seq.resize(cap);
    p.qual.resize(cap);
    p.nl.resize(cap / 4 + 8);
    p.sl.resize(cap / 4 + 8);
    const int64_t n = pe ? sa_parse_pe(j.t1.data(), j.t1.size(), j.t2.data(), j.t2.size(), p.names.data(), p.nl.data(),
                                       p.seq.data(), p.sl.data(), p.qual.data())
                         : sa_parse_se(j.t1.data(), j.t1.size(), p.names.data(), p.nl.data(), p.seq.data(),
                                       p.sl.data(), p.qual.data());
    if (n < 0) return false;
    p.nreads = (uint32_t)n;
    p.text1 = j.t1.size();
    p.text2 = j.t2.size();
    uint64_t nb = 0, sb = 0;
    for (uint32_t r = 0; r < p.nreads; r++) {
        nb += p.nl[r];
        sb += (uint64_t)p.sl[r];
    }
    p.names.n = nb;
    p.seq.n = sb;
    p.qual.n = sb;
    p.nl.n = p.nreads;
    p.sl.n = p.nreads;
    j.nreads = p.nreads;
    for (uint32_t r = 0; r < p.nreads; r++) j.len_long |= p.sl[r] > 0xffff;
    if (!keep_text) give_back(j, texts);
    return true;
}

struct Options {
    const char *f1 = nullptr, *f2 = nullptr, *out = nullptr, *arc = nullptr, *ref = nullptr;
    bool compress = false, decompress = false, index = false, force = false, in_dir = false, share_device = false,
         verbose = false, host_only = false, host_parse = false, ingest_only = false, ramp = false,
         release = false, stage_ahead = false, shm = false, maxmis_set = false, ingest_crc = false;
    // --read-threads: the plain-file reader's fill threads (SegReader).  16 since
    // round 6: the whole-node ingest (--ingest-only --devices 8) 34.3 / 35.8
    // against 18.2 / 28.7 GB/s with 8 (r6s; the reader two or three batches
    // ahead instead: 21.5-25.4)
    int read_threads = 16;
    int writers = 8;        // --writers: the archive writer's copy threads (ArcWriter; 1: write(2) in order)
    int threads = 0, pipe = 0, device = 0, devices = 1, contexts = 2, batch = 32, block_mib = 50, maxmis = 7;
    int insert = 0;
    sa_cfg cfg{3, 2, 1, 0, 0.0};
};

bool shm_publish(const char* ref, const uint8_t* p, size_t n, const uint8_t* md5, bool verbose);

// ---- SeqArc -i ref.fa: the HASH index (HashAlignment::buildRefIndex@0x410190,
//      HashRefIndex32::writeIndexFile@0x41ed00 -> "<ref>.hash"; MD5File@0x405950 of
//      the FASTA -> "<ref>.md5", 16 bytes) ----
int build_index(const Options& o)
{
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<uint8_t> fa;
    if (!slurp(o.ref, fa) || fa.empty()) {
        fprintf(stderr, "Error:The file %s may be not exist or empty!\n", o.ref);
        return 1;
    }
    sa_ctx* c = sa_create(o.device);
    if (!c) {
        fprintf(stderr, "seqarc_amd: no usable gfx950 device %d\n", o.device);
        return 1;
    }
    const auto t1 = std::chrono::steady_clock::now();
    sa_hash_index* ix = sa_hash_build(c, (const char*)fa.data(), fa.size(), 14, 2, 1u << 16);
    if (!ix) {
        fprintf(stderr, "seqarc_amd: index build failed: %s\n", sa_last_error(c));
        sa_destroy(c);
        return 1;
    }
    const auto t2 = std::chrono::steady_clock::now();
    std::vector<uint8_t> file(sa_hash_file_bytes(ix));
    int rc = sa_hash_serialize(c, ix, file.data(), file.size());
    uint8_t md[16];
    sa_md5(fa.data(), fa.size(), md);
    if (rc || !spill(std::string(o.ref) + ".hash", file.data(), file.size()) ||
        !spill(std::string(o.ref) + ".md5", md, 16)) {
        fprintf(stderr, "seqarc_amd: cannot write the index files of %s\n", o.ref);
        rc = 1;
    }
    if (rc == 0 && o.shm && !shm_publish(o.ref, file.data(), file.size(), md, o.verbose)) rc = 1;
    const double s_load = std::chrono::duration<double>(t1 - t0).count(),
                 s_build = std::chrono::duration<double>(t2 - t1).count(),
                 s_all = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "seqarc_amd: index of %u bases (%s.hash, %zu bytes): read %.3f s, build %.3f s, total %.3f s\n",
            sa_hash_genome_length(ix), o.ref, file.size(), s_load, s_build, s_all);
    sa_hash_destroy(ix);
    sa_destroy(c);
    return rc;
}

// The reference of -c / -d: its index file (or the FASTA to build it from) and
// the MD5 the archive records (getMd5@0x416810 reads "<ref>.md5")
struct RefFiles {
    std::vector<uint8_t> hash, fasta;
    // the index image: hash's bytes, or (-s) a /dev/shm object mapped read-only
    const uint8_t* hp = nullptr;
    size_t hn = 0;
    void* map = nullptr;
    size_t map_len = 0;
    uint8_t md5[16] = {0};
    bool have_hash() const { return hn > 16; }
    void drop_hash()
    {
        hash.clear();
        hash.shrink_to_fit();
        if (map) munmap(map, map_len);
        map = nullptr;
        hp = nullptr;
        hn = 0;
    }
    ~RefFiles() { drop_hash(); }
};

// the bytes an index image's header announces (HashRefIndex32::loadRefIndexShm@0x41ef80:
// K, bases, words, positions; words, num[4^K], ind[4^K], positions), 0 if no header
uint64_t hash_image_bytes(const uint8_t* p, size_t n)
{
    if (n < 16) return 0;
    uint32_t h[4];
    memcpy(h, p, 16);
    if (h[0] < 1 || h[0] > 16) return 0;
    return 16 + 4ull * (h[2] + 2 * (1ull << (2 * h[0])) + h[3]);
}

// -s: the index image in POSIX shared memory under the reference's file name
// (IHashRefIndex::createShm@0x41f280: shm_open of the basename, an existing
// object of the announced size is kept, one of another size replaced;
// HashRefIndex32::createRefIndexShm@0x41f520 copies the image in after the
// file was read).  Later runs map it instead of reading <ref>.hash.
std::string shm_name(const char* ref)
{
    const std::string r(ref);
    return r.substr(r.rfind('/') + 1);
}

// The object is bound to its reference by a sidecar object "<name>.sa_ref":
// the FASTA's MD5 (the archive's encap 8) and the image size.  The reference
// keys the object by the file's basename alone, so two references of the same
// name would otherwise share one image (and -c would align against the wrong
// genome while recording the right MD5).
struct ShmTag {
    char magic[8];
    uint8_t md5[16];
    uint64_t bytes;
};
constexpr char kShmTagMagic[8] = {'S', 'A', 'R', 'E', 'F', '0', '0', '1'};

std::string shm_tag_name(const char* ref) { return shm_name(ref) + ".sa_ref"; }

// 1: the tag names this reference and size, 0: no tag, -1: another reference or size
int shm_tag_check(const char* ref, const uint8_t* md5, uint64_t bytes)
{
    const int fd = shm_open(shm_tag_name(ref).c_str(), O_RDONLY, 0);
    if (fd < 0) return 0;
    ShmTag t{};
    const bool got = ::pread(fd, &t, sizeof t, 0) == (ssize_t)sizeof t;
    close(fd);
    return got && !memcmp(t.magic, kShmTagMagic, 8) && !memcmp(t.md5, md5, 16) && t.bytes == bytes ? 1 : -1;
}

bool shm_tag_write(const char* ref, const uint8_t* md5, uint64_t bytes)
{
    const std::string nm = shm_tag_name(ref);
    shm_unlink(nm.c_str());
    const int fd = shm_open(nm.c_str(), O_CREAT | O_EXCL | O_RDWR, 0644);
    if (fd < 0) return false;
    ShmTag t{};
    memcpy(t.magic, kShmTagMagic, 8);
    memcpy(t.md5, md5, 16);
    t.bytes = bytes;
    const bool ok = ::pwrite(fd, &t, sizeof t, 0) == (ssize_t)sizeof t;
    close(fd);
    return ok;
}

// <ref>.hash on disk: 1 its header and size equal the image's, 0 no file, -1 they differ
int hash_file_matches(const char* ref, const uint8_t* p, size_t n)
{
    const std::string f = std::string(ref) + ".hash";
    const int fd = ::open(f.c_str(), O_RDONLY);
    if (fd < 0) return 0;
    struct stat sb;
    uint8_t h[16];
    const bool same = fstat(fd, &sb) == 0 && (uint64_t)sb.st_size == n && n >= 16 &&
                      ::pread(fd, h, 16, 0) == 16 && !memcmp(h, p, 16);
    close(fd);
    return same ? 1 : -1;
}

bool shm_publish(const char* ref, const uint8_t* p, size_t n, const uint8_t* md5, bool verbose)
{
    const std::string nm = shm_name(ref);
    int fd = shm_open(nm.c_str(), O_RDWR, 0);
    if (fd >= 0) {
        struct stat sb;
        const bool same = fstat(fd, &sb) == 0 && (uint64_t)sb.st_size == n;
        close(fd);
        // kept only when it is this reference's image (an object of the same
        // size but another reference, or an untagged one, is replaced)
        if (same && shm_tag_check(ref, md5, n) == 1) {
            fprintf(stderr, "createHashShm %s has existed.\n", nm.c_str());
            return true;
        }
        shm_unlink(nm.c_str());
    }
    fd = shm_open(nm.c_str(), O_CREAT | O_EXCL | O_RDWR, 0644);
    if (fd < 0) {
        fprintf(stderr, "shm_open fail.\n");
        return false;
    }
    bool ok = ftruncate(fd, (off_t)n) == 0;
    if (!ok) fprintf(stderr, "ftruncate fail.\n");
    void* m = ok ? mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : MAP_FAILED;
    close(fd);
    if (ok && m == MAP_FAILED) {
        fprintf(stderr, "mmap fail.\n");
        ok = false;
    }
    if (!ok) {
        shm_unlink(nm.c_str());
        return false;
    }
    memcpy(m, p, n);
    munmap(m, n);
    if (!shm_tag_write(ref, md5, n)) {
        fprintf(stderr, "shm_open fail.\n");
        shm_unlink(nm.c_str());
        return false;
    }
    if (verbose) fprintf(stderr, "seqarc_amd: index image in /dev/shm/%s (%zu bytes)\n", nm.c_str(), n);
    return true;
}

// 1: mapped, 0: no such object, or the object of another reference while
// <ref>.hash exists (the caller reads the file and republishes), -1: an object
// that is not an index image, or one that cannot be shown to be this
// reference's (md5: the FASTA's, from <ref>.md5 or the FASTA itself)
int shm_map(const char* ref, const uint8_t* md5, RefFiles& rf)
{
    const std::string nm = shm_name(ref);
    const int fd = shm_open(nm.c_str(), O_RDONLY, 0);
    if (fd < 0) return 0;
    struct stat sb;
    void* m = MAP_FAILED;
    size_t n = 0;
    if (fstat(fd, &sb) == 0 && sb.st_size >= 16) {
        n = (size_t)sb.st_size;
        m = mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
    }
    close(fd);
    if (m == MAP_FAILED || hash_image_bytes((const uint8_t*)m, n) != n) {
        if (m != MAP_FAILED) munmap(m, n);
        fprintf(stderr, "/dev/shm/ %s is wrong file, please delete\n", nm.c_str());
        return -1;
    }
    // bound to this reference: its tag, else (an object without one, e.g. made
    // by SeqArc itself) <ref>.hash's header and size
    const int tag = shm_tag_check(ref, md5, n);
    const int file = tag == 1 ? 1 : hash_file_matches(ref, (const uint8_t*)m, n);
    if (tag < 0 || file < 0 || (tag == 0 && file == 0)) {
        munmap(m, n);
        if (file != 0) return 0;   // (stale or another reference's image: <ref>.hash is read and republished)
        fprintf(stderr, "/dev/shm/ %s is not the index of %s (another reference of the same name?), please delete\n",
                nm.c_str(), ref);
        return -1;
    }
    rf.map = m;
    rf.map_len = n;
    rf.hp = (const uint8_t*)m;
    rf.hn = n;
    return 1;
}

bool load_ref(const char* ref, bool need_fasta, RefFiles& rf, bool use_shm = false, bool verbose = false)
{
    const std::string r(ref);
    auto read_fasta = [&]() {
        if (!rf.fasta.empty()) return true;
        if (!slurp(r, rf.fasta) || rf.fasta.empty()) {
            fprintf(stderr, "Error:The file %s may be not exist or empty!\n", ref);
            return false;
        }
        return true;
    };
    // the reference's MD5 first: the shared-memory image must be this reference's
    std::vector<uint8_t> m;
    const bool have_md5 = slurp(r + ".md5", m) && m.size() == 16;
    if ((!have_md5 || need_fasta) && !read_fasta()) return false;
    if (have_md5) memcpy(rf.md5, m.data(), 16);
    else sa_md5(rf.fasta.data(), rf.fasta.size(), rf.md5);
    bool have_hash = false;
    if (use_shm) {   // (HashAlignment::loadRefIndex: loadRefIndexShm, else loadRefIndexFile)
        const int sm = shm_map(ref, rf.md5, rf);
        if (sm < 0) return false;
        have_hash = sm == 1;
        if (have_hash && verbose) fprintf(stderr, "seqarc_amd: index image from /dev/shm/%s\n", shm_name(ref).c_str());
    }
    if (!have_hash) {
        have_hash = slurp(r + ".hash", rf.hash) && rf.hash.size() > 16;
        if (!have_hash) rf.hash.clear();
        if (have_hash) {
            rf.hp = rf.hash.data();
            rf.hn = rf.hash.size();
            if (use_shm && hash_image_bytes(rf.hp, rf.hn) == rf.hn) (void)shm_publish(ref, rf.hp, rf.hn, rf.md5, verbose);
        }
    }
    return have_hash || read_fasta();
}

// ---- compression: the streaming pipeline ------------------------------------
bool g_fast_exit = false;   // compress() left the device buffers to the process exit

double mono_s()   // CLOCK_MONOTONIC (the clock of Python's time.monotonic: bench.py splits its wall clock)
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
double g_main_s = 0.0;

// the -v stamps bench.py reads (process start -> main and exit -> reaped are the
// caller's to see), then, after a compression that left its device buffers to
// the exit, the exit itself: no runtime teardown, and none of compress()'s
// destructors either (freeing the reader's ~24 GB of page-locked windows took
// 1.35 s after the archive was closed, round 3 g4f)
[[noreturn]] void fast_exit(int rc, bool verbose)
{
    if (verbose) fprintf(stderr, "seqarc_amd: monotonic clock: main %.6f, exit %.6f\n", g_main_s, mono_s());
    fflush(stdout);
    fflush(stderr);
    std::_Exit(rc);
}

int compress(const Options& o)
{
    const auto t_start = std::chrono::steady_clock::now();
    const bool pe = o.f2 && *o.f2;
    // inflate threads per BGZF input: the -t share (the device parse leaves the host threads free)
    g_gz_workers = std::max(2, (o.threads > 0 ? o.threads : 16) / (pe ? 2 : 1));
    Input in1, in2;
    struct stat sb;
    for (const char* f : {o.f1, pe ? o.f2 : nullptr}) {
        if (f && (stat(f, &sb) != 0 || sb.st_size == 0)) {   // doCheckSetEncodeOpt@0x407fa0
            fprintf(stderr, "Error:The Src file %s may be not exist or empty!\n", f);
            return 1;
        }
    }
    if (!in1.open(o.f1) || (pe && !in2.open(o.f2))) {
        fprintf(stderr, "seqarc_amd: cannot open the input\n");
        return 1;
    }
    std::string outp = o.out;
    if (o.in_dir && outp.find('/') == std::string::npos) outp = dir_of(o.f1) + outp;
    const std::string path = outp + ".arc";
    if (!may_write(path, o.force)) return 1;

    const uint64_t bs = (uint64_t)o.block_mib << 20;   // BlockSize(M), default 50 (param+0x1b78)
    const int nparse = !o.host_parse && !o.host_only ? 1   // (device parse: block 0 only, for the ID template)
                       : o.threads > 0 ? o.threads
                                       : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    // Device parse (default): the reader's text windows are page-locked, the
    // encoder threads stage them with sa_stage_text (H2D DMA + parse in HBM)
    // and recycle them at once; only block 0 is parsed here, for the ID
    // template.  --host-parse / --host-only: -t parser threads build the SoA.
    const bool dev_parse = !o.host_parse && !o.host_only;
    ParsedPool pool;   // (declared before the jobs: outlive them)
    OutPool outpool;
    // (round 6) the device-parse path sizes each block's output buffer by its
    // encoded size (sa_fetch_sizes after sa_run) instead of its output bound:
    // the pool held ~270 buffers of ~180 MB of address space for ~7 MB blocks,
    // whose teardown was most of the exit (r6z).  SA_CLI_OUT_EXACT=0: the bound (A/B)
    const bool out_exact = !(std::getenv("SA_CLI_OUT_EXACT") && std::atoi(std::getenv("SA_CLI_OUT_EXACT")) == 0);
    TextPool texts;
    texts.pinned = dev_parse && !o.ingest_only;
    texts.win = (pe ? (size_t)((uint32_t)bs >> 1) : (size_t)bs) + (64u << 10);   // a window + slack for the carry
    // the windows the reader will hold (two batches ahead of the staging, both
    // mates), pinned by a thread of their own beside the reader (an input that
    // is smaller needs fewer)
    struct Joiner {
        std::thread t;
        ~Joiner()
        {
            if (t.joinable()) t.join();
        }
    } prefill;
    // plain regular files (not gzip, not a pipe) are read by the segment reader
    // (SegReader, started below), the others in per-block windows (TextPool)
    uint64_t fsize[2] = {0, 0};
    bool seg_plain = o.read_threads > 0 && !in1.is_gz && (!pe || !in2.is_gz) && !std::getenv("SA_CLI_WINDOWS");
    for (int i = 0; i < (pe ? 2 : 1) && seg_plain; i++) {
        struct stat st;
        if (fstat(i ? in2.fd : in1.fd, &st) != 0 || !S_ISREG(st.st_mode)) seg_plain = false;
        else fsize[i] = (uint64_t)st.st_size;
    }
    size_t prefill_chunks = 0;
    if (texts.pinned && !seg_plain) {
        size_t wins = (size_t)(pe ? 2 : 1) * (2 * (size_t)std::max(1, o.batch) + 4);
        uint64_t tot = 0;
        bool known = true;
        struct stat st;
        for (const char* f : {o.f1, pe ? o.f2 : nullptr})
            if (f) {
                if (stat(f, &st) == 0 && S_ISREG(st.st_mode) && !in1.is_gz && !in2.is_gz) tot = std::max<uint64_t>(tot, (uint64_t)st.st_size);
                else known = false;
            }
        if (known) wins = std::min(wins, (size_t)(pe ? 2 : 1) * (size_t)(tot / (texts.win - (64u << 10)) + 3));
        if (const char* e = std::getenv("SA_CLI_PREFILL_WINDOWS")) wins = std::strtoull(e, nullptr, 10);   // (A/B)
        prefill_chunks = (wins + TextPool::kChunk - 1) / TextPool::kChunk;
    }
    // contexts: K per device; every device's contexts share one front scratch
    std::vector<sa_ctx*> ctxs;
    std::vector<int> ctx_dev;   // (the device of each context)
    // reference path: the index on every device in use, one align_info chain
    // through all batches in input order (the reference's -t 1 thread)
    RefFiles rf;
    std::map<sa_ctx*, sa_align_cfg> acfg;
    std::vector<sa_hash_index*> indexes;
    sa_align_chain* chain = nullptr;
    // The plain-file reader starts before the device contexts exist (round 5):
    // creating five contexts takes ~0.35 s, which the reader's first batch
    // then overlaps instead of following.  (SA_CLI_EARLY_READ=0: contexts
    // first, A/B.)  The contexts and the reference index: false with a message.
    const bool early_read =
        !(std::getenv("SA_CLI_EARLY_READ") && std::atoi(std::getenv("SA_CLI_EARLY_READ")) == 0) && seg_plain;
    std::string ctx_err;
    auto create_contexts = [&]() -> bool {
        // --ingest-only: the reader and the block cut alone, feeding devices x
        // contexts consumers that take batches as the device parse would (no device)
        if (o.host_only || o.ingest_only) ctxs.assign((size_t)o.contexts * (o.ingest_only ? o.devices : 1), nullptr);
        for (int d = 0; d < o.devices && !o.host_only && !o.ingest_only; d++) {
            sa_ctx* first = nullptr;
            for (int k = 0; k < o.contexts; k++) {
                const int dev = o.device + (o.share_device ? 0 : d);
                sa_ctx* c = first ? sa_create_shared(dev, first) : sa_create(dev);
                if (!c) break;
                if (!first) first = c;
                ctxs.push_back(c);
                ctx_dev.push_back(dev);
            }
            if (!first) break;
        }
        // (started once the contexts exist: pinning beside their creation held
        // it up, 0.25 -> 0.83 s, round 3 g4j)
        if (prefill_chunks && !ctxs.empty() && ctxs[0])
            prefill.t = std::thread([&texts, prefill_chunks]() {
                for (size_t i = 0; i < prefill_chunks; i++)
                    if (!texts.grow()) break;
            });
        if (o.verbose)
            for (sa_ctx* c : ctxs)
                if (c) sa_set_timing(c, 1);
        if (ctxs.empty()) {
            ctx_err = "no usable gfx950 device " + std::to_string(o.device);
            return false;
        }
        if (o.ref && !o.host_only && !o.ingest_only) {
            if (!load_ref(o.ref, false, rf, o.shm, o.verbose)) {
                ctx_err = std::string("cannot load the reference ") + o.ref;
                return false;
            }
            const double ti = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
            sa_ctx* owner = nullptr;
            sa_hash_index* ix = nullptr;
            for (size_t k = 0; k < ctxs.size(); k++) {
                if (k % (size_t)o.contexts == 0 && !(o.share_device && ix)) {   // the first context of a device
                    owner = ctxs[k];
                    ix = rf.have_hash() ? sa_hash_load(owner, rf.hp, rf.hn)
                                          : sa_hash_build(owner, (const char*)rf.fasta.data(), rf.fasta.size(), 14, 2,
                                                          1u << 16);
                    if (!ix) {
                        ctx_err = std::string("reference index: ") + sa_last_error(owner);
                        return false;
                    }
                    indexes.push_back(ix);
                }
                acfg[ctxs[k]] = sa_align_cfg{ix, pe ? 1 : 0, o.maxmis, 1, (uint32_t)o.insert};
            }
            chain = sa_align_chain_create(0, 0);   // a fresh encode thread's AlignParam (nmis 0)
            if (o.verbose)
                fprintf(stderr, "seqarc_amd: reference %s: index %s in %.3f s\n", o.ref,
                        rf.have_hash() ? "loaded" : "built",
                        std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() - ti);
        }
        return true;
    };
    if (!early_read && !create_contexts()) {
        fprintf(stderr, "seqarc_amd: %s\n", ctx_err.c_str());
        return 1;
    }
    if (!early_read && !o.host_only && !o.ingest_only && (int64_t)ctxs.size() != (int64_t)o.contexts * o.devices)
        fprintf(stderr, "seqarc_amd: warning: %zu of %lld encoder contexts created\n", ctxs.size(),
                (long long)o.contexts * o.devices);
    int64_t B = std::max(1, o.batch);
    // (the contexts the options ask for: with early_read they do not exist yet)
    const int64_t C = early_read ? (int64_t)o.contexts * (o.host_only ? 1 : o.devices) : (int64_t)ctxs.size();
    // batch k = blocks [bstart(k), bstart(k + 1)).  --ramp: the first batch of
    // each context ramps up (B (k+1) / (C+1) blocks: the first encode starts
    // after a fraction of a batch is read, and the contexts' first tails are
    // staggered); the contexts allocate for B from the start (sa_set_reserve).
    // Off by default since round 4: a batch's latency is its longest chain's
    // whatever its size, so the ramp's five small batches cost a round of
    // throughput (42.8 GB: 5,390 MB/s with it, 6,642 without, r4m).
    // A plain-file input that fits one round (C batches of B blocks, by its
    // size) is dealt as C equal batches (round 3 g4g: with the ramp its last
    // blocks waited for a second round of batch latencies).
    bool ramp = o.ramp;
    if (!o.host_only && !o.ingest_only && !in1.is_gz && (!pe || !in2.is_gz)) {
        uint64_t tot = 0;
        struct stat st;
        for (const char* f : {o.f1, pe ? o.f2 : nullptr})
            if (f && stat(f, &st) == 0 && S_ISREG(st.st_mode)) tot += (uint64_t)st.st_size;
            else tot = ~0ull >> 1;   // (a pipe: size unknown)
        const int64_t est = (int64_t)((tot + bs - 1) / bs) + 1;   // blocks (cut at record ends: <= bs each)
        if (tot < (~0ull >> 2) && est <= C * B) {
            ramp = false;
            B = (est + C - 1) / C;
        }
    }
    // blocks read but not yet written: C batches encoding and two ahead; with the
    // streamed staging (below) each context's helper holds one more batch on the
    // device, its text already back with the reader
    const bool stream_opt = dev_parse && !o.ingest_only && !o.stage_ahead && std::getenv("SA_CLI_STREAM") &&
                            std::atoi(std::getenv("SA_CLI_STREAM")) != 0;
    const size_t max_inflight = (size_t)B * ((size_t)C * (stream_opt ? 2 : 1) + 2);
    std::vector<int64_t> ramp_start{0};
    for (int64_t k = 0; ramp && k < C; k++) ramp_start.push_back(ramp_start.back() + std::max<int64_t>(1, B * (k + 1) / (C + 1)));
    auto bstart = [&](int64_t k) -> int64_t {
        const int64_t r = (int64_t)ramp_start.size() - 1;
        return k <= r ? ramp_start[(size_t)k] : ramp_start.back() + (k - r) * B;
    };
    auto reserve = [&]() {
        if (ramp)
            for (sa_ctx* c : ctxs)
                if (c) sa_set_reserve(c, (uint32_t)B);
    };
    if (!early_read) reserve();

    std::mutex mu;
    std::condition_variable cv;
    std::atomic<double> stage_busy{0};
    std::map<int64_t, std::unique_ptr<Job>> jobs;
    // -v: when the stages first / last did something (seconds from the start)
    auto now_s = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
    double t_ctx = now_s();   // (early_read: set once the contexts exist)
    std::atomic<double> t_read_done{0}, t_first_enc{1e30}, t_last_enc{0}, enc_busy{0}, parse_busy{0};
    double fill_busy = 0, cut_busy = 0;   // (reader thread only)
    std::deque<int64_t> to_parse;
    int64_t nread = 0, nblocks = -1, written = 0, next_batch = 0, staged = 0;
    bool failed = false, tmpl_ready = false;
    std::string err;
    uint8_t tmpl[512] = {0};
    sa_cfg cfg = o.cfg;
    int plus_bare = 1;
    uint64_t total_in = 0;
    auto fail = [&](const std::string& m) {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!failed) err = m;
            failed = true;
            cv.notify_all();
        }
        // contexts waiting on the alignment chain for a batch that will never
        // reach it return instead of waiting forever
        if (chain) sa_align_chain_fail(chain);
    };

    // plain regular files (not gzip, not a pipe): the segment reader (SegReader)
    std::unique_ptr<SegReader> segr;
    {
        if (seg_plain) {
            const uint64_t win = pe ? (uint64_t)((uint32_t)bs >> 1) : bs;
            segr.reset(new SegReader());
            const int fds[2] = {in1.fd, in2.fd};
            // the reader runs at most two batches of blocks ahead of the staging (below)
            // (one batch of windows ahead of the staging, SA_CLI_AHEAD_BATCHES to change;
            // two until round 5: the contexts take batches as fast as the reader
            // cuts them until all are busy, then the device sets the pace)
            const char* ab = std::getenv("SA_CLI_AHEAD_BATCHES");
            const int64_t ahead = ab ? std::max(1, std::atoi(ab)) : 1;
            segr->start(fds, fsize, pe ? 2 : 1, win + (64u << 10), (int64_t)(ahead * B + 2) * (int64_t)win,
                        o.read_threads, dev_parse, (uint64_t)B);   // (page-locked for the device parse; --ingest-only too)
        }
    }
    // the segments are released as soon as every block is staged (device parse)
    std::atomic<double> t_seg_freed{0};
    std::thread seg_free;
    bool seg_stop = false;
    // (SA_CLI_RING_FREE=0, A/B: the ring is left to the process exit)
    const bool ring_free = !(std::getenv("SA_CLI_RING_FREE") && std::atoi(std::getenv("SA_CLI_RING_FREE")) == 0);
    if (segr && dev_parse && ring_free)
        seg_free = std::thread([&]() {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return failed || seg_stop || (nblocks >= 0 && staged >= nblocks); });
                if (failed || seg_stop) return;
            }
            segr->free_all();
            t_seg_freed = now_s();
        });
    // reader: cuts blocks as the input arrives
    std::thread reader([&]() {
        if (segr) {   // blocks are views into the segments
            const uint64_t want = pe ? (uint64_t)((uint32_t)bs >> 1) : bs;
            std::vector<uint8_t> first;
            uint64_t o1 = 0, o2 = 0;
            for (int64_t i = 0;; i++) {
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] {
                        return failed || ((size_t)(nread - written) < max_inflight && (!dev_parse || nread - staged < 2 * B));
                    });
                    if (failed) return;
                }
                if (o1 >= fsize[0] && (!pe || o2 >= fsize[1])) {   // the input ended on a block boundary
                    segr->finish();
                    std::lock_guard<std::mutex> g(mu);
                    nblocks = i;
                    cv.notify_all();
                    return;
                }
                const double tf0 = now_s();
                uint64_t av1 = 0, av2 = 0;
                int64_t s1 = -1, s2 = -1;
                const uint8_t* w1 = segr->window(0, o1, av1, s1);
                const uint8_t* w2 = pe ? segr->window(1, o2, av2, s2) : nullptr;
                if (!w1 || (pe && !w2)) return fail("read error on the input");
                const bool eof1 = o1 + av1 >= fsize[0], eof2 = pe && o2 + av2 >= fsize[1];
                if (i == 0) {
                    const void* nl = memchr(w1, '\n', (size_t)std::min(av1, want));
                    first.assign(w1, nl ? (const uint8_t*)nl + 1 : w1 + std::min(av1, want));
                    plus_bare = pe ? bare_plus(w2, (size_t)std::min(av2, want)) : bare_plus(w1, (size_t)std::min(av1, want));
                }
                const double tc0 = now_s();
                fill_busy += tc0 - tf0;   // (waiting for the fill threads)
                uint64_t e1 = 0, e2 = 0;
                if (pe) {
                    const uint64_t k1 = segr->newlines(0, o1, std::min(av1, want), w1);
                    const uint64_t k2 = segr->newlines(1, o2, std::min(av2, want), w2);
                    if (sa_cut_next_pe_nl(w1, av1, eof1, k1, w2, av2, eof2, k2, bs, first.data(), first.size(), &e1,
                                          &e2) != 0)
                        return fail("PE block cut failed (mates out of step)");
                } else {
                    const int64_t e = sa_cut_next_se(w1, av1, eof1, bs, first.data(), first.size());
                    if (e < 0) return fail("block cut failed");
                    e1 = (uint64_t)e;
                }
                cut_busy += now_s() - tc0;
                if (e1 + e2 == 0) return fail("block cut made no progress");
                std::unique_ptr<Job> j(new Job());
                auto view = [](Buf<uint8_t>& b, const uint8_t* p, uint64_t n) {
                    b.d = const_cast<uint8_t*>(p);
                    b.n = n;
                    b.cap = 0;   // (not a window: TextPool::put leaves it)
                    b.external = true;
                };
                view(j->t1, w1, e1);
                if (pe) view(j->t2, w2, e2);
                j->segr = segr.get();
                j->seg[0] = s1;
                j->seg[1] = s2;
                o1 += e1;
                o2 += e2;
                const bool last = o1 >= fsize[0] && (!pe || o2 >= fsize[1]);
                if (last) {
                    t_read_done = now_s();
                    segr->finish();
                }
                j->text1 = e1;
                j->text2 = e2;
                if (dev_parse && i > 0) j->state = 1;   // (parsed on the device when staged)
                {
                    std::lock_guard<std::mutex> g(mu);
                    total_in += e1 + e2;
                    jobs[i] = std::move(j);
                    if (!dev_parse || i == 0) to_parse.push_back(i);
                    nread = i + 1;
                    if (last) nblocks = nread;
                }
                cv.notify_all();
                if (last) return;
            }
        }
        Buf<uint8_t> b1 = texts.get(), b2 = texts.get();
        std::vector<uint8_t> first;
        const uint64_t want = pe ? (uint64_t)((uint32_t)bs >> 1) : bs;
        for (int64_t i = 0;; i++) {
            {
                std::unique_lock<std::mutex> lk(mu);
                // device parse: at most two batches of page-locked text ahead of the staging
                cv.wait(lk, [&] {
                    return failed || ((size_t)(nread - written) < max_inflight && (!dev_parse || nread - staged < 2 * B));
                });
                if (failed) return;
            }
            b1.reserve(want);
            if (pe) b2.reserve(want);
            const double tf0 = now_s();
            {   // the two mate files are read concurrently
                std::future<bool> r2;
                if (pe && b2.size() < want && !in2.eof)
                    r2 = std::async(std::launch::async, [&]() { return in2.fill(b2, want - b2.size()); });
                const bool ok1 = b1.size() >= want || in1.eof || in1.fill(b1, want - b1.size());
                const bool ok2 = !r2.valid() || r2.get();
                if (!ok1) return fail("read error on input 1");
                if (!ok2) return fail("read error on input 2");
            }
            if (b1.empty() && (!pe || b2.empty())) {   // the input ended on a block boundary
                std::lock_guard<std::mutex> g(mu);
                nblocks = i;
                cv.notify_all();
                return;
            }
            if (i == 0) {
                const void* nl = memchr(b1.data(), '\n', b1.size());
                const uint8_t* f0 = b1.data();
                first.assign(f0, nl ? (const uint8_t*)nl + 1 : f0 + b1.size());
                plus_bare = pe ? bare_plus(b2.data(), b2.size()) : bare_plus(b1.data(), b1.size());
            }
            const double tc0 = now_s();
            fill_busy += tc0 - tf0;
            uint64_t e1 = 0, e2 = 0;
            if (pe) {
                if (sa_cut_next_pe(b1.data(), b1.size(), in1.eof, b2.data(), b2.size(), in2.eof, bs, first.data(),
                                   first.size(), &e1, &e2) != 0)
                    return fail("PE block cut failed (mates out of step)");
            } else {
                const int64_t e = sa_cut_next_se(b1.data(), b1.size(), in1.eof, bs, first.data(), first.size());
                if (e < 0) return fail("block cut failed");
                e1 = (uint64_t)e;
            }
            cut_busy += now_s() - tc0;
            std::unique_ptr<Job> j(new Job());
            auto hand_over = [&](Buf<uint8_t>& b, Buf<uint8_t>& to, uint64_t e) {
                Buf<uint8_t> carry = texts.get();   // the bytes after the cut start the next window
                carry.reserve(want);
                memcpy(carry.data(), b.data() + e, b.size() - e);
                carry.n = b.size() - e;
                b.n = e;
                to = std::move(b);
                b = std::move(carry);
            };
            hand_over(b1, j->t1, e1);
            if (pe) hand_over(b2, j->t2, e2);
            const bool last = b1.empty() && b2.empty() && in1.eof && (!pe || in2.eof);
            if (last) t_read_done = now_s();
            j->text1 = e1;
            j->text2 = e2;
            if (dev_parse && i > 0) j->state = 1;   // (parsed on the device when staged)
            {
                std::lock_guard<std::mutex> g(mu);
                total_in += e1 + e2;
                jobs[i] = std::move(j);
                if (!dev_parse || i == 0) to_parse.push_back(i);
                nread = i + 1;
                if (last) nblocks = nread;
            }
            cv.notify_all();
            if (last) return;
        }
    });

    // parsers
    std::vector<std::thread> parsers;
    for (int t = 0; t < nparse; t++)
        parsers.emplace_back([&]() {
            for (;;) {
                int64_t i;
                Job* j;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return failed || !to_parse.empty() || nblocks >= 0; });
                    if (failed || (to_parse.empty() && nblocks >= 0)) return;
                    i = to_parse.front();
                    to_parse.pop_front();
                    j = jobs[i].get();
                }
                const double tp = now_s();
                if (!parse_job(*j, pe, pool, texts, dev_parse)) return fail("parse failed");
                {
                    double cur = parse_busy.load();
                    while (!parse_busy.compare_exchange_weak(cur, cur + now_s() - tp)) {}
                }
                if (i == 0) {   // the ID template of the first block
                    const sa_block fb = j->p->view();
                    if (sa_analyze_ids(&fb, pe ? 0 : 1, tmpl) != 0) return fail("ID analysis failed");
                }
                if (dev_parse) pool.put(std::move(j->p));   // (only the template needed it)
                {
                    std::lock_guard<std::mutex> g(mu);
                    j->state = 1;
                    if (i == 0) {
                        cfg.bin_mode = tmpl[0];
                        tmpl_ready = true;
                    }
                }
                cv.notify_all();
            }
        });

    // early_read: the contexts now, beside the reader's first batch
    if (early_read) {
        if (create_contexts()) {
            reserve();
            t_ctx = now_s();
            // (B, the ring and the in-flight bound were sized for C contexts
            // before they existed: fewer only cost pace, but say so)
            if ((int64_t)ctxs.size() != C)
                fprintf(stderr, "seqarc_amd: warning: %zu of %lld encoder contexts created\n", ctxs.size(),
                        (long long)C);
        } else {
            fail(ctx_err);
        }
    }
    // encoders: one host thread per context, batches of B blocks in order
    auto batch_ready = [&](int64_t k) {   // under mu
        if (!tmpl_ready) return false;
        const int64_t b0 = bstart(k);
        const int64_t b1 = nblocks >= 0 ? std::min(nblocks, bstart(k + 1)) : bstart(k + 1);
        if (nblocks < 0 && nread < b1) return false;
        for (int64_t i = b0; i < b1; i++)
            if (jobs.count(i) == 0 || jobs[i]->state < 1) return false;
        return true;
    };
    std::vector<std::thread> encoders;
    // --stage-ahead (device parse): each context stages its next batch into a
    // second device input -- with a staging context of its own (stream,
    // mailbox) on a helper thread -- while it encodes the current one, so the
    // H2D copy and the parse leave the context's cycle.  Measured slower (4.7-5.0
    // against 6.6-6.7 GB/s on 42.8 GB, round 3 g4d: the staging contexts' streams
    // outnumber the hardware queues, and the tails slowed under the concurrent
    // parse), so by default the stage is part of the cycle (sa_stage_text into
    // the context's own input).
    const bool stage_ahead = dev_parse && !o.ingest_only && o.stage_ahead && !ctxs.empty() && ctxs[0];
    std::vector<sa_ctx*> stagers;
    std::vector<sa_input*> sinputs;   // two per context
    if (stage_ahead) {
        for (size_t i = 0; i < ctxs.size(); i++) {
            sa_ctx* s = sa_create(ctx_dev[i]);
            sa_input* a = sa_input_empty(ctx_dev[i]);
            sa_input* b = sa_input_empty(ctx_dev[i]);
            if (!s || !a || !b) {
                fprintf(stderr, "seqarc_amd: cannot create the staging contexts\n");
                return 1;
            }
            if (ramp) sa_set_reserve(s, (uint32_t)B);
            stagers.push_back(s);
            sinputs.push_back(a);
            sinputs.push_back(b);
        }
    }
    // takes batch k (in order) once the reader has cut it: false when the input
    // is exhausted or the run failed
    auto claim = [&](int64_t& k, std::vector<Job*>& js) -> bool {
        std::unique_lock<std::mutex> lk(mu);
        if (failed) return false;
        k = next_batch++;
        cv.wait(lk, [&] { return failed || (nblocks >= 0 && bstart(k) >= nblocks) || batch_ready(k); });
        if (failed || (nblocks >= 0 && bstart(k) >= nblocks)) return false;
        const int64_t b0 = bstart(k), b1 = nblocks >= 0 ? std::min(nblocks, bstart(k + 1)) : bstart(k + 1);
        js.clear();
        for (int64_t i = b0; i < b1; i++) js.push_back(jobs[i].get());
        return true;
    };
    // stages the batch's texts into input I with staging context s (the text
    // windows go back to the reader at once)
    auto stage_into = [&](sa_ctx* s, sa_input* I, std::vector<Job*>& js) -> bool {
        const double t0 = now_s();
        std::vector<sa_text_block> tin(js.size());
        std::vector<sa_text_info> ti(js.size());
        for (size_t i = 0; i < js.size(); i++)
            tin[i] = sa_text_block{js[i]->t1.data(), js[i]->t1.size(), pe ? js[i]->t2.data() : nullptr,
                                   pe ? js[i]->t2.size() : 0};
        if (sa_stage_text_input(s, I, tin.data(), (int)tin.size(), ti.data()) != 0) {
            fail(std::string("staging failed: ") + sa_last_error(s));
            return false;
        }
        {
            double cur = stage_busy.load();
            while (!stage_busy.compare_exchange_weak(cur, cur + now_s() - t0)) {}
        }
        {
            std::lock_guard<std::mutex> g(mu);
            staged += (int64_t)js.size();
            for (size_t i = 0; i < js.size(); i++) {
                give_back(*js[i], texts);   // (the device holds the text now)
                js[i]->nreads = ti[i].nreads;
                js[i]->len_long = ti[i].len_long;
                outpool.take(js[i]->out, ti[i].out_bound);
            }
        }
        cv.notify_all();
        return true;
    };
    for (size_t ci = 0; stage_ahead && ci < ctxs.size(); ci++)
        encoders.emplace_back([&, ci]() {
            sa_ctx* ctx = ctxs[ci];
            sa_ctx* stg = stagers[ci];
            sa_input* in2[2] = {sinputs[2 * ci], sinputs[2 * ci + 1]};
            int64_t k = 0;
            std::vector<Job*> js;
            double tw = now_s();
            if (!claim(k, js)) return;
            double te = now_s();
            if (!stage_into(stg, in2[0], js)) return;
            for (int cur = 0;; cur ^= 1) {
                // the next batch is claimed and staged while this one encodes
                int64_t k2 = -1;
                std::vector<Job*> js2;
                double tw2 = 0, te2 = 0;
                std::future<int> next = std::async(std::launch::async, [&]() -> int {
                    tw2 = now_s();
                    if (!claim(k2, js2)) return 0;
                    te2 = now_s();
                    return stage_into(stg, in2[cur ^ 1], js2) ? 1 : -1;
                });
                {
                    double c0 = t_first_enc.load();
                    while (te < c0 && !t_first_enc.compare_exchange_weak(c0, te)) {}
                }
                std::vector<sa_out> outs(js.size());
                for (size_t i = 0; i < js.size(); i++) outs[i] = sa_out{js[i]->out.data(), js[i]->out.size(), 0};
                const sa_cfg c = cfg;
                const double tr = now_s();
                if ((chain ? sa_run_input_aligned(ctx, in2[cur], &c, &acfg[ctx], chain, (uint64_t)k)
                           : sa_run_input(ctx, in2[cur], &c)) != 0)
                    return fail(std::string("encode failed: ") + sa_last_error(ctx));
                const double tf = now_s();
                if (sa_fetch(ctx, outs.data(), (int)outs.size()) != 0)
                    return fail(std::string("fetch failed: ") + sa_last_error(ctx));
                if (o.verbose) {
                    const char* pn[16];
                    float pm[16];
                    const int np = sa_phase_times(ctx, pn, pm, 16);
                    std::string ph;
                    for (int x = 0; x < np; x++) {
                        char pb[48];
                        snprintf(pb, sizeof pb, " %s %.0f", pn[x], pm[x]);
                        ph += pb;
                    }
                    fprintf(stderr,
                            "seqarc_amd: batch %lld (%zu blocks) context %p: asked %.3f s, ready %.3f s, staged ahead, "
                            "run from %.3f s for %.3f s, fetch %.3f s; device ms:%s\n",
                            (long long)k, js.size(), (void*)ctx, tw, te, tr, tf - tr, now_s() - tf, ph.c_str());
                }
                {
                    const double t1 = now_s();
                    double c0 = enc_busy.load();
                    while (!enc_busy.compare_exchange_weak(c0, c0 + t1 - tr)) {}
                    c0 = t_last_enc.load();
                    while (t1 > c0 && !t_last_enc.compare_exchange_weak(c0, t1)) {}
                }
                {
                    std::lock_guard<std::mutex> g(mu);
                    for (size_t i = 0; i < js.size(); i++) {
                        js[i]->out.n = outs[i].size;
                        js[i]->state = 2;
                    }
                }
                cv.notify_all();
                const int r = next.get();
                if (r <= 0) return;   // (no more batches, or the staging failed: fail() was called)
                k = k2;
                js = std::move(js2);
                tw = tw2;
                te = te2;
            }
        });
    const double t_enc_start = now_s();
    // (round 6) the device parse, streamed: a context takes its batch as soon as
    // the reader has cut the batch's first block and copies each block's text to
    // the device as it is cut (sa_text_upload: the reader's segments are free
    // again at once, so the reader is not held to the pace of whole-batch
    // staging), then parses the batch (sa_text_parse) and encodes it; meanwhile
    // a helper thread takes the next batch and uploads it into the input's other
    // text arena, so the next cycle starts with its text already on the device.
    // SA_CLI_STREAM=1 (A/B; off by default): the reader ran faster with it
    // (17.8 GB read in 0.69 against 0.92 s, 42.8 GB in 1.84 against 2.39 s) but
    // the device pipeline slower -- pass R 744-1,019 against 605-694 ms a batch,
    // the run's end 2.28 / 4.46 against 2.08-2.14 / 3.48-3.59 s (r6e, one box):
    // with every batch on the device at once the fronts queue up all the same
    // and the concurrent uploads slow the chains.  By default the round-5 path:
    // sa_stage_text of a whole batch once the reader has cut it.
    const bool stream_stage = stream_opt && !stage_ahead && !ctxs.empty() && ctxs[0];
    // bytes reserved per text on the device: the reader's window (a block's text
    // never exceeds it) and some slack
    const uint64_t tstride = (pe ? (uint64_t)((uint32_t)bs >> 1) : bs) + (128u << 10);
    // batch k once its first block is cut (and the ID template known): false
    // when the input ended before it or the run failed
    auto claim_first = [&](int64_t& k) -> bool {
        std::unique_lock<std::mutex> lk(mu);
        if (failed) return false;
        k = next_batch++;
        cv.wait(lk, [&] { return failed || (nblocks >= 0 && bstart(k) >= nblocks) || (tmpl_ready && nread > bstart(k)); });
        return !(failed || (nblocks >= 0 && bstart(k) >= nblocks));
    };
    // the blocks of batch k to the device (text arena `slot` of ctx's input),
    // each as soon as the reader has cut it; its text goes back to the reader
    auto upload = [&](sa_ctx* ctx, int slot, int64_t k, std::vector<Job*>& js) -> bool {
        js.clear();
        const int nmax = (int)(bstart(k + 1) - bstart(k));
        for (int64_t i = bstart(k); i < bstart(k + 1); i++) {
            Job* j;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return failed || (nblocks >= 0 && i >= nblocks) || (jobs.count(i) && jobs[i]->state >= 1); });
                if (failed) return false;
                if (nblocks >= 0 && i >= nblocks) break;
                j = jobs[i].get();
            }
            const sa_text_block tb{j->t1.data(), j->t1.size(), pe ? j->t2.data() : nullptr, pe ? j->t2.size() : 0};
            const double t0 = now_s();
            if (sa_text_upload(ctx, nullptr, slot, (int)(i - bstart(k)), nmax, &tb, tstride) != 0) {
                fail(std::string("staging failed: ") + sa_last_error(ctx));
                return false;
            }
            give_back(*j, texts);   // (the device holds the text now)
            {
                std::lock_guard<std::mutex> g(mu);
                staged++;
                double cur = stage_busy.load();
                while (!stage_busy.compare_exchange_weak(cur, cur + now_s() - t0)) {}
            }
            cv.notify_all();
            js.push_back(j);
        }
        return true;
    };
    static const char kPe = 0;   // (a non-NULL text2 marks a PE block for sa_text_parse)
    const bool prefetch = !(std::getenv("SA_CLI_PREFETCH") && std::atoi(std::getenv("SA_CLI_PREFETCH")) == 0);
    for (size_t ci = 0; stream_stage && ci < ctxs.size(); ci++)
        encoders.emplace_back([&, ctx = ctxs[ci]]() {
            int slot = 0;
            int64_t k = -1;
            std::vector<Job*> js;
            double tw = now_s();
            if (!claim_first(k) || !upload(ctx, slot, k, js)) return;
            double te = now_s();
            for (;;) {
                const double tp = now_s();
                std::vector<sa_text_block> lens(js.size());
                std::vector<sa_text_info> ti(js.size());
                for (size_t i = 0; i < js.size(); i++)
                    lens[i] = sa_text_block{nullptr, js[i]->text1, pe ? reinterpret_cast<const uint8_t*>(&kPe) : nullptr,
                                            pe ? js[i]->text2 : 0};
                if (sa_text_parse(ctx, nullptr, slot, lens.data(), (int)js.size(), tstride, ti.data()) != 0)
                    return fail(std::string("staging failed: ") + sa_last_error(ctx));
                std::vector<sa_out> outs(js.size());
                for (size_t i = 0; i < js.size(); i++) {
                    js[i]->nreads = ti[i].nreads;
                    js[i]->len_long = ti[i].len_long;
                    outpool.take(js[i]->out, ti[i].out_bound);
                    outs[i] = sa_out{js[i]->out.data(), js[i]->out.size(), 0};
                }
                // the next batch into the other arena while this one encodes
                // (SA_CLI_PREFETCH=0: after it, A/B)
                int64_t k2 = -1;
                std::vector<Job*> js2;
                double tw2 = 0, te2 = 0;
                auto take_next = [&, slot2 = slot ^ 1]() -> int {
                    tw2 = now_s();
                    if (!claim_first(k2)) return 0;
                    const bool ok = upload(ctx, slot2, k2, js2);
                    te2 = now_s();
                    return ok ? 1 : -1;
                };
                std::future<int> next;
                if (prefetch) next = std::async(std::launch::async, take_next);
                {
                    double c0 = t_first_enc.load();
                    while (te < c0 && !t_first_enc.compare_exchange_weak(c0, te)) {}
                }
                const sa_cfg c = cfg;
                const double tr = now_s();
                if ((chain ? sa_run_aligned(ctx, &c, &acfg[ctx], chain, (uint64_t)k) : sa_run(ctx, &c)) != 0)
                    return fail(std::string("encode failed: ") + sa_last_error(ctx));
                const double tf = now_s();
                if (sa_fetch(ctx, outs.data(), (int)outs.size()) != 0)
                    return fail(std::string("fetch failed: ") + sa_last_error(ctx));
                if (o.verbose) {
                    const char* pn[16];
                    float pm[16];
                    const int np = sa_phase_times(ctx, pn, pm, 16);
                    std::string ph;
                    for (int x = 0; x < np; x++) {
                        char pb[48];
                        snprintf(pb, sizeof pb, " %s %.0f", pn[x], pm[x]);
                        ph += pb;
                    }
                    fprintf(stderr,
                            "seqarc_amd: batch %lld (%zu blocks) context %p: asked %.3f s, uploaded %.3f s, parse %.3f s, "
                            "run %.3f s, fetch %.3f s; device ms:%s\n",
                            (long long)k, js.size(), (void*)ctx, tw, te, tr - tp, tf - tr, now_s() - tf, ph.c_str());
                }
                {
                    const double t1 = now_s();
                    double c0 = enc_busy.load();
                    while (!enc_busy.compare_exchange_weak(c0, c0 + t1 - tp)) {}
                    c0 = t_last_enc.load();
                    while (t1 > c0 && !t_last_enc.compare_exchange_weak(c0, t1)) {}
                }
                {
                    std::lock_guard<std::mutex> g(mu);
                    for (size_t i = 0; i < js.size(); i++) {
                        js[i]->out.n = outs[i].size;
                        js[i]->state = 2;
                    }
                }
                cv.notify_all();
                const int r = prefetch ? next.get() : take_next();
                if (r <= 0) return;   // (no more batches, or the upload failed: fail() was called)
                k = k2;
                js = std::move(js2);
                slot ^= 1;
                tw = tw2;
                te = te2;
            }
        });
    for (size_t ci = 0; !stage_ahead && !stream_stage && ci < ctxs.size(); ci++)
        encoders.emplace_back([&, ctx = ctxs[ci]]() {
            for (;;) {
                int64_t k, b0, b1;
                std::vector<Job*> js;
                const double tw = now_s();
                {
                    std::unique_lock<std::mutex> lk(mu);
                    if (failed) return;
                    k = next_batch++;
                    cv.wait(lk, [&] { return failed || (nblocks >= 0 && bstart(k) >= nblocks) || batch_ready(k); });
                    if (failed || (nblocks >= 0 && bstart(k) >= nblocks)) return;
                    b0 = bstart(k);
                    b1 = nblocks >= 0 ? std::min(nblocks, bstart(k + 1)) : bstart(k + 1);
                    for (int64_t i = b0; i < b1; i++) js.push_back(jobs[i].get());
                }
                std::vector<sa_out> outs(js.size());
                const sa_cfg c = cfg;
                const double te = now_s();
                {
                    double cur = t_first_enc.load();
                    while (te < cur && !t_first_enc.compare_exchange_weak(cur, te)) {}
                }
                if (dev_parse && !ctx) {   // --ingest-only: the batch is taken, its windows recycled
                    for (size_t i = 0; i < js.size(); i++) {
                        if (o.ingest_crc) {   // (a check of the delivered bytes, for the tests: CPU work no device path does)
                            uint32_t c = (uint32_t)crc32(0L, js[i]->t1.data(), (uInt)js[i]->t1.size());
                            if (pe) c = (uint32_t)crc32(c, js[i]->t2.data(), (uInt)js[i]->t2.size());
                            js[i]->crc = c;
                        }
                        give_back(*js[i], texts);
                        outs[i] = sa_out{nullptr, 0, 0};
                    }
                    {
                        std::lock_guard<std::mutex> g(mu);
                        staged += (int64_t)js.size();
                    }
                    cv.notify_all();
                } else if (dev_parse) {
                    std::vector<sa_text_block> tin(js.size());
                    std::vector<sa_text_info> ti(js.size());
                    for (size_t i = 0; i < js.size(); i++)
                        tin[i] = sa_text_block{js[i]->t1.data(), js[i]->t1.size(), pe ? js[i]->t2.data() : nullptr,
                                               pe ? js[i]->t2.size() : 0};
                    if (sa_stage_text(ctx, tin.data(), (int)tin.size(), ti.data()) != 0)
                        return fail(std::string("staging failed: ") + sa_last_error(ctx));
                    {
                        const double ts = now_s() - te;
                        double cur = stage_busy.load();
                        while (!stage_busy.compare_exchange_weak(cur, cur + ts)) {}
                    }
                    {
                        std::lock_guard<std::mutex> g(mu);
                        staged += (int64_t)js.size();
                    }
                    for (size_t i = 0; i < js.size(); i++) {
                        give_back(*js[i], texts);   // (the device holds the text now)
                        js[i]->nreads = ti[i].nreads;
                        js[i]->len_long = ti[i].len_long;
                        if (!out_exact) {
                            outpool.take(js[i]->out, ti[i].out_bound);
                            outs[i] = sa_out{js[i]->out.data(), js[i]->out.size(), 0};
                        }
                    }
                    cv.notify_all();   // (text windows are free for the reader)
                    const double tr = now_s();
                    if ((chain ? sa_run_aligned(ctx, &c, &acfg[ctx], chain, (uint64_t)k) : sa_run(ctx, &c)) != 0)
                        return fail(std::string("encode failed: ") + sa_last_error(ctx));
                    if (out_exact) {   // the output buffers sized by the encoded blocks
                        std::vector<uint64_t> fs(js.size());
                        if (sa_fetch_sizes(ctx, fs.data(), (int)fs.size()) != 0)
                            return fail(std::string("fetch failed: ") + sa_last_error(ctx));
                        for (size_t i = 0; i < js.size(); i++) {
                            outpool.take(js[i]->out, fs[i]);
                            outs[i] = sa_out{js[i]->out.data(), js[i]->out.size(), 0};
                        }
                    }
                    const double tf = now_s();
                    if (sa_fetch(ctx, outs.data(), (int)outs.size()) != 0)
                        return fail(std::string("fetch failed: ") + sa_last_error(ctx));
                    if (o.verbose) {   // per batch: when it became ready, what each step took, device phases
                        const char* pn[16];
                        float pm[16];
                        const int np = sa_phase_times(ctx, pn, pm, 16);
                        std::string ph;
                        for (int x = 0; x < np; x++) {
                            char pb[48];
                            snprintf(pb, sizeof pb, " %s %.0f", pn[x], pm[x]);
                            ph += pb;
                        }
                        uint32_t grows = 0;
                        double alloc_ms = 0;
                        sa_alloc_stats(&grows, &alloc_ms);
                        fprintf(stderr,
                                "seqarc_amd: batch %lld (%zu blocks) context %p: asked %.3f s, ready %.3f s, stage %.3f s, "
                                "run %.3f s, fetch %.3f s; grows %u, alloc %.0f ms; device ms:%s\n",
                                (long long)k, js.size(), (void*)ctx, tw, te, tr - te, tf - tr, now_s() - tf, grows, alloc_ms,
                                ph.c_str());
                    }
                } else {
                    std::vector<sa_block> in(js.size());
                    for (size_t i = 0; i < js.size(); i++) {
                        in[i] = js[i]->p->view();
                        outpool.take(js[i]->out, sa_output_bound(&in[i]));   // (uninitialised: only the real bytes are touched)
                        outs[i] = sa_out{js[i]->out.data(), js[i]->out.size(), 0};
                    }
                    if (!ctx) {   // --host-only
                        // (tests: SA_CLI_TEST_OUT=n gives each block n bytes of filler, so the
                        // archive writer runs without a device)
                        static const uint64_t test_out =
                            std::getenv("SA_CLI_TEST_OUT") ? std::strtoull(std::getenv("SA_CLI_TEST_OUT"), nullptr, 10) : 0;
                        for (sa_out& x : outs) {
                            x.size = std::min<uint64_t>(test_out, x.cap);
                            if (x.size) memset(x.data, 0x5a, x.size);
                        }
                    } else if (chain) {   // (the batch's place in the chain: k)
                        if (sa_stage(ctx, in.data(), (int)in.size()) != 0 ||
                            sa_run_aligned(ctx, &c, &acfg[ctx], chain, (uint64_t)k) != 0 ||
                            sa_fetch(ctx, outs.data(), (int)outs.size()) != 0)
                            return fail(std::string("encode failed: ") + sa_last_error(ctx));
                    } else if (sa_encode_blocks(ctx, in.data(), (int)in.size(), &c, outs.data()) != 0)
                        return fail(std::string("encode failed: ") + sa_last_error(ctx));
                }
                {
                    const double tf = now_s();
                    double cur = enc_busy.load();
                    while (!enc_busy.compare_exchange_weak(cur, cur + tf - te)) {}
                    cur = t_last_enc.load();
                    while (tf > cur && !t_last_enc.compare_exchange_weak(cur, tf)) {}
                }
                {
                    std::lock_guard<std::mutex> g(mu);
                    for (size_t i = 0; i < js.size(); i++) {
                        js[i]->out.n = outs[i].size;
                        js[i]->state = 2;
                    }
                }
                cv.notify_all();
            }
        });

    // writer (this thread): blocks in input order, each handed to the archive
    // writer's threads at its offset (ArcWriter); `written` counts the blocks
    // whose copy is done (the reader's bound on blocks in flight)
    int rc = 0;
    std::vector<sa_arc_block> info;
    uint64_t total = 0;
    uint32_t text_crc = 0;
    uint8_t hdr[16] = {0};
    ArcWriter aw;
    const int nwriters = std::max(1, std::min(8, o.writers));
    const bool opened = aw.open(path, nwriters, [&](std::unique_ptr<Job> j) {
        if (j->p) pool.put(std::move(j->p));
        outpool.give(j->out);
        j.reset();
        {
            std::lock_guard<std::mutex> g(mu);
            written++;
        }
        cv.notify_all();
    });
    if (!opened || !aw.lead(hdr, 16))   // patched at the end (createOutFile@0x417480 / writeFileInfo@0x4171b0)
        fail("cannot write " + path);
    for (int64_t i = 0;; i++) {
        std::unique_ptr<Job> j;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] {
                return failed || (nblocks >= 0 && i >= nblocks) || (jobs.count(i) && jobs[i]->state == 2);
            });
            if (failed || (nblocks >= 0 && i >= nblocks)) break;
            j = std::move(jobs[i]);
            jobs.erase(i);
        }
        if (aw.bad()) {   // writeData@0x40e070: exit(1)
            fail("write error on " + path);
            break;
        }
        info.push_back(sa_arc_block{(uint32_t)j->out.size(), j->len_long, j->text1, j->text2});
        text_crc = (uint32_t)crc32_combine(text_crc, j->crc, (z_off_t)(j->text1 + j->text2));
        const uint64_t off = 16 + total;
        total += j->out.size();
        aw.put(std::move(j), off);
    }
    const double t_written = now_s();
    reader.join();
    for (auto& t : parsers) t.join();
    for (auto& t : encoders) t.join();
    if (seg_free.joinable()) {
        {
            std::lock_guard<std::mutex> g(mu);
            seg_stop = true;   // (wakes it when the run ended early)
            cv.notify_all();
        }
        seg_free.join();
    }
    const double t_joined = now_s();
    // the archive is finished (trailer, header, closed) before the contexts'
    // device buffers are released (~1.4 s for five contexts' ~200 GB)
    auto release = [&]() {
        for (sa_hash_index* ix : indexes) sa_hash_destroy(ix);
        indexes.clear();
        if (chain) sa_align_chain_destroy(chain);
        chain = nullptr;
        for (sa_input*& I : sinputs) {
            sa_input_destroy(I);
            I = nullptr;
        }
        for (sa_ctx*& s : stagers) {
            sa_destroy(s);
            s = nullptr;
        }
        for (sa_ctx*& c : ctxs)
            if (c) {
                sa_destroy(c);
                c = nullptr;
            }
    };
    if (failed) {
        aw.finish(nullptr, 0, 0, nullptr, 0);
        release();
        fprintf(stderr, "seqarc_amd: %s\n", err.c_str());
        return 1;
    }
    sa_arc_info ai{o.f1, pe ? o.f2 : nullptr, pe ? 1 : 0, in1.is_gz ? 1 : 0, plus_bare, cfg.md5,
                   cfg.lossy > 0.0 ? 1 : 0, tmpl, o.ref ? rf.md5 : nullptr, (uint32_t)o.insert};
    std::vector<uint8_t> tr(4096 + 40 * info.size());
    const int64_t tl = sa_arc_trailer2(&ai, o.maxmis, info.data(), (uint32_t)info.size(), tr.data(), tr.size());
    if (tl < 0) {
        fprintf(stderr, "seqarc_amd: trailer failed\n");
        rc = 1;
    } else {
        sa_arc_header(total, hdr);
    }
    if (!aw.finish(tl < 0 ? nullptr : tr.data(), tl < 0 ? 0 : (size_t)tl, 16 + total, tl < 0 ? nullptr : hdr, 16)) {
        if (tl >= 0) fprintf(stderr, "seqarc_amd: write error on %s\n", path.c_str());
        rc = 1;
    }
    const double t_closed = now_s();
    // (diagnostics, SA_CLI_EXIT_PROBE=1: what the exit would tear down, timed
    // here instead -- the output pool's buffers, then the contexts)
    if (std::getenv("SA_CLI_EXIT_PROBE") && std::atoi(std::getenv("SA_CLI_EXIT_PROBE")) != 0) {
        size_t nb = 0, cap = 0;
        const double p0 = now_s();
        {
            std::lock_guard<std::mutex> g(outpool.mu);
            nb = outpool.free.size();
            for (auto& b : outpool.free) cap += b.cap;
            outpool.free.clear();
        }
        const double p1 = now_s();
        release();
        const double p2 = now_s();
        fprintf(stderr, "seqarc_amd: exit probe: output pool %zu buffers, %.3f GB reserved, freed in %.3f s; contexts "
                        "released in %.3f s\n", nb, (double)cap / 1e9, p1 - p0, p2 - p1);
    }
    // the contexts' device buffers (~200 GB for five contexts) are left to the
    // process exit unless --release: the command line exits right after this
    // (main, g_fast_exit), and the driver reclaims them without the ~1.4 s of
    // hipFree calls (round 3 g3n)
    if (o.release) release();
    else g_fast_exit = true;
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    if (o.verbose)
        fprintf(stderr, "seqarc_amd: blocks written %.3f s, segment ring freed %.3f s, encoders done %.3f s, archive closed %.3f s, contexts %s %.3f s\n",
                t_written, t_seg_freed.load(), t_joined, t_closed, o.release ? "released" : "left to the exit", secs);
    if (tl >= 0) {
        if (o.verbose)
            fprintf(stderr,
                    "seqarc_amd: contexts ready %.3f s, encoders started %.3f s, input read %.3f s, first encode %.3f s, last encode "
                    "done %.3f s; encode busy %.3f s over %zu contexts, parse busy %.3f s over %d threads; "
                    "reader: fill %.3f s, cut %.3f s; stage %.3f s (%s parse)\n",
                    t_ctx, t_enc_start, t_read_done.load(), t_first_enc.load(), t_last_enc.load(), enc_busy.load(), ctxs.size(),
                    parse_busy.load(), nparse, fill_busy, cut_busy, stage_busy.load(),
                    dev_parse ? "device" : "host");
        if (o.verbose && texts.pinned) {
            size_t nch;
            {
                std::lock_guard<std::mutex> g(texts.mu);
                nch = texts.chunks.size();
            }
            fprintf(stderr, "seqarc_amd: text windows: %zu chunks of %zu pinned (%zu ahead, %u on demand, the last at "
                            "%.3f s)\n", nch, TextPool::kChunk, prefill_chunks, texts.on_demand.load(),
                    texts.last_on_demand.load());
        }
        if (o.ingest_only) fprintf(stderr, "seqarc_amd: ingest text crc32 %08x\n", text_crc);
        fprintf(stderr, "seqarc_amd: %zu block(s), %llu -> %llu bytes (%.2fx), %.3f s, %.1f MB/s\n", info.size(),
                (unsigned long long)total_in, (unsigned long long)(16 + total + tl),
                (double)total_in / (double)(16 + total + tl), secs, (double)total_in / secs / 1e6);
    }
    if (g_fast_exit) fast_exit(rc, o.verbose);   // (every thread joined, the archive closed)
    return rc;
}

// ---- decompression --------------------------------------------------------
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

// One decoded block, written as FASTQ records.  mate: -1 all reads in order,
// 0 / 1 only the r1 / r2 reads of a PE block (DecodePipeOutJob::recoverData*,
// mode 1 / 2); bare: '+' lines without the ID.
void write_reads(FILE* f, FILE* f2, const std::vector<uint8_t>& names, const std::vector<uint16_t>& nl,
                 const std::vector<uint8_t>& seq, const std::vector<int32_t>& sl, const std::vector<uint8_t>& qual,
                 uint32_t n, bool paired, int mate, bool bare)
{
    const uint8_t *nm = names.data(), *sq = seq.data(), *ql = qual.data();
    for (uint32_t r = 0; r < n; r++) {
        const size_t L = (size_t)sl[r], N = nl[r];
        const bool keep = mate < 0 || (int)(r & 1) == mate;
        FILE* o = (paired && mate < 0 && f2 && (r & 1)) ? f2 : f;
        if (keep) {
            fputc('@', o);
            fwrite(nm, 1, N, o);
            fputc('\n', o);
            fwrite(sq, 1, L, o);
            fputs("\n+", o);
            if (!bare) fwrite(nm, 1, N, o);
            fputc('\n', o);
            fwrite(ql, 1, L, o);
            fputc('\n', o);
        }
        nm += N;
        sq += L;
        ql += L;
    }
}

// SeqArc -d: SeqArcFile::readFileInfo@0x419660 (header, trailer params, block
// table), -t blocks decoded at once (ISeqArcDecodeThread::doJob@0x435580),
// written in block order.  Output names (SeqArcParam::getDecodeFile@0x405f70,
// appendname@0x405f10): PREFIX_1.fastq / PREFIX_2.fastq (PE) or PREFIX.fastq
// (SE); without a prefix the stored input names (3 more bytes cut when input 1
// was gzip, as the binary does).  -P writes to stdout instead.
int decompress(const Options& o)
{
    std::vector<uint8_t> a;
    {
        FILE* f = fopen(o.arc, "rb");
        if (!f) { fprintf(stderr, "Error:The file %s may be not exist!\n", o.arc); return 1; }
        fseek(f, 0, SEEK_END);
        a.resize((size_t)ftell(f));
        fseek(f, 0, SEEK_SET);
        if (fread(a.data(), 1, a.size(), f) != a.size()) { fclose(f); return 1; }
        fclose(f);
    }
    if (a.size() < 16 || memcmp(a.data(), ".arc", 4) || a[7] != 0x82) {
        fprintf(stderr, "seqarc_amd: %s is not a SeqArc 1.6 archive\n", o.arc);
        return 1;
    }
    const uint64_t region = be(a.data() + 8, 8) & ((1ull << 56) - 1);
    if (16 + region > a.size()) return 1;
    const uint8_t *t = a.data() + 16 + region, *end = a.data() + a.size();
    int w;
    if (vint(t, end, w) != 3 || !w) return 1;
    t += w + 4;
    // params encap (ID 1, 2-byte size): fields 1-18 (writeParam@0x416450)
    if (vint(t, end, w) != 1 || !w) return 1;
    t += w;
    const uint64_t psz = be(t, 2) & 0x3fff;
    t += 2;
    const uint8_t* pend = t + psz;
    uint8_t tmpl[512] = {0};
    int bare = 1, paired = 0, lossy = 0, md5 = 1, gz1 = 0, noref = 1;
    uint32_t nblocks = 0, insert = 0;
    // SeqArc's default (param+0x1b60); field 19 when the archive was made with
    // another; an archive without field 19 (SeqArc's own, made with a
    // seqarc.config maxmis, or an earlier build of this tool) takes -d --maxmis
    int maxmis = o.maxmis_set ? o.maxmis : 7;
    std::string name1, name2;
    while (t < pend) {
        const uint64_t id = vint(t, pend, w);
        if (!w) return 1;
        t += w;
        const int sw = id == 15 ? 2 : 1;
        const uint64_t ln = be(t, sw) & ((1ull << (7 * sw)) - 1);
        t += sw;
        if (t + ln > pend) return 1;
        if (id == 1) noref = t[0];
        else if (id == 10 && ln >= 2) insert = (uint32_t)(t[0] | t[1] << 8);
        else if (id == 2) bare = t[0];
        else if (id == 4) gz1 = t[0];
        else if (id == 11 && ln >= 4) nblocks = (uint32_t)(t[0] | t[1] << 8 | t[2] << 16 | (uint32_t)t[3] << 24);
        else if (id == 13) name1.assign((const char*)t, ln);
        else if (id == 14 && ln) { paired = 1; name2.assign((const char*)t, ln); }
        else if (id == 15 && ln == 512) memcpy(tmpl, t, 512);
        else if (id == 16) lossy = t[0];
        else if (id == 17) md5 = t[0];
        else if (id == 19 && ln >= 1) maxmis = t[0];   // (ours: a non-default --maxmis)
        t += ln;
    }
    // writeMd5@0x416b10: the reference FASTA's MD5 (ID 8), archives made with one
    uint8_t arc_md5[16] = {0};
    bool have_md5 = false;
    if (vint(t, end, w) == 8 && w) {
        t += w;
        if (t + 17 > end || (be(t, 1) & 0x7f) != 16) return 1;
        memcpy(arc_md5, t + 1, 16);
        have_md5 = true;
        t += 17;
    }
    // the genome of an archive made with a reference (Decompress::loadRef: the
    // index's packed bases, or the FASTA packed the same way)
    RefFiles rf;
    std::vector<uint32_t> gwords;
    uint64_t gbases = 0;
    if (!noref) {
        if (!o.ref) {
            fprintf(stderr, "seqarc_amd: %s was made with a reference: give ref.fa\n", o.arc);
            return 1;
        }
        if (!load_ref(o.ref, false, rf, o.shm, o.verbose)) return 1;
        if (have_md5 && memcmp(arc_md5, rf.md5, 16)) {   // checkMd5@0x416c40
            fprintf(stderr, "seqarc_amd: the reference %s is not the one %s was made with (MD5)\n", o.ref, o.arc);
            return 1;
        }
        if (rf.have_hash()) {   // K, bases, words, positions; words follow
            uint32_t hdr[4];
            memcpy(hdr, rf.hp, 16);
            if (16 + 4ull * hdr[2] > rf.hn) {
                fprintf(stderr, "seqarc_amd: %s.hash is truncated\n", o.ref);
                return 1;
            }
            gbases = hdr[1];
            gwords.resize(hdr[2]);
            memcpy(gwords.data(), rf.hp + 16, 4ull * hdr[2]);
            rf.drop_hash();
        } else if (!pack_fasta(rf.fasta, gwords, gbases)) {
            fprintf(stderr, "seqarc_amd: %s: not a FASTA file\n", o.ref);
            return 1;
        }
    }
    if (maxmis < 0 || maxmis > 8) {
        fprintf(stderr, "seqarc_amd: maxmis %d in the archive trailer (0..8 expected)\n", maxmis);
        return 1;
    }
    const sa_ref gref{gwords.data(), gbases, paired, maxmis, insert};
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
    sa_cfg cfg = o.cfg;
    cfg.md5 = md5;
    cfg.lossy = lossy ? 1.0 : 0.0;
    cfg.bin_mode = tmpl[0];

    // outputs
    FILE *o1 = nullptr, *o2 = nullptr;
    int mate = -1;
    if (o.pipe) {   // DecodePipeOutJob ctor@0x42fd00: SE -> all reads; PE: 1 -> r1, 2 -> r2, 3 -> pairs in order
        if (o.pipe < 1 || o.pipe > 3) return usage();
        o1 = stdout;
        mate = !paired ? -1 : o.pipe == 1 ? 0 : o.pipe == 2 ? 1 : -1;
    } else {
        const std::string dir = o.in_dir ? dir_of(o.arc) : std::string();
        auto name = [&](int i) {   // getDecodeFile(i)
            if (o.out && *o.out) {
                std::string p = o.out;
                if (o.in_dir && p.find('/') == std::string::npos) p = dir + p;
                return p + (i == 0 ? ".fastq" : i == 1 ? "_1.fastq" : "_2.fastq");
            }
            std::string s = i <= 1 ? name1 : name2;
            if (gz1 && s.size() >= 3) s = s.substr(0, s.size() - 3);
            // the archive's stored names (trailer fields 13/14) are untrusted: the
            // encoder only ever stores basenames (compressStr@0x4160f0), so keep the
            // part after the last '/' and refuse '.', '..' and control characters
            const size_t sl = s.rfind('/');
            if (sl != std::string::npos) s = s.substr(sl + 1);
            bool bad = s == "." || s == "..";
            for (unsigned char ch : s) bad |= ch < 0x20 || ch == 0x7f;
            if (bad || s == "@empty*" || s.empty())
                s = std::string("decode") + (i == 0 ? ".fastq" : i == 1 ? "_1.fastq" : "_2.fastq");
            return dir + s;
        };
        const std::string p1 = name(paired ? 1 : 0), p2 = paired ? name(2) : std::string();
        if (!may_write(p1, o.force) || (paired && !may_write(p2, o.force))) return 1;
        o1 = fopen(p1.c_str(), "wb");
        o2 = paired ? fopen(p2.c_str(), "wb") : nullptr;
        if (!o1 || (paired && !o2)) { fprintf(stderr, "seqarc_amd: cannot write %s\n", p1.c_str()); return 1; }
    }
    struct Dec {
        std::vector<uint8_t> names, seq, qual;
        std::vector<uint16_t> nl;
        std::vector<int32_t> sl;
        sa_decoded d{};
        int64_t rc = -1;
    };
    int rc = 0, bad_md5 = 0;
    const uint32_t nt = (uint32_t)std::max(1, o.threads > 0 ? o.threads : 1);
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
                d.rc = noref ? sa_decode_block(a.data() + bk.off, bk.size, &cfg, tmpl, (int32_t)bk.lng, &d.d)
                             : sa_decode_block_ref(a.data() + bk.off, bk.size, &cfg, tmpl, (int32_t)bk.lng, &gref, &d.d);
            });
        for (auto& x : th) x.join();
        for (uint32_t i = 0; i < n && !rc; i++) {
            Dec& d = ds[i];
            if (d.rc < 0) { fprintf(stderr, "seqarc_amd: block %u does not decode\n", b0 + i); rc = 1; break; }
            if (!d.d.md5_ok)   // (-l archives: a range-coder desync fills the rest of the block with N)
                fprintf(stderr, "seqarc_amd: block %u: Name/Seq/Qual md5 unequal%s\n", b0 + i,
                        lossy ? " (made with -l: its bases past a desync are N)" : "");
            bad_md5 |= !d.d.md5_ok;
            write_reads(o1, o2, d.names, d.nl, d.seq, d.sl, d.qual, d.d.nreads, paired, mate, bare);
        }
    }
    if (o1 && o1 != stdout) fclose(o1);
    else if (o1) fflush(o1);
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
    g_main_s = mono_s();
    setenv("SA_SYNC", "block", 0);   // encoder threads sleep on their streams (sa_create)
    Options o;
    std::vector<const char*> pos;
    for (int i = 1; i < argc; i++) {
        const char* a = argv[i];
        auto val = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
        auto ival = [&](int& dst, int lo) -> bool {
            const char* v = val();
            if (!v) return false;
            dst = std::max(lo, atoi(v));
            return true;
        };
        if (!strcmp(a, "-c")) o.compress = true;
        else if (!strcmp(a, "-d")) o.decompress = true;
        else if (!strcmp(a, "-1")) { if (!(o.f1 = val())) return usage(); }
        else if (!strcmp(a, "-2")) { if (!(o.f2 = val())) return usage(); }
        else if (!strcmp(a, "-o")) { if (!(o.out = val())) return usage(); }
        else if (!strcmp(a, "-n")) o.cfg.md5 = 0;
        else if (!strcmp(a, "-f")) o.force = true;
        else if (!strcmp(a, "-p")) o.in_dir = true;
        else if (!strcmp(a, "-l")) { const char* v = val(); if (!v) return usage(); o.cfg.lossy = atof(v); }
        else if (!strcmp(a, "-P")) { if (!ival(o.pipe, 0)) return usage(); }
        else if (!strcmp(a, "-t")) { if (!ival(o.threads, 1)) return usage(); }
        else if (!strcmp(a, "--slevel")) { if (!ival(o.cfg.slevel, 0)) return usage(); }
        else if (!strcmp(a, "--qlevel")) { if (!ival(o.cfg.qlevel, 0)) return usage(); }
        else if (!strcmp(a, "--device")) { if (!ival(o.device, 0)) return usage(); }
        else if (!strcmp(a, "--devices")) { if (!ival(o.devices, 1)) return usage(); }
        else if (!strcmp(a, "--contexts")) { if (!ival(o.contexts, 1)) return usage(); }
        else if (!strcmp(a, "--batch")) { if (!ival(o.batch, 1)) return usage(); }
        else if (!strcmp(a, "--block-size")) { if (!ival(o.block_mib, 1)) return usage(); }
        else if (!strcmp(a, "--share-device")) o.share_device = true;
        else if (!strcmp(a, "--host-only")) o.host_only = true;
        else if (!strcmp(a, "--ingest-only")) o.ingest_only = true;
        else if (!strcmp(a, "--ingest-crc")) o.ingest_crc = true;
        else if (!strcmp(a, "--read-threads")) { if (!ival(o.read_threads, 0)) return usage(); }
        else if (!strcmp(a, "--writers")) { if (!ival(o.writers, 1)) return usage(); }
        else if (!strcmp(a, "--no-ramp")) o.ramp = false;
        else if (!strcmp(a, "--ramp")) o.ramp = true;
        else if (!strcmp(a, "--release")) o.release = true;
        else if (!strcmp(a, "--stage-ahead")) o.stage_ahead = true;
        else if (!strcmp(a, "--host-parse")) o.host_parse = true;
        else if (!strcmp(a, "-v")) o.verbose = true;
        else if (!strcmp(a, "-i")) { o.index = true; if (!(o.ref = val())) return usage(); }
        else if (!strcmp(a, "-s")) o.shm = true;
        else if (!strcmp(a, "-q")) {   // -q -i: the minimizer index (MINI_INDEX) is not part of this build
            fprintf(stderr, "seqarc_amd: -q (minimizer index) is not part of this build; the HASH index is\n");
            return 2;
        }
        else if (!strcmp(a, "-I")) { if (!ival(o.insert, 0)) return usage(); o.insert = std::min(o.insert, 65535); }
        else if (!strcmp(a, "--maxmis")) {   // the Mis model (compressAlignInfo_Mis@0x425ff0) exists for 1..8
            if (!ival(o.maxmis, 0) || o.maxmis > 8) {
                fprintf(stderr, "seqarc_amd: --maxmis takes 0..8\n");
                return usage();
            }
            o.maxmis_set = true;
        }
        else if (a[0] != '-') pos.push_back(a);
        else return usage();
    }
    if (o.index) {
        if (o.compress || o.decompress || !pos.empty()) return usage();
        return build_index(o);
    }
    if (o.compress == o.decompress) return usage();
    if (o.compress && o.cfg.lossy > 0.0)   // (the reference's R-Block decoder loses sync on N / IUPAC bases)
        fprintf(stderr, "seqarc_amd: warning: -l: blocks with N / IUPAC bases may not decode back to their "
                        "bases (as in SeqArc 1.6); -d reports such blocks\n");
    // the first positional argument is the reference when it names a FASTA
    // (SeqArcParam::parseOptFromCmd@0x40b460: the argument before the inputs)
    if (!pos.empty() && is_fasta_name(pos[0])) {
        o.ref = pos[0];
        pos.erase(pos.begin());
    }
    if (o.decompress) {   // SeqArc -d [ref.fa] ARCHIVE [PREFIX]
        if (pos.empty() || pos.size() > 2) return usage();
        o.arc = pos[0];
        if (pos.size() == 2 && !o.out) o.out = pos[1];
        return decompress(o);
    }
    // SeqArc -c [ref.fa] -1 A [-2 B] OUT
    for (const char* p : pos) {
        if (o.out) return usage();
        o.out = p;
    }
    if (!o.f1 || !o.out) return usage();
    // one hardware queue per stream (four per context): with the runtime's
    // default of four queues (which the GPU boxes preset), the contexts' streams
    // share queues and one context's packets wait behind another's (DESIGN.md
    // 5); set before the device is used, overriding a preset value
    // (round 6: five per context with the streamed staging's copy stream;
    // SA_CLI_HWQ=n: n per context, A/B)
    {
        const bool stream = std::getenv("SA_CLI_STREAM") && std::atoi(std::getenv("SA_CLI_STREAM")) != 0;
        int per = stream ? 5 : 4;
        if (const char* e = std::getenv("SA_CLI_HWQ")) per = std::max(1, std::atoi(e));
        char q[16];
        snprintf(q, sizeof q, "%d", std::min(32, per * o.contexts + 4));   // (per device)
        setenv("GPU_MAX_HW_QUEUES", q, 1);
    }
    const int rc = compress(o);
    if (o.verbose && !o.decompress)   // (a compression that released its buffers: the same stamps)
        fprintf(stderr, "seqarc_amd: monotonic clock: main %.6f, exit %.6f\n", g_main_s, mono_s());
    return rc;
}
