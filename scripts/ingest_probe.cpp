// ingest_probe.cpp -- round 5: what the host ingest of `seqarc_amd -c` can be
// built from, measured on the GPU box (one call, scripts/gpu_r5a.sh).
//   a) pread from a tmpfs file into page-locked memory, 1..16 threads
//   b) mmap of the file: fault-in by touching / MADV_POPULATE_READ, N threads
//   c) hipHostRegister of the mapped file (read-only), chunk sizes, threads
//   d) H2D DMA from the registered mapping, from plain pageable mapping
//   e) newline counting over the mapping on N threads
//   f) a kernel reading the registered mapping directly (zero copy)
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -o ingest_probe ingest_probe.cpp -lpthread
#include <hip/hip_runtime.h>
#include <emmintrin.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                            \
        }                                                                                       \
    } while (0)

template <class F>
static void par(int nt, F f)
{
    std::vector<std::thread> ts;
    for (int i = 0; i < nt; i++) ts.emplace_back(f, i);
    for (auto& t : ts) t.join();
}

static uint64_t count_nl(const uint8_t* t, uint64_t len)
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

__global__ void k_count(const uint4* __restrict__ p, uint64_t n16, unsigned long long* out)
{
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned c = 0;
    for (; i < n16; i += stride) {
        const uint4 v = p[i];
        const unsigned w[4] = {v.x, v.y, v.z, v.w};
        for (int k = 0; k < 4; k++) {
            const unsigned x = w[k] ^ 0x0a0a0a0au;
            c += __popc((x - 0x01010101u) & ~x & 0x80808080u);
        }
    }
    atomicAdd(out, (unsigned long long)c);
}

int main(int argc, char** argv)
{
    const char* path = argc > 1 ? argv[1] : "/dev/shm/ingest_probe.fq";
    const uint64_t GB = 1ull << 30;
    const uint64_t fsize = (argc > 2 ? strtoull(argv[2], nullptr, 10) : 8) * GB;
    // ---- the file: FASTQ-like records, 150 bp ----
    {
        const double t0 = now();
        std::string rec;
        std::vector<uint8_t> buf;
        buf.reserve(64u << 20);
        unsigned s = 1;
        while (buf.size() < (64u << 20)) {
            char hdr[64];
            int h = snprintf(hdr, sizeof hdr, "@SRR000%u/1\n", s);
            buf.insert(buf.end(), hdr, hdr + h);
            for (int i = 0; i < 150; i++) buf.push_back("ACGT"[(s = s * 1103515245u + 12345u) >> 30]);
            buf.push_back('\n');
            buf.push_back('+');
            buf.push_back('\n');
            for (int i = 0; i < 150; i++) buf.push_back('!' + ((s = s * 1103515245u + 12345u) >> 27));
            buf.push_back('\n');
        }
        int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
        if (fd < 0) { perror("open"); return 1; }
        for (uint64_t w = 0; w < fsize; w += buf.size()) {
            const size_t k = (size_t)std::min<uint64_t>(buf.size(), fsize - w);
            if (write(fd, buf.data(), k) != (ssize_t)k) { perror("write"); return 1; }
        }
        close(fd);
        printf("file %s: %.1f GB written in %.2f s\n", path, fsize / 1e9, now() - t0);
    }
    int ndev = 0;
    CK(hipGetDeviceCount(&ndev));
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    const int fd = open(path, O_RDONLY);
    const uint64_t slice = 4 * GB;

    // ---- a) pread into page-locked memory ----
    uint8_t* pinned = nullptr;
    CK(hipHostMalloc((void**)&pinned, slice, hipHostMallocDefault));
    memset(pinned, 0, slice);
    for (int nt : {1, 2, 4, 8, 12, 16}) {
        const double t0 = now();
        par(nt, [&](int i) {
            const uint64_t part = slice / nt, a = i * part;
            uint64_t got = 0;
            while (got < part) {
                ssize_t r = pread(fd, pinned + a + got, part - got, a + got);
                if (r <= 0) break;
                got += r;
            }
        });
        const double dt = now() - t0;
        printf("a) pread 4 GiB into pinned, %2d threads: %.3f s, %.1f GB/s\n", nt, dt, slice / dt / 1e9);
    }

    // ---- b) mmap + fault-in ----
    for (int mode = 0; mode < 2; mode++)
        for (int nt : {1, 4, 8, 16}) {
            uint8_t* m = (uint8_t*)mmap(nullptr, fsize, PROT_READ, MAP_SHARED, fd, 0);
            if (m == MAP_FAILED) { perror("mmap"); return 1; }
            const double t0 = now();
            std::atomic<uint64_t> sink{0};
            par(nt, [&](int i) {
                const uint64_t part = (fsize / nt) & ~4095ull, a = i * part, e = i == nt - 1 ? fsize : a + part;
                if (mode == 0) {
                    uint64_t s = 0;
                    for (uint64_t p = a; p < e; p += 4096) s += m[p];
                    sink += s;
                } else {
                    if (madvise(m + a, e - a, MADV_POPULATE_READ) != 0) perror("madvise");
                }
            });
            const double dt = now() - t0;
            printf("b) mmap %.1f GB, fault-in by %s, %2d threads: %.3f s (%.1f GB/s)\n", fsize / 1e9,
                   mode ? "MADV_POPULATE_READ" : "touch", nt, dt, fsize / dt / 1e9);
            if (nt == 16 && mode == 1) {
                // ---- e) newline count on the mapped pages ----
                for (int nt2 : {1, 4, 8, 16}) {
                    const double t1 = now();
                    std::atomic<uint64_t> tot{0};
                    par(nt2, [&](int i) {
                        const uint64_t part = fsize / nt2, a = i * part, e = i == nt2 - 1 ? fsize : a + part;
                        tot += count_nl(m + a, e - a);
                    });
                    const double dt2 = now() - t1;
                    printf("e) newline count over the mapping, %2d threads: %.3f s, %.1f GB/s (%llu)\n", nt2, dt2,
                           fsize / dt2 / 1e9, (unsigned long long)tot.load());
                }
            }
            munmap(m, fsize);
        }

    // ---- c) register the mapping; d) DMA from it ----
    uint8_t* dbuf = nullptr;
    CK(hipMalloc((void**)&dbuf, slice));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    unsigned long long* dcnt = nullptr;
    CK(hipMalloc((void**)&dcnt, 8));
    for (int populate = 0; populate < 2; populate++)
        for (uint64_t chunk : {256ull << 20, 1ull << 30, 4ull << 30}) {
            for (int nt : {1, 4}) {
                uint8_t* m = (uint8_t*)mmap(nullptr, fsize, PROT_READ, MAP_SHARED, fd, 0);
                if (populate) par(16, [&](int i) {
                    const uint64_t part = (fsize / 16) & ~4095ull, a = i * part, e = i == 15 ? fsize : a + part;
                    madvise(m + a, e - a, MADV_POPULATE_READ);
                });
                const uint64_t nch = std::min<uint64_t>(fsize / chunk, 16);
                std::vector<int> ok(nch, 0);
                std::vector<double> per(nch, 0);
                const double t0 = now();
                par(nt, [&](int i) {
                    for (uint64_t c = i; c < nch; c += nt) {
                        const double a = now();
                        hipError_t e = hipHostRegister(m + c * chunk, chunk, hipHostRegisterReadOnly);
                        per[c] = now() - a;
                        ok[c] = e == hipSuccess;
                        if (e != hipSuccess && c == 0) fprintf(stderr, "register: %s\n", hipGetErrorString(e));
                    }
                });
                const double dt = now() - t0;
                int nok = 0;
                for (int x : ok) nok += x;
                double pmax = 0;
                for (double x : per) pmax = std::max(pmax, x);
                printf("c) hipHostRegister(ReadOnly) %s mapping, %llu MiB chunks x %llu, %d threads: %.3f s (%.1f GB/s), "
                       "%d ok, slowest chunk %.3f s\n",
                       populate ? "populated" : "unpopulated", (unsigned long long)(chunk >> 20),
                       (unsigned long long)nch, nt, dt, nch * chunk / dt / 1e9, nok, pmax);
                if (nok == (int)nch && chunk == (1ull << 30) && nt == 1) {
                    // d) DMA from the registered mapping (4 GiB, 1 GiB copies)
                    for (int rep = 0; rep < 2; rep++) {
                        const double t1 = now();
                        for (uint64_t c = 0; c < 4 && c < nch; c++)
                            CK(hipMemcpyAsync(dbuf + c * chunk, m + c * chunk, chunk, hipMemcpyHostToDevice, st));
                        CK(hipStreamSynchronize(st));
                        const double dt1 = now() - t1;
                        printf("d) H2D DMA from the registered mapping, 4 x 1 GiB: %.3f s, %.1f GB/s\n", dt1,
                               4.0 * chunk / dt1 / 1e9);
                    }
                    // smaller copies, as the staging issues them (25 MiB per text)
                    {
                        const uint64_t sz = 25ull << 20, n = (4 * chunk) / sz;
                        const double t1 = now();
                        for (uint64_t c = 0; c < n; c++)
                            CK(hipMemcpyAsync(dbuf + c * sz, m + c * sz, sz, hipMemcpyHostToDevice, st));
                        CK(hipStreamSynchronize(st));
                        const double dt1 = now() - t1;
                        printf("d) H2D DMA from the registered mapping, %llu x 25 MiB: %.3f s, %.1f GB/s\n",
                               (unsigned long long)n, dt1, n * sz / dt1 / 1e9);
                    }
                    // f) zero copy: a kernel reads the registered pages
                    {
                        void* dp = nullptr;
                        CK(hipHostGetDevicePointer(&dp, m, 0));
                        for (int rep = 0; rep < 2; rep++) {
                            CK(hipMemsetAsync(dcnt, 0, 8, st));
                            const double t1 = now();
                            hipLaunchKernelGGL(k_count, dim3(4096), dim3(256), 0, st, (const uint4*)dp,
                                               (uint64_t)(4 * chunk / 16), dcnt);
                            CK(hipGetLastError());
                            CK(hipStreamSynchronize(st));
                            const double dt1 = now() - t1;
                            unsigned long long h = 0;
                            CK(hipMemcpy(&h, dcnt, 8, hipMemcpyDeviceToHost));
                            printf("f) kernel reading 4 GiB of the registered mapping: %.3f s, %.1f GB/s (%llu newlines, "
                                   "CPU %llu)\n",
                                   dt1, 4.0 * chunk / dt1 / 1e9, h, (unsigned long long)count_nl(m, 4 * chunk));
                        }
                    }
                }
                const double t2 = now();
                for (uint64_t c = 0; c < nch; c++)
                    if (ok[c]) CK(hipHostUnregister(m + c * chunk));
                printf("c) hipHostUnregister x %llu: %.3f s\n", (unsigned long long)nch, now() - t2);
                munmap(m, fsize);
            }
        }
    // d') pageable H2D from the mapping (no registration)
    {
        uint8_t* m = (uint8_t*)mmap(nullptr, fsize, PROT_READ, MAP_SHARED, fd, 0);
        for (int rep = 0; rep < 2; rep++) {
            const double t1 = now();
            for (uint64_t c = 0; c < 4; c++)
                CK(hipMemcpyAsync(dbuf + c * GB, m + c * GB, GB, hipMemcpyHostToDevice, st));
            CK(hipStreamSynchronize(st));
            const double dt1 = now() - t1;
            printf("d') H2D from the pageable mapping, 4 x 1 GiB: %.3f s, %.1f GB/s\n", dt1, 4.0 * GB / dt1 / 1e9);
        }
        munmap(m, fsize);
    }
    // d'') DMA from hipHostMalloc memory (the reference point)
    for (int rep = 0; rep < 2; rep++) {
        const double t1 = now();
        CK(hipMemcpyAsync(dbuf, pinned, slice, hipMemcpyHostToDevice, st));
        CK(hipStreamSynchronize(st));
        const double dt1 = now() - t1;
        printf("d'') H2D from hipHostMalloc memory, 4 GiB: %.3f s, %.1f GB/s\n", dt1, slice / dt1 / 1e9);
    }
    CK(hipHostFree(pinned));
    CK(hipFree(dbuf));
    close(fd);
    unlink(path);
    printf("done\n");
    return 0;
}
