// pin_probe: page-locking cost of host memory (hipHostRegister / unregister,
// hipHostMalloc) against how it was allocated: 2 MiB-aligned with the
// transparent-huge-page hint, registered untouched or after the first touch;
// plain 4 KiB pages; and what the kernel gave (AnonHugePages).  The command
// line's segment ring is page-locked at ~12 GB/s (round 5, r5a), which bounds
// how fast its first pass over the ring can go.
//   hipcc -O2 -o pin_probe scripts/micro/pin_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include <thread>
#include <vector>

static double now()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static long anon_huge_kb()
{
    FILE* f = fopen("/proc/self/smaps_rollup", "r");
    if (!f) return -1;
    char line[256];
    long kb = -1;
    while (fgets(line, sizeof line, f))
        if (!strncmp(line, "AnonHugePages:", 14)) kb = atol(line + 14);
    fclose(f);
    return kb;
}

int main(int argc, char** argv)
{
    const size_t gb = argc > 1 ? (size_t)atol(argv[1]) : 8;
    const size_t n = gb << 30;
    hipInit(0);
    struct Case {
        const char* name;
        bool huge, touch;
        int threads;
    } cases[] = {{"2M-aligned + THP hint, untouched", true, false, 1},
                 {"2M-aligned + THP hint, touched first (8 threads)", true, true, 1},
                 {"2M-aligned + THP hint, touched, 4 register threads", true, true, 4},
                 {"4K pages (no hint), touched first", false, true, 1}};
    for (const Case& c : cases) {
        void* p = nullptr;
        if (posix_memalign(&p, 2u << 20, n) != 0) return 1;
        madvise(p, n, c.huge ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
        double tt = 0;
        if (c.touch) {
            const double t0 = now();
            std::vector<std::thread> th;
            for (int i = 0; i < 8; i++)
                th.emplace_back([=]() { memset((char*)p + n / 8 * i, 0, n / 8); });
            for (auto& t : th) t.join();
            tt = now() - t0;
        }
        const long huge = anon_huge_kb();
        const double t0 = now();
        std::vector<std::thread> th;
        const size_t part = n / c.threads;
        bool ok = true;
        for (int i = 0; i < c.threads; i++)
            th.emplace_back([&, i]() {
                if (hipHostRegister((char*)p + part * i, part, hipHostRegisterPortable) != hipSuccess) ok = false;
            });
        for (auto& t : th) t.join();
        const double tr = now() - t0;
        const double t1 = now();
        for (int i = 0; i < c.threads; i++) hipHostUnregister((char*)p + part * i);
        const double tu = now() - t1;
        const double t2 = now();
        free(p);
        printf("%-52s %zu GB: touch %.3f s, register %.3f s (%.1f GB/s)%s, unregister %.3f s, free %.3f s, AnonHugePages %ld MB\n",
               c.name, gb, tt, tr, gb / tr, ok ? "" : " FAILED", tu, now() - t2, huge / 1024);
    }
    // the command line's segment ring: 512 MiB segments, touched, registered,
    // each the source of an H2D copy; then released (unregister + free) on one
    // thread or on eight
    for (int rel_threads : {1, 8}) {
        const size_t seg = 512ull << 20, ns = n / seg;
        std::vector<void*> segs(ns, nullptr);
        void* d = nullptr;
        if (hipMalloc(&d, seg) != hipSuccess) return 1;
        for (size_t k = 0; k < ns; k++) {
            if (posix_memalign(&segs[k], 2u << 20, seg) != 0) return 1;
            madvise(segs[k], seg, MADV_HUGEPAGE);
            memset(segs[k], 1, seg);
            if (hipHostRegister(segs[k], seg, hipHostRegisterPortable) != hipSuccess) return 1;
            if (hipMemcpy(d, segs[k], seg, hipMemcpyHostToDevice) != hipSuccess) return 1;
        }
        const double t0 = now();
        std::vector<std::thread> th;
        double tu_sum[8] = {0}, tf_sum[8] = {0};
        for (int i = 0; i < rel_threads; i++)
            th.emplace_back([&, i]() {
                for (size_t k = i; k < ns; k += rel_threads) {
                    const double a = now();
                    hipHostUnregister(segs[k]);
                    const double b = now();
                    free(segs[k]);
                    tu_sum[i] += b - a;
                    tf_sum[i] += now() - b;
                }
            });
        for (auto& t : th) t.join();
        const double tr = now() - t0;
        double tu = 0, tf = 0;
        for (int i = 0; i < rel_threads; i++) {
            tu += tu_sum[i];
            tf += tf_sum[i];
        }
        (void)hipFree(d);
        printf("segment ring %zu x 512 MiB, released on %d thread(s): %.3f s (unregister %.3f s, free %.3f s summed)\n",
               ns, rel_threads, tr, tu, tf);
    }
    {
        void* p = nullptr;
        const double t0 = now();
        const hipError_t e = hipHostMalloc(&p, n, hipHostMallocPortable);
        const double ta = now() - t0;
        const double t1 = now();
        if (e == hipSuccess) hipHostFree(p);
        printf("%-52s %zu GB: alloc %.3f s (%.1f GB/s), free %.3f s\n", "hipHostMalloc", gb, ta, gb / ta, now() - t1);
    }
    return 0;
}
