// Probe: host time of device allocations and releases at the command line's
// sizes (five contexts x ~33 GB + ~41 GB of front scratch), as hipMalloc /
// hipFree and from a stream-ordered pool (hipMallocAsync with the release
// threshold at its maximum, so freed memory stays in the pool), each from
// several host threads at once as the command line's contexts do.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_touch(uint32_t* p, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (uint32_t)i;
}

// spins for `cycles` of the wall clock (s_memrealtime, 100 MHz) on every lane
__global__ void k_spin(uint64_t ticks, uint32_t* out)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[0] = x;
}

int main(int argc, char** argv)
{
    const int threads = argc > 1 ? std::atoi(argv[1]) : 5;
    const double gb_per_thread = argc > 2 ? std::atof(argv[2]) : 33.0;
    const size_t chunk = (size_t)(argc > 3 ? std::atof(argv[3]) : 2.0) * (1ull << 30);
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    size_t fr = 0, tot = 0;
    CK(hipMemGetInfo(&fr, &tot));
    std::printf("device memory: %.1f GB free of %.1f GB\n", fr / 1e9, tot / 1e9);
    const size_t per = (size_t)(gb_per_thread * 1e9);
    const int nchunks = (int)((per + chunk - 1) / chunk);

    // 1. hipMalloc / touch / hipFree, `threads` host threads at once
    for (int touch = 0; touch < 2; touch++) {
        std::vector<std::vector<void*>> ptr(threads);
        std::vector<double> ta(threads), tf(threads);
        double t0 = now();
        {
            std::vector<std::thread> th;
            for (int t = 0; t < threads; t++)
                th.emplace_back([&, t]() {
                    CK(hipSetDevice(0));
                    const double a = now();
                    for (int c = 0; c < nchunks; c++) {
                        void* p = nullptr;
                        CK(hipMalloc(&p, chunk));
                        ptr[t].push_back(p);
                    }
                    ta[t] = now() - a;
                });
            for (auto& x : th) x.join();
        }
        const double t_alloc = now() - t0;
        double t_touch = 0;
        if (touch) {
            const double a = now();
            for (auto& v : ptr)
                for (void* p : v) hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, 0, (uint32_t*)p, chunk / 4);
            CK(hipDeviceSynchronize());
            t_touch = now() - a;
        }
        t0 = now();
        {
            std::vector<std::thread> th;
            for (int t = 0; t < threads; t++)
                th.emplace_back([&, t]() {
                    CK(hipSetDevice(0));
                    const double a = now();
                    for (void* p : ptr[t]) CK(hipFree(p));
                    tf[t] = now() - a;
                });
            for (auto& x : th) x.join();
        }
        const double t_free = now() - t0;
        const double gb = (double)threads * nchunks * chunk / 1e9;
        std::printf("hipMalloc%s: %d threads x %d x %.1f GB = %.0f GB: alloc %.3f s (%.1f ms/GB), touch %.3f s, free %.3f s "
                    "(%.1f ms/GB); per thread alloc %.3f..%.3f s\n",
                    touch ? "+touch" : "", threads, nchunks, chunk / 1e9, gb, t_alloc, t_alloc / gb * 1e3, t_touch,
                    t_free, t_free / gb * 1e3, ta[0], ta[threads - 1]);
    }

    // 2. stream-ordered pool: allocate, free back to the pool, allocate again
    hipMemPool_t pool;
    CK(hipDeviceGetDefaultMemPool(&pool, 0));
    uint64_t thr = UINT64_MAX;
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    for (int round = 0; round < 2; round++) {
        std::vector<void*> ptr;
        double a = now();
        for (int t = 0; t < threads; t++)
            for (int c = 0; c < nchunks; c++) {
                void* p = nullptr;
                CK(hipMallocAsync(&p, chunk, st));
                ptr.push_back(p);
            }
        CK(hipStreamSynchronize(st));
        const double t_alloc = now() - a;
        for (void* p : ptr) hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, st, (uint32_t*)p, chunk / 4);
        a = now();
        for (void* p : ptr) CK(hipFreeAsync(p, st));
        CK(hipStreamSynchronize(st));
        const double t_free = now() - a;
        const double gb = (double)ptr.size() * chunk / 1e9;
        std::printf("pool round %d: %.0f GB: alloc %.3f s (%.1f ms/GB), touch+free %.3f s\n", round, gb, t_alloc,
                    t_alloc / gb * 1e3, t_free);
    }
    // 3. hipMalloc / hipFree of 4 GB while a kernel keeps the device busy for ~2 s
    {
        uint32_t* sink = nullptr;
        CK(hipMalloc(&sink, 256));
        hipStream_t busy;
        CK(hipStreamCreate(&busy));
        hipLaunchKernelGGL(k_spin, dim3(256), dim3(64), 0, busy, (uint64_t)200000000, sink);   // 2 s at 100 MHz
        const double a0 = now();
        void* p = nullptr;
        CK(hipMalloc(&p, 4ull << 30));
        const double a1 = now();
        CK(hipFree(p));
        const double a2 = now();
        CK(hipStreamSynchronize(busy));
        std::printf("while a 2 s kernel runs: hipMalloc(4 GB) %.3f s, hipFree %.3f s, kernel done at %.3f s\n", a1 - a0,
                    a2 - a1, now() - a0);
    }
    double a = now();
    CK(hipMemPoolTrimTo(pool, 0));
    CK(hipDeviceSynchronize());
    std::printf("pool trim: %.3f s\n", now() - a);
    return 0;
}
