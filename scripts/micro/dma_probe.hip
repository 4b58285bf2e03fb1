// Probe: does a large host-to-device copy (the command line's text staging,
// sa_stage_text: ~3.6 GB per batch from page-locked host memory) slow the
// kernels running beside it?  Times a scattered-store kernel (k_replay_seq's
// pattern: 4-byte stores at random positions of a 6 GB array) and a streaming
// copy kernel alone, then while hipMemcpyAsync moves 3.6 GB host -> device on
// another stream, from hipHostMalloc memory and from hipHostRegister'ed
// 2 MiB-aligned memory (madvise huge pages).
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

__global__ void k_scatter(uint32_t* __restrict__ out, size_t n_out, size_t n_items, uint32_t seed)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_items; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t h = (i + seed) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        out[h % n_out] = (uint32_t)i;
    }
}

__global__ void k_stream(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

static float time_kernel(hipStream_t s, int which, uint32_t* big, size_t n_big, uint4* a, uint4* b, size_t n_ab)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    if (which == 0)
        hipLaunchKernelGGL(k_scatter, dim3(8192), dim3(256), 0, s, big, n_big, (size_t)1500000000, 7u);
    else
        hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, s, a, b, n_ab);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms;
}

int main()
{
    CK(hipSetDevice(0));
    const size_t n_big = (6ull << 30) / 4, n_ab = (4ull << 30) / 16, copy = 3600ull << 20;
    uint32_t* big;
    uint4 *a, *b;
    uint8_t* dst;
    CK(hipMalloc(&big, n_big * 4));
    CK(hipMalloc(&a, n_ab * 16));
    CK(hipMalloc(&b, n_ab * 16));
    CK(hipMalloc(&dst, copy));
    CK(hipMemset(big, 0, n_big * 4));
    CK(hipMemset(a, 1, n_ab * 16));
    uint8_t* pinned;
    CK(hipHostMalloc(reinterpret_cast<void**>(&pinned), copy, hipHostMallocDefault));
    std::memset(pinned, 7, copy);
    void* huge = nullptr;
    if (posix_memalign(&huge, 2u << 20, copy) != 0) return 1;
    madvise(huge, copy, MADV_HUGEPAGE);
    std::memset(huge, 9, copy);
    CK(hipHostRegister(huge, copy, hipHostRegisterDefault));
    hipStream_t sk, sc;
    CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
    for (int which = 0; which < 2; which++) {
        const char* nm = which ? "stream copy 4 GB" : "scatter 1.5G x 4 B into 6 GB";
        time_kernel(sk, which, big, n_big, a, b, n_ab);   // warm
        const float alone = time_kernel(sk, which, big, n_big, a, b, n_ab);
        for (int src = 0; src < 2; src++) {
            const void* h = src ? huge : pinned;
            const auto t0 = std::chrono::steady_clock::now();
            CK(hipMemcpyAsync(dst, h, copy, hipMemcpyHostToDevice, sc));
            float during = 0;
            int runs = 0;
            while (hipStreamQuery(sc) == hipErrorNotReady) {
                during += time_kernel(sk, which, big, n_big, a, b, n_ab);
                runs++;
            }
            CK(hipStreamSynchronize(sc));
            const double cs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            std::printf("%s: alone %.2f ms; during a %.1f GB H2D copy from %s: %.2f ms (%d runs), copy %.3f s "
                        "(%.1f GB/s)\n",
                        nm, alone, copy / 1e9, src ? "registered huge-page memory" : "hipHostMalloc memory",
                        runs ? during / runs : 0.f, runs, cs, copy / 1e9 / cs);
        }
    }
    CK(hipHostUnregister(huge));
    free(huge);
    CK(hipHostFree(pinned));
    return 0;
}
