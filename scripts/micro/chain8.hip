// Microbenchmark 8: the pass R chain fed from VGPRs -- one lane-parallel
// vector load per 64-record segment, LA segments ahead (vector loads return in
// order, so the lookahead can be deep), v_readlane into SGPRs per symbol.
// Microbenchmark 3: range chain on the scalar unit with SMEM-double-buffered
// inputs (16 symbols x {Mlo, Mhi, f} per chunk = 3 x s_load_dwordx16) and one
// range checkpoint stored per 64 symbols.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#ifndef LA
#define LA 2
#endif
struct Chunk { uint32_t w[32]; };   // 16 symbols x {m = ceil(2^32/t), t | f << 16}

__device__ __forceinline__ uint32_t step(uint32_t r, uint32_t m, uint32_t tf, uint32_t)
{
#ifdef ASM_STEP
    uint32_t t, f, q, p;
    asm volatile(
        "s_and_b32 %1, %5, 0xffff\n\t"
        "s_lshr_b32 %2, %5, 16\n\t"
        "s_mul_hi_u32 %3, %0, %6\n\t"
        "s_mul_i32 %4, %3, %1\n\t"
        "s_cmp_lt_u32 %0, %4\n\t"
        "s_subb_u32 %3, %3, 0\n\t"
        "s_mul_i32 %3, %3, %2\n\t"
        "s_flbit_i32_b32 %4, %3\n\t"
        "s_and_b32 %4, %4, 24\n\t"
        "s_lshl_b32 %0, %3, %4"
        : "+s"(r), "=&s"(t), "=&s"(f), "=&s"(q), "=&s"(p)
        : "s"(tf), "s"(m)
        : "scc");
    return r;
#else
    const uint32_t t = tf & 0xffff, f = tf >> 16;
    uint32_t q = __umulhi(r, m);
    q -= (r < q * t) ? 1u : 0u;
    const uint32_t rr = q * f;
    return rr << (__builtin_clz(rr) & 24);
#endif
}

__global__ __launch_bounds__(64) void k_passr2(const Chunk* __restrict__ chunks, uint32_t nchunks, uint32_t* __restrict__ ckpt, uint32_t* res)
{
    const uint32_t lane = threadIdx.x;
    const uint2* P = reinterpret_cast<const uint2*>(chunks + (size_t)blockIdx.x * (nchunks + 4 + 8 * LA)) + lane;
    uint32_t* K = ckpt + (size_t)blockIdx.x * (nchunks / 4 + 64);
    uint32_t r = 0xffffffffu;
    uint32_t kv = 0;
    const uint32_t nseg = nchunks / 4;
    uint2 buf[LA + 1];
#pragma unroll
    for (int k = 0; k < LA; k++) buf[k] = P[(size_t)k * 64];
    for (uint32_t g = 0; g < nseg; g += LA + 1) {
#pragma unroll
        for (int k = 0; k <= LA; k++) {
            buf[(k + LA) % (LA + 1)] = P[(size_t)(g + k + LA) * 64];
            const uint32_t m = buf[k].x, tf = buf[k].y;
#pragma unroll
            for (int j = 0; j < 64; j++)
                r = step(r, __builtin_amdgcn_readlane(m, j), __builtin_amdgcn_readlane(tf, j), 0);
            const uint32_t s = g + k;
            kv = lane == (s & 63) ? r : kv;
            if ((s & 63) == 63) K[s - 63 + lane] = kv;
        }
    }
    if (lane == 0) res[blockIdx.x] = r;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main()
{
    const uint32_t nchunks = 65536;     // 1M symbols per stream
    const int W = 128;
    std::vector<Chunk> h((size_t)(nchunks + 4 + 8 * LA) * W);
    std::vector<uint32_t> tt((size_t)nchunks * 16 * W);
    uint32_t x = 777;
    for (int s = 0; s < W; s++)
        for (uint32_t c = 0; c < nchunks + 4 + 8 * LA; c++)
            for (int j = 0; j < 16; j++) {
                x = x * 1664525u + 1013904223u;
                uint32_t t = 12 + (x >> 8) % 240, f = 1 + (x >> 20) % (t - 1);
                Chunk& ch = h[(size_t)s * (nchunks + 4 + 8 * LA) + c];
                ch.w[2 * j] = (uint32_t)((0x100000000ull + t - 1) / t); ch.w[2 * j + 1] = t | (f << 16);
                if (c < nchunks) tt[((size_t)s * nchunks + c) * 16 + j] = t;
            }
    Chunk* d; uint32_t *dk, *dres;
    CK(hipMalloc(&d, h.size() * sizeof(Chunk)));
    CK(hipMalloc(&dk, (size_t)W * (nchunks / 4 + 64) * 4)); CK(hipMalloc(&dres, 4096 * 4));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(Chunk), hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    for (int w : {1, 32, W}) {
        hipLaunchKernelGGL(k_passr2, dim3(w), dim3(64), 0, 0, d, nchunks, dk, dres);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_passr2, dim3(w), dim3(64), 0, 0, d, nchunks, dk, dres); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("LA=%d vgpr streams=%3d : %.2f ns/sym/stream\n", LA, w, ms * 1e6 / (nchunks * 16.0));
    }
    std::vector<uint32_t> res(W);
    CK(hipMemcpy(res.data(), dres, W * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (int s = 0; s < W; s++) {
        uint32_t r = 0xffffffffu;
        for (uint32_t c = 0; c < nchunks; c++)
            for (int j = 0; j < 16; j++) {
                const Chunk& ch = h[(size_t)s * (nchunks + 4 + 8 * LA) + c];
                uint32_t q = r / tt[((size_t)s * nchunks + c) * 16 + j];
                uint32_t rr = q * (ch.w[2 * j + 1] >> 16);
                r = rr << (__builtin_clz(rr) & 24);
            }
        bad += r != res[s];
    }
    printf("final range check: %zu of %d streams differ\n", bad, W);
    return 0;
}
