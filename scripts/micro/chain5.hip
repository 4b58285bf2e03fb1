// Microbenchmark 5: pass-R range chain, 2-dword records {m, t | f << 16}
// (10 SALU / symbol) against 3-dword records {m, t, f} (8 SALU / symbol).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int W, int R = 16> struct Chunk { uint32_t w[R * W]; };

__device__ __forceinline__ void step2(uint32_t& r, uint32_t m, uint32_t tf)
{
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
}

__device__ __forceinline__ void step3(uint32_t& r, uint32_t m, uint32_t t, uint32_t f)
{
    uint32_t q, p;
    asm volatile(
        "s_mul_hi_u32 %1, %0, %3\n\t"
        "s_mul_i32 %2, %1, %4\n\t"
        "s_cmp_lt_u32 %0, %2\n\t"
        "s_subb_u32 %1, %1, 0\n\t"
        "s_mul_i32 %1, %1, %5\n\t"
        "s_flbit_i32_b32 %2, %1\n\t"
        "s_and_b32 %2, %2, 24\n\t"
        "s_lshl_b32 %0, %1, %2"
        : "+s"(r), "=&s"(q), "=&s"(p)
        : "s"(m), "s"(t), "s"(f)
        : "scc");
}

template <int W>
__device__ __forceinline__ void steps(uint32_t& r, const Chunk<W>& A, int j0)
{
#pragma unroll
    for (int j = j0; j < 16; j++) {
        if constexpr (W == 2) step2(r, A.w[2 * j], A.w[2 * j + 1]);
        else step3(r, A.w[3 * j], A.w[3 * j + 1], A.w[3 * j + 2]);
    }
}

template <int W>
__device__ __forceinline__ void first(uint32_t& r, const Chunk<W>& A)
{
    if constexpr (W == 2) step2(r, A.w[0], A.w[1]);
    else step3(r, A.w[0], A.w[1], A.w[2]);
}

template <int W, int PF = 0>
__global__ __launch_bounds__(64) void k_passr(const Chunk<W>* __restrict__ chunks, uint32_t nchunks,
                                              uint32_t* __restrict__ ckpt, uint32_t* res,
                                              const uint32_t* __restrict__ pfp = nullptr)
{
    uint32_t pf_acc = 0, pf_prev = 0;
    const uint32_t lane = threadIdx.x;
    const Chunk<W>* C = chunks + (size_t)blockIdx.x * (nchunks + 4);
    uint32_t* K = ckpt + (size_t)blockIdx.x * (nchunks / 4 + 64);
    uint32_t r = 0xffffffffu, kv = 0;
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    Chunk<W> A = C[0], B;
    for (uint32_t c = 0; c < nchunks; c += 2) {
        first<W>(r, A);   // waits for A; then B is requested while A is coded
        __builtin_amdgcn_sched_barrier(0);
        B = C[c + 1];
        __builtin_amdgcn_sched_barrier(0);
        steps<W>(r, A, 1);
        first<W>(r, B);
        __builtin_amdgcn_sched_barrier(0);
        A = C[c + 2];
        __builtin_amdgcn_sched_barrier(0);
        steps<W>(r, B, 1);
        if (PF > 0 && c + PF + 2 <= nchunks) {   // touch the records PF chunks ahead (lane-parallel: 2 chunks) into L2
            pf_acc += pf_prev;
            pf_prev = pfp[(size_t)blockIdx.x * (nchunks + 4) * (16 * W) + (size_t)(c + PF) * (16 * W) + lane];
        }
        if ((c & 3) == 2) {
            const uint32_t slot = (c >> 2) & 63;
            kv = lane == slot ? r : kv;
            if (slot == 63) K[(c >> 2) - 63 + lane] = kv;
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    if (pf_acc + pf_prev == 0x12345678u) res[8000] = 1;   // keeps the prefetch loads
    if (lane == 0) {
        res[blockIdx.x] = r;
        res[4096 + 2 * blockIdx.x] = (uint32_t)(c1 - c0);
        res[4096 + 2 * blockIdx.x + 1] = (uint32_t)(t1 - t0);
    }
}

// 3-dword records, 8 per chunk, three chunks in flight (SGPR budget: 72 of 102)
using C8 = Chunk<3, 8>;
__device__ __forceinline__ void steps8(uint32_t& r, const C8& A, int j0)
{
#pragma unroll
    for (int j = j0; j < 8; j++) step3(r, A.w[3 * j], A.w[3 * j + 1], A.w[3 * j + 2]);
}
__global__ __launch_bounds__(64) void k_passr8(const C8* __restrict__ chunks, uint32_t nchunks, uint32_t* __restrict__ ckpt,
                                               uint32_t* res)
{
    const uint32_t lane = threadIdx.x;
    const C8* C = chunks + (size_t)blockIdx.x * (nchunks + 8);
    uint32_t* K = ckpt + (size_t)blockIdx.x * (nchunks / 8 + 64);
    uint32_t r = 0xffffffffu, kv = 0;
    C8 A = C[0], B = C[1], D;
    for (uint32_t c = 0; c < nchunks; c += 3) {
        steps8(r, A, 0);
        __builtin_amdgcn_sched_barrier(0);
        D = C[c + 2];
        __builtin_amdgcn_sched_barrier(0);
        steps8(r, B, 0);
        __builtin_amdgcn_sched_barrier(0);
        A = C[c + 3];
        __builtin_amdgcn_sched_barrier(0);
        steps8(r, D, 0);
        __builtin_amdgcn_sched_barrier(0);
        B = C[c + 4];
        __builtin_amdgcn_sched_barrier(0);
        if ((c & 7) == 0) {
            const uint32_t slot = (c >> 3) & 63;
            kv = lane == slot ? r : kv;
            if (slot == 63) K[(c >> 3) - 63 + lane] = kv;
        }
    }
    if (lane == 0) res[blockIdx.x] = r;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int W>
int run(const char* name)
{
    const uint32_t nchunks = 65536;   // 1M symbols per stream
    const int NS = 256;
    std::vector<Chunk<W>> h((size_t)(nchunks + 4) * NS);
    std::vector<uint32_t> tt((size_t)(nchunks + 4) * 16 * NS), ff(tt.size());
    uint32_t x = 777;
    for (size_t i = 0; i < h.size(); i++)
        for (int j = 0; j < 16; j++) {
            x = x * 1664525u + 1013904223u;
            uint32_t t = 12 + (x >> 8) % 240, f = 1 + (x >> 20) % (t - 1);
            uint32_t m = (uint32_t)((0x100000000ull + t - 1) / t);
            if (W == 2) { h[i].w[2 * j] = m; h[i].w[2 * j + 1] = t | (f << 16); }
            else { h[i].w[3 * j] = m; h[i].w[3 * j + 1] = t; h[i].w[3 * j + 2] = f; }
            tt[i * 16 + j] = t; ff[i * 16 + j] = f;
        }
    Chunk<W>* d; uint32_t *dk, *dres;
    CK(hipMalloc(&d, h.size() * sizeof(Chunk<W>)));
    CK(hipMalloc(&dk, (size_t)NS * (nchunks / 4 + 64) * 4)); CK(hipMalloc(&dres, 3 * 4096 * 4));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(Chunk<W>), hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    for (int pfv : {0, 8, 32}) {
        for (int w : {32, 64, 128}) {
            auto kern = pfv == 0 ? k_passr<W, 0> : pfv == 8 ? k_passr<W, 8> : k_passr<W, 32>;
            hipLaunchKernelGGL(kern, dim3(w), dim3(64), 0, 0, d, nchunks, dk, dres, (const uint32_t*)d);
            CK(hipEventRecord(a)); hipLaunchKernelGGL(kern, dim3(w), dim3(64), 0, 0, d, nchunks, dk, dres, (const uint32_t*)d); CK(hipEventRecord(b));
            CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
            printf("%s prefetch %2d chunks ahead, streams=%3d : %.2f ns/sym\n", name, pfv, w, ms * 1e6 / (nchunks * 16.0));
        }
    }
    for (int lds : {0})
    for (int w : {1}) {
        hipLaunchKernelGGL(k_passr<W>, dim3(w), dim3(64), lds, 0, d, nchunks, dk, dres);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_passr<W>, dim3(w), dim3(64), lds, 0, d, nchunks, dk, dres); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        std::vector<uint32_t> cr(2 * w);
        CK(hipMemcpy(cr.data(), dres + 4096, 8 * w, hipMemcpyDeviceToHost));
        double cyc = 0, rt = 0;
        for (int i = 0; i < w; i++) { cyc += cr[2 * i]; rt += cr[2 * i + 1]; }
        printf("%s streams=%3d lds=%6d : %.2f ns/sym/stream, %.1f cycles/sym, clock %.0f MHz (memtime / memrealtime at 100 MHz)\n",
               name, w, lds, ms * 1e6 / (nchunks * 16.0), cyc / w / (nchunks * 16.0), cyc / rt * 100.0);
    }
    {
        hipDeviceProp_t prop;
        CK(hipGetDeviceProperties(&prop, 0));
        const int ncu = prop.multiProcessorCount;
        for (int every : {2, 4}) {
            for (int phase = 0; phase < 2; phase++) {
                std::vector<uint32_t> m((ncu + 31) / 32, 0u);
                for (int cu = 0; cu < ncu; cu++)
                    if (cu % every == phase) m[cu / 32] |= 1u << (cu % 32);
                hipStream_t sm;
                CK(hipExtStreamCreateWithCUMask(&sm, (uint32_t)ncu, m.data()));
                for (int w : {32, 64, 128}) {
                    hipLaunchKernelGGL(k_passr<W>, dim3(w), dim3(64), 0, sm, d, nchunks, dk, dres);
                    CK(hipEventRecord(a, sm));
                    hipLaunchKernelGGL(k_passr<W>, dim3(w), dim3(64), 0, sm, d, nchunks, dk, dres);
                    CK(hipEventRecord(b, sm));
                    CK(hipEventSynchronize(b));
                    CK(hipEventElapsedTime(&ms, a, b));
                    std::vector<uint32_t> cr(2 * w);
                    CK(hipMemcpy(cr.data(), dres + 4096, 8 * w, hipMemcpyDeviceToHost));
                    double cyc = 0;
                    for (int i = 0; i < w; i++) cyc += cr[2 * i];
                    printf("%s CU mask cu%%%d==%d streams=%3d : %.2f ns/sym, %.1f cycles/sym\n", name, every, phase, w,
                           ms * 1e6 / (nchunks * 16.0), cyc / w / (nchunks * 16.0));
                }
                CK(hipStreamDestroy(sm));
            }
        }
    }
    std::vector<uint32_t> res(NS);
    CK(hipMemcpy(res.data(), dres, NS * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (int s = 0; s < NS; s++) {
        uint32_t r = 0xffffffffu;
        for (size_t i = (size_t)s * (nchunks + 4) * 16; i < ((size_t)s * (nchunks + 4) + nchunks) * 16; i++) {
            uint32_t q = r / tt[i], rr = q * ff[i];
            r = rr << (__builtin_clz(rr) & 24);
        }
        bad += r != res[s];
    }
    printf("%s final range check: %zu of %d streams differ\n", name, bad, NS);
    CK(hipFree(d)); CK(hipFree(dk)); CK(hipFree(dres));
    return 0;
}

int run8()
{
    const uint32_t nchunks = 3 * 43690;   // ~1M symbols per stream
    const int NS = 128;
    std::vector<C8> h((size_t)(nchunks + 8) * NS);
    std::vector<uint32_t> tt((size_t)(nchunks + 8) * 8 * NS), ff(tt.size());
    uint32_t x = 777;
    for (size_t i = 0; i < h.size(); i++)
        for (int j = 0; j < 8; j++) {
            x = x * 1664525u + 1013904223u;
            uint32_t t = 12 + (x >> 8) % 240, f = 1 + (x >> 20) % (t - 1);
            h[i].w[3 * j] = (uint32_t)((0x100000000ull + t - 1) / t); h[i].w[3 * j + 1] = t; h[i].w[3 * j + 2] = f;
            tt[i * 8 + j] = t; ff[i * 8 + j] = f;
        }
    C8* d; uint32_t *dk, *dres;
    CK(hipMalloc(&d, h.size() * sizeof(C8)));
    CK(hipMalloc(&dk, (size_t)NS * (nchunks / 8 + 64) * 4)); CK(hipMalloc(&dres, 4096 * 4));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(C8), hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    for (int w : {1, 32, NS}) {
        hipLaunchKernelGGL(k_passr8, dim3(w), dim3(64), 0, 0, d, nchunks, dk, dres);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_passr8, dim3(w), dim3(64), 0, 0, d, nchunks, dk, dres); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("3-dword/8 SALU, 8-rec x3 streams=%3d : %.2f ns/sym/stream\n", w, ms * 1e6 / (nchunks * 8.0));
    }
    std::vector<uint32_t> res(NS);
    CK(hipMemcpy(res.data(), dres, NS * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (int s = 0; s < NS; s++) {
        uint32_t r = 0xffffffffu;
        for (size_t i = (size_t)s * (nchunks + 8) * 8; i < ((size_t)s * (nchunks + 8) + nchunks) * 8; i++) {
            uint32_t q = r / tt[i], rr = q * ff[i];
            r = rr << (__builtin_clz(rr) & 24);
        }
        bad += r != res[s];
    }
    printf("8-rec final range check: %zu of %d streams differ\n", bad, NS);
    return 0;
}

int main()
{
    if (run<2>("2-dword/10 SALU")) return 1;
    return 0;
}
