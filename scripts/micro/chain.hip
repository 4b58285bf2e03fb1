// Microbenchmark: latency of the range-coder "range chain" and of MD5 on one
// wave, VALU (per-lane streams) vs SALU (wave-uniform) code generation.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <chrono>

struct Sym { uint32_t mlo, mhi, f, pad; };

// SALU form: one stream per wave, inputs through s_load (uniform addresses)
__global__ __launch_bounds__(64) void k_chain_salu(const Sym* __restrict__ syms, uint32_t n, uint32_t* __restrict__ qout, uint32_t* res)
{
    const uint32_t lane = threadIdx.x;
    const Sym* S = syms + (size_t)blockIdx.x * n;
    uint32_t* Q = qout + (size_t)blockIdx.x * n;
    uint32_t r = 0xffffffffu;
    for (uint32_t base = 0; base < n; base += 64) {
        uint32_t qv = 0;
#pragma unroll 8
        for (uint32_t j = 0; j < 64; j++) {
            const Sym s = S[base + j];
            const uint32_t t1 = (uint32_t)(((uint64_t)s.mlo * r) >> 32);
            const uint32_t q = (uint32_t)(((uint64_t)s.mhi * r + t1) >> 32);
            const uint32_t rr = q * s.f;
            r = rr << (__builtin_clz(rr) & 24);
            qv = lane == j ? q : qv;
        }
        Q[base + lane] = qv;
    }
    if (lane == 0) res[blockIdx.x] = r;
}

// VALU form: each lane its own stream (lane-strided layout), per-lane loads
__global__ __launch_bounds__(64) void k_chain_valu(const Sym* __restrict__ syms, uint32_t n, uint32_t* __restrict__ qout, uint32_t* res)
{
    const uint32_t lane = threadIdx.x;
    const uint32_t stream = blockIdx.x * 64 + lane;
    uint32_t r = 0xffffffffu;
    const uint32_t nstreams = gridDim.x * 64;
#pragma unroll 8
    for (uint32_t i = 0; i < n; i++) {
        const Sym s = syms[(size_t)i * nstreams + stream];
        const uint32_t t1 = __umulhi(s.mlo, r);
        const uint32_t q = (uint32_t)(((uint64_t)s.mhi * r + t1) >> 32);
        const uint32_t rr = q * s.f;
        r = rr << (__builtin_clz(rr) & 24);
        qout[(size_t)i * nstreams + stream] = q;
    }
    res[stream] = r;
}

// f64 form (VALU, per lane)
__global__ __launch_bounds__(64) void k_chain_f64(const double* __restrict__ inv, const uint32_t* __restrict__ fs, uint32_t n, uint32_t* __restrict__ qout, uint32_t* res)
{
    const uint32_t lane = threadIdx.x;
    const uint32_t stream = blockIdx.x * 64 + lane;
    const uint32_t nstreams = gridDim.x * 64;
    double r = 4294967295.0;
#pragma unroll 8
    for (uint32_t i = 0; i < n; i++) {
        const size_t k = (size_t)i * nstreams + stream;
        const double q = __builtin_trunc(r * inv[k]);
        const double rr = q * (double)fs[k];
        const int e = __builtin_amdgcn_frexp_exp(rr);   // rr in [2^(e-1), 2^e)
        const int sh = ((32 - e) >> 3) << 3;
        r = __builtin_ldexp(rr, sh);
        qout[k] = (uint32_t)q;
    }
    res[stream] = (uint32_t)r;
}

__device__ inline uint32_t rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }
#define STEP(F, a, b, c, d, x, k, s) a = b + rotl(a + F(b, c, d) + x + k, s)
#define FF(b, c, d) (((c ^ d) & b) ^ d)
#define GG(b, c, d) (((b ^ c) & d) ^ c)
#define HH(b, c, d) (b ^ c ^ d)
#define II(b, c, d) (c ^ (b | ~d))
__device__ inline void md5_block(uint32_t h[4], const uint32_t* M)
{
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    STEP(FF,a,b,c,d,M[0],0xd76aa478,7); STEP(FF,d,a,b,c,M[1],0xe8c7b756,12); STEP(FF,c,d,a,b,M[2],0x242070db,17); STEP(FF,b,c,d,a,M[3],0xc1bdceee,22);
    STEP(FF,a,b,c,d,M[4],0xf57c0faf,7); STEP(FF,d,a,b,c,M[5],0x4787c62a,12); STEP(FF,c,d,a,b,M[6],0xa8304613,17); STEP(FF,b,c,d,a,M[7],0xfd469501,22);
    STEP(FF,a,b,c,d,M[8],0x698098d8,7); STEP(FF,d,a,b,c,M[9],0x8b44f7af,12); STEP(FF,c,d,a,b,M[10],0xffff5bb1,17); STEP(FF,b,c,d,a,M[11],0x895cd7be,22);
    STEP(FF,a,b,c,d,M[12],0x6b901122,7); STEP(FF,d,a,b,c,M[13],0xfd987193,12); STEP(FF,c,d,a,b,M[14],0xa679438e,17); STEP(FF,b,c,d,a,M[15],0x49b40821,22);
    STEP(GG,a,b,c,d,M[1],0xf61e2562,5); STEP(GG,d,a,b,c,M[6],0xc040b340,9); STEP(GG,c,d,a,b,M[11],0x265e5a51,14); STEP(GG,b,c,d,a,M[0],0xe9b6c7aa,20);
    STEP(GG,a,b,c,d,M[5],0xd62f105d,5); STEP(GG,d,a,b,c,M[10],0x02441453,9); STEP(GG,c,d,a,b,M[15],0xd8a1e681,14); STEP(GG,b,c,d,a,M[4],0xe7d3fbc8,20);
    STEP(GG,a,b,c,d,M[9],0x21e1cde6,5); STEP(GG,d,a,b,c,M[14],0xc33707d6,9); STEP(GG,c,d,a,b,M[3],0xf4d50d87,14); STEP(GG,b,c,d,a,M[8],0x455a14ed,20);
    STEP(GG,a,b,c,d,M[13],0xa9e3e905,5); STEP(GG,d,a,b,c,M[2],0xfcefa3f8,9); STEP(GG,c,d,a,b,M[7],0x676f02d9,14); STEP(GG,b,c,d,a,M[12],0x8d2a4c8a,20);
    STEP(HH,a,b,c,d,M[5],0xfffa3942,4); STEP(HH,d,a,b,c,M[8],0x8771f681,11); STEP(HH,c,d,a,b,M[11],0x6d9d6122,16); STEP(HH,b,c,d,a,M[14],0xfde5380c,23);
    STEP(HH,a,b,c,d,M[1],0xa4beea44,4); STEP(HH,d,a,b,c,M[4],0x4bdecfa9,11); STEP(HH,c,d,a,b,M[7],0xf6bb4b60,16); STEP(HH,b,c,d,a,M[10],0xbebfbc70,23);
    STEP(HH,a,b,c,d,M[13],0x289b7ec6,4); STEP(HH,d,a,b,c,M[0],0xeaa127fa,11); STEP(HH,c,d,a,b,M[3],0xd4ef3085,16); STEP(HH,b,c,d,a,M[6],0x04881d05,23);
    STEP(HH,a,b,c,d,M[9],0xd9d4d039,4); STEP(HH,d,a,b,c,M[12],0xe6db99e5,11); STEP(HH,c,d,a,b,M[15],0x1fa27cf8,16); STEP(HH,b,c,d,a,M[2],0xc4ac5665,23);
    STEP(II,a,b,c,d,M[0],0xf4292244,6); STEP(II,d,a,b,c,M[7],0x432aff97,10); STEP(II,c,d,a,b,M[14],0xab9423a7,15); STEP(II,b,c,d,a,M[5],0xfc93a039,21);
    STEP(II,a,b,c,d,M[12],0x655b59c3,6); STEP(II,d,a,b,c,M[3],0x8f0ccc92,10); STEP(II,c,d,a,b,M[10],0xffeff47d,15); STEP(II,b,c,d,a,M[1],0x85845dd1,21);
    STEP(II,a,b,c,d,M[8],0x6fa87e4f,6); STEP(II,d,a,b,c,M[15],0xfe2ce6e0,10); STEP(II,c,d,a,b,M[6],0xa3014314,15); STEP(II,b,c,d,a,M[13],0x4e0811a1,21);
    STEP(II,a,b,c,d,M[4],0xf7537e82,6); STEP(II,d,a,b,c,M[11],0xbd3af235,10); STEP(II,c,d,a,b,M[2],0x2ad7d2bb,15); STEP(II,b,c,d,a,M[9],0xeb86d391,21);
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}

// SALU MD5: message read with uniform addresses (s_load)
__global__ __launch_bounds__(64) void k_md5_salu(const uint32_t* __restrict__ msg, uint32_t nblk, uint32_t* out)
{
    const uint32_t* M = msg + (size_t)blockIdx.x * nblk * 16;
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    for (uint32_t b = 0; b < nblk; b++) md5_block(h, M + (size_t)b * 16);
    if (threadIdx.x == 0) for (int k = 0; k < 4; k++) out[blockIdx.x * 4 + k] = h[k];
}
// VALU MD5: one message per lane
__global__ __launch_bounds__(64) void k_md5_valu(const uint32_t* __restrict__ msg, uint32_t nblk, uint32_t* out)
{
    const uint32_t id = blockIdx.x * 64 + threadIdx.x;
    const uint4* M4 = reinterpret_cast<const uint4*>(msg + (size_t)id * nblk * 16);
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    for (uint32_t b = 0; b < nblk; b++) {
        uint32_t M[16];
        for (int k = 0; k < 4; k++) { uint4 v = M4[b * 4 + k]; M[4*k]=v.x; M[4*k+1]=v.y; M[4*k+2]=v.z; M[4*k+3]=v.w; }
        md5_block(h, M);
    }
    for (int k = 0; k < 4; k++) out[id * 4 + k] = h[k];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main()
{
    const uint32_t n = 1u << 20;       // symbols per stream
    const int nwaves[] = {1, 64, 256};
    std::vector<Sym> hs((size_t)n * 64);
    uint32_t x = 12345;
    for (auto& s : hs) {
        x = x * 1664525u + 1013904223u;
        uint32_t t = 12 + (x >> 8) % 240;   // BASE_MODEL-like totals
        uint32_t f = 1 + (x >> 20) % (t - 1);
        uint64_t m = ~0ull / t + 1;
        s = Sym{(uint32_t)m, (uint32_t)(m >> 32), f, t};
    }
    Sym* d_s; uint32_t *d_q, *d_res;
    CK(hipMalloc(&d_s, hs.size() * sizeof(Sym)));
    CK(hipMalloc(&d_q, hs.size() * 4 * 4));
    CK(hipMalloc(&d_res, 4096 * 4));
    CK(hipMemcpy(d_s, hs.data(), hs.size() * sizeof(Sym), hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    for (int w : {1, 64}) {
        uint32_t per = (uint32_t)((size_t)n * 64 / w / 64 * 64);
        if (per > n) per = n;
        hipLaunchKernelGGL(k_chain_salu, dim3(w), dim3(64), 0, 0, d_s, per, d_q, d_res);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_chain_salu, dim3(w), dim3(64), 0, 0, d_s, per, d_q, d_res); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("chain_salu  waves=%4d syms/stream=%u : %.2f ns/sym/stream\n", w, per, ms * 1e6 / per);
    }
    for (int w : {1, 16}) {
        uint32_t per = (uint32_t)((size_t)n * 64 / (w * 64)); if (per > 1u << 18) per = 1u << 18;
        hipLaunchKernelGGL(k_chain_valu, dim3(w), dim3(64), 0, 0, d_s, per, d_q, d_res);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_chain_valu, dim3(w), dim3(64), 0, 0, d_s, per, d_q, d_res); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("chain_valu  waves=%4d lanes=%d syms/stream=%u : %.2f ns/sym/stream\n", w, w * 64, per, ms * 1e6 / per);
    }
    {
        std::vector<double> inv(hs.size()); std::vector<uint32_t> fs(hs.size());
        for (size_t i = 0; i < hs.size(); i++) { inv[i] = (1.0 + 0x1p-45) / hs[i].pad; fs[i] = hs[i].f; }
        double* d_inv; uint32_t* d_f;
        CK(hipMalloc(&d_inv, inv.size() * 8)); CK(hipMalloc(&d_f, fs.size() * 4));
        CK(hipMemcpy(d_inv, inv.data(), inv.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_f, fs.data(), fs.size() * 4, hipMemcpyHostToDevice));
        for (int w : {1, 16}) {
            uint32_t per = (uint32_t)((size_t)n * 64 / (w * 64)); if (per > 1u << 18) per = 1u << 18;
            hipLaunchKernelGGL(k_chain_f64, dim3(w), dim3(64), 0, 0, d_inv, d_f, per, d_q, d_res);
            CK(hipEventRecord(a)); hipLaunchKernelGGL(k_chain_f64, dim3(w), dim3(64), 0, 0, d_inv, d_f, per, d_q, d_res); CK(hipEventRecord(b));
            CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
            printf("chain_f64   waves=%4d lanes=%d syms/stream=%u : %.2f ns/sym/stream\n", w, w * 64, per, ms * 1e6 / per);
        }
        // verify f64 == integer on a stream
        std::vector<uint32_t> q1(1024), q2(1024);
        hipLaunchKernelGGL(k_chain_valu, dim3(1), dim3(64), 0, 0, d_s, 1024u, d_q, d_res);
        CK(hipMemcpy(q1.data(), d_q, 4096, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(k_chain_f64, dim3(1), dim3(64), 0, 0, d_inv, d_f, 1024u, d_q, d_res);
        CK(hipMemcpy(q2.data(), d_q, 4096, hipMemcpyDeviceToHost));
        printf("f64 vs int q identical: %d\n", (int)(q1 == q2));
    }
    // MD5
    {
        const uint32_t nblk = 1u << 14;   // 1 MiB per message
        uint32_t* d_m; uint32_t* d_o;
        CK(hipMalloc(&d_m, (size_t)nblk * 64 * 64)); CK(hipMemset(d_m, 0x5a, (size_t)nblk * 64 * 64));
        CK(hipMalloc(&d_o, 64 * 16 * 64));
        for (int w : {1, 64}) {
            hipLaunchKernelGGL(k_md5_salu, dim3(w), dim3(64), 0, 0, d_m, nblk, d_o);
            CK(hipEventRecord(a)); hipLaunchKernelGGL(k_md5_salu, dim3(w), dim3(64), 0, 0, d_m, nblk, d_o); CK(hipEventRecord(b));
            CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
            printf("md5_salu waves=%d : %.2f ns/64B-block  (%.3f GB/s per message)\n", w, ms * 1e6 / nblk, nblk * 64.0 / (ms * 1e6));
        }
        const uint32_t nb2 = 1u << 10;
        hipLaunchKernelGGL(k_md5_valu, dim3(1), dim3(64), 0, 0, d_m, nb2, d_o);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_md5_valu, dim3(1), dim3(64), 0, 0, d_m, nb2, d_o); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("md5_valu 64 lanes : %.2f ns/64B-block/lane (%.3f GB/s per message)\n", ms * 1e6 / nb2, nb2 * 64.0 / (ms * 1e6));
    }
    return 0;
}
