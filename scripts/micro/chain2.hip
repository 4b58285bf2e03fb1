// Microbenchmark 2: range chain and MD5 on one wave with VMEM-prefetched
// inputs broadcast by v_readlane into SALU arithmetic.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define RL(v, j) __builtin_amdgcn_readlane((int)(v), (j))
#define WL(v, q, j) asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(q), "i"(j))

// R1: 64-bit reciprocal (3 readlanes / symbol)
__global__ __launch_bounds__(64) void k_r1(const uint4* __restrict__ syms, uint32_t n, uint32_t* __restrict__ qout, uint32_t* res)
{
    const uint32_t lane = threadIdx.x;
    const uint4* S = syms + (size_t)blockIdx.x * n;
    uint32_t* Q = qout + (size_t)blockIdx.x * n;
    uint32_t r = 0xffffffffu;
    auto proc = [&](const uint4& c0, uint32_t base) {
        uint32_t qv = 0;
#pragma unroll
        for (int j = 0; j < 64; j++) {
            const uint32_t mlo = RL(c0.x, j), mhi = RL(c0.y, j), f = RL(c0.z, j);
            const uint32_t t1 = (uint32_t)(((uint64_t)mlo * r) >> 32);
            const uint32_t q = (uint32_t)(((uint64_t)mhi * r + t1) >> 32);
            const uint32_t rr = q * f;
            r = rr << (__builtin_clz(rr) & 24);
            WL(qv, q, j);
        }
        Q[base + lane] = qv;
    };
    uint4 c0 = S[lane], c1 = S[64 + lane], c2;
    for (uint32_t base = 0; base < n; base += 192) {
        __builtin_amdgcn_sched_barrier(0); c2 = S[base + 128 + lane]; __builtin_amdgcn_sched_barrier(0);
        proc(c0, base);
        __builtin_amdgcn_sched_barrier(0); c0 = S[base + 192 + lane]; __builtin_amdgcn_sched_barrier(0);
        proc(c1, base + 64);
        __builtin_amdgcn_sched_barrier(0); c1 = S[base + 256 + lane]; __builtin_amdgcn_sched_barrier(0);
        proc(c2, base + 128);
    }
    if (lane == 0) res[blockIdx.x] = r;
}

// R2: 32-bit reciprocal m = ceil(2^32/t) with one correction (2 readlanes / symbol)
__global__ __launch_bounds__(64) void k_r2(const uint2* __restrict__ syms, uint32_t n, uint32_t* __restrict__ qout, uint32_t* res)
{
    const uint32_t lane = threadIdx.x;
    const uint2* S = syms + (size_t)blockIdx.x * n;
    uint32_t* Q = qout + (size_t)blockIdx.x * n;
    uint32_t r = 0xffffffffu;
    auto proc = [&](const uint2& c0, uint32_t base) {
        uint32_t qv = 0;
#pragma unroll
        for (int j = 0; j < 64; j++) {
            const uint32_t m = RL(c0.x, j), tf = RL(c0.y, j);
            const uint32_t t = tf & 0xffff, f = tf >> 16;
            uint32_t q = __umulhi(r, m);
            q -= (q * t > r) ? 1u : 0u;
            const uint32_t rr = q * f;
            r = rr << (__builtin_clz(rr) & 24);
            WL(qv, q, j);
        }
        Q[base + lane] = qv;
    };
    uint2 c0 = S[lane], c1 = S[64 + lane], c2;
    for (uint32_t base = 0; base < n; base += 192) {
        __builtin_amdgcn_sched_barrier(0); c2 = S[base + 128 + lane]; __builtin_amdgcn_sched_barrier(0);
        proc(c0, base);
        __builtin_amdgcn_sched_barrier(0); c0 = S[base + 192 + lane]; __builtin_amdgcn_sched_barrier(0);
        proc(c1, base + 64);
        __builtin_amdgcn_sched_barrier(0); c1 = S[base + 256 + lane]; __builtin_amdgcn_sched_barrier(0);
        proc(c2, base + 128);
    }
    if (lane == 0) res[blockIdx.x] = r;
}

__device__ inline uint32_t rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }
#define STEP(F, a, b, c, d, x, k, s) a = b + rotl(a + F(b, c, d) + x + k, s)
#define FF(b, c, d) (((c ^ d) & b) ^ d)
#define GG(b, c, d) (((b ^ c) & d) ^ c)
#define HH(b, c, d) (b ^ c ^ d)
#define II(b, c, d) (c ^ (b | ~d))
#define MD5_ROUNDS(M) \
    STEP(FF,a,b,c,d,M(0),0xd76aa478,7); STEP(FF,d,a,b,c,M(1),0xe8c7b756,12); STEP(FF,c,d,a,b,M(2),0x242070db,17); STEP(FF,b,c,d,a,M(3),0xc1bdceee,22); \
    STEP(FF,a,b,c,d,M(4),0xf57c0faf,7); STEP(FF,d,a,b,c,M(5),0x4787c62a,12); STEP(FF,c,d,a,b,M(6),0xa8304613,17); STEP(FF,b,c,d,a,M(7),0xfd469501,22); \
    STEP(FF,a,b,c,d,M(8),0x698098d8,7); STEP(FF,d,a,b,c,M(9),0x8b44f7af,12); STEP(FF,c,d,a,b,M(10),0xffff5bb1,17); STEP(FF,b,c,d,a,M(11),0x895cd7be,22); \
    STEP(FF,a,b,c,d,M(12),0x6b901122,7); STEP(FF,d,a,b,c,M(13),0xfd987193,12); STEP(FF,c,d,a,b,M(14),0xa679438e,17); STEP(FF,b,c,d,a,M(15),0x49b40821,22); \
    STEP(GG,a,b,c,d,M(1),0xf61e2562,5); STEP(GG,d,a,b,c,M(6),0xc040b340,9); STEP(GG,c,d,a,b,M(11),0x265e5a51,14); STEP(GG,b,c,d,a,M(0),0xe9b6c7aa,20); \
    STEP(GG,a,b,c,d,M(5),0xd62f105d,5); STEP(GG,d,a,b,c,M(10),0x02441453,9); STEP(GG,c,d,a,b,M(15),0xd8a1e681,14); STEP(GG,b,c,d,a,M(4),0xe7d3fbc8,20); \
    STEP(GG,a,b,c,d,M(9),0x21e1cde6,5); STEP(GG,d,a,b,c,M(14),0xc33707d6,9); STEP(GG,c,d,a,b,M(3),0xf4d50d87,14); STEP(GG,b,c,d,a,M(8),0x455a14ed,20); \
    STEP(GG,a,b,c,d,M(13),0xa9e3e905,5); STEP(GG,d,a,b,c,M(2),0xfcefa3f8,9); STEP(GG,c,d,a,b,M(7),0x676f02d9,14); STEP(GG,b,c,d,a,M(12),0x8d2a4c8a,20); \
    STEP(HH,a,b,c,d,M(5),0xfffa3942,4); STEP(HH,d,a,b,c,M(8),0x8771f681,11); STEP(HH,c,d,a,b,M(11),0x6d9d6122,16); STEP(HH,b,c,d,a,M(14),0xfde5380c,23); \
    STEP(HH,a,b,c,d,M(1),0xa4beea44,4); STEP(HH,d,a,b,c,M(4),0x4bdecfa9,11); STEP(HH,c,d,a,b,M(7),0xf6bb4b60,16); STEP(HH,b,c,d,a,M(10),0xbebfbc70,23); \
    STEP(HH,a,b,c,d,M(13),0x289b7ec6,4); STEP(HH,d,a,b,c,M(0),0xeaa127fa,11); STEP(HH,c,d,a,b,M(3),0xd4ef3085,16); STEP(HH,b,c,d,a,M(6),0x04881d05,23); \
    STEP(HH,a,b,c,d,M(9),0xd9d4d039,4); STEP(HH,d,a,b,c,M(12),0xe6db99e5,11); STEP(HH,c,d,a,b,M(15),0x1fa27cf8,16); STEP(HH,b,c,d,a,M(2),0xc4ac5665,23); \
    STEP(II,a,b,c,d,M(0),0xf4292244,6); STEP(II,d,a,b,c,M(7),0x432aff97,10); STEP(II,c,d,a,b,M(14),0xab9423a7,15); STEP(II,b,c,d,a,M(5),0xfc93a039,21); \
    STEP(II,a,b,c,d,M(12),0x655b59c3,6); STEP(II,d,a,b,c,M(3),0x8f0ccc92,10); STEP(II,c,d,a,b,M(10),0xffeff47d,15); STEP(II,b,c,d,a,M(1),0x85845dd1,21); \
    STEP(II,a,b,c,d,M(8),0x6fa87e4f,6); STEP(II,d,a,b,c,M(15),0xfe2ce6e0,10); STEP(II,c,d,a,b,M(6),0xa3014314,15); STEP(II,b,c,d,a,M(13),0x4e0811a1,21); \
    STEP(II,a,b,c,d,M(4),0xf7537e82,6); STEP(II,d,a,b,c,M(11),0xbd3af235,10); STEP(II,c,d,a,b,M(2),0x2ad7d2bb,15); STEP(II,b,c,d,a,M(9),0xeb86d391,21);

// M1: SALU MD5, message prefetched with VMEM (4 x 64-B blocks per wave load), readlane broadcast
__global__ __launch_bounds__(64) void k_md5_rl(const uint32_t* __restrict__ msg, uint32_t nblk, uint32_t* out)
{
    const uint32_t lane = threadIdx.x;
    const uint32_t* Mp = msg + (size_t)blockIdx.x * nblk * 16;
    uint32_t h0 = 0x67452301u, h1 = 0xefcdab89u, h2 = 0x98badcfeu, h3 = 0x10325476u;
    auto proc = [&](uint32_t v0) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            uint32_t a = h0, bb = h1, c = h2, d = h3;
#define MW(i) ((uint32_t)RL(v0, s * 16 + (i)))
            {
                uint32_t& b_ = bb;
#define b b_
                MD5_ROUNDS(MW)
#undef b
            }
            h0 += a; h1 += bb; h2 += c; h3 += d;
        }
    };
    uint32_t v0 = Mp[lane], v1 = Mp[64 + lane], v2;
    for (uint32_t b = 0; b < nblk; b += 12) {
        __builtin_amdgcn_sched_barrier(0); v2 = Mp[(size_t)(b + 8) * 16 + lane]; __builtin_amdgcn_sched_barrier(0);
        proc(v0);
        __builtin_amdgcn_sched_barrier(0); v0 = Mp[(size_t)(b + 12) * 16 + lane]; __builtin_amdgcn_sched_barrier(0);
        proc(v1);
        __builtin_amdgcn_sched_barrier(0); v1 = Mp[(size_t)(b + 16) * 16 + lane]; __builtin_amdgcn_sched_barrier(0);
        proc(v2);
    }
    if (lane == 0) { out[blockIdx.x * 4] = h0; out[blockIdx.x * 4 + 1] = h1; out[blockIdx.x * 4 + 2] = h2; out[blockIdx.x * 4 + 3] = h3; }
}

// reference VALU MD5 (one lane) for checking
__global__ void k_md5_ref(const uint32_t* __restrict__ msg, uint32_t nblk, uint32_t* out)
{
    if (threadIdx.x) return;
    const uint32_t* Mp = msg + (size_t)blockIdx.x * nblk * 16;
    uint32_t h0 = 0x67452301u, h1 = 0xefcdab89u, h2 = 0x98badcfeu, h3 = 0x10325476u;
    for (uint32_t blk = 0; blk < nblk; blk++) {
        uint32_t a = h0, b = h1, c = h2, d = h3;
#define MR(i) (Mp[(size_t)blk * 16 + (i)])
        MD5_ROUNDS(MR)
        h0 += a; h1 += b; h2 += c; h3 += d;
    }
    out[blockIdx.x * 4] = h0; out[blockIdx.x * 4 + 1] = h1; out[blockIdx.x * 4 + 2] = h2; out[blockIdx.x * 4 + 3] = h3;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main()
{
    const uint32_t n = 192u * 5462;
    const int W = 128;
    std::vector<uint4> h1((size_t)n * W);
    std::vector<uint2> h2((size_t)n * W);
    uint32_t x = 12345;
    for (size_t i = 0; i < h1.size(); i++) {
        x = x * 1664525u + 1013904223u;
        uint32_t t = 12 + (x >> 8) % 240;
        uint32_t f = 1 + (x >> 20) % (t - 1);
        uint64_t m = ~0ull / t + 1;
        h1[i] = uint4{(uint32_t)m, (uint32_t)(m >> 32), f, t};
        uint32_t m32 = (uint32_t)((0x100000000ull + t - 1) / t);
        h2[i] = uint2{m32, t | (f << 16)};
    }
    uint4* d1; uint2* d2; uint32_t *dq, *dq2, *dres;
    CK(hipMalloc(&d1, h1.size() * 16 + 16384)); CK(hipMalloc(&d2, h2.size() * 8 + 8192));
    CK(hipMalloc(&dq, h1.size() * 4)); CK(hipMalloc(&dq2, h1.size() * 4)); CK(hipMalloc(&dres, 4096 * 4));
    CK(hipMemcpy(d1, h1.data(), h1.size() * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(d2, h2.data(), h2.size() * 8, hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    for (int w : {1, 32, W}) {
        hipLaunchKernelGGL(k_r1, dim3(w), dim3(64), 0, 0, d1, n, dq, dres);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_r1, dim3(w), dim3(64), 0, 0, d1, n, dq, dres); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("r1 (u64 recip, 3 readlane) streams=%3d : %.2f ns/sym/stream\n", w, ms * 1e6 / n);
        hipLaunchKernelGGL(k_r2, dim3(w), dim3(64), 0, 0, d2, n, dq2, dres);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_r2, dim3(w), dim3(64), 0, 0, d2, n, dq2, dres); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("r2 (u32 recip, 2 readlane) streams=%3d : %.2f ns/sym/stream\n", w, ms * 1e6 / n);
    }
    {   // check r1 == r2 == host
        std::vector<uint32_t> q1(n), q2(n);
        CK(hipMemcpy(q1.data(), dq, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(q2.data(), dq2, n * 4, hipMemcpyDeviceToHost));
        uint32_t r = 0xffffffffu; size_t bad = 0;
        for (uint32_t i = 0; i < n; i++) {
            uint32_t q = r / h1[i].w; uint32_t rr = q * h1[i].z; r = rr << (__builtin_clz(rr) & 24);
            bad += (q != q1[i]) + (q != q2[i]);
        }
        printf("chain check vs host: %zu mismatches\n", bad);
    }
    {
        const uint32_t nblk = 12u * 1366;
        uint32_t *dm, *o1, *o2;
        CK(hipMalloc(&dm, (size_t)nblk * 64 * 128 + 8192));
        std::vector<uint32_t> hm((size_t)nblk * 16 * 128);
        for (auto& v : hm) { x = x * 1664525u + 1013904223u; v = x; }
        CK(hipMemcpy(dm, hm.data(), hm.size() * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&o1, 128 * 16)); CK(hipMalloc(&o2, 128 * 16));
        for (int w : {1, 32, 128}) {
            hipLaunchKernelGGL(k_md5_rl, dim3(w), dim3(64), 0, 0, dm, nblk, o1);
            CK(hipEventRecord(a)); hipLaunchKernelGGL(k_md5_rl, dim3(w), dim3(64), 0, 0, dm, nblk, o1); CK(hipEventRecord(b));
            CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
            printf("md5 salu+readlane streams=%3d : %.1f ns/64B (%.3f GB/s per message)\n", w, ms * 1e6 / nblk, nblk * 64.0 / (ms * 1e6));
        }
        hipLaunchKernelGGL(k_md5_ref, dim3(4), dim3(64), 0, 0, dm, nblk, o2);
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_md5_ref, dim3(4), dim3(64), 0, 0, dm, nblk, o2); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("md5 one-lane VALU ref : %.1f ns/64B\n", ms * 1e6 / nblk);
        std::vector<uint32_t> r1(16), r2(16);
        CK(hipMemcpy(r1.data(), o1, 64, hipMemcpyDeviceToHost)); CK(hipMemcpy(r2.data(), o2, 64, hipMemcpyDeviceToHost));
        printf("md5 check: %s\n", r1 == r2 ? "match" : "MISMATCH");
    }
    return 0;
}
