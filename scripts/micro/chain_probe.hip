// chain_probe: shader cycles per step of pass R's range step run in the VALU
// (one chain per lane, k_coder_rl) against the same step on the scalar unit
// (k_coder_rv's eight SALU instructions), one wave alone on the GPU; and the
// issue cost of the integer multiplies the VALU step needs.
//   hipcc --offload-arch=gfx950 -O3 -o chain_probe scripts/micro/chain_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define N_STEPS 4096

// VALU: records from registers (a rotating set of 8), one chain per lane
__global__ void k_valu(uint32_t* out, uint64_t* cyc, uint32_t seed)
{
    const uint32_t lane = threadIdx.x;
    uint32_t m[8], t[8], f[8];
    for (int k = 0; k < 8; k++) {
        t[k] = 200 + ((seed * (k + 3) + lane * 7) & 0x3fff);
        f[k] = 1 + (t[k] >> 3);
        m[k] = 0xffffffffu / t[k] + 1u;
    }
    uint32_t r = 0xfffffff0u - lane;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N_STEPS; i += 8) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint32_t q = __umulhi(r, m[k]);
            q -= r < q * t[k] ? 1u : 0u;
            const uint32_t x = q * f[k];
            r = x << (__builtin_clz(x) & 24);
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    out[lane] = r;
    if (lane == 0) cyc[0] = c1 - c0;
}

// VALU with the correction's two products off each other: q*t and q*f both from q0
__global__ void k_valu2(uint32_t* out, uint64_t* cyc, uint32_t seed)
{
    const uint32_t lane = threadIdx.x;
    uint32_t m[8], t[8], f[8];
    for (int k = 0; k < 8; k++) {
        t[k] = 200 + ((seed * (k + 3) + lane * 7) & 0x3fff);
        f[k] = 1 + (t[k] >> 3);
        m[k] = 0xffffffffu / t[k] + 1u;
    }
    uint32_t r = 0xfffffff0u - lane;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N_STEPS; i += 8) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t q = __umulhi(r, m[k]);
            const uint32_t p = q * t[k], x0 = q * f[k];
            const uint32_t x = r < p ? x0 - f[k] : x0;
            r = x << (__builtin_clz(x) & 24);
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    out[lane] = r;
    if (lane == 0) cyc[0] = c1 - c0;
}

// two independent chain sets per lane interleaved (latency vs issue)
__global__ void k_valu_x2(uint32_t* out, uint64_t* cyc, uint32_t seed)
{
    const uint32_t lane = threadIdx.x;
    uint32_t m[8], t[8], f[8];
    for (int k = 0; k < 8; k++) {
        t[k] = 200 + ((seed * (k + 3) + lane * 7) & 0x3fff);
        f[k] = 1 + (t[k] >> 3);
        m[k] = 0xffffffffu / t[k] + 1u;
    }
    uint32_t r = 0xfffffff0u - lane, s = 0xfffff000u - lane;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N_STEPS; i += 8) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint32_t q = __umulhi(r, m[k]), u = __umulhi(s, m[7 - k]);
            q -= r < q * t[k] ? 1u : 0u;
            u -= s < u * t[7 - k] ? 1u : 0u;
            const uint32_t x = q * f[k], y = u * f[7 - k];
            r = x << (__builtin_clz(x) & 24);
            s = y << (__builtin_clz(y) & 24);
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    out[lane] = r ^ s;
    if (lane == 0) cyc[0] = c1 - c0;
}

// throughput of independent v_mul_lo_u32 / v_mul_hi_u32 / v_add_u32
template <int OP>
__global__ void k_issue(uint32_t* out, uint64_t* cyc, uint32_t seed)
{
    uint32_t a[8];
    for (int k = 0; k < 8; k++) a[k] = seed * (k + 1) + threadIdx.x;
    const uint32_t b = seed | 1u;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N_STEPS; i += 8) {
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = OP == 0 ? a[k] * b : OP == 1 ? __umulhi(a[k], b) : a[k] + b;
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
    for (int k = 0; k < 8; k++) x ^= a[k];
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

// SALU: the same step on the scalar unit (wave-uniform values)
__global__ void k_salu(uint32_t* out, uint64_t* cyc, uint32_t seed)
{
    uint32_t m[8], t[8], f[8];
    for (int k = 0; k < 8; k++) {
        t[k] = 200 + ((seed * (k + 3)) & 0x3fff);
        f[k] = 1 + (t[k] >> 3);
        m[k] = 0xffffffffu / t[k] + 1u;
    }
    uint32_t r = 0xfffffff0u;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N_STEPS; i += 8) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
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
                : "s"(m[k]), "s"(t[k]), "s"(f[k])
                : "scc");
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

int main()
{
    uint32_t* out;
    uint64_t* cyc;
    hipMalloc(&out, 4096);
    hipMalloc(&cyc, 64);
    struct K {
        const char* name;
        void (*k)(uint32_t*, uint64_t*, uint32_t);
        double per;   // chain steps (or ops) per loop step
    } ks[] = {{"valu chain (k_coder_rl step)", k_valu, 1.0},
              {"valu chain, both products from q0", k_valu2, 1.0},
              {"valu two chains interleaved (per chain step)", k_valu_x2, 2.0},
              {"salu chain (k_coder_rv step)", k_salu, 1.0},
              {"v_mul_lo_u32 independent", k_issue<0>, 1.0},
              {"v_mul_hi_u32 independent", k_issue<1>, 1.0},
              {"v_add_u32 independent", k_issue<2>, 1.0}};
    for (const K& k : ks) {
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, out, cyc, 12345u + rep);
            hipDeviceSynchronize();
        }
        uint64_t c = 0;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-48s %8.1f cycles per step\n", k.name, (double)c / N_STEPS / k.per);
    }
    return 0;
}
