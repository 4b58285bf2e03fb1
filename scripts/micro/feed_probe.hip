// feed_probe (round 6): shader cycles per symbol of pass R's range chain under
// different ways of feeding the scalar unit its (reciprocal, total, frequency)
// operands.  Every variant runs the same chain over the same records and must
// end with the host's range; one wave per chain, chains of N symbols.
//   V0 salu    : operands constant in SGPRs (the step alone)
//   V1 rl3     : k_coder_rv today -- records loaded 4 segments ahead into
//                VGPRs, m / t / f per lane, 24 v_readlane per 8 steps
//   V2 rl2     : m and tf per lane, 16 v_readlane per 8 steps, t / f split
//                in the SALU
//   V3 ring3x8 : the lanes write (m, t, f) of segment g+2 to a per-wave ring
//                (vector stores), the chain reads 8 symbols per s_load group
//                (glc), two groups in flight (48 SGPRs)
//   V4 ring2x16: (m, tf) triples... pairs, 16 symbols a group, split in SALU
//   V5 mtf2x16 : (m, tf) pairs precomputed in memory by an earlier kernel,
//                s_load without glc, 16 symbols a group; the lanes only touch
//                the lines 4 segments ahead (L2 prefetch)
//   V6 mtf3x8  : (m, t, f) precomputed, 8 symbols a group
//   hipcc --offload-arch=gfx950 -O3 -o feed_probe scripts/micro/feed_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>

constexpr int SEG = 64;
constexpr int LA = 4;

__device__ __forceinline__ uint32_t recip32(uint32_t t) { return 0xffffffffu / t + 1u; }

#define STEP(M, T, F)                                                                                  \
    "s_mul_hi_u32 %[q], %[r], " M "\n\ts_mul_i32 %[p], %[q], " T "\n\ts_cmp_lt_u32 %[r], %[p]\n\t"   \
    "s_subb_u32 %[q], %[q], 0\n\ts_mul_i32 %[q], %[q], " F "\n\ts_flbit_i32_b32 %[p], %[q]\n\t"        \
    "s_and_b32 %[p], %[p], 24\n\ts_lshl_b32 %[r], %[q], %[p]\n\t"
// (m, tf) pair: split first (off the chain's dependency)
#define STEP2(M, TF)                                                                                   \
    "s_and_b32 %[t], " TF ", 0xffff\n\ts_lshr_b32 %[f], " TF ", 16\n\t" STEP(M, "%[t]", "%[f]")

// ---------------------------------------------------------------- V0
__global__ void k_v0(const uint32_t* rec, uint32_t n, uint32_t* out, uint64_t* cyc)
{
    uint32_t m[8], t[8], f[8];
    for (int k = 0; k < 8; k++) {
        const uint32_t tf = __builtin_amdgcn_readfirstlane(rec[k]);
        t[k] = tf & 0xffff;
        f[k] = tf >> 16;
        m[k] = recip32(t[k]);
    }
    uint32_t r = 0xffffffffu;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; i += 8) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint32_t q, p;
            asm volatile(STEP("%[m]", "%[tt]", "%[ff]") : [r] "+s"(r), [q] "=&s"(q), [p] "=&s"(p)
                         : [m] "s"(m[k]), [tt] "s"(t[k]), [ff] "s"(f[k]) : "scc");
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = r;
        cyc[blockIdx.x] = c1 - c0;
    }
}

// ---------------------------------------------------------------- V1 / V2
#define RL3(k)                                                                                         \
    "v_readlane_b32 %[m" #k "], %[cm], %[l" #k "]\n\tv_readlane_b32 %[t" #k "], %[vt], %[l" #k "]\n\t" \
    "v_readlane_b32 %[f" #k "], %[vf], %[l" #k "]\n\t"
#define ST3(k) STEP("%[m" #k "]", "%[t" #k "]", "%[f" #k "]")
template <int J, bool NOP = false>
__device__ __forceinline__ void rl3_step8(uint32_t& r, uint32_t cm, uint32_t vt, uint32_t vf)
{
    uint32_t q, p, m0, m1, m2, m3, m4, m5, m6, m7, t0, t1, t2, t3, t4, t5, t6, t7, f0, f1, f2, f3, f4, f5, f6, f7;
    if constexpr (NOP) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    asm volatile(RL3(0) RL3(1) RL3(2) RL3(3) RL3(4) RL3(5) RL3(6) RL3(7) ST3(0) ST3(1) ST3(2) ST3(3) ST3(4) ST3(5)
                     ST3(6) ST3(7)
                 : [r] "+s"(r), [q] "=&s"(q), [p] "=&s"(p), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2),
                   [m3] "=&s"(m3), [m4] "=&s"(m4), [m5] "=&s"(m5), [m6] "=&s"(m6), [m7] "=&s"(m7), [t0] "=&s"(t0),
                   [t1] "=&s"(t1), [t2] "=&s"(t2), [t3] "=&s"(t3), [t4] "=&s"(t4), [t5] "=&s"(t5), [t6] "=&s"(t6),
                   [t7] "=&s"(t7), [f0] "=&s"(f0), [f1] "=&s"(f1), [f2] "=&s"(f2), [f3] "=&s"(f3), [f4] "=&s"(f4),
                   [f5] "=&s"(f5), [f6] "=&s"(f6), [f7] "=&s"(f7)
                 : [cm] "v"(cm), [vt] "v"(vt), [vf] "v"(vf), [l0] "i"(J), [l1] "i"(J + 1), [l2] "i"(J + 2),
                   [l3] "i"(J + 3), [l4] "i"(J + 4), [l5] "i"(J + 5), [l6] "i"(J + 6), [l7] "i"(J + 7)
                 : "scc");
}
#define RL2(k) "v_readlane_b32 %[m" #k "], %[cm], %[l" #k "]\n\tv_readlane_b32 %[x" #k "], %[vx], %[l" #k "]\n\t"
#define ST2(k) STEP2("%[m" #k "]", "%[x" #k "]")
template <int J>
__device__ __forceinline__ void rl2_step8(uint32_t& r, uint32_t cm, uint32_t vx)
{
    uint32_t q, p, t, f, m0, m1, m2, m3, m4, m5, m6, m7, x0, x1, x2, x3, x4, x5, x6, x7;
    asm volatile(RL2(0) RL2(1) RL2(2) RL2(3) RL2(4) RL2(5) RL2(6) RL2(7) ST2(0) ST2(1) ST2(2) ST2(3) ST2(4) ST2(5)
                     ST2(6) ST2(7)
                 : [r] "+s"(r), [q] "=&s"(q), [p] "=&s"(p), [t] "=&s"(t), [f] "=&s"(f), [m0] "=&s"(m0),
                   [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3), [m4] "=&s"(m4), [m5] "=&s"(m5), [m6] "=&s"(m6),
                   [m7] "=&s"(m7), [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), [x3] "=&s"(x3), [x4] "=&s"(x4),
                   [x5] "=&s"(x5), [x6] "=&s"(x6), [x7] "=&s"(x7)
                 : [cm] "v"(cm), [vx] "v"(vx), [l0] "i"(J), [l1] "i"(J + 1), [l2] "i"(J + 2), [l3] "i"(J + 3),
                   [l4] "i"(J + 4), [l5] "i"(J + 5), [l6] "i"(J + 6), [l7] "i"(J + 7)
                 : "scc");
}

template <int V>
__global__ __launch_bounds__(256) void k_rl(const uint32_t* rec, uint32_t n, uint32_t* out, uint64_t* cyc)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t* G = rec + (size_t)w * n + lane;
    const uint32_t nseg = n / SEG;
    uint32_t buf[LA];
#pragma unroll
    for (int k = 0; k < LA; k++) buf[k] = G[(size_t)k * SEG];
    uint32_t r = 0xffffffffu;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (uint32_t g = 0; g < nseg; g += LA) {
#pragma unroll
        for (int k = 0; k < LA; k++) {
            const uint32_t tf = buf[k];
            buf[k] = G[(size_t)min(g + k + LA, nseg - 1) * SEG];
            const uint32_t vt = tf & 0xffff, cm = recip32(vt);
            r = __builtin_amdgcn_readfirstlane(r);
            if constexpr (V == 1 || V == 3) {
                constexpr bool N = V == 3;
                const uint32_t vf = tf >> 16;
                rl3_step8<0, N>(r, cm, vt, vf); rl3_step8<8, N>(r, cm, vt, vf); rl3_step8<16, N>(r, cm, vt, vf);
                rl3_step8<24, N>(r, cm, vt, vf); rl3_step8<32, N>(r, cm, vt, vf); rl3_step8<40, N>(r, cm, vt, vf);
                rl3_step8<48, N>(r, cm, vt, vf); rl3_step8<56, N>(r, cm, vt, vf);
            } else {
                rl2_step8<0>(r, cm, tf); rl2_step8<8>(r, cm, tf); rl2_step8<16>(r, cm, tf);
                rl2_step8<24>(r, cm, tf); rl2_step8<32>(r, cm, tf); rl2_step8<40>(r, cm, tf);
                rl2_step8<48>(r, cm, tf); rl2_step8<56>(r, cm, tf);
            }
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[w] = r;
        cyc[w] = c1 - c0;
    }
}

// ---------------------------------------------------------------- SMEM groups
// Two buffers at fixed SGPRs: A = s[52:75], B = s[76:99] (3 dwords x 8
// symbols), or A = s[36:67], B = s[68:99] (2 dwords x 16 symbols).  One asm
// block per group: wait for everything (SMEM returns out of order), issue the
// OTHER buffer's load for the group after this one, run this group's steps.
#define CLOB_52_99                                                                                     \
    "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", \
        "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", \
        "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", \
        "s94", "s95", "s96", "s97", "s98", "s99"
#define CLOB_36_51                                                                                     \
    "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", \
        "s50", "s51"

// 3 x 8: symbol k of buffer A = (s[52+3k], s[53+3k], s[54+3k]); 2 x 16: (m, tf)
// pairs (the preprocessor cannot add numbers: the buffers are spelt out)
#define A3_STEPS                                                                                       \
    STEP("s52", "s53", "s54") STEP("s55", "s56", "s57") STEP("s58", "s59", "s60") STEP("s61", "s62", "s63") \
    STEP("s64", "s65", "s66") STEP("s67", "s68", "s69") STEP("s70", "s71", "s72") STEP("s73", "s74", "s75")
#define B3_STEPS                                                                                       \
    STEP("s76", "s77", "s78") STEP("s79", "s80", "s81") STEP("s82", "s83", "s84") STEP("s85", "s86", "s87") \
    STEP("s88", "s89", "s90") STEP("s91", "s92", "s93") STEP("s94", "s95", "s96") STEP("s97", "s98", "s99")
#define A2_STEPS                                                                                       \
    STEP2("s36", "s37") STEP2("s38", "s39") STEP2("s40", "s41") STEP2("s42", "s43") STEP2("s44", "s45")   \
    STEP2("s46", "s47") STEP2("s48", "s49") STEP2("s50", "s51") STEP2("s52", "s53") STEP2("s54", "s55")   \
    STEP2("s56", "s57") STEP2("s58", "s59") STEP2("s60", "s61") STEP2("s62", "s63") STEP2("s64", "s65")   \
    STEP2("s66", "s67")
#define B2_STEPS                                                                                       \
    STEP2("s68", "s69") STEP2("s70", "s71") STEP2("s72", "s73") STEP2("s74", "s75") STEP2("s76", "s77")   \
    STEP2("s78", "s79") STEP2("s80", "s81") STEP2("s82", "s83") STEP2("s84", "s85") STEP2("s86", "s87")   \
    STEP2("s88", "s89") STEP2("s90", "s91") STEP2("s92", "s93") STEP2("s94", "s95") STEP2("s96", "s97")   \
    STEP2("s98", "s99")
#define LOAD_A3(GLC) "s_load_dwordx16 s[52:67], %[nx], 0x0" GLC "\n\ts_load_dwordx8 s[68:75], %[nx], 0x40" GLC "\n\t"
#define LOAD_B3(GLC) "s_load_dwordx16 s[76:91], %[nx], 0x0" GLC "\n\ts_load_dwordx8 s[92:99], %[nx], 0x40" GLC "\n\t"
#define LOAD_A2(GLC) "s_load_dwordx16 s[36:51], %[nx], 0x0" GLC "\n\ts_load_dwordx16 s[52:67], %[nx], 0x40" GLC "\n\t"
#define LOAD_B2(GLC) "s_load_dwordx16 s[68:83], %[nx], 0x0" GLC "\n\ts_load_dwordx16 s[84:99], %[nx], 0x40" GLC "\n\t"

// a pointer the wave holds in SGPRs
__device__ __forceinline__ const uint32_t* uni(const uint32_t* p)
{
    const uint64_t x = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x), hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return (const uint32_t*)((uint64_t)hi << 32 | lo);
}

// group bytes: 3x8 -> 96, 2x16 -> 128.  W3: 3 dwords per symbol.
template <bool W3, bool GLC>
__device__ __forceinline__ void grp_first(const uint32_t* p)
{
    p = uni(p);
    if constexpr (W3) {
        if constexpr (GLC) asm volatile(LOAD_A3(" glc") ::[nx] "s"(p) : CLOB_52_99);
        else asm volatile(LOAD_A3("") ::[nx] "s"(p) : CLOB_52_99);
    } else {
        if constexpr (GLC) asm volatile(LOAD_A2(" glc") ::[nx] "s"(p) : CLOB_52_99, CLOB_36_51);
        else asm volatile(LOAD_A2("") ::[nx] "s"(p) : CLOB_52_99, CLOB_36_51);
    }
}
// consume buffer A (ODD = 0) or B (ODD = 1) while the other one loads from nx
template <bool W3, bool GLC, int ODD>
__device__ __forceinline__ void grp(uint32_t& r, const uint32_t* nx)
{
    nx = uni(nx);
    uint32_t q, p, t, f;
#define GRP_OPS : [r] "+s"(r), [q] "=&s"(q), [p] "=&s"(p), [t] "=&s"(t), [f] "=&s"(f) : [nx] "s"(nx)
    if constexpr (W3) {
        if constexpr (ODD == 0) {
            if constexpr (GLC) asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_B3(" glc") A3_STEPS GRP_OPS : "scc", CLOB_52_99);
            else asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_B3("") A3_STEPS GRP_OPS : "scc", CLOB_52_99);
        } else {
            if constexpr (GLC) asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_A3(" glc") B3_STEPS GRP_OPS : "scc", CLOB_52_99);
            else asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_A3("") B3_STEPS GRP_OPS : "scc", CLOB_52_99);
        }
    } else {
        if constexpr (ODD == 0) {
            if constexpr (GLC)
                asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_B2(" glc") A2_STEPS GRP_OPS : "scc", CLOB_52_99, CLOB_36_51);
            else asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_B2("") A2_STEPS GRP_OPS : "scc", CLOB_52_99, CLOB_36_51);
        } else {
            if constexpr (GLC)
                asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_A2(" glc") B2_STEPS GRP_OPS : "scc", CLOB_52_99, CLOB_36_51);
            else asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_A2("") B2_STEPS GRP_OPS : "scc", CLOB_52_99, CLOB_36_51);
        }
    }
#undef GRP_OPS
}

// the groups of one segment: data of this segment at cur, of the next at nxt
template <bool W3, bool GLC>
__device__ __forceinline__ void seg_groups(uint32_t& r, const uint32_t* cur, const uint32_t* nxt)
{
    constexpr int GD = W3 ? 24 : 32;   // dwords per group
    constexpr int NG = W3 ? 8 : 4;     // groups per segment (even)
#pragma unroll
    for (int j = 0; j < NG; j += 2) {
        grp<W3, GLC, 0>(r, cur + (j + 1) * GD);
        grp<W3, GLC, 1>(r, j + 2 < NG ? cur + (j + 2) * GD : nxt);
    }
}

// V3 / V4: the lanes fill a per-wave ring of 4 segment slots, 2 segments ahead
template <bool W3>
__global__ __launch_bounds__(256) void k_ring(const uint32_t* rec, uint32_t n, uint32_t* ring, uint32_t* out,
                                              uint64_t* cyc)
{
    constexpr int SD = W3 ? 3 * SEG : 2 * SEG;   // dwords per segment slot
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t* G = rec + (size_t)w * n + lane;
    uint32_t* R = ring + (size_t)w * 4 * SD;
    const uint32_t nseg = n / SEG;
    auto put = [&](uint32_t slot, uint32_t tf) {
        const uint32_t t = tf & 0xffff;
        uint32_t* d = R + slot * SD;
        if constexpr (W3) {
            d[3 * lane] = recip32(t);
            d[3 * lane + 1] = t;
            d[3 * lane + 2] = tf >> 16;
        } else {
            d[2 * lane] = recip32(t);
            d[2 * lane + 1] = tf;
        }
    };
    uint32_t buf[LA];
#pragma unroll
    for (int k = 0; k < LA; k++) buf[k] = G[(size_t)k * SEG];
    // segments 0 and 1 into the ring before the start
    put(0, buf[0]);
    put(1, buf[1]);
    buf[0] = G[(size_t)min(LA, nseg - 1) * SEG];
    buf[1] = G[(size_t)min(LA + 1, nseg - 1) * SEG];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t r = 0xffffffffu;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    grp_first<W3, true>(R);
    for (uint32_t g = 0; g < nseg; g += LA) {
#pragma unroll
        for (int k = 0; k < LA; k++) {
            // segment g+k+2's slot from buf[(k+2)%LA], then its refill
            const int kk = (k + 2) % LA;
            put((g + k + 2) & 3, buf[kk]);
            buf[kk] = G[(size_t)min(g + k + 2 + LA, nseg - 1) * SEG];
            // the slot of segment g+k+1 (stored one segment ago) must be in L2
            // before its first group is loaded at the end of this segment:
            // younger than that store are this segment's store and load
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            seg_groups<W3, true>(r, R + ((g + k) & 3) * SD, R + ((g + k + 1) & 3) * SD);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[w] = r;
        cyc[w] = c1 - c0;
    }
}

// V5 / V6: operands precomputed in memory (an earlier kernel); the lanes only
// touch each segment's lines LA segments ahead
template <bool W3>
__global__ __launch_bounds__(256) void k_direct(const uint32_t* mtf, uint32_t n, uint32_t* out, uint64_t* cyc)
{
    constexpr int SD = W3 ? 3 * SEG : 2 * SEG;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t* D = mtf + (size_t)w * n * (W3 ? 3 : 2);
    const uint32_t nseg = n / SEG;
    // touch loads: one dword per 64-byte line of segment g+LA (lanes < SD/16)
    const uint32_t* T = D + (lane < SD / 16 ? lane * 16 : 0);
    uint32_t tb[LA], acc = 0;
#pragma unroll
    for (int k = 0; k < LA; k++) tb[k] = T[(size_t)k * SD];
    uint32_t r = 0xffffffffu;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    grp_first<W3, false>(D);
    for (uint32_t g = 0; g < nseg; g += LA) {
#pragma unroll
        for (int k = 0; k < LA; k++) {
            acc ^= tb[k];
            tb[k] = T[(size_t)min(g + k + LA, nseg - 1) * SD];
            seg_groups<W3, false>(r, D + (size_t)(g + k) * SD, D + (size_t)min(g + k + 1, nseg - 1) * SD);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[w] = r + (acc & 0u) * (acc == 0x12345678u);
        cyc[w] = c1 - c0;
    }
}


// ---------------------------------------------------------------- V7
// (m, t) pairs through SMEM from the ring (buffers s[36:67] / s[68:99]), f
// through one v_readlane per symbol from the lanes' copy of the segment's
// records: 8 SALU + 1 VALU + 1/8 SMEM per symbol (V4: 10 SALU)
#define RL7(k) "v_readlane_b32 %[f" #k "], %[vf], %[l" #k "]\n\t"
#define A7_LO STEP("s36", "s37", "%[f0]") STEP("s38", "s39", "%[f1]") STEP("s40", "s41", "%[f2]") STEP("s42", "s43", "%[f3]") \
              STEP("s44", "s45", "%[f4]") STEP("s46", "s47", "%[f5]") STEP("s48", "s49", "%[f6]") STEP("s50", "s51", "%[f7]")
#define A7_HI STEP("s52", "s53", "%[f0]") STEP("s54", "s55", "%[f1]") STEP("s56", "s57", "%[f2]") STEP("s58", "s59", "%[f3]") \
              STEP("s60", "s61", "%[f4]") STEP("s62", "s63", "%[f5]") STEP("s64", "s65", "%[f6]") STEP("s66", "s67", "%[f7]")
#define B7_LO STEP("s68", "s69", "%[f0]") STEP("s70", "s71", "%[f1]") STEP("s72", "s73", "%[f2]") STEP("s74", "s75", "%[f3]") \
              STEP("s76", "s77", "%[f4]") STEP("s78", "s79", "%[f5]") STEP("s80", "s81", "%[f6]") STEP("s82", "s83", "%[f7]")
#define B7_HI STEP("s84", "s85", "%[f0]") STEP("s86", "s87", "%[f1]") STEP("s88", "s89", "%[f2]") STEP("s90", "s91", "%[f3]") \
              STEP("s92", "s93", "%[f4]") STEP("s94", "s95", "%[f5]") STEP("s96", "s97", "%[f6]") STEP("s98", "s99", "%[f7]")
#define RL7_8 RL7(0) RL7(1) RL7(2) RL7(3) RL7(4) RL7(5) RL7(6) RL7(7)
#define OPS7(J)                                                                                                \
    : [r] "+s"(r), [q] "=&s"(q), [p] "=&s"(p), [f0] "=&s"(f0), [f1] "=&s"(f1), [f2] "=&s"(f2), [f3] "=&s"(f3),      \
      [f4] "=&s"(f4), [f5] "=&s"(f5), [f6] "=&s"(f6), [f7] "=&s"(f7)                                            \
    : [nx] "s"(nx), [vf] "v"(vf), [l0] "i"(J), [l1] "i"(J + 1), [l2] "i"(J + 2), [l3] "i"(J + 3), [l4] "i"(J + 4), \
      [l5] "i"(J + 5), [l6] "i"(J + 6), [l7] "i"(J + 7)
template <int ODD, int J>
__device__ __forceinline__ void grp7(uint32_t& r, const uint32_t* nx, uint32_t vf)
{
    nx = uni(nx);
    uint32_t q, p, f0, f1, f2, f3, f4, f5, f6, f7;
    if constexpr (ODD == 0) {
        asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_B2(" glc") RL7_8 A7_LO OPS7(J) : "scc", CLOB_52_99, CLOB_36_51);
        asm volatile(RL7_8 A7_HI OPS7(J + 8) : "scc", CLOB_52_99, CLOB_36_51);
    } else {
        asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_A2(" glc") RL7_8 B7_LO OPS7(J) : "scc", CLOB_52_99, CLOB_36_51);
        asm volatile(RL7_8 B7_HI OPS7(J + 8) : "scc", CLOB_52_99, CLOB_36_51);
    }
}
__global__ __launch_bounds__(256) void k_ring7(const uint32_t* rec, uint32_t n, uint32_t* ring, uint32_t* out,
                                               uint64_t* cyc)
{
    constexpr int SD = 2 * SEG;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t* G = rec + (size_t)w * n + lane;
    uint32_t* R = ring + (size_t)w * 4 * SD;
    const uint32_t nseg = n / SEG;
    auto put = [&](uint32_t slot, uint32_t tf) {
        const uint32_t t = tf & 0xffff;
        uint32_t* d = R + slot * SD;
        d[2 * lane] = recip32(t);
        d[2 * lane + 1] = t;
    };
    uint32_t buf[LA], fv[LA];
#pragma unroll
    for (int k = 0; k < LA; k++) buf[k] = G[(size_t)k * SEG];
    put(0, buf[0]);
    put(1, buf[1]);
    fv[0] = buf[0] >> 16;
    fv[1] = buf[1] >> 16;
    buf[0] = G[(size_t)min(LA, nseg - 1) * SEG];
    buf[1] = G[(size_t)min(LA + 1, nseg - 1) * SEG];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t r = 0xffffffffu;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    grp_first<false, true>(R);
    for (uint32_t g = 0; g < nseg; g += LA) {
#pragma unroll
        for (int k = 0; k < LA; k++) {
            const int kk = (k + 2) % LA;
            put((g + k + 2) & 3, buf[kk]);
            fv[kk] = buf[kk] >> 16;
            buf[kk] = G[(size_t)min(g + k + 2 + LA, nseg - 1) * SEG];
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            const uint32_t* cur = R + ((g + k) & 3) * SD;
            const uint32_t vf = fv[k];
            grp7<0, 0>(r, cur + 32, vf);
            grp7<1, 16>(r, cur + 64, vf);
            grp7<0, 32>(r, cur + 96, vf);
            grp7<1, 48>(r, R + ((g + k + 1) & 3) * SD, vf);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[w] = r;
        cyc[w] = c1 - c0;
    }
}


// V8: the same with each f read one step ahead of its use (two SGPRs)
#define ST8(M, T, F, FN, LN) "v_readlane_b32 " FN ", %[vf], " LN "\n\t" STEP(M, T, F)
#define A8(J0)                                                                                                         \
    ST8("s36", "s37", "%[fa]", "%[fb]", "%[l1]") ST8("s38", "s39", "%[fb]", "%[fa]", "%[l2]")                          \
    ST8("s40", "s41", "%[fa]", "%[fb]", "%[l3]") ST8("s42", "s43", "%[fb]", "%[fa]", "%[l4]")                          \
    ST8("s44", "s45", "%[fa]", "%[fb]", "%[l5]") ST8("s46", "s47", "%[fb]", "%[fa]", "%[l6]")                          \
    ST8("s48", "s49", "%[fa]", "%[fb]", "%[l7]") ST8("s50", "s51", "%[fb]", "%[fa]", "%[l8]")                          \
    ST8("s52", "s53", "%[fa]", "%[fb]", "%[l9]") ST8("s54", "s55", "%[fb]", "%[fa]", "%[l10]")                         \
    ST8("s56", "s57", "%[fa]", "%[fb]", "%[l11]") ST8("s58", "s59", "%[fb]", "%[fa]", "%[l12]")                        \
    ST8("s60", "s61", "%[fa]", "%[fb]", "%[l13]") ST8("s62", "s63", "%[fb]", "%[fa]", "%[l14]")                        \
    ST8("s64", "s65", "%[fa]", "%[fb]", "%[l15]") ST8("s66", "s67", "%[fb]", "%[fa]", "%[l16]")
#define B8(J0)                                                                                                         \
    ST8("s68", "s69", "%[fa]", "%[fb]", "%[l1]") ST8("s70", "s71", "%[fb]", "%[fa]", "%[l2]")                          \
    ST8("s72", "s73", "%[fa]", "%[fb]", "%[l3]") ST8("s74", "s75", "%[fb]", "%[fa]", "%[l4]")                          \
    ST8("s76", "s77", "%[fa]", "%[fb]", "%[l5]") ST8("s78", "s79", "%[fb]", "%[fa]", "%[l6]")                          \
    ST8("s80", "s81", "%[fa]", "%[fb]", "%[l7]") ST8("s82", "s83", "%[fb]", "%[fa]", "%[l8]")                          \
    ST8("s84", "s85", "%[fa]", "%[fb]", "%[l9]") ST8("s86", "s87", "%[fb]", "%[fa]", "%[l10]")                         \
    ST8("s88", "s89", "%[fa]", "%[fb]", "%[l11]") ST8("s90", "s91", "%[fb]", "%[fa]", "%[l12]")                        \
    ST8("s92", "s93", "%[fa]", "%[fb]", "%[l13]") ST8("s94", "s95", "%[fb]", "%[fa]", "%[l14]")                        \
    ST8("s96", "s97", "%[fa]", "%[fb]", "%[l15]") ST8("s98", "s99", "%[fb]", "%[fa]", "%[l16]")
// fa holds f of the group's first symbol on entry (read by the previous group);
// the last step reads the next group's first f (lane J+16, masked to 63)
#define OPS8(J)                                                                                                \
    : [r] "+s"(r), [q] "=&s"(q), [p] "=&s"(p), [fa] "+s"(fa), [fb] "=&s"(fb)                                       \
    : [nx] "s"(nx), [vf] "v"(vf), [vn] "v"(vn), [l1] "i"(J + 1), [l2] "i"(J + 2), [l3] "i"(J + 3), [l4] "i"(J + 4), \
      [l5] "i"(J + 5), [l6] "i"(J + 6), [l7] "i"(J + 7), [l8] "i"(J + 8), [l9] "i"(J + 9), [l10] "i"(J + 10),       \
      [l11] "i"(J + 11), [l12] "i"(J + 12), [l13] "i"(J + 13), [l14] "i"(J + 14), [l15] "i"(J + 15),              \
      [l16] "i"((J + 16) & 63)
template <int ODD, int J>
__device__ __forceinline__ void grp8(uint32_t& r, uint32_t& fa, const uint32_t* nx, uint32_t vf, uint32_t vn)
{
    nx = uni(nx);
    uint32_t q, p, fb;
    // (the last step's read is of the next segment's lane 0 when J = 48: vn)
    if constexpr (J == 48) {
#define A8L A8(0)
        if constexpr (ODD == 0)
            asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_B2(" glc")
                         ST8("s36", "s37", "%[fa]", "%[fb]", "%[l1]") ST8("s38", "s39", "%[fb]", "%[fa]", "%[l2]")
                         ST8("s40", "s41", "%[fa]", "%[fb]", "%[l3]") ST8("s42", "s43", "%[fb]", "%[fa]", "%[l4]")
                         ST8("s44", "s45", "%[fa]", "%[fb]", "%[l5]") ST8("s46", "s47", "%[fb]", "%[fa]", "%[l6]")
                         ST8("s48", "s49", "%[fa]", "%[fb]", "%[l7]") ST8("s50", "s51", "%[fb]", "%[fa]", "%[l8]")
                         ST8("s52", "s53", "%[fa]", "%[fb]", "%[l9]") ST8("s54", "s55", "%[fb]", "%[fa]", "%[l10]")
                         ST8("s56", "s57", "%[fa]", "%[fb]", "%[l11]") ST8("s58", "s59", "%[fb]", "%[fa]", "%[l12]")
                         ST8("s60", "s61", "%[fa]", "%[fb]", "%[l13]") ST8("s62", "s63", "%[fb]", "%[fa]", "%[l14]")
                         ST8("s64", "s65", "%[fa]", "%[fb]", "%[l15]")
                         "v_readlane_b32 %[fa], %[vn], 0\n\t" STEP("s66", "s67", "%[fb]") OPS8(J)
                         : "scc", CLOB_52_99, CLOB_36_51);
        else
            asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_A2(" glc")
                         ST8("s68", "s69", "%[fa]", "%[fb]", "%[l1]") ST8("s70", "s71", "%[fb]", "%[fa]", "%[l2]")
                         ST8("s72", "s73", "%[fa]", "%[fb]", "%[l3]") ST8("s74", "s75", "%[fb]", "%[fa]", "%[l4]")
                         ST8("s76", "s77", "%[fa]", "%[fb]", "%[l5]") ST8("s78", "s79", "%[fb]", "%[fa]", "%[l6]")
                         ST8("s80", "s81", "%[fa]", "%[fb]", "%[l7]") ST8("s82", "s83", "%[fb]", "%[fa]", "%[l8]")
                         ST8("s84", "s85", "%[fa]", "%[fb]", "%[l9]") ST8("s86", "s87", "%[fb]", "%[fa]", "%[l10]")
                         ST8("s88", "s89", "%[fa]", "%[fb]", "%[l11]") ST8("s90", "s91", "%[fb]", "%[fa]", "%[l12]")
                         ST8("s92", "s93", "%[fa]", "%[fb]", "%[l13]") ST8("s94", "s95", "%[fb]", "%[fa]", "%[l14]")
                         ST8("s96", "s97", "%[fa]", "%[fb]", "%[l15]")
                         "v_readlane_b32 %[fa], %[vn], 0\n\t" STEP("s98", "s99", "%[fb]") OPS8(J)
                         : "scc", CLOB_52_99, CLOB_36_51);
    } else {
        if constexpr (ODD == 0)
            asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_B2(" glc") A8(J) OPS8(J) : "scc", CLOB_52_99, CLOB_36_51);
        else
            asm volatile("s_waitcnt lgkmcnt(0)\n\t" LOAD_A2(" glc") B8(J) OPS8(J) : "scc", CLOB_52_99, CLOB_36_51);
    }
}
__global__ __launch_bounds__(256) void k_ring8(const uint32_t* rec, uint32_t n, uint32_t* ring, uint32_t* out,
                                               uint64_t* cyc)
{
    constexpr int SD = 2 * SEG;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t* G = rec + (size_t)w * n + lane;
    uint32_t* R = ring + (size_t)w * 4 * SD;
    const uint32_t nseg = n / SEG;
    auto put = [&](uint32_t slot, uint32_t tf) {
        const uint32_t t = tf & 0xffff;
        uint32_t* d = R + slot * SD;
        d[2 * lane] = recip32(t);
        d[2 * lane + 1] = t;
    };
    uint32_t buf[LA], fv[LA];
#pragma unroll
    for (int k = 0; k < LA; k++) buf[k] = G[(size_t)k * SEG];
    put(0, buf[0]);
    put(1, buf[1]);
    fv[0] = buf[0] >> 16;
    fv[1] = buf[1] >> 16;
    buf[0] = G[(size_t)min(LA, nseg - 1) * SEG];
    buf[1] = G[(size_t)min(LA + 1, nseg - 1) * SEG];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t r = 0xffffffffu;
    uint32_t fa = __builtin_amdgcn_readlane(fv[0], 0);
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    grp_first<false, true>(R);
    for (uint32_t g = 0; g < nseg; g += LA) {
#pragma unroll
        for (int k = 0; k < LA; k++) {
            const int kk = (k + 2) % LA;
            put((g + k + 2) & 3, buf[kk]);
            fv[kk] = buf[kk] >> 16;
            buf[kk] = G[(size_t)min(g + k + 2 + LA, nseg - 1) * SEG];
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            const uint32_t* cur = R + ((g + k) & 3) * SD;
            const uint32_t vf = fv[k], vn = fv[(k + 1) % LA];
            grp8<0, 0>(r, fa, cur + 32, vf, vn);
            grp8<1, 16>(r, fa, cur + 64, vf, vn);
            grp8<0, 32>(r, fa, cur + 96, vf, vn);
            grp8<1, 48>(r, fa, R + ((g + k + 1) & 3) * SD, vf, vn);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[w] = r;
        cyc[w] = c1 - c0;
    }
}

__global__ void k_prep(const uint32_t* rec, size_t total, uint32_t* d2, uint32_t* d3)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t tf = rec[i], t = tf & 0xffff;
        d2[2 * i] = recip32(t);
        d2[2 * i + 1] = tf;
        d3[3 * i] = recip32(t);
        d3[3 * i + 1] = t;
        d3[3 * i + 2] = tf >> 16;
    }
}

static uint32_t host_chain(const uint32_t* rec, uint32_t n, uint32_t n_salu)
{
    uint32_t r = 0xffffffffu;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t tf = rec[n_salu ? (i & 7) : i], t = tf & 0xffff, f = tf >> 16;
        const uint32_t m = 0xffffffffu / t + 1u;
        uint32_t q = (uint32_t)(((uint64_t)r * m) >> 32);
        if (r < q * t) q--;
        const uint32_t x = q * f;
        r = x << (__builtin_clz(x) & 24);
    }
    return r;
}

int main(int argc, char** argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);   // symbols per chain
    const int chains_max = 1024;
    std::vector<uint32_t> h((size_t)n * chains_max);
    uint64_t s = 88172645463325252ull;
    for (auto& x : h) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const uint32_t t = 12 + (uint32_t)(s % 242), f = 1 + (uint32_t)((s >> 20) % t);   // BASE_MODEL-like
        x = t | f << 16;
    }
    uint32_t *rec, *out, *ring, *d2, *d3;
    uint64_t* cyc;
    const size_t total = (size_t)n * chains_max;
    hipMalloc(&rec, total * 4);
    hipMalloc(&d2, total * 8);
    hipMalloc(&d3, total * 12);
    hipMalloc(&ring, (size_t)chains_max * 4 * 3 * SEG * 4);
    hipMalloc(&out, chains_max * 4);
    hipMalloc(&cyc, chains_max * 8);
    hipMemcpy(rec, h.data(), total * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_prep, dim3(4096), dim3(256), 0, 0, rec, total, d2, d3);
    hipDeviceSynchronize();
    std::vector<uint32_t> ref(chains_max);
    for (int c = 0; c < chains_max; c++) ref[c] = host_chain(h.data() + (size_t)c * n, n, 0);
    const uint32_t ref_salu = host_chain(h.data(), n, 1);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // configurations: (workgroups, waves per workgroup)
    const int cfgs[][2] = {{1, 1}, {1, 4}, {256, 4}};
    const char* names[] = {"V0 salu (operands in SGPRs)", "V1 rl3 (today)", "V2 rl2 + split",
                           "V3 ring 3x8 glc", "V4 ring 2x16 glc + split", "V5 direct 2x16 + split",
                           "V6 direct 3x8", "V7 ring (m,t) + readlane f", "V1n rl3 + s_nop before blocks",
                           "V8 ring (m,t) + readlane f 1 ahead"};
    for (int v = 0; v < 10; v++) {
        if (v == 7) continue;   // (k_ring7: the compiler uses s36-s39 between its asm blocks -- unsafe, not run)
        for (auto& cf : cfgs) {
            const int nb = cf[0], wpg = cf[1], nw = nb * wpg;
            hipMemset(out, 0, chains_max * 4);
            float best = 1e30f;
            for (int rep = 0; rep < 3; rep++) {
                hipEventRecord(e0, 0);
                switch (v) {
                case 0: hipLaunchKernelGGL(k_v0, dim3(nw), dim3(64), 0, 0, rec, n, out, cyc); break;
                case 1: hipLaunchKernelGGL(k_rl<1>, dim3(nb), dim3(64 * wpg), 0, 0, rec, n, out, cyc); break;
                case 2: hipLaunchKernelGGL(k_rl<2>, dim3(nb), dim3(64 * wpg), 0, 0, rec, n, out, cyc); break;
                case 3: hipLaunchKernelGGL(k_ring<true>, dim3(nb), dim3(64 * wpg), 0, 0, rec, n, ring, out, cyc); break;
                case 4: hipLaunchKernelGGL(k_ring<false>, dim3(nb), dim3(64 * wpg), 0, 0, rec, n, ring, out, cyc); break;
                case 5: hipLaunchKernelGGL(k_direct<false>, dim3(nb), dim3(64 * wpg), 0, 0, d2, n, out, cyc); break;
                case 6: hipLaunchKernelGGL(k_direct<true>, dim3(nb), dim3(64 * wpg), 0, 0, d3, n, out, cyc); break;
                case 7: hipLaunchKernelGGL(k_ring7, dim3(nb), dim3(64 * wpg), 0, 0, rec, n, ring, out, cyc); break;
                case 8: hipLaunchKernelGGL(k_rl<3>, dim3(nb), dim3(64 * wpg), 0, 0, rec, n, out, cyc); break;
                case 9: hipLaunchKernelGGL(k_ring8, dim3(nb), dim3(64 * wpg), 0, 0, rec, n, ring, out, cyc); break;
                }
                hipEventRecord(e1, 0);
                if (hipEventSynchronize(e1) != hipSuccess) {
                    printf("%s: launch failed\n", names[v]);
                    return 1;
                }
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            std::vector<uint32_t> ho(nw);
            std::vector<uint64_t> hc(nw);
            hipMemcpy(ho.data(), out, nw * 4, hipMemcpyDeviceToHost);
            hipMemcpy(hc.data(), cyc, nw * 8, hipMemcpyDeviceToHost);
            int bad = 0;
            double cs = 0;
            for (int c = 0; c < nw; c++) {
                bad += ho[c] != (v == 0 ? ref_salu : ref[c]);
                cs += (double)hc[c];
            }
            printf("%-28s wg %4d x %d waves: %6.1f cycles/symbol (mean over waves), %6.2f ns/symbol wall, %s\n",
                   names[v], nb, wpg, cs / nw / n, best * 1e6 / n, bad ? "MISMATCH" : "ok");
            fflush(stdout);
        }
    }
    return 0;
}
