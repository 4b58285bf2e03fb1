// sa_kernels.hip -- gfx950 kernels of the SeqArc no-reference block encoder.
//
// Pipeline per batch of blocks:
//   k_prep        per read: symbol counts of every stream, name prefix/suffix
//   k_scan_reads  per block: exclusive scan of the counts over its reads
//   k_emit        per read: (model id, symbol, stream position) of every symbol
//   k_sort_*      per block: stable LSD radix sort of the symbols by model id
//   k_replay_*    per model: replay the adaptive model in stream order
//   k_coder       per (block, stream): the serial carry-less range coder
//   k_md5         per (block, field): RFC1321 digest (runs on a second stream)
//   k_assemble    per block: encaps in doFqzEncode@0x42d2d0 order
#include <hip/hip_runtime.h>

#include <utility>

#include "sa_common.h"
#include "sa_device.h"
#include "sa_logic.h"

namespace sa {

// ---------------------------------------------------------------------------
// wave / workgroup helpers (wave64)
// ---------------------------------------------------------------------------
__device__ inline uint32_t lane_id() { return __lane_id(); }

__device__ inline uint32_t wave_incl_scan(uint32_t v)
{
    const uint32_t lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v += t;
    }
    return v;
}

__device__ inline uint32_t lanes_below(uint64_t m)   // popc(m & ((1 << lane) - 1))
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// inclusive add-scan of a wave64 on DPP (row shifts, then row broadcasts 15/31):
// register-to-register, no LDS round trip
__device__ inline uint32_t wave_incl_scan_dpp(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// exclusive scan across a 1024-thread workgroup; returns the workgroup total
__device__ inline uint32_t wg1024_excl_scan(uint32_t v, uint32_t& excl, uint32_t* sh /*16*/)
{
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(v);
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    if (w == 0) {
        uint32_t s = lane < 16 ? sh[lane] : 0;
        s = wave_incl_scan(s);
        if (lane < 16) sh[lane] = s;
    }
    __syncthreads();
    uint32_t wpre = w ? sh[w - 1] : 0;
    uint32_t total = sh[15];
    excl = wpre + inc - v;
    __syncthreads();
    return total;
}

// exclusive scan across a 256-thread workgroup (called once per kernel: sh is
// not reset)
__device__ inline void wg256_excl_scan(uint32_t v, uint32_t& excl, uint32_t* sh /*4*/)
{
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan_dpp(v);
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    uint32_t wpre = 0;
    for (uint32_t k = 0; k < w; k++) wpre += sh[k];
    excl = wpre + inc - v;
}

// s_setprio 3 when `prio` (a kernel argument, so uniform): the branch is scalar
// code of its own, outside the compiler's control flow
__device__ __forceinline__ void set_l_prio(uint32_t prio)
{
    asm volatile(
        "s_cmp_eq_u32 %0, 0\n\t"
        "s_cbranch_scc1 1f\n\t"
        "s_setprio 2\n"
        "1:" ::"s"(prio)
        : "scc");
}

__device__ __forceinline__ void set_chain_prio(uint32_t prio)
{
    asm volatile(
        "s_cmp_eq_u32 %0, 0\n\t"
        "s_cbranch_scc1 1f\n\t"
        "s_setprio 3\n"
        "1:" ::"s"(prio)
        : "scc");
}

// ---------------------------------------------------------------------------
// k_prep: one thread per read, grid-stride (name prefix / suffix, length and
// tip columns);
// k_prep_sq: one wave per read (SEQ, QUAL and N-IUPAC columns, input checks).
// ---------------------------------------------------------------------------
__global__ void k_prep(const BatchView bv, uint32_t* __restrict__ counts,
                       int16_t* __restrict__ name_p, int16_t* __restrict__ name_s,
                       uint32_t* __restrict__ err)
{
    uint32_t e = 0;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < bv.nreads_total; r += gridDim.x * blockDim.x)
        e |= prep_read(bv, r, counts, name_p, name_s, false);
    if (e) atomicOr(err, e);
}

constexpr uint32_t EMIT_WAVES = 4;
enum : uint32_t { EMIT_SEQ = 1, EMIT_QUAL = 2, EMIT_DEGE = 4 };   // k_emit_sq parts
constexpr uint32_t EMIT_STAGE = 256;   // bases / quals of a read staged in LDS up front

// Stages the first EMIT_STAGE bases and quals of a read in LDS: every load is
// issued before any is used (one memory latency per read instead of one per
// step and loop).
__device__ __forceinline__ void stage_read(const uint8_t* s, const uint8_t* q, uint32_t len,
                                           uint8_t (&st)[2][EMIT_STAGE])
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t pre = len < EMIT_STAGE ? len : EMIT_STAGE;
    uint32_t sb[EMIT_STAGE / 64], qb[EMIT_STAGE / 64];
    __builtin_amdgcn_wave_barrier();   // after the previous read's reads of the stage
    asm volatile("" ::: "memory");
#pragma unroll
    for (uint32_t k = 0; k < EMIT_STAGE / 64; k++) {
        const uint32_t i = 64 * k + lane;
        sb[k] = i < pre ? s[i] : 0u;
        qb[k] = i < pre ? q[i] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < EMIT_STAGE / 64; k++) {
        st[0][64 * k + lane] = (uint8_t)sb[k];
        st[1][64 * k + lane] = (uint8_t)qb[k];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

__device__ inline int wave_max_i32(int v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const int o = __shfl_xor(v, d, 64);
        v = o > v ? o : v;
    }
    return v;
}

// seq_stat + qual_nonhash + the quality range check of one read (sa_common.h),
// 64 positions per step; the gap statistics of reads with an N/IUPAC base run
// on one lane over the staged bytes.
__device__ __forceinline__ void prep_sq_read(const BatchView& bv, const uint32_t r, const uint32_t lane,
                                             uint8_t (&stg)[2][EMIT_STAGE], uint32_t* __restrict__ counts,
                                             uint32_t* __restrict__ err)
{
    const uint32_t b = bv.read_block[r];
    const DevBlock& blk = bv.blocks[b];
    const uint8_t* s = bv.seq + blk.seq_base + bv.seq_off[r];
    const uint8_t* q = bv.qual + blk.seq_base + bv.seq_off[r];
    const uint32_t len = bv.seq_len[r];
    const uint8_t* qv = bv.qual_q + blk.seq_base + bv.seq_off[r];   // QUAL stream (rblock output with -l)
    stage_read(s, q, len, stg);
    auto S = [&](uint32_t i) __attribute__((always_inline)) { return i < EMIT_STAGE ? stg[0][i] : s[i]; };
    auto Q = [&](uint32_t i) __attribute__((always_inline)) { return i < EMIT_STAGE ? stg[1][i] : q[i]; };
    uint32_t valid = 0, nch = 0, n = 0;
    int maxq = 0;
    bool nonascii = false;
    for (uint32_t i0 = 0; i0 < len; i0 += 64) {
        const uint32_t i = i0 + lane;
        const bool in = i < len;
        const uint32_t c = in ? S(i) : (uint32_t)'A', qq = in ? Q(i) : (uint32_t)'#';
        const uint32_t cd = base_code((uint8_t)c);
        nonascii |= __ballot(in && c >= 0x80) != 0;
        const uint64_t vm = __ballot(in && cd <= 3), nm = __ballot(in && cd > 3);
        valid += (uint32_t)__popcll(vm);
        nch += (uint32_t)__popcll(nm);
        if (nm) {
            const int m = wave_max_i32(in && cd > 3 ? (int)(int8_t)qq : 0);
            maxq = m > maxq ? m : maxq;
        }
        const uint32_t qc = bv.lossy ? (in ? (uint32_t)qv[i] : (uint32_t)'#') : qq;   // the QUAL stream's byte
        const uint64_t nz = __ballot(in && qc != '#');
        if (nz) n = i0 + 64 - (uint32_t)__builtin_clzll(nz);
    }
    bool qbad = false;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + lane;
        const uint32_t qq = i < n ? (bv.lossy ? (uint32_t)qv[i] : Q(i)) : 33u;
        qbad |= __ballot(qq < 33 || qq > 126) != 0;
    }
    SeqStat st{valid, nch, (uint32_t)maxq & 0xffu, 0u, 0u, nonascii ? (uint32_t)E_NONASCII : 0u};
    if (nch && lane == 0) {   // seq_stat's second loop
        uint32_t gap = 0;
        for (uint32_t i = 0; i < len; i++) {
            if ((int)st.maxq < (int)(int8_t)Q(i)) continue;
            if (base_code(S(i)) > 3) {
                gap++;
            } else {
                st.exc++;
                st.npos_syms += 1 + (uint32_t)nbits_u32(gap);
                gap = 0;
            }
        }
    }
    if (lane == 0) {
        const uint32_t e = prep_sq_cols(counts + (size_t)r * NCOL, len, n, st, qbad, bv.seq_skip && bv.seq_skip[r]);
        if (e) atomicOr(err, e);
    }
}

// a wave per read, grid-stride (a launch of one tiny workgroup per 4 reads is
// bound by workgroup dispatch)
__global__ __launch_bounds__(64 * EMIT_WAVES) void k_prep_sq(const BatchView bv, uint32_t* __restrict__ counts,
                                                              uint32_t* __restrict__ err)
{
    __shared__ uint8_t stage[EMIT_WAVES][2][EMIT_STAGE];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t r = blockIdx.x * EMIT_WAVES + w; r < bv.nreads_total; r += gridDim.x * EMIT_WAVES)
        prep_sq_read(bv, r, lane, stage[w], counts, err);
}

// k_prep_sq16: the same columns, one 16-lane row per read (four reads per
// wave), each lane taking 16 bytes of the read per step with SWAR byte tests:
// a 150 bp read is one step instead of three wave-wide steps of ballots.
// Bytes are loaded as aligned dwords and funnel-shifted (the reads start at
// any byte).  The gap statistics of reads with an N/IUPAC base (seq_stat's
// second loop) run on the row's first lane.
__device__ __forceinline__ uint32_t bytes_nonzero(uint32_t v)   // 0x80 in every non-zero byte
{
    return (((v & 0x7f7f7f7fu) + 0x7f7f7f7fu) | v) & 0x80808080u;
}

__device__ __forceinline__ void load16(const uint8_t* p, uint32_t w[4])
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* al = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[5];
#pragma unroll
    for (int k = 0; k < 5; k++) d[k] = al[k];
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

template <int W>
__device__ __forceinline__ uint32_t row_sum(uint32_t v)
{
#pragma unroll
    for (int d = W / 2; d >= 1; d >>= 1) v += __shfl_xor(v, d, W);
    return v;
}
template <int W>
__device__ __forceinline__ uint32_t row_max(uint32_t v)
{
#pragma unroll
    for (int d = W / 2; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(v, d, W);
        v = o > v ? o : v;
    }
    return v;
}
template <int W>
__device__ __forceinline__ uint32_t row_min(uint32_t v)
{
#pragma unroll
    for (int d = W / 2; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(v, d, W);
        v = o < v ? o : v;
    }
    return v;
}

constexpr uint32_t PREP_ROW = 16;

// k_prep's name columns, row-parallel (name_prefix_suffix of sa_common.h,
// encode_name@0x421070's prefix / suffix against the previous name of the
// block): each lane compares 16 bytes per step, from the front for the common
// prefix and from the back for the common suffix; the row minimum of the first
// mismatches.  Loop bounds are wave-uniform (every row of the wave steps).
__device__ __forceinline__ uint32_t first_diff16(const uint32_t a[4], const uint32_t b[4], uint32_t cnt)
{
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t nb = cnt > 4u * k ? (cnt - 4u * k < 4 ? cnt - 4u * k : 4) : 0;
        const uint32_t inm = nb >= 4 ? 0x80808080u : (0x80808080u & ((1u << (8 * nb)) - 1u));
        const uint32_t d = bytes_nonzero(a[k] ^ b[k]) & inm;
        if (d) return 4u * k + (uint32_t)(__ffs(d) - 1) / 8;
        if (nb < 4) break;
    }
    return 0xffffffffu;
}

template <int W>
__device__ __forceinline__ void name_cols16(const BatchView& bv, bool live, uint32_t r, uint32_t rl, int& p, int& sfx)
{
    const uint8_t *nm = nullptr, *pv = nullptr;
    uint32_t nl = 0, pl = 0;
    if (live) {
        const DevBlock& blk = bv.blocks[bv.read_block[r]];
        nm = bv.names + blk.name_base + bv.name_off[r];
        nl = bv.name_len[r];
        if (r > blk.read0) {
            pv = bv.names + blk.name_base + bv.name_off[r - 1];
            pl = bv.name_len[r - 1];
        }
    }
    const uint32_t lim = nl < pl ? nl : pl;   // (0 for a block's first read: p = s = 0)
    const uint32_t wlim = (uint32_t)wave_max_i32((int)lim);
    uint32_t lcp = lim, lcs = lim;
    bool pdone = false, sdone = false;
    for (uint32_t i0 = 0; i0 < wlim; i0 += 16 * W) {
        const uint32_t t0 = i0 + 16 * rl;
        uint32_t dp = 0xffffffffu, ds = 0xffffffffu;
        if (t0 < lim) {
            const uint32_t cnt = lim - t0 < 16 ? lim - t0 : 16;
            if (!pdone) {   // from the front: bytes t0 .. t0 + cnt of both names
                uint32_t a[4], b[4];
                load16(nm + t0, a);
                load16(pv + t0, b);
                const uint32_t f = first_diff16(a, b, cnt);
                if (f != 0xffffffffu) dp = t0 + f;
            }
            if (!sdone) {   // from the back: the 16 bytes ending at name[len - t0] of both names
                if (nl - t0 >= 16 && pl - t0 >= 16) {
                    uint32_t a[4], b[4];
                    load16(nm + nl - t0 - 16, a);
                    load16(pv + pl - t0 - 16, b);
                    // window byte i is t = t0 + 15 - i; valid for i >= 16 - cnt; the first
                    // mismatch from the back is the highest mismatching byte of the window
                    const uint32_t first_ok = 16u - cnt;
#pragma unroll
                    for (int w = 3; w >= 0; w--) {
                        uint32_t inm = 0;
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            if (4u * (uint32_t)w + (uint32_t)j >= first_ok) inm |= 0x80u << (8 * j);
                        const uint32_t d = bytes_nonzero(a[w] ^ b[w]) & inm;
                        if (d && ds == 0xffffffffu) ds = t0 + 15u - (4u * (uint32_t)w + (uint32_t)(31 - __clz(d)) / 8);
                    }
                } else {   // (a window reaching the front of a name: byte by byte)
                    for (uint32_t j = 0; j < cnt; j++) {
                        const uint32_t t = t0 + j;
                        if (nm[nl - 1 - t] != pv[pl - 1 - t]) {
                            ds = t;
                            break;
                        }
                    }
                }
            }
        }
        dp = row_min<W>(dp);
        ds = row_min<W>(ds);
        if (!pdone && dp != 0xffffffffu) {
            lcp = dp;
            pdone = true;
        }
        if (!sdone && ds != 0xffffffffu) {
            lcs = ds;
            sdone = true;
        }
        if (__ballot(live && !(pdone && sdone)) == 0) break;
    }
    p = (int)lcp;
    sfx = (int)lcs;
    if ((int)nl - sfx - p < 0) sfx = (int)nl - p;
}

// (round 5) Reads handed to a wave of four 16-lane rows, four at a time.
// Static: grid stride (the round-4 form, wq == nullptr).  Dynamic: the wave
// takes WQ_CHUNK reads at a time from a counter, so the waves on CUs whose
// scalar unit other batches' pass-R chains keep busy (their loops and address
// arithmetic wait for it) take fewer reads instead of finishing last: a
// grid-stride kernel's time is its slowest CU's.
// (round 6) `chunk`, the reads a wave takes at a time, is the host's choice
// per batch (front_wq_chunk): WQ_CHUNK for short reads, down to one wave's
// reads for long ones -- 64 reads of 10-50 kbp a take left an ONT batch's
// 60,000 reads to ~940 waves, each walking 64 reads in series.
constexpr uint32_t WQ_CHUNK = 64;
template <bool DYN, uint32_t RPW = 4>   // (RPW: reads per wave)
struct WaveReads {
    uint32_t* wq;
    uint32_t base, stride, chunk, cur = 0, lim = 0;
    __device__ WaveReads(uint32_t* q, uint32_t wrow0, uint32_t rows, uint32_t ch)
        : wq(q), base(wrow0), stride(rows), chunk(ch) {}
    // the wave's next first row (wave-uniform); false when the reads are done
    __device__ __forceinline__ bool next(uint32_t nr, uint32_t& b)
    {
        if constexpr (!DYN) {
            b = base;
            base += stride;
            return b < nr;
        } else {
            if (cur >= lim) {
                uint32_t g = 0;
                if ((threadIdx.x & 63) == 0) g = atomicAdd(wq, chunk);
                cur = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)g, 0, 64));
                lim = cur + chunk;
            }
            b = cur;
            cur += RPW;
            return b < nr;
        }
    }
};

// W = 64 (round 6): one read per wave, for batches of long reads -- four reads
// of 10-50 kbp in a wave all walked the longest one's length
template <bool DYN, int W = PREP_ROW>
__global__ __launch_bounds__(256) void k_prep_sq16(const BatchView bv, uint32_t* __restrict__ counts,
                                                   uint32_t* __restrict__ err, uint8_t* __restrict__ dege_maxq,
                                                   int16_t* __restrict__ name_p, int16_t* __restrict__ name_s,
                                                   uint32_t* __restrict__ wq, uint32_t wq_chunk)
{
    constexpr uint32_t RPW = 64 / W;   // rows (reads) per wave
    const uint32_t rl = threadIdx.x & (W - 1);
    const uint32_t rows = gridDim.x * (blockDim.x / W);
    const uint32_t row0 = (blockIdx.x * blockDim.x + threadIdx.x) / W;
    const uint32_t nr = bv.nreads_total;
    // wave-uniform trip count: every row of the wave loops while any row has a read
    WaveReads<DYN, RPW> wr(wq, row0 & ~(RPW - 1), rows, wq_chunk);
    for (uint32_t base; wr.next(nr, base);) {
        const uint32_t r = base + (row0 & (RPW - 1));
        const bool live = r < nr;
        uint32_t len = 0;
        const uint8_t *s = nullptr, *q = nullptr, *qv = nullptr;
        if (live) {
            const DevBlock& blk = bv.blocks[bv.read_block[r]];
            const uint64_t o = blk.seq_base + bv.seq_off[r];
            s = bv.seq + o;
            q = bv.qual + o;
            qv = bv.qual_q + o;
            len = bv.seq_len[r];
        }
        uint32_t valid = 0, nonascii = 0, lastnz = 0, firstbad = 0xffffffffu, maxq = 0, hasn = 0;
        const uint32_t wlen = (uint32_t)wave_max_i32((int)len);   // (the wave's longest read)
        for (uint32_t i0 = 0; i0 < wlen; i0 += 16 * W) {
            const uint32_t pos = i0 + 16 * rl;
            if (pos < len) {
                const uint32_t cnt = len - pos < 16 ? len - pos : 16;
                uint32_t sw[4], qw[4], cw[4];
                load16(s + pos, sw);
                load16(q + pos, qw);
                if (bv.lossy) load16(qv + pos, cw);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t nb = cnt > 4u * k ? (cnt - 4u * k < 4 ? cnt - 4u * k : 4) : 0;
                    const uint32_t inm = nb >= 4 ? 0x80808080u : (0x80808080u & ((1u << (8 * nb)) - 1u));
                    const uint32_t x = sw[k] | 0x20202020u;
                    const uint32_t acgt = ~(bytes_nonzero(x ^ 0x61616161u) & bytes_nonzero(x ^ 0x63636363u) &
                                            bytes_nonzero(x ^ 0x67676767u) & bytes_nonzero(x ^ 0x74747474u)) & inm;
                    valid += __popc(acgt);
                    nonascii |= sw[k] & inm;
                    const uint32_t nonb = ~acgt & inm;   // N / IUPAC bytes: max of their (signed) qualities
                    if (nonb) {
                        hasn = 1;
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            if (nonb & (0x80u << (8 * j))) {
                                const int qi = (int)(int8_t)(qw[k] >> (8 * j));
                                if (qi > (int)maxq) maxq = (uint32_t)qi;
                            }
                    }
                    const uint32_t qc = bv.lossy ? cw[k] : qw[k];   // the QUAL stream's bytes
                    const uint32_t nh = bytes_nonzero(qc ^ 0x23232323u) & inm;
                    if (nh) lastnz = pos + 4 * k + (31 - __clz(nh)) / 8 + 1;
                    const uint32_t lo = qc & 0x7f7f7f7fu;
                    const uint32_t bad = ((qc & 0x80808080u) | (~(lo + 0x5f5f5f5fu) & 0x80808080u) |
                                          ((lo + 0x01010101u) & 0x80808080u)) & inm;
                    if (bad && firstbad == 0xffffffffu) firstbad = pos + 4 * k + (__ffs(bad) - 1) / 8;
                }
            }
        }
        valid = row_sum<W>(valid);
        nonascii = row_max<W>(nonascii ? 1u : 0u);
        lastnz = row_max<W>(lastnz);
        firstbad = row_min<W>(firstbad);
        maxq = row_max<W>(maxq);
        hasn = row_max<W>(hasn);
        // seq_stat's second loop, row-parallel (long reads carry N / IUPAC bases
        // in nearly every read): over the positions with quality <= maxq, an
        // ACGT base adds 1 + bits(gap) symbols, gap = the eligible non-ACGT
        // bases since the previous eligible ACGT base.  Each lane summarises its
        // 16 bytes as (g, h) = (eligible non-ACGT after its last eligible ACGT,
        // has one); a row scan gives each lane the gap entering it.
        uint32_t exc = 0, nsym = 0;
        if (__ballot(hasn != 0)) {   // (rows without such a base take no bytes: cnt = 0)
            uint32_t cg = 0;         // the row's carry from the previous step: gap after its last eligible ACGT
            const int mq = (int)(maxq & 0xffu);   // (0..127: the max of signed qualities, from 0)
            const uint32_t mq4 = 0x80808080u | ((uint32_t)mq * 0x01010101u);
            for (uint32_t i0 = 0; i0 < wlen; i0 += 16 * W) {
                const uint32_t pos = i0 + 16 * rl;
                uint32_t sw[4] = {0, 0, 0, 0}, qw[4] = {0, 0, 0, 0}, cnt = 0;
                if (hasn && pos < len) {
                    cnt = len - pos < 16 ? len - pos : 16;
                    load16(s + pos, sw);
                    load16(q + pos, qw);
                }
                // the lane's 16 bytes as bit masks (round 5: SWAR instead of a
                // byte loop): E = eligible (signed quality <= maxq: a byte with
                // the top bit set is negative, else (0x80 + maxq) - q keeps the
                // top bit), A = ACGT; Y = eligible ACGT, N = eligible other bases
                uint32_t E = 0, A = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t nb = cnt > 4u * k ? (cnt - 4u * k < 4 ? cnt - 4u * k : 4) : 0;
                    const uint32_t inm = nb >= 4 ? 0x80808080u : (0x80808080u & ((1u << (8 * nb)) - 1u));
                    const uint32_t x = sw[k] | 0x20202020u;
                    const uint32_t acgt = ~(bytes_nonzero(x ^ 0x61616161u) & bytes_nonzero(x ^ 0x63636363u) &
                                            bytes_nonzero(x ^ 0x67676767u) & bytes_nonzero(x ^ 0x74747474u)) & inm;
                    const uint32_t el = ((mq4 - (qw[k] & 0x7f7f7f7fu)) | qw[k]) & inm;
                    // the four top bits -> four mask bits (bit 7 + 8j -> bit j)
                    E |= ((((el >> 7) & 0x01010101u) * 0x01020408u) >> 24 & 0xfu) << (4 * k);
                    A |= ((((acgt >> 7) & 0x01010101u) * 0x01020408u) >> 24 & 0xfu) << (4 * k);
                }
                const uint32_t Y = E & A, N = E & ~A;
                // the lane's summary: eligible non-ACGT after its last eligible ACGT, and whether it has one
                const uint32_t h = Y ? 1u : 0u;
                const uint32_t g = Y ? (uint32_t)__popc(N >> (32 - __clz(Y))) : (uint32_t)__popc(N);
                // inclusive row scan of (g, h): (A then B) = (hB ? gB : gA + gB, hA | hB)
                uint32_t ig = g, ih = h;
#pragma unroll
                for (int d = 1; d < W; d <<= 1) {
                    const uint32_t pg = __shfl_up(ig, d, W), ph = __shfl_up(ih, d, W);
                    if ((int)rl >= d) {
                        ig = ih ? ig : pg + ig;
                        ih |= ph;
                    }
                }
                uint32_t eg = __shfl_up(ig, 1, W), eh = __shfl_up(ih, 1, W);
                if (rl == 0) eg = eh = 0;
                // the gap entering this lane: the carry, then the lanes before it
                const uint32_t gap = eh ? eg : cg + eg;
                // each eligible ACGT base: 1 + bits(gap before it) symbols; only the
                // first one of the lane and those after an eligible N have a gap
                exc += (uint32_t)__popc(Y);
                nsym += (uint32_t)__popc(Y);
                if (Y) nsym += (uint32_t)nbits_u32(gap + (uint32_t)__popc(N & ((Y & (0u - Y)) - 1u)));
                if (N && (Y & (Y - 1u))) {
                    // (rare: eligible N bases between eligible ACGT bases of the lane)
                    uint32_t yy = Y & (Y - 1u), from = (uint32_t)__ffs(Y);   // bits below `from` are done
                    while (yy) {
                        const uint32_t y = (uint32_t)__ffs(yy) - 1u;
                        nsym += (uint32_t)nbits_u32((uint32_t)__popc(N & ((1u << y) - 1u) & ~((1u << from) - 1u)));
                        from = y + 1u;
                        yy &= yy - 1u;
                    }
                }
                // the row's total (lane 15's inclusive value) continues the carry
                const uint32_t tg = __shfl(ig, W - 1, W), th = __shfl(ih, W - 1, W);
                cg = th ? tg : cg + tg;
            }
            exc = row_sum<W>(exc);
            nsym = row_sum<W>(nsym);
        }
        // k_prep's columns (name_p == nullptr: k_prep runs, SA_PREP_WAVE)
        int np = 0, ns = 0;
        if (name_p && !bv.bin_mode) name_cols16<W>(bv, live, r, rl, np, ns);
        if (live && rl == 0) {
            SeqStat st{valid, len - valid, maxq & 0xffu, hasn ? exc : 0u, hasn ? nsym : 0u,
                       nonascii ? (uint32_t)E_NONASCII : 0u};
            uint32_t* c = counts + (size_t)r * NCOL;
            uint32_t e = prep_sq_cols(c, len, lastnz, st, firstbad < lastnz, bv.seq_skip && bv.seq_skip[r]);
            dege_maxq[r] = (uint8_t)st.maxq;   // (k_emit / k_emit_sq: the side streams)
            if (name_p) {   // (prep_read with bulk = false)
                c[C_LEN] = len == 0 ? 1 : (bv.blocks[bv.read_block[r]].len_long ? 5 : 3);
                c[C_TIP] = 1;
                if (bv.bin_mode) {
                    c[C_NAME] = 0;
                } else {
                    const int nl = bv.name_len[r];
                    if (nl > 255) e |= E_NAME;
                    name_p[r] = (int16_t)np;
                    name_s[r] = (int16_t)ns;
                    const int mid = nl - ns - np;
                    c[C_NAME] = 3 + (mid > 0 ? (uint32_t)mid : 0);
                }
            }
            if (e) atomicOr(err, e);
        }
    }
}

// ---------------------------------------------------------------------------
// R-Block lossy pre-pass (rblock@0x426c10; sa_logic.h): speculative chunk
// passes, one carry lane per block, chunk replay writing every run once.
// ---------------------------------------------------------------------------
// (round 5) the R decision tables (sa_logic.h RbTab) in LDS, 16 KB per
// workgroup of four waves; k_rb_fix (a lane per block, rarely past a compare)
// reads them from global memory
constexpr uint32_t RB_THREADS = 256;

__device__ __forceinline__ RbTab rb_stage_tab(const uint32_t* __restrict__ tab, uint32_t* sh)
{
    for (uint32_t k = threadIdx.x; k < 2 * RB_TAB_WORDS; k += blockDim.x) sh[k] = tab[k];
    __syncthreads();
    return RbTab{sh, sh + RB_TAB_WORDS};
}

__global__ __launch_bounds__(RB_THREADS) void k_rb_spec(const uint8_t* __restrict__ q, const RbChunk* __restrict__ ck,
                                                        uint32_t nck, const uint32_t* __restrict__ tab,
                                                        uint32_t* __restrict__ opens, RbRun* __restrict__ spec_exit,
                                                        uint8_t* __restrict__ vals, RbInfo* __restrict__ info,
                                                        uint32_t cs, uint32_t* __restrict__ wq)
{
    __shared__ uint32_t sh[2 * RB_TAB_WORDS];
    const RbTab t = rb_stage_tab(tab, sh);
    auto one = [&](uint32_t c) __attribute__((always_inline)) {
        if (vals) spec_exit[c] = rb_spec_vals(q, ck[c], t, opens + (size_t)c * (cs / 32), vals + (size_t)c * cs, info[c], cs);
        else spec_exit[c] = rb_spec(q, ck[c], t, opens + (size_t)c * (cs / 32), cs / 32);
    };
    if (!wq) {   // a lane per chunk, one grid
        const uint32_t c = blockIdx.x * RB_THREADS + threadIdx.x;
        if (c < nck) one(c);
        return;
    }
    // (round 6, the default: SA_RB_SPEC_WG workgroups per CU) a smaller grid
    // whose waves take 64 chunks at a time from a counter, so the waves on CUs
    // that other batches' chains keep busy take fewer
    const uint32_t lane = threadIdx.x & 63;
    for (;;) {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(wq, 64u);
        b = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)b, 0, 64));
        if (b >= nck) break;
        if (b + lane < nck) one(b + lane);
    }
}

// k_rb_guess: one lane per chunk, the chunk's exit if the run open before it
// is the previous chunk's speculative exit -- what it is whenever the previous
// chunk converged, i.e. nearly always.  k_rb_fix then only compares states,
// and runs rb_carry itself (serial byte loads at memory latency: ~50 us per
// chunk, 214 ms per ONT batch, r3r) where the guess does not apply.
__global__ __launch_bounds__(RB_THREADS) void k_rb_guess(const uint8_t* __restrict__ q, const RbChunk* __restrict__ ck,
                                                         uint32_t nck, const uint32_t* __restrict__ tab,
                                                         const uint32_t* __restrict__ opens,
                                                         const RbRun* __restrict__ spec_exit, RbRun* __restrict__ guess,
                                                         uint32_t cs)
{
    __shared__ uint32_t sh[2 * RB_TAB_WORDS];
    const RbTab t = rb_stage_tab(tab, sh);
    const uint32_t c = blockIdx.x * RB_THREADS + threadIdx.x;
    if (c >= nck || c == 0 || (ck[c].flags & RB_FIRST)) return;
    guess[c] = rb_carry(q, ck[c], spec_exit[c - 1], t, opens + (size_t)c * (cs / 32), spec_exit[c]);
}

__global__ __launch_bounds__(64) void k_rb_fix(const uint8_t* __restrict__ q, const RbChunk* __restrict__ ck,
                                               const uint32_t* __restrict__ ck0, uint32_t nblk,
                                               const uint32_t* __restrict__ tab, const uint32_t* __restrict__ opens,
                                               const RbRun* __restrict__ spec_exit, const RbRun* __restrict__ guess,
                                               RbRun* __restrict__ entry, uint32_t cs)
{
    const uint32_t b = blockIdx.x * 64 + threadIdx.x;
    if (b >= nblk) return;
    const RbTab t{tab, tab + RB_TAB_WORDS};
    const uint32_t c0 = ck0[b], c1 = ck0[b + 1];
    if (c0 == c1) return;
    RbRun cur = spec_exit[c0];
    for (uint32_t c = c0 + 1; c < c1; c++) {
        entry[c] = cur;
        const RbRun sp = spec_exit[c - 1];
        if (cur.start == sp.start && cur.mn == sp.mn && cur.mx == sp.mx) cur = guess[c];
        else cur = rb_carry(q, ck[c], cur, t, opens + (size_t)c * (cs / 32), spec_exit[c]);
    }
}

// (round 6) k_rb_fix_w: the same entries, a wave per block and 64 chunks a
// step.  While every check passes, the entry of chunk c is the speculative
// exit of chunk c - 1 (the guess of chunk c - 1 equals it whenever the check
// at chunk c passes), so the checks of a window are independent: lane i tests
// chunk c + i's entry -- `cur` for lane 0, guess[c + i - 1] for the others --
// against spec_exit[c + i - 1]; the window's entries up to the first failing
// lane are written at once, and only that lane runs rb_carry.  k_rb_fix walked
// a block's ~3,300 chunks of an ONT batch one dependent load pair at a time
// (1.6 ms alone, 2.5 ms under the batch's load, r6f / r6j).
__device__ __forceinline__ RbRun rb_shfl(const RbRun& r, uint32_t src)
{
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)r.start, (int)src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(r.start >> 32), (int)src, 64);
    return RbRun{(uint64_t)hi << 32 | lo, (uint32_t)__shfl((int)r.mn, (int)src, 64),
                 (uint32_t)__shfl((int)r.mx, (int)src, 64)};
}

__global__ __launch_bounds__(64) void k_rb_fix_w(const uint8_t* __restrict__ q, const RbChunk* __restrict__ ck,
                                                 const uint32_t* __restrict__ ck0, uint32_t nblk,
                                                 const uint32_t* __restrict__ tab, const uint32_t* __restrict__ opens,
                                                 const RbRun* __restrict__ spec_exit, const RbRun* __restrict__ guess,
                                                 RbRun* __restrict__ entry, uint32_t cs)
{
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    if (b >= nblk) return;
    const RbTab t{tab, tab + RB_TAB_WORDS};
    const uint32_t c0 = ck0[b], c1 = ck0[b + 1];
    if (c0 == c1) return;
    RbRun cur = spec_exit[c0];   // (wave-uniform: the true run open after chunk c)
    for (uint32_t c = c0 + 1; c < c1;) {
        const uint32_t n = c1 - c < 64 ? c1 - c : 64;
        const uint32_t ci = c + lane;
        RbRun e = cur;
        bool ok = true;
        if (lane < n) {
            if (lane > 0) e = guess[ci - 1];
            const RbRun sp = spec_exit[ci - 1];
            ok = e.start == sp.start && e.mn == sp.mn && e.mx == sp.mx;
        }
        const uint64_t bad = __ballot(!ok);
        const uint32_t f = bad ? (uint32_t)__ffsll((unsigned long long)bad) - 1u : n;   // first failing chunk
        if (lane < n && lane <= f) entry[ci] = e;
        if (f < n) {
            RbRun nx = e;
            if (lane == f) nx = rb_carry(q, ck[ci], e, t, opens + (size_t)ci * (cs / 32), spec_exit[ci]);
            cur = rb_shfl(nx, f);
            c += f + 1;
        } else {
            cur = guess[c + n - 1];
            c += n;
        }
    }
}

__global__ __launch_bounds__(RB_THREADS) void k_rb_apply(const uint8_t* __restrict__ q, uint8_t* __restrict__ out,
                                                         const RbChunk* __restrict__ ck, uint32_t nck,
                                                         const uint32_t* __restrict__ tab,
                                                         const RbRun* __restrict__ entry)
{
    __shared__ uint32_t sh[2 * RB_TAB_WORDS];
    const RbTab t = rb_stage_tab(tab, sh);
    const uint32_t c = blockIdx.x * RB_THREADS + threadIdx.x;
    if (c >= nck) return;
    const RbChunk k = ck[c];
    rb_apply(q, out, k, (k.flags & RB_FIRST) ? RbRun{k.base, 0u, 0u} : entry[c], t);
}

// (round 5) k_rb_true: a lane per chunk after a block's first, the true pass
// from its entry until it converges with the speculative one (rb_true);
// k_rb_fill: a workgroup of RB_WORDS threads per chunk, 32 output bytes each
// from the open bits and the run values (rb_fill_word): the last open before
// each thread's word is an exclusive max-scan over the workgroup's words.
__global__ __launch_bounds__(RB_THREADS) void k_rb_true(const uint8_t* __restrict__ q, const RbChunk* __restrict__ ck,
                                                        uint32_t nck, const uint32_t* __restrict__ tab,
                                                        uint32_t* __restrict__ opens, uint8_t* __restrict__ vals,
                                                        RbInfo* __restrict__ info, const RbRun* __restrict__ entry,
                                                        uint32_t cs)
{
    __shared__ uint32_t sh[2 * RB_TAB_WORDS];
    const RbTab t = rb_stage_tab(tab, sh);
    const uint32_t c = blockIdx.x * RB_THREADS + threadIdx.x;
    if (c >= nck || (ck[c].flags & RB_FIRST)) return;
    rb_true(q, ck[c], entry[c], t, opens + (size_t)c * (cs / 32), vals + (size_t)c * cs, info[c]);
}

__global__ __launch_bounds__(RB_WORDS) void k_rb_fill(uint8_t* __restrict__ out, const RbChunk* __restrict__ ck,
                                                      const uint32_t* __restrict__ opens,
                                                      const uint8_t* __restrict__ vals, const RbInfo* __restrict__ info,
                                                      uint32_t cs)
{
    __shared__ int32_t wl[RB_WORDS / 64];
    __shared__ uint32_t ev[2];
    const uint32_t c = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const RbChunk k = ck[c];
    if (t == 0) {
        ev[0] = info[c].entry_val & 0xffu;
        ev[1] = rb_chase(info, ck, c);
    }
    const uint32_t word = t < cs / 32 ? opens[(size_t)c * (cs / 32) + t] : 0u;
    // the last open at or before the end of each word, then exclusive over the words
    int32_t m = word ? (int32_t)(32 * t + 31 - __clz(word)) : -1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int32_t o = __shfl_up(m, d, 64);
        if (lane >= (uint32_t)d) m = m > o ? m : o;
    }
    if (lane == 63) wl[w] = m;
    __syncthreads();
    int32_t prev = __shfl_up(m, 1, 64);
    if (lane == 0) prev = -1;
    for (uint32_t k2 = 0; k2 < w; k2++) prev = prev > wl[k2] ? prev : wl[k2];
    if (32 * t < k.len) rb_fill_word(out, k, t, word, prev, vals + (size_t)c * cs, info[c], ev[0], ev[1]);
}

// ---------------------------------------------------------------------------
// k_scan_reads: one 1024-thread workgroup per block; exclusive scan of the
// count columns over the block's reads (in place) and per-block totals.  Also
// the running maximum of name lengths before each read (name_maxlen).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_scan_reads(const BatchView bv, uint32_t* __restrict__ counts,
                                                     uint32_t* __restrict__ totals,
                                                     uint16_t* __restrict__ name_maxlen)
{
    __shared__ uint32_t sh[16];
    __shared__ uint32_t shmax[16];
    const uint32_t b = blockIdx.x;
    const DevBlock& blk = bv.blocks[b];
    const uint32_t r0 = blk.read0, n = blk.nreads;
    uint32_t carry[NCOL];
#pragma unroll
    for (int k = 0; k < NCOL; k++) carry[k] = 0;
    uint32_t mcarry = 0;
    for (uint32_t base = 0; base < n; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const bool in = i < n;
        uint32_t* c = counts + (size_t)(r0 + i) * NCOL;
#pragma unroll
        for (int k = 0; k < NCOL; k++) {
            uint32_t v = in ? c[k] : 0;
            uint32_t ex;
            uint32_t tot = wg1024_excl_scan(v, ex, sh);
            if (in) c[k] = carry[k] + ex;
            carry[k] += tot;
        }
        // exclusive running max of name lengths
        uint32_t v = in ? bv.name_len[r0 + i] : 0;
        const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
        uint32_t m = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t t = __shfl_up(m, d, 64);
            if (lane >= (uint32_t)d) m = m > t ? m : t;
        }
        if (lane == 63) shmax[w] = m;
        __syncthreads();
        uint32_t wmax = mcarry;
        for (uint32_t k = 0; k < w; k++) wmax = wmax > shmax[k] ? wmax : shmax[k];
        uint32_t prev_incl = __shfl_up(m, 1, 64);
        uint32_t excl = lane ? (prev_incl > wmax ? prev_incl : wmax) : wmax;
        if (in) name_maxlen[r0 + i] = (uint16_t)excl;
        uint32_t all = mcarry;
        for (uint32_t k = 0; k < 16; k++) all = all > shmax[k] ? all : shmax[k];
        __syncthreads();
        mcarry = all;
    }
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NCOL; k++) totals[(size_t)b * NCOL + k] = carry[k];
    }
}

// ---------------------------------------------------------------------------
// k_emit: one thread per read (grid-stride); the length, name and degenerate-base symbols
// (the serial per-read tokenizers).  k_emit_sq: one wave per read; the SEQ and
// QUAL symbols, 64 positions per step, written coalesced.
// ---------------------------------------------------------------------------
__global__ void k_emit(const BatchView bv, const uint32_t* __restrict__ counts, const uint32_t* __restrict__ totals,
                       const int16_t* __restrict__ name_p, const int16_t* __restrict__ name_s,
                       const uint16_t* __restrict__ name_maxlen,
                       uint32_t* __restrict__ seq_key, uint32_t* __restrict__ seq_val,
                       uint32_t* __restrict__ aux_key, uint32_t* __restrict__ aux_val,
                       uint32_t* __restrict__ err, const uint8_t* __restrict__ dege_maxq)
{
    uint32_t e = 0;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < bv.nreads_total; r += gridDim.x * blockDim.x)
        e |= emit_read(bv, r, counts, totals, name_p, name_s, name_maxlen, seq_key, seq_val, aux_key, aux_val, false,
                       dege_maxq);
    if (e) atomicOr(err, e);
}

__device__ inline uint32_t shfl_up0(uint32_t v, uint32_t d)   // lane - d's value, 0 below lane d
{
    const uint32_t x = (uint32_t)__shfl_up((int)v, d, 64);
    return lane_id() >= d ? x : 0u;
}

// SEQ (encode_seq@0x421f30): the context of an ACGT base is the seed
// 0x7616c7 shifted by two bits per earlier ACGT base of the read, plus those
// bases' codes, masked -- i.e. the packed codes of the up to 16 previous ACGT
// bases over the seed.  The step's ACGT bases are compacted (LDS, only when a
// step holds another character), then a shuffle ladder packs 1, 2, 4, 8, 16
// previous codes.  QUAL (encode_qual@0x422180): the context after symbol i
// depends on symbols i-1, i-2 and the running sum delta of the drops, an
// inclusive scan.
__device__ __forceinline__ void emit_sq_read(const BatchView& bv, const uint32_t r, const uint32_t lane,
                                             uint32_t (&comp)[64], uint8_t (&stg)[2][EMIT_STAGE],
                                             const uint32_t* __restrict__ counts, uint32_t* __restrict__ seq_key,
                                             uint32_t* __restrict__ seq_val, uint32_t* __restrict__ aux_key,
                                             uint32_t* __restrict__ aux_val, const uint32_t* __restrict__ totals,
                                             const uint8_t* __restrict__ dege_maxq, const uint32_t seq_sh,
                                             const uint32_t parts)
{
    const uint32_t b = bv.read_block[r];
    const DevBlock& blk = bv.blocks[b];
    const uint8_t* s = bv.seq + blk.seq_base + bv.seq_off[r];
    const uint8_t* q = bv.qual_q + blk.seq_base + bv.seq_off[r];   // QUAL stream only (rblock output with -l)
    const uint32_t len = bv.seq_len[r];
    const uint32_t* off = counts + (size_t)r * NCOL;
    stage_read(s, q, len, stg);
    auto S = [&](uint32_t i) __attribute__((always_inline)) { return i < EMIT_STAGE ? stg[0][i] : s[i]; };
    auto Q = [&](uint32_t i) __attribute__((always_inline)) { return i < EMIT_STAGE ? stg[1][i] : q[i]; };
    if ((parts & EMIT_SEQ) && !(bv.seq_skip && bv.seq_skip[r])) {   // (reference path: aligned reads leave the SEQ stream)
        uint32_t* K = seq_key + blk.seq_sym_base;
        uint32_t* V = seq_val + blk.seq_sym_base;
        uint32_t d = off[C_SEQ];
        const uint32_t mask = bv.seq_mask;
        uint32_t carry = 0x7616c7u & mask;   // the context after the previous step
        for (uint32_t i0 = 0; i0 < len; i0 += 64) {
            const uint32_t i = i0 + lane;
            const uint32_t cd = i < len ? base_code(S(i)) : 4u;
            const uint64_t vm = __ballot(cd <= 3);
            const uint32_t nv = (uint32_t)__popcll(vm);
            const uint32_t in_step = len - i0 < 64 ? len - i0 : 64;
            uint32_t c = cd;
            if (vm != (in_step == 64 ? ~0ull : (1ull << in_step) - 1ull)) {   // compact the ACGT codes
                if (cd <= 3) comp[lanes_below(vm)] = cd;
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
                c = lane < nv ? comp[lane] : 0u;
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
            }
            uint32_t x = shfl_up0(c, 1);
            x |= shfl_up0(x, 1) << 2;
            x |= shfl_up0(x, 2) << 4;
            x |= shfl_up0(x, 4) << 8;
            x |= shfl_up0(x, 8) << 16;
            const uint32_t ctx = ((lane < 16 ? carry << (2 * lane) : 0u) | x) & mask;
            if (lane < nv) {   // seq_sh = 2: the base rides in the key, the value is the index (implicit)
                if (seq_sh) {
                    K[d + lane] = (ctx << 2) | c;
                } else {
                    K[d + lane] = ctx;
                    V[d + lane] = ((d + lane) << 2) | c;
                }
            }
            if (nv) carry = __builtin_amdgcn_readlane(((ctx << 2) + c) & mask, (int)nv - 1);
            d += nv;
        }
    }
    if (parts & EMIT_QUAL) {
        // trailing '#' are not coded (qual_nonhash); one symbol 94 marks them
        uint32_t n = 0;
        for (uint32_t i0 = 0; i0 < len; i0 += 64) {
            const uint32_t i = i0 + lane;
            const uint64_t nz = __ballot(i < len && Q(i) != '#');
            if (nz) n = i0 + 64 - (uint32_t)__builtin_clzll(nz);
        }
        uint32_t* K = aux_key + blk.aux_sym_base;
        uint32_t* V = aux_val ? aux_val + blk.aux_sym_base : nullptr;
        const uint32_t pos0 = blk.sbase[ST_QUAL] + off[C_QUAL];
        const int ql = bv.qlevel;
        uint32_t p1 = 0, p2 = 0, ctx_c = 0;   // sym i0-1, sym i0-2, the context after i0-1
        int delta_c = 5;
        for (uint32_t i0 = 0; i0 < n; i0 += 64) {
            const uint32_t i = i0 + lane;
            const uint32_t sym = i < n ? (uint32_t)(uint8_t)(Q(i) - 33) : 0u;
            const uint32_t u1 = (uint32_t)__shfl_up((int)sym, 1, 64), u2 = (uint32_t)__shfl_up((int)sym, 2, 64);
            const uint32_t q1 = lane >= 1 ? u1 : p1;
            const uint32_t q2 = lane >= 2 ? u2 : lane == 1 ? p1 : p2;
            const uint32_t drop = i < n && q1 > sym ? q1 - sym : 0u;
            const int delta = delta_c + (int)wave_incl_scan_dpp(drop);
            uint32_t ctx = (((q1 > q2 ? q1 : q2) << 6) + sym) & 0xfffu;
            if (ql > 1) {
                ctx += q1 == q2 ? 0x1000u : 0u;
                ctx += (uint32_t)(((delta <= 56 ? delta : 56) & 0xf8) << 10);
                if (ql > 2) ctx += i <= 0x6f ? (uint32_t)(((i + 15) & 0x78) << 13) : 0xf0000u;
            }
            const uint32_t uc = (uint32_t)__shfl_up((int)ctx, 1, 64);
            const uint32_t last = lane >= 1 ? uc : ctx_c;
            if (i < n) {
                K[pos0 + i] = ((M_QUAL + last) << AUX_SYM_BITS) | sym;
                if (aux_val) V[pos0 + i] = pos0 + i;
            }
            const int tail = (int)(n - i0 < 64 ? n - i0 : 64) - 1;   // last lane of the step
            p1 = __builtin_amdgcn_readlane(sym, tail);
            p2 = __builtin_amdgcn_readlane(sym, tail >= 1 ? tail - 1 : 0);
            delta_c = __builtin_amdgcn_readlane(delta, tail);
            ctx_c = __builtin_amdgcn_readlane(ctx, tail);
        }
        if (n != len && lane == 0) {
            K[pos0 + n] = ((M_QUAL + ctx_c) << AUX_SYM_BITS) | 94u;
            if (aux_val) V[pos0 + n] = pos0 + n;
        }
    }
    // N / IUPAC side streams (DegeInfoProcess@0x433a10), 64 positions per step,
    // when k_prep_sq16 left the read's maxq (long reads carry such bases in
    // nearly every read; k_emit's serial loops took four passes per read):
    // the CH codes in order, and per eligible ACGT base (quality <= maxq, the
    // original qualities) the kModel symbols of the gap before it -- a wave
    // scan of (gap, has-ACGT) gives each lane its gap, an exclusive scan of the
    // symbol counts its slots.
    if ((parts & EMIT_DEGE) && dege_maxq && read_col_count(bv, counts, totals, r, C_CH)) {
        const int mq = (int)dege_maxq[r];
        const uint8_t* qo = bv.qual + blk.seq_base + bv.seq_off[r];
        uint32_t* K = aux_key + blk.aux_sym_base;
        uint32_t pch = blk.sbase[ST_CH] + off[C_CH];
        uint32_t pnp = blk.sbase[ST_NPOS] + off[C_NPOS];
        uint32_t gcarry = 0;   // eligible non-ACGT bases since the last eligible ACGT base
        const uint64_t below = (1ull << lane) - 1ull;
        for (uint32_t i0 = 0; i0 < len; i0 += 64) {
            const uint32_t i = i0 + lane;
            const bool in = i < len;
            const uint32_t cd = in ? base_code(S(i)) : 0u;
            const bool isn = in && cd > 3;
            const uint64_t nm = __ballot(isn);
            if (isn) K[pch + (uint32_t)__popcll(nm & below)] = (M_CH << AUX_SYM_BITS) | (cd - 4);
            pch += (uint32_t)__popcll(nm);
            const bool elig = in && (int)(int8_t)(i < EMIT_STAGE && !bv.lossy ? stg[1][i] : qo[i]) <= mq;
            uint32_t g = elig && isn ? 1u : 0u, h = elig && !isn ? 1u : 0u;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {   // inclusive scan: (A then B) = (hB ? gB : gA + gB, hA | hB)
                const uint32_t pg = (uint32_t)__shfl_up((int)g, d, 64), ph = (uint32_t)__shfl_up((int)h, d, 64);
                if (lane >= (uint32_t)d) {
                    g = h ? g : pg + g;
                    h |= ph;
                }
            }
            uint32_t eg = (uint32_t)__shfl_up((int)g, 1, 64), eh = (uint32_t)__shfl_up((int)h, 1, 64);
            if (lane == 0) eg = eh = 0;
            const uint32_t gap = eh ? eg : gcarry + eg;
            const bool emit = elig && !isn;
            const uint32_t nb = emit ? (uint32_t)nbits_u32(gap) : 0u;
            const uint32_t cnt = emit ? 1 + nb : 0u;
            const uint32_t incl = wave_incl_scan_dpp(cnt);
            if (emit) {
                uint32_t at = pnp + incl - cnt;
                K[at++] = (M_KBITS << AUX_SYM_BITS) | nb;
                for (uint32_t k = 0; k < nb; k++) K[at++] = ((M_KBIT0 + k) << AUX_SYM_BITS) | ((gap >> k) & 1u);
            }
            pnp += (uint32_t)__builtin_amdgcn_readlane(incl, 63);
            const uint32_t tg = (uint32_t)__builtin_amdgcn_readlane(g, 63), th = (uint32_t)__builtin_amdgcn_readlane(h, 63);
            gcarry = th ? tg : gcarry + tg;
        }
    }
}

// The reads with N / IUPAC bases (a nonzero CH count): a wave tests 64 reads
// at once (each lane one read's CH count, four dependent loads; one read per
// wave step was 5.6 ms of dependent loads per batch, r4n) and appends the
// flagged ones to list[1..] (list[0]: their number; zeroed before).
__global__ __launch_bounds__(256) void k_dege_list(const BatchView bv, const uint32_t* __restrict__ counts,
                                                   const uint32_t* __restrict__ totals, uint32_t* __restrict__ list)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * (blockDim.x >> 6) * 64;
    for (uint32_t r0 = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; r0 < bv.nreads_total; r0 += stride) {
        const uint32_t r = r0 + lane;
        const bool has = r < bv.nreads_total && read_col_count(bv, counts, totals, r, C_CH) != 0;
        const uint64_t m = __ballot(has);
        if (!m) continue;
        uint32_t at = 0;
        if (lane == 0) at = atomicAdd(list, (uint32_t)__popcll(m));
        at = (uint32_t)__shfl((int)at, 0, 64);
        if (has) list[1 + at + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = r;
    }
}

__global__ __launch_bounds__(64 * EMIT_WAVES) void k_emit_sq(const BatchView bv, const uint32_t* __restrict__ counts,
                                                              uint32_t* __restrict__ seq_key,
                                                              uint32_t* __restrict__ seq_val,
                                                              uint32_t* __restrict__ aux_key,
                                                              uint32_t* __restrict__ aux_val,
                                                              const uint32_t* __restrict__ totals,
                                                              const uint8_t* __restrict__ dege_maxq, const uint32_t seq_sh,
                                                              const uint32_t parts,
                                                              const uint32_t* __restrict__ dege_list,
                                                              uint32_t* __restrict__ wq)
{
    __shared__ uint32_t comp[EMIT_WAVES][64];
    __shared__ uint8_t stage[EMIT_WAVES][2][EMIT_STAGE];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (parts == EMIT_DEGE) {
        // only the reads with N / IUPAC bases have work: k_dege_list listed
        // them, a wave per listed read (round 5: the waves had walked the
        // flagged reads of their own 64-read group -- for long reads, where
        // nearly every read has some, 60,000 reads on ~940 waves, 76 ms per
        // ONT batch, profiles/round5_r5b_ont_kernel_stats.txt)
        // (round 6) wq: long-read batches take the listed reads one at a time
        // from a counter, so the waves on CUs that other batches' chains keep
        // busy take fewer of the 10-50 kbp reads instead of finishing last
        const uint32_t n = dege_list[0];
        if (wq) {
            for (;;) {
                uint32_t i = 0;
                if (lane == 0) i = atomicAdd(wq, 1u);
                i = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)i, 0, 64));
                if (i >= n) break;
                emit_sq_read(bv, dege_list[1 + i], lane, comp[w], stage[w], counts, seq_key, seq_val, aux_key,
                             aux_val, totals, dege_maxq, seq_sh, parts);
            }
            return;
        }
        for (uint32_t i = blockIdx.x * EMIT_WAVES + w; i < n; i += gridDim.x * EMIT_WAVES)
            emit_sq_read(bv, dege_list[1 + i], lane, comp[w], stage[w], counts, seq_key, seq_val, aux_key, aux_val,
                         totals, dege_maxq, seq_sh, parts);
        return;
    }
    for (uint32_t r = blockIdx.x * EMIT_WAVES + w; r < bv.nreads_total; r += gridDim.x * EMIT_WAVES)
        emit_sq_read(bv, r, lane, comp[w], stage[w], counts, seq_key, seq_val, aux_key, aux_val, totals, dege_maxq,
                     seq_sh, parts);
}

// ---------------------------------------------------------------------------
// k_emit_sq16: the SEQ and QUAL symbols of every read, one 16-lane row per read
// (four reads per wave, grid-stride like k_prep_sq16), each lane 16 consecutive
// bytes per step (256 bytes of a read per step: a 150 bp read is one step
// instead of k_emit_sq's three dependent wave steps per stream).
//   SEQ: a lane packs the codes of its ACGT bases (2 bits each, the last 16);
//   a row scan concatenates them, so each lane knows the codes of the <= 16
//   ACGT bases before its first one (the context, encode_seq@0x421f30, seed
//   0x7616c7); the lane then walks its bytes.
//   QUAL (encode_qual@0x422180): the context after symbol i needs symbols
//   i-1, i-2 (from the previous lane's last two) and the running sum of drops
//   (a row scan of the lanes' drop sums).
// Keys are staged per row in LDS and written out row-contiguous.  The N /
// IUPAC side streams stay in k_emit_sq (parts = EMIT_DEGE).
// ---------------------------------------------------------------------------
constexpr uint32_t ER = 16;              // lanes per row
constexpr uint32_t ER_STEP = 16 * ER;    // bytes of a read per step

__device__ __forceinline__ uint32_t cat_codes(uint32_t a, uint32_t b, uint32_t nb)   // a's codes, then nb codes b
{
    return nb >= 16 ? b : (a << (2 * nb)) | b;
}

__device__ __forceinline__ uint32_t byte_at(const uint32_t (&w)[4], uint32_t j)
{
    return (w[j >> 2] >> (8 * (j & 3))) & 0xffu;
}

// seq_sh SH: 2 = the base in the SEQ key, values implicit; 0 = values position << 2 | base.
// DYN: reads from a counter (WaveReads)
template <uint32_t SH, bool DYN>
__global__ __launch_bounds__(256, 4) void k_emit_sq16(const BatchView bv, const uint32_t* __restrict__ counts,
                                                   uint32_t* __restrict__ seq_key, uint32_t* __restrict__ seq_val,
                                                   uint32_t* __restrict__ aux_key, uint32_t* __restrict__ aux_val,
                                                   uint32_t* __restrict__ wq, uint32_t wq_chunk)
{
    // (one slot past each row's ER_STEP: the stores of the branch-free loops
    // below that carry no symbol land there)
    __shared__ uint32_t stk[256 / ER][ER_STEP + 1];
    __shared__ uint32_t stv[SH ? 1 : 256 / ER][SH ? 1 : ER_STEP + 1];
    const uint32_t rl = threadIdx.x & (ER - 1), rw = threadIdx.x / ER;
    const uint32_t rows = gridDim.x * (blockDim.x / ER);
    const uint32_t row0 = (blockIdx.x * blockDim.x + threadIdx.x) / ER;
    const uint32_t nr = bv.nreads_total;
    const uint32_t mask = bv.seq_mask;
    const int ql = bv.qlevel;
    uint32_t* sk = stk[rw];
    uint32_t* sv = stv[SH ? 0 : rw];
    auto sync_row = [&]() __attribute__((always_inline)) {
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
    };
    WaveReads<DYN> wr(wq, row0 & ~3u, rows, wq_chunk);   // (wave-uniform: the rows of a wave shuffle together)
    for (uint32_t base; wr.next(nr, base);) {
        const uint32_t r = base + (row0 & 3u);
        const bool live = r < nr;
        uint32_t len = 0;
        const uint8_t *s = nullptr, *q = nullptr;
        uint32_t* KS = nullptr;
        uint32_t* VS = nullptr;
        uint32_t* KA = nullptr;
        uint32_t* VA = nullptr;
        uint32_t dseq = 0, pos0 = 0;
        bool skip = true;
        if (live) {
            const DevBlock& blk = bv.blocks[bv.read_block[r]];
            const uint64_t o = blk.seq_base + bv.seq_off[r];
            s = bv.seq + o;
            q = bv.qual_q + o;   // QUAL stream only (rblock output with -l)
            len = bv.seq_len[r];
            const uint32_t* off = counts + (size_t)r * NCOL;
            KS = seq_key + blk.seq_sym_base;
            VS = seq_val + blk.seq_sym_base;
            KA = aux_key + blk.aux_sym_base;
            VA = aux_val ? aux_val + blk.aux_sym_base : nullptr;
            dseq = off[C_SEQ];
            pos0 = blk.sbase[ST_QUAL] + off[C_QUAL];
            skip = bv.seq_skip && bv.seq_skip[r];
        }
        const uint32_t wlen = (uint32_t)wave_max_i32((int)len);
        // ---- SEQ ----
        uint32_t carry = 0x7616c7u;   // the packed codes before the step (seed, masked at use)
        for (uint32_t i0 = 0; i0 < wlen; i0 += ER_STEP) {
            const uint32_t pos = i0 + 16 * rl;
            const uint32_t cnt = !skip && pos < len ? (len - pos < 16 ? len - pos : 16) : 0u;
            uint32_t sw[4] = {0, 0, 0, 0};
            if (cnt) load16(s + pos, sw);
            uint32_t P = 0, nv = 0, vmask = 0, codes = 0;
#pragma unroll
            for (uint32_t j = 0; j < 16; j++) {   // (branch-free: selects, no per-lane branches)
                const uint32_t c = j < cnt ? base_code((uint8_t)byte_at(sw, j)) : 4u;
                const bool ok = c <= 3;
                const uint32_t cc = c & 3u;
                P = ok ? (P << 2) | cc : P;
                nv += ok ? 1u : 0u;
                vmask |= (ok ? 1u : 0u) << j;
                codes |= (ok ? cc : 0u) << (2 * j);
            }
            uint32_t ip = P, in = nv;   // inclusive row scan of (codes, count): concatenation
#pragma unroll
            for (uint32_t d = 1; d < ER; d <<= 1) {
                const uint32_t pp = __shfl_up(ip, d, ER), pn = __shfl_up(in, d, ER);
                if (rl >= d) {
                    ip = cat_codes(pp, ip, in);
                    in += pn;
                }
            }
            uint32_t ep = __shfl_up(ip, 1, ER), en = __shfl_up(in, 1, ER);
            if (rl == 0) ep = en = 0;
            uint32_t ctx = cat_codes(carry, ep, en);
            uint32_t k = en;
#pragma unroll
            for (uint32_t j = 0; j < 16; j++) {   // (branch-free: a base that is not coded stores to the dummy slot)
                const bool ok = (vmask >> j) & 1u;
                const uint32_t c = (codes >> (2 * j)) & 3u;
                const uint32_t cm = ctx & mask;
                const uint32_t at = ok ? k : ER_STEP;
                if constexpr (SH != 0) {
                    sk[at] = (cm << 2) | c;
                } else {
                    sk[at] = cm;
                    sv[at] = ((dseq + k) << 2) | c;
                }
                ctx = ok ? (ctx << 2) | c : ctx;
                k += ok ? 1u : 0u;
            }
            const uint32_t tp = __shfl(ip, ER - 1, ER), tn = __shfl(in, ER - 1, ER);
            carry = cat_codes(carry, tp, tn);
            sync_row();
            for (uint32_t t = rl; t < tn; t += ER) {
                KS[dseq + t] = sk[t];
                if constexpr (SH == 0) VS[dseq + t] = sv[t];
            }
            dseq += tn;
            sync_row();
        }
        // ---- QUAL: trailing '#' are not coded (qual_nonhash); one symbol 94 marks them ----
        uint32_t n = 0;
        for (uint32_t i0 = 0; i0 < wlen; i0 += ER_STEP) {
            const uint32_t pos = i0 + 16 * rl;
            const uint32_t cnt = pos < len ? (len - pos < 16 ? len - pos : 16) : 0u;
            uint32_t qw[4] = {0, 0, 0, 0};
            if (cnt) load16(q + pos, qw);
            uint32_t last = 0;
#pragma unroll
            for (uint32_t j = 0; j < 16; j++) last = (j < cnt && byte_at(qw, j) != '#') ? pos + j + 1 : last;
            last = row_max<ER>(last);
            n = last > n ? last : n;
        }
        const uint32_t nw = (uint32_t)wave_max_i32((int)n);
        uint32_t p1 = 0, p2 = 0, ctx_c = 0;   // symbols i0-1, i0-2, the context after i0-1
        int delta_c = 5;
        for (uint32_t i0 = 0; i0 < nw; i0 += ER_STEP) {
            const uint32_t pos = i0 + 16 * rl;
            const uint32_t cnt = pos < n ? (n - pos < 16 ? n - pos : 16) : 0u;
            uint32_t qw[4] = {0, 0, 0, 0};
            if (cnt) load16(q + pos, qw);
            // entering symbols: the previous lane's last two (every earlier lane of a step holds 16)
            const uint32_t l2 = (byte_at(qw, 15) - 33u) & 0xffu, l1 = (byte_at(qw, 14) - 33u) & 0xffu;
            const uint32_t u = __shfl_up(l2 | l1 << 8, 1, ER);
            uint32_t q1 = rl ? (u & 0xffu) : p1, q2 = rl ? (u >> 8) : p2;
            uint32_t dsum = 0;
            {
                uint32_t a1 = q1;
#pragma unroll
                for (uint32_t j = 0; j < 16; j++) {   // (branch-free)
                    const uint32_t sym = (byte_at(qw, j) - 33u) & 0xffu;
                    const bool in = j < cnt;
                    dsum += in && a1 > sym ? a1 - sym : 0u;
                    a1 = in ? sym : a1;
                }
            }
            uint32_t id = dsum;   // inclusive row scan of the drop sums
#pragma unroll
            for (uint32_t d = 1; d < ER; d <<= 1) {
                const uint32_t pd = __shfl_up(id, d, ER);
                if (rl >= d) id += pd;
            }
            int delta = delta_c + (int)(id - dsum);
            // the context before the lane's first symbol: after the previous
            // lane's last symbol, i.e. from its last three symbols and the delta
            // entering this lane (every earlier lane of a step holds 16 symbols)
            const auto qctx = [&](uint32_t a1, uint32_t a2, uint32_t sym, int d, uint32_t i) {
                uint32_t cx = (((a1 > a2 ? a1 : a2) << 6) + sym) & 0xfffu;
                if (ql > 1) {
                    cx += a1 == a2 ? 0x1000u : 0u;
                    cx += (uint32_t)(((d <= 56 ? d : 56) & 0xf8) << 10);
                    if (ql > 2) cx += i <= 0x6f ? (uint32_t)(((i + 15) & 0x78) << 13) : 0xf0000u;
                }
                return cx;
            };
            const uint32_t l3 = (byte_at(qw, 13) - 33u) & 0xffu;
            const uint32_t s3 = __shfl_up(l3, 1, ER);
            uint32_t prev = rl ? qctx(q2, s3, q1, delta, pos - 1) : ctx_c;
            uint32_t cl = 0;   // the context after the lane's last symbol
#pragma unroll
            for (uint32_t j = 0; j < 16; j++) {   // (branch-free: past cnt the state holds)
                const bool in = j < cnt;
                const uint32_t sym = (byte_at(qw, j) - 33u) & 0xffu;
                delta += in ? (int)(q1 > sym ? q1 - sym : 0u) : 0;
                const uint32_t cx = qctx(q1, q2, sym, delta, pos + j);
                sk[in ? 16 * rl + j : ER_STEP] = ((M_QUAL + prev) << AUX_SYM_BITS) | sym;
                prev = in ? cx : prev;
                cl = in ? cx : cl;
                q2 = in ? q1 : q2;
                q1 = in ? sym : q1;
            }
            // the step's last symbol: its lane carries the state on
            const uint32_t tot = n > i0 ? (n - i0 < ER_STEP ? n - i0 : ER_STEP) : 0u;
            const uint32_t src = tot ? (tot - 1) / 16 : 0u;
            const uint32_t dl = (uint32_t)(delta_c + (int)id);   // (the lane's delta after its symbols)
            const uint32_t n1 = __shfl(q1, src, ER), n2 = __shfl(q2, src, ER), nc = __shfl(cl, src, ER),
                           nd = __shfl(dl, src, ER);
            if (tot) {   // (a row whose read ended: its carry stays)
                p1 = n1;
                p2 = n2;
                ctx_c = nc;
                delta_c = (int)nd;
            }
            sync_row();
            for (uint32_t t = rl; t < tot; t += ER) {
                KA[pos0 + i0 + t] = sk[t];
                if (VA) VA[pos0 + i0 + t] = pos0 + i0 + t;
            }
            sync_row();
        }
        if (live && n != len && rl == 0) {
            KA[pos0 + n] = ((M_QUAL + ctx_c) << AUX_SYM_BITS) | 94u;
            if (VA) VA[pos0 + n] = pos0 + n;
        }
    }
}

// ---------------------------------------------------------------------------
// Reference path (doAlignEncode@0x42d4c0): the alignment streams' per-read
// columns, their per-block scan and their keys (sa_logic.h align_read_*).
// ---------------------------------------------------------------------------
// per read: the alignment columns and whether the SEQ stream leaves it out
__global__ __launch_bounds__(256) void k_align_counts(const BatchView bv, const AlignView av,
                                                      uint32_t* __restrict__ acounts, uint8_t* __restrict__ seq_skip)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= bv.nreads_total) return;
    seq_skip[r] = align_read_counts(bv, av, r, acounts + (size_t)r * NACOL) ? 1 : 0;
}

// exclusive scan of the alignment columns per block (one workgroup a block)
__global__ __launch_bounds__(1024) void k_scan_align(const BatchView bv, uint32_t* __restrict__ acounts,
                                                     uint32_t* __restrict__ atot)
{
    __shared__ uint32_t sh[16];
    const DevBlock& blk = bv.blocks[blockIdx.x];
    const uint32_t r0 = blk.read0, n = blk.nreads;
    uint32_t carry[NACOL];
#pragma unroll
    for (int k = 0; k < NACOL; k++) carry[k] = 0;
    for (uint32_t base = 0; base < n; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const bool in = i < n;
        uint32_t* c = acounts + (size_t)(r0 + i) * NACOL;
#pragma unroll
        for (int k = 0; k < NACOL; k++) {
            const uint32_t v = in ? c[k] : 0u;
            uint32_t ex;
            const uint32_t tot = wg1024_excl_scan(v, ex, sh);
            if (in) c[k] = carry[k] + ex;
            carry[k] += tot;
        }
    }
    if (threadIdx.x == 0)
#pragma unroll
        for (int k = 0; k < NACOL; k++) atot[(size_t)blockIdx.x * NACOL + k] = carry[k];
}

__global__ __launch_bounds__(256) void k_align_emit(const BatchView bv, const AlignView av,
                                                    const uint32_t* __restrict__ acounts, uint32_t* __restrict__ aux_key)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= bv.nreads_total) return;
    align_read_emit(bv, av, r, acounts + (size_t)r * NACOL, aux_key, nullptr);
}

// SORT_PAD into the key slots no symbol is written to: each segment's tail up to
// its last tile (ping buffer), and the slack slots past the space (both buffers;
// the replays read past a run's end).
constexpr uint32_t KEY_SLACK = 128;

__global__ __launch_bounds__(256) void k_pad_keys(const SortView sv, uint32_t* __restrict__ k0,
                                                  uint32_t* __restrict__ k1)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t seg = i / SORT_TILE, off = i % SORT_TILE;
    if (seg < sv.nsegs) {
        const SortSeg& g = sv.segs[seg];
        const uint64_t pos = g.base + g.count + off;
        if (pos < g.base + (uint64_t)g.ntiles * SORT_TILE) k0[pos] = SORT_PAD;
    } else if (seg == sv.nsegs && off < KEY_SLACK) {
        k0[sv.total + off] = SORT_PAD;
        k1[sv.total + off] = SORT_PAD;
    }
}

// ---------------------------------------------------------------------------
// Segmented stable LSD radix sort, DB-bit digits (DB = 8 or 9; the host
// picks the widths of a sort's passes, sort_digits()).
// A segment is one block's symbol space, padded with key 0xffffffff to a whole
// number of tiles.  Tile = 256 threads x 16 keys; each wave owns 1024
// consecutive keys processed in 16 rounds of 64, ranked with a DB-ballot
// match (the wavefront "multi-split"), so the scatter is stable.  The scatter
// stages the tile in digit order in LDS and writes each digit's run with
// consecutive threads.  Digit counts are tile-major: row t (global tile index)
// holds tile t's 2^DB counts.
// ---------------------------------------------------------------------------
constexpr uint32_t HIST_TILES = 2;
// (10-bit digits measured slower than 8: a 4096-key tile scatters ~4 keys per
// digit run, too short for coalesced writes)
constexpr int SORT_MIN_DB = 7, SORT_MAX_DB = 9;   // (SA_SORT_MIN_DB=8: round 1's floor, for A/B)

// ---------------------------------------------------------------------------
// Dense AUX model ids.  A block's AUX symbols use a few hundred of the 2^17
// model ids (Qlevel <= 2: 16384 + 65536 quality contexts and the other
// streams' models), so the AUX sort can order them by their rank among the
// block's present models -- the same order as by model id -- in one 9-bit pass
// instead of two passes over the 17-bit id.  k_aux_presence marks the models of
// each tile in an LDS bitmap and ORs its non-zero words into the block's
// bitmap; k_aux_dense turns each block's bitmap into the rank table.
// ---------------------------------------------------------------------------
constexpr uint32_t AUX_DENSE_BITS = 17;                             // model ids < 2^17
constexpr uint32_t AUX_DENSE_WORDS = 1u << (AUX_DENSE_BITS - 5);    // 4096 bitmap words per block

constexpr uint32_t PRESENCE_TILES = 16;   // tiles per k_aux_presence workgroup

__global__ __launch_bounds__(SORT_THREADS) void k_aux_presence(const SortView sv, const uint32_t* __restrict__ keys,
                                                               uint32_t* __restrict__ bm)
{
    // PRESENCE_TILES consecutive tiles per workgroup (one block's, mostly):
    // the LDS bitmap is flushed to the block's global bitmap once per block
    // seen, not once per tile (a tile flushed up to one atomicOr per nonzero
    // word, ~37 M global atomics per batch onto a few hot words); and a key
    // whose model equals its left neighbour's (consecutive stream positions:
    // quality contexts repeat) sets nothing
    __shared__ uint32_t lb[AUX_DENSE_WORDS];
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = threadIdx.x; i < AUX_DENSE_WORDS; i += SORT_THREADS) lb[i] = 0;
    __syncthreads();
    const uint32_t t0 = blockIdx.x * PRESENCE_TILES;
    const uint32_t t1 = t0 + PRESENCE_TILES < sv.ntiles ? t0 + PRESENCE_TILES : sv.ntiles;
    auto flush = [&](uint32_t seg) __attribute__((always_inline)) {
        __syncthreads();
        uint32_t* B = bm + (size_t)seg * AUX_DENSE_WORDS;
        for (uint32_t i = threadIdx.x; i < AUX_DENSE_WORDS; i += SORT_THREADS) {
            if (lb[i]) atomicOr(&B[i], lb[i]);
            lb[i] = 0;
        }
        __syncthreads();
    };
    uint32_t cur = t0 < t1 ? sv.tile_seg[t0] : 0;
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t seg = sv.tile_seg[t];   // (workgroup-uniform)
        if (seg != cur) {
            flush(cur);
            cur = seg;
        }
        const SortSeg& sg = sv.segs[seg];
        const uint32_t* K = keys + sg.base + (size_t)(t - sg.tile0) * SORT_TILE;
        uint32_t k[SORT_ITEMS];
#pragma unroll
        for (int r = 0; r < SORT_ITEMS; r++) k[r] = K[threadIdx.x + r * SORT_THREADS];
#pragma unroll
        for (int r = 0; r < SORT_ITEMS; r++) {
            const uint32_t m = k[r] == SORT_PAD ? 0xffffffffu : k[r] >> AUX_SYM_BITS;
            const uint32_t left = __shfl_up(m, 1, 64);
            if (m < (1u << AUX_DENSE_BITS) && (lane == 0 || left != m)) atomicOr(&lb[m >> 5], 1u << (m & 31));
        }
    }
    if (t0 < t1) flush(cur);
}

// per block (one workgroup): the rank table and the number of models
__global__ __launch_bounds__(256) void k_aux_dense(const uint32_t* __restrict__ bm, uint64_t* __restrict__ tab,
                                                   uint32_t* __restrict__ nmodels)
{
    __shared__ uint32_t sh[4];
    constexpr uint32_t PER = AUX_DENSE_WORDS / 256;
    const uint32_t* B = bm + (size_t)blockIdx.x * AUX_DENSE_WORDS;
    uint64_t* T = tab + (size_t)blockIdx.x * AUX_DENSE_WORDS;
    uint32_t w[PER], s = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
        w[j] = B[threadIdx.x * PER + j];
        s += (uint32_t)__popc(w[j]);
    }
    uint32_t ex;
    wg256_excl_scan(s, ex, sh);
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
        T[threadIdx.x * PER + j] = (uint64_t)ex << 32 | w[j];
        ex += (uint32_t)__popc(w[j]);
    }
    if (threadIdx.x == 255) nmodels[blockIdx.x] = ex;
}

// the digit of a key in a sort pass: bits [shift, shift + DB) of the key, or
// (DENSE) of the dense id of its model; pad keys take the last digit
template <int DB, bool DENSE>
__device__ __forceinline__ uint32_t sort_digit(uint32_t k, uint32_t shift, const uint64_t* __restrict__ T)
{
    constexpr uint32_t ND = 1u << DB;
    if constexpr (!DENSE) {
        return (k >> shift) & (ND - 1);
    } else {
        if (k == SORT_PAD) return ND - 1;
        const uint32_t m = (k >> AUX_SYM_BITS) & ((1u << AUX_DENSE_BITS) - 1u);
        const uint64_t e = T[m >> 5];
        const uint32_t d = (uint32_t)(e >> 32) + (uint32_t)__popc((uint32_t)e & ((1u << (m & 31)) - 1u));
        return (d >> shift) & (ND - 1);
    }
}

template <int DB, bool DENSE>
__global__ __launch_bounds__(SORT_THREADS) void k_sort_hist(const SortView sv, const uint32_t* __restrict__ keys,
                                                            uint32_t shift)
{
    constexpr uint32_t ND = 1u << DB;
    // HIST_TILES consecutive tiles per workgroup (amortises the per-workgroup
    // prologue; each tile's counts still go to its own row)
    __shared__ uint32_t h[HIST_TILES][ND];
    uint32_t k[HIST_TILES][SORT_ITEMS];
    const SortSeg* sgp[HIST_TILES];
#pragma unroll
    for (int j = 0; j < HIST_TILES; j++) {
        const uint32_t t = blockIdx.x * HIST_TILES + j;
        for (uint32_t i = threadIdx.x; i < ND; i += SORT_THREADS) h[j][i] = 0;   // (ND may be < the threads)
        sgp[j] = t < sv.ntiles ? &sv.segs[sv.tile_seg[t]] : nullptr;
    }
#pragma unroll
    for (int j = 0; j < HIST_TILES; j++) {
        if (!sgp[j]) continue;
        const uint32_t t = blockIdx.x * HIST_TILES + j;
        const uint32_t* K = keys + sgp[j]->base + (size_t)(t - sgp[j]->tile0) * SORT_TILE;
#pragma unroll
        for (int i = 0; i < SORT_ITEMS; i++) k[j][i] = K[threadIdx.x + i * SORT_THREADS];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < HIST_TILES; j++) {
        if (!sgp[j]) continue;
        const uint64_t* T = DENSE ? sv.dense + (size_t)sv.tile_seg[blockIdx.x * HIST_TILES + j] * AUX_DENSE_WORDS
                                  : nullptr;
#pragma unroll
        for (int i = 0; i < SORT_ITEMS; i++) atomicAdd(&h[j][sort_digit<DB, DENSE>(k[j][i], shift, T)], 1u);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < HIST_TILES; j++)   // one coalesced row per tile
        if (sgp[j]) {
            const uint32_t t = blockIdx.x * HIST_TILES + j;
            for (uint32_t i = threadIdx.x; i < ND; i += SORT_THREADS) sv.hist[(size_t)t * ND + i] = h[j][i];
        }
}

// The segment's digit counts -> in place, each (tile, digit)'s start in the
// sorted segment: base[d] + the counts of d in earlier tiles.  G groups of
// threads take 1/G of the tiles each; a thread walks DPT digit columns, reading
// rows coalesced across the digits.
template <int DB>
__global__ __launch_bounds__(1024) void k_sort_scan(const SortView sv)
{
    constexpr uint32_t ND = 1u << DB;
    constexpr uint32_t TG = ND < 1024 ? ND : 1024;   // threads per group
    constexpr uint32_t G = 1024 / TG, DPT = ND / TG;
    constexpr uint32_t C = ND >= 1024 ? ND / 1024 : 1;   // digits per thread in the digit scan
    __shared__ uint32_t part[G][ND];
    __shared__ uint32_t sh[16];
    const SortSeg& sg = sv.segs[blockIdx.x];
    uint32_t* H = sv.hist + (size_t)sg.tile0 * ND;
    const uint32_t dl = threadIdx.x % TG, g = threadIdx.x / TG;
    const uint32_t nt = sg.ntiles, q = (nt + G - 1) / G;
    const uint32_t t0 = g * q < nt ? g * q : nt, t1 = t0 + q < nt ? t0 + q : nt;
#pragma unroll
    for (uint32_t j = 0; j < DPT; j++) {
        const uint32_t d = dl + j * TG;
        uint32_t sum = 0;
        uint32_t t = t0;
        for (; t + 8 <= t1; t += 8) {
            uint32_t v[8];
#pragma unroll
            for (int i = 0; i < 8; i++) v[i] = H[(size_t)(t + i) * ND + d];
#pragma unroll
            for (int i = 0; i < 8; i++) sum += v[i];
        }
        for (; t < t1; t++) sum += H[(size_t)t * ND + d];
        part[g][d] = sum;
    }
    __syncthreads();
    // digit bases: exclusive scan of the digit totals in digit order (thread i
    // owns digits [i C, i C + C)); then each group's start per digit
    uint32_t tot[C], s = 0;
#pragma unroll
    for (uint32_t c = 0; c < C; c++) {
        const uint32_t d = threadIdx.x * C + c;
        tot[c] = 0;
        if (d < ND)
#pragma unroll
            for (uint32_t gg = 0; gg < G; gg++) tot[c] += part[gg][d];
        s += tot[c];
    }
    uint32_t ex;
    wg1024_excl_scan(s, ex, sh);
#pragma unroll
    for (uint32_t c = 0; c < C; c++) {
        const uint32_t d = threadIdx.x * C + c;
        if (d < ND) {
            uint32_t acc = ex;
#pragma unroll
            for (uint32_t gg = 0; gg < G; gg++) {
                const uint32_t p = part[gg][d];
                part[gg][d] = acc;
                acc += p;
            }
        }
        ex += tot[c];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < DPT; j++) {
        const uint32_t d = dl + j * TG;
        uint32_t run = part[g][d];
        uint32_t t = t0;
        for (; t + 8 <= t1; t += 8) {
            uint32_t v[8];
#pragma unroll
            for (int i = 0; i < 8; i++) v[i] = H[(size_t)(t + i) * ND + d];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                H[(size_t)(t + i) * ND + d] = run;
                run += v[i];
            }
        }
        for (; t < t1; t++) {
            const uint32_t v = H[(size_t)t * ND + d];
            H[(size_t)t * ND + d] = run;
            run += v;
        }
    }
}

// WIDE: a segment of >= 2^30 keys (the HASH index of a genome of > 2^31
// bases sorts all its seeds as one segment): 64-bit element offsets
// IDX: the input values are the elements' index in the segment (vin unused;
// each value is computed where it is written, so no register holds it)
// INV (with IDX, one pass): vout gets the inverse permutation instead, in
// input order -- vout[index] = the element's sorted slot in its segment --
// coalesced, where the positions would go out scattered (k_seq_unpermute)
template <int DB, bool WIDE, bool DENSE, bool IDX, bool INV = false>
__global__ __launch_bounds__(SORT_THREADS) void k_sort_scatter(const SortView sv,
                                                               const uint32_t* __restrict__ kin,
                                                               const uint32_t* __restrict__ vin,
                                                               uint32_t* __restrict__ kout,
                                                               uint32_t* __restrict__ vout, uint32_t shift)
{
    constexpr uint32_t ND = 1u << DB, NW = SORT_THREADS / 64, C = ND >= SORT_THREADS ? ND / SORT_THREADS : 1;
    // per wave and digit: count, then the wave's slot base in the tile (<= 4096:
    // 16 bits); one tile buffer, keys then values: 22 KB for the 9-bit pass, so
    // three workgroups fit beside pass R's 82 KB of LDS (two with a key and a
    // value buffer)
    __shared__ uint16_t wc[NW][ND];
    __shared__ uint32_t gstart[ND], dsum[NW];
    __shared__ uint32_t sb[SORT_TILE];
    const uint32_t t = blockIdx.x;
    const SortSeg& sg = sv.segs[sv.tile_seg[t]];
    const uint32_t lt = t - sg.tile0;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    for (uint32_t i = threadIdx.x; i < NW * ND; i += SORT_THREADS) (&wc[0][0])[i] = 0;
    __syncthreads();
    const size_t wbase = sg.base + (size_t)lt * SORT_TILE + (size_t)w * (64 * SORT_ITEMS);
    uint32_t k[SORT_ITEMS], v[IDX ? 1 : SORT_ITEMS], rk[SORT_ITEMS];
    // IDX: the values are the index in the segment (a space's first pass: the
    // emitters leave the values out)
    auto val = [&](int r) __attribute__((always_inline)) -> uint32_t {
        return IDX ? lt * SORT_TILE + w * (64 * SORT_ITEMS) + (uint32_t)r * 64 + lane : v[IDX ? 0 : r];
    };
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) {
        k[r] = kin[wbase + (size_t)r * 64 + lane];
        if constexpr (!IDX) v[r] = vin[wbase + (size_t)r * 64 + lane];
    }
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    const uint64_t* T = DENSE ? sv.dense + (size_t)sv.tile_seg[t] * AUX_DENSE_WORDS : nullptr;
    uint32_t dg[SORT_ITEMS];   // (the keys' digits: DENSE ones cost a table read)
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) dg[r] = sort_digit<DB, DENSE>(k[r], shift, T);
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) {
        const uint32_t d = dg[r];
        uint64_t peers = ~0ull;
#pragma unroll
        for (int bit = 0; bit < DB; bit++) {
            const uint64_t bal = __ballot((d >> bit) & 1);
            peers &= ((d >> bit) & 1) ? bal : ~bal;
        }
        const uint32_t before = wc[w][d];
        rk[r] = before + (uint32_t)__popcll(peers & lt_mask);
        if ((peers & lt_mask) == 0) wc[w][d] = (uint16_t)(before + (uint32_t)__popcll(peers));
    }
    __syncthreads();
    {
        // per digit (thread i owns digits [i C, i C + C)): each wave's start
        // within the tile's run of that digit, the run's start in the tile (scan
        // over digits), folded into wc; and the run's start in the output (the
        // scanned counts) minus its start in the tile
        uint32_t cnt[C], s = 0;
#pragma unroll
        for (uint32_t c = 0; c < C; c++) {
            const uint32_t d = threadIdx.x * C + c;
            uint32_t acc = 0;
            if (d < ND) {   // (7-bit digits: half the threads own none)
#pragma unroll
                for (uint32_t ww = 0; ww < NW; ww++) {
                    const uint32_t tcount = wc[ww][d];
                    wc[ww][d] = (uint16_t)acc;
                    acc += tcount;
                }
            }
            cnt[c] = acc;
            s += acc;
        }
        uint32_t ex;
        wg256_excl_scan(s, ex, dsum);
#pragma unroll
        for (uint32_t c = 0; c < C; c++) {
            const uint32_t d = threadIdx.x * C + c;
            if (d < ND) {
#pragma unroll
                for (uint32_t ww = 0; ww < NW; ww++) wc[ww][d] = (uint16_t)(wc[ww][d] + ex);
                gstart[d] = sv.hist[(size_t)t * ND + d] - ex;
            }
            ex += cnt[c];
        }
    }
    __syncthreads();
    // stage the tile in digit order in LDS, then write it out: consecutive
    // threads write consecutive slots of one digit's run (coalesced); the keys
    // first (each thread keeps the output slots of its tile slots), then the
    // values through the same buffer
    // the keys' digits in tile order, for the output offsets
    __shared__ uint16_t sd[DENSE ? SORT_TILE : 1];
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) {
        const uint32_t d = dg[r];
        rk[r] += wc[w][d];   // (the key's slot in the tile)
        sb[rk[r]] = k[r];
        if constexpr (DENSE) sd[rk[r]] = (uint16_t)d;
    }
    __syncthreads();
    if constexpr (WIDE) {
        uint32_t* const ko = kout + sg.base;
        uint32_t* const vo = vout + sg.base;
        uint32_t ro[SORT_ITEMS];   // element offsets in the segment (< 2^32)
#pragma unroll
        for (int r = 0; r < SORT_ITEMS; r++) {
            const uint32_t i = threadIdx.x + (uint32_t)r * SORT_THREADS;
            const uint32_t kk = sb[i];
            ro[r] = gstart[DENSE ? (uint32_t)sd[i] : (kk >> shift) & (ND - 1)] + i;
            ko[(uint64_t)ro[r]] = kk;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < SORT_ITEMS; r++) sb[rk[r]] = val(r);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < SORT_ITEMS; r++) vo[(uint64_t)ro[r]] = sb[threadIdx.x + (uint32_t)r * SORT_THREADS];
    } else {
        // (byte offsets in the segment, 32-bit: a segment of a block's symbols
        // holds < 2^30 keys (plan_batch refuses larger blocks), so the stores take
        // a scalar base and a 32-bit lane offset)
        char* const ko = reinterpret_cast<char*>(kout + sg.base);
        char* const vo = reinterpret_cast<char*>(vout + sg.base);
        uint32_t ro[SORT_ITEMS];
#pragma unroll
        for (int r = 0; r < SORT_ITEMS; r++) {
            const uint32_t i = threadIdx.x + (uint32_t)r * SORT_THREADS;
            const uint32_t kk = sb[i];
            ro[r] = (gstart[DENSE ? (uint32_t)sd[i] : (kk >> shift) & (ND - 1)] + i) << 2;
            *reinterpret_cast<uint32_t*>(ko + ro[r]) = kk;
        }
        if constexpr (INV) {
            static_assert(IDX && !DENSE, "INV: one pass over implicit values");
            uint32_t* const vi = vout + sg.base;
#pragma unroll
            for (int r = 0; r < SORT_ITEMS; r++) vi[val(r)] = gstart[dg[r]] + rk[r];
            return;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < SORT_ITEMS; r++) sb[rk[r]] = val(r);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < SORT_ITEMS; r++)
            *reinterpret_cast<uint32_t*>(vo + ro[r]) = sb[threadIdx.x + (uint32_t)r * SORT_THREADS];
    }
}

// ---------------------------------------------------------------------------
// Sequence model replay: BASE_MODEL<u8> of encode_seq@0x421f30.
// Before the j-th symbol of a context run the model's counts are 3 + the
// occurrences of each base among the run's first j symbols, as long as no
// halving happened; the first halving comes at j = 242 (total 12 + j > 253).
// k_replay_seq: one workgroup per sort tile (4096 sorted symbols, 16 per
// thread): a segmented exclusive scan of one-hot packed counts (4 x 8 bit)
// gives every symbol's model state directly.  The run that continues from the
// previous tile gets its counts from a backwards scan by the first wave.  A
// run reaching j = 242 is queued (its symbol j = 242 appends it) and replayed
// from its start by one lane in k_replay_seq_long.
// ---------------------------------------------------------------------------
constexpr uint32_t SEQ_HALVE_J = 242;   // first in-run index that can halve

// Packed counts: 4 x 16 bit (a run can hold more than 255 of one base; only
// in-run indices < SEQ_HALVE_J are coded here, but the sums must not wrap).
struct SegCnt {   // segmented-scan element
    uint64_t cnt;
    uint32_t head;
};
__device__ inline SegCnt segcnt_op(const SegCnt& a, const SegCnt& b)   // a then b
{
    return SegCnt{b.head ? b.cnt : a.cnt + b.cnt, a.head | b.head};
}
__device__ inline uint64_t onehot16(uint32_t b) { return 1ull << (16 * b); }
__device__ inline uint32_t sum16(uint64_t c)
{
    return (uint32_t)(c & 0xffff) + (uint32_t)((c >> 16) & 0xffff) + (uint32_t)((c >> 32) & 0xffff) +
           (uint32_t)(c >> 48);
}

// sh = 2: keys are context << 2 | base and values the stream position (k <= 14);
// sh = 0: keys are the context and values position << 2 | base
__global__ __launch_bounds__(SORT_THREADS) void k_replay_seq(const SortView sv, const uint32_t* __restrict__ keys,
                                                             const uint32_t* __restrict__ vals, const SymSink rec,
                                                             uint64_t* __restrict__ long_runs,
                                                             uint32_t* __restrict__ nlong, const uint32_t sh)
{
    __shared__ SegCnt part[SORT_THREADS / 64];
    __shared__ uint64_t carry_cnt;
    __shared__ uint32_t last_key[SORT_THREADS];
    const uint32_t t = blockIdx.x;
    const SortSeg& sg = sv.segs[sv.tile_seg[t]];
    const uint32_t lt = t - sg.tile0;
    const size_t tile0 = sg.base + (size_t)lt * SORT_TILE;
    const uint32_t tid = threadIdx.x;
    const size_t i0 = tile0 + (size_t)tid * SORT_ITEMS;
    uint32_t k[SORT_ITEMS], v[SORT_ITEMS];
    {
        const uint4* K4 = reinterpret_cast<const uint4*>(keys + i0);
        const uint4* V4 = reinterpret_cast<const uint4*>(vals + i0);
#pragma unroll
        for (int q = 0; q < SORT_ITEMS / 4; q++) {
            const uint4 a = K4[q], b = V4[q];
            k[4 * q] = a.x; k[4 * q + 1] = a.y; k[4 * q + 2] = a.z; k[4 * q + 3] = a.w;
            v[4 * q] = b.x; v[4 * q + 1] = b.y; v[4 * q + 2] = b.z; v[4 * q + 3] = b.w;
        }
    }
    last_key[tid] = k[SORT_ITEMS - 1];
    const uint32_t before_tile = lt > 0 ? keys[tile0 - 1] : SORT_PAD;
    // counts of the run continued from the previous tile; only its first
    // SEQ_HALVE_J + 64 symbols are counted (later ones are not coded here)
    if (tid < 64) {
        uint64_t cc = 0;
        const uint32_t key0 = keys[tile0];
        if (lt > 0 && (before_tile >> sh) == (key0 >> sh) && key0 != SORT_PAD) {
            for (uint32_t back = 0; back < SEQ_HALVE_J + 64; back += 64) {
                const size_t at = tile0 - 1 - back - tid;
                const bool ok = at >= sg.base && at < tile0 && (keys[at] >> sh) == (key0 >> sh);
                const uint64_t miss = ~__ballot(ok);
                const uint64_t lead = miss ? ((1ull << __builtin_ctzll(miss)) - 1ull) : ~0ull;
                if ((lead >> tid) & 1ull) cc += onehot16((sh ? keys[at] : vals[at]) & 3u);
                if (miss) break;
            }
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) cc += __shfl_xor(cc, d, 64);
        }
        if (tid == 0) carry_cnt = cc;
    }
    __syncthreads();
    const uint32_t prev_key = tid ? last_key[tid - 1] : before_tile;
    // per-thread segmented reduction, then a block-wide scan of the aggregates
    SegCnt acc{0ull, 0u};
    uint32_t pk = prev_key;
#pragma unroll
    for (int e = 0; e < SORT_ITEMS; e++) {
        if ((k[e] >> sh) != (pk >> sh)) {
            acc.cnt = 0;
            acc.head = 1;
        }
        if (k[e] != SORT_PAD) acc.cnt += onehot16((sh ? k[e] : v[e]) & 3u);
        pk = k[e];
    }
    // block-wide exclusive segmented scan of the aggregates: a wave scan
    // (shuffles), then the waves' totals through LDS
    const uint32_t lane = tid & 63, w = tid >> 6;
    SegCnt x = acc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const SegCnt y{__shfl_up(x.cnt, d, 64), __shfl_up(x.head, d, 64)};
        if (lane >= (uint32_t)d) x = segcnt_op(y, x);
    }
    if (lane == 63) part[w] = x;
    __syncthreads();
    SegCnt run{0ull, 0u};
    for (uint32_t k = 0; k < w; k++) run = segcnt_op(run, part[k]);
    {
        const SegCnt y{__shfl_up(x.cnt, 1, 64), __shfl_up(x.head, 1, 64)};
        if (lane > 0) run = segcnt_op(run, y);
    }
    if (!run.head) run.cnt += carry_cnt;   // still inside the run continued from the previous tile
    uint64_t cnt = run.cnt;
    pk = prev_key;
    const SymSink out{rec.prs + sg.base, nullptr};   // packed SEQ records
#pragma unroll
    for (int e = 0; e < SORT_ITEMS; e++) {
        if ((k[e] >> sh) != (pk >> sh)) cnt = 0;
        pk = k[e];
        if (k[e] == SORT_PAD) continue;
        const uint32_t b = (sh ? k[e] : v[e]) & 3u, pos = sh ? v[e] : v[e] >> 2;
        const uint32_t j = sum16(cnt);
        if (j < SEQ_HALVE_J) {
            const uint32_t c0 = 3u + (uint32_t)(cnt & 0xffff), c1 = 3u + (uint32_t)((cnt >> 16) & 0xffff);
            const uint32_t c2 = 3u + (uint32_t)((cnt >> 32) & 0xffff), c3 = 3u + (uint32_t)(cnt >> 48);
            const uint32_t cum = (b > 0 ? c0 : 0u) + (b > 1 ? c1 : 0u) + (b > 2 ? c2 : 0u);
            const uint32_t f = b == 0 ? c0 : b == 1 ? c1 : b == 2 ? c2 : c3;
            sink_put(out, pos, cum, f, j + 12u);
        } else if (j == SEQ_HALVE_J) {
            long_runs[atomicAdd(nlong, 1u)] = i0 + e - SEQ_HALVE_J;   // the run's first symbol
        }
        cnt += onehot16(b);
    }
}

// ---------------------------------------------------------------------------
// k_replay_seq_bkt (round 5): BASE_MODEL replay after ONE sort pass.  The SEQ
// space is sorted stably by the low TB bits of the context only -- a bucket
// (the low bits: the first bases of every read have contexts made of the seed
// 0x7616c7's bits, so by the top bits the first seven positions of all reads
// would share one bucket, many to one context);
// inside it the symbols stay in stream order -- and one wave walks each
// (block, bucket) in stream order with the models of the bucket's 2^SB
// contexts in LDS (4 x u8 counts each, init 3, updated exactly as
// replay_seq_run / encode_seq@0x421f30 do, the halving inline: no run goes to
// k_replay_seq_long).  64 symbols a step: a lane writes its lane id to its
// context's tag and reads it back; the lanes whose context no other lane of the
// step has update their model directly (the common case), the lanes that share
// one take their counts before them from ballots, or one after the other where
// the shared run crosses a halving.  This replaces the further sort passes
// (hist, scan, scatter each) and the tile-wide replay.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bm_tot(uint32_t s) { return (s * 0x01010101u) >> 24; }   // byte sum (< 256)

// the record of base b under model s (tot | cum << 8 | freq << 16); s halved
// first when its total is above 253 (replay_seq_run)
__device__ __forceinline__ uint32_t bm_rec(uint32_t& s, uint32_t b)
{
    uint32_t tot = bm_tot(s);
    if (tot > 253) {
        s -= (s >> 1) & 0x7f7f7f7fu;
        tot = bm_tot(s);
    }
    const uint32_t below = b ? (s & (0xffffffffu >> (32 - 8 * b))) : 0u;
    return tot | (bm_tot(below) << 8) | (((s >> (8 * b)) & 0xffu) << 16);
}

__device__ __forceinline__ uint32_t bm_counts(uint64_t m, uint64_t b0, uint64_t b1, uint64_t b2, uint64_t b3)
{
    return (uint32_t)__popcll(m & b0) | (uint32_t)__popcll(m & b1) << 8 | (uint32_t)__popcll(m & b2) << 16 |
           (uint32_t)__popcll(m & b3) << 24;
}

// grid: nsegs << tb workgroups of one wave; dynamic LDS 5 * ((1 << sb) + 64) bytes;
// spare: 64 records per workgroup (the inactive lanes' stores).
// hist: the bucket pass's scanned histogram (row tile0 of a segment = its
// digit starts); keys = context << 2 | base, values = stream positions.
// SORTED: vals unused, each record goes to its symbol's sorted slot (the
// wave's 64 stores of a step are one run of 256 bytes); k_seq_unpermute puts
// them in stream order
template <bool SORTED>
__global__ __launch_bounds__(64) void k_replay_seq_bkt(const SortView sv, const uint32_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ vals, const SymSink rec,
                                                       uint32_t tb, uint32_t sb, uint32_t subsh,
                                                       PRec* __restrict__ spare, uint64_t* __restrict__ probe,
                                                       const uint32_t* __restrict__ order)
{
    extern __shared__ uint32_t bkt_lds[];
    const uint64_t t0 = probe ? __builtin_amdgcn_s_memrealtime() : 0ull, c0 = probe ? __builtin_amdgcn_s_memtime() : 0ull;
    __shared__ uint32_t fl[128];
    const uint32_t nsub = 1u << sb, nd = 1u << tb;
    // (plain LDS pointers and compiler barriers, not volatile ones: a volatile
    // access becomes a flat access, and every flat access waits for all the
    // wave's outstanding global stores -- the scattered records -- r5e / r5g)
    uint32_t* mst = bkt_lds;   // (nsub models, then 64 lanes' spare slots)
    uint8_t* tag = reinterpret_cast<uint8_t*>(bkt_lds + nsub + 64);
    uint32_t* vfl = fl;
    // (order: workgroup r * nsegs + seg takes the r-th largest digit, see
    // k_bkt_order; without it, workgroup seg << tb | d)
    const uint32_t seg = order ? blockIdx.x % sv.nsegs : blockIdx.x >> tb;
    const uint32_t d = order ? order[blockIdx.x / sv.nsegs] : blockIdx.x & (nd - 1);
    const SortSeg& sg = sv.segs[seg];
    if (sg.count == 0) return;
    const uint32_t* H = sv.hist + (size_t)sg.tile0 * nd;
    const uint32_t start = H[d];
    const uint32_t end = d + 1 < nd ? H[d + 1] : sg.count;   // (the pad keys sort last)
    if (start >= end) return;
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < nsub; i += 64) mst[i] = 0x03030303u;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const uint32_t* K = keys + sg.base;
    const uint32_t* V = vals + sg.base;
    PRec* out = rec.prs + sg.base;
    const uint32_t smask = nsub - 1;
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t nshared = 0;   // (probe: steps with a context shared by lanes)
    // one step: 64 symbols of the bucket in stream order (k: key); the lane's
    // record (for an inactive lane: anything)
    // (round 6) The common path has no lane branches: an inactive lane works on
    // a slot of its own past the bucket's models (sub = nsub + lane: its tag
    // names itself, it shares nothing, its model write lands there), and a
    // shared context's lanes write their (unused) uncontested update there too.
    // Every exec-mask branch is scalar-unit work, which the other batches'
    // pass-R chains hold: under the bench's load this kernel ran 2.4x its time
    // alone, the VALU-only gather beside it 1.1x (r6p).
    auto step = [&](const uint32_t k, const bool act) __attribute__((always_inline)) -> uint32_t {
        const uint32_t sub = act ? (k >> subsh) & smask : nsub + lane, b = k & 3u;
        tag[sub] = (uint8_t)lane;
        asm volatile("" ::: "memory");   // (LDS operations of a wave complete in order)
        const uint32_t t = tag[sub];
        const uint32_t s = mst[sub];
        const bool loser = t != lane;   // another lane of the step has this context
        const uint64_t lm = __ballot(loser);
        bool member = false;            // shares its context with another lane
        if (lm) {
            nshared++;
            vfl[lane] = 0u;
            asm volatile("" ::: "memory");
            vfl[loser ? t : 64 + lane] = 1u;
            asm volatile("" ::: "memory");
            member = loser || vfl[lane] != 0u;
        }
        uint32_t s1 = s;
        uint32_t r = bm_rec(s1, b);
        mst[member ? nsub + lane : sub] = s1 + (1u << (8 * b));
        if (lm) {
            const uint64_t b0 = __ballot(member && b == 0), b1 = __ballot(member && b == 1),
                           b2 = __ballot(member && b == 2), b3 = __ballot(member && b == 3);
            uint64_t M = __ballot(member);
            while (M) {   // one group of lanes with the same context at a time
                const uint32_t L = (uint32_t)__builtin_ctzll(M);
                const uint32_t gs = (uint32_t)__builtin_amdgcn_readlane((int)sub, (int)L);
                const uint64_t G = __ballot(member && sub == gs);
                const uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane((int)s, (int)L);
                const bool in_g = (G >> lane) & 1ull;
                // at most one halving inside a group: the symbol with group index
                // h = 254 - tot halves the model (tot > 253), and after it the
                // total is ~127, which 63 more symbols cannot take past 253
                const uint32_t tot0 = bm_tot(s0), h = tot0 >= 254 ? 0u : 254u - tot0;
                const uint32_t gi = (uint32_t)__popcll(G & below);
                const uint64_t lo = __ballot(in_g && gi < h);   // the members before the halving
                uint32_t sh = s0 + bm_counts(lo, b0, b1, b2, b3);
                sh -= (sh >> 1) & 0x7f7f7f7fu;   // (the model at the halving symbol, halved)
                if (in_g) {
                    uint32_t si = gi < h ? s0 + bm_counts(G & below, b0, b1, b2, b3)
                                         : sh + bm_counts(G & below & ~lo, b0, b1, b2, b3);
                    r = bm_rec(si, b);   // (no halving left for bm_rec: total <= 253)
                }
                if (lane == L)
                    mst[gs] = G == lo ? s0 + bm_counts(G, b0, b1, b2, b3) : sh + bm_counts(G & ~lo, b0, b1, b2, b3);
                M &= ~G;
            }
        }
        asm volatile("" ::: "memory");
        return r;
    };
    // (round 6) Every step issues exactly one store -- an inactive lane's goes
    // to `spare` -- and every step runs (past the bucket's end with no lane
    // active), so the number of stores between two points of the loop is
    // fixed and the waits for the keys (vmcnt, which counts the stores too) are
    // exact: the keys of two chunks ahead are in flight, and a wait never
    // covers the stores of the last eight steps.  Before, a step's store sat
    // in the branches and steps past the end were skipped, so the loop waited
    // for every outstanding store once per chunk -- a full store round trip
    // per eight steps.  The prologue's eight stores to `spare` give the first
    // pass through the loop the same count as every later one.
    constexpr uint32_t BKT_AHEAD = 8;
    uint32_t ka[BKT_AHEAD], pa[SORTED ? 1 : BKT_AHEAD], kb[BKT_AHEAD], pb[SORTED ? 1 : BKT_AHEAD];
    auto load = [&](uint32_t* kk, uint32_t* pp, uint32_t b0) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t j = 0; j < BKT_AHEAD; j++) {
            const uint32_t i = min(b0 + 64 * j + lane, end - 1);   // (branch-free loads)
            kk[j] = K[i];
            if constexpr (!SORTED) pp[j] = V[i];
        }
    };
    auto run = [&](const uint32_t* kk, const uint32_t* pp, uint32_t b0) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t j = 0; j < BKT_AHEAD; j++) {
            const uint32_t i = b0 + 64 * j + lane;
            const bool act = i < end;
            const uint32_t r = step(kk[j], act);
            PRec* dst = act ? out + (SORTED ? i : pp[SORTED ? 0 : j]) : spare + 64 * blockIdx.x + lane;
            *dst = PRec{r};
        }
    };
    load(ka, pa, start);
#pragma unroll
    for (uint32_t j = 0; j < BKT_AHEAD; j++) spare[64 * blockIdx.x + lane] = PRec{0u};
    load(kb, pb, start + 64 * BKT_AHEAD);
    for (uint32_t base = start; base < end; base += 128 * BKT_AHEAD) {
        run(ka, pa, base);
        load(ka, pa, base + 128 * BKT_AHEAD);
        run(kb, pb, base + 64 * BKT_AHEAD);
        load(kb, pb, base + 192 * BKT_AHEAD);
    }
    if (probe) {   // (SA_BKT_PROBE) this wave's clocks, steps and placement
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if (lane == 0) {
            uint64_t* pr = probe + 4ull * blockIdx.x;
            pr[0] = t0;
            pr[1] = t1;
            pr[2] = c1 - c0;
            pr[3] = (uint64_t)((end - start + 63) / 64) | (uint64_t)nshared << 24 | (uint64_t)(xcc & 0xffu) << 48;
        }
    }
}

// (round 6) The bucket replay's digits, largest first over all segments: a
// bucket's wave walks all its symbols in steps of 64, the heavy digits' waves
// run 3-5x the median (SA_BKT_PROBE, r6l: 8-12 ms against 0.7 ms), and
// started last they set the kernel's span.  One workgroup of nd threads.
__global__ __launch_bounds__(1024) void k_bkt_order(const SortView sv, uint32_t nd, uint32_t* __restrict__ order)
{
    __shared__ uint32_t sz[1024];
    const uint32_t d = threadIdx.x;
    if (d < nd) {
        uint32_t n = 0;
        for (uint32_t g = 0; g < sv.nsegs; g++) {
            const SortSeg& sg = sv.segs[g];
            if (sg.count == 0) continue;
            const uint32_t* H = sv.hist + (size_t)sg.tile0 * nd;
            n += (d + 1 < nd ? H[d + 1] : sg.count) - H[d];
        }
        sz[d] = n;
    }
    __syncthreads();
    if (d < nd) {
        const uint32_t n = sz[d];
        uint32_t r = 0;
        for (uint32_t e = 0; e < nd; e++) r += sz[e] > n || (sz[e] == n && e < d) ? 1u : 0u;
        order[r] = d;
    }
}

// The SEQ records from sorted order (rs, k_replay_seq_bkt<true>) to stream
// order: prs[p] = rs[inv[p]] in every segment, inv from the bucket pass
// (k_sort_scatter<INV>).  One workgroup per sort tile; inv read and prs written
// coalesced.  The records of one bucket are consecutive in rs, so the tiles
// near each other in the stream gather from the same lines: tile ranges go
// to the XCDs contiguously (workgroup g runs on XCD g % 8) to meet in one L2.
__global__ __launch_bounds__(SORT_THREADS) void k_seq_unpermute(const SortView sv, const uint32_t* __restrict__ inv,
                                                                const PRec* __restrict__ rs, PRec* __restrict__ prs)
{
    const uint32_t g = blockIdx.x, per = (sv.ntiles + 7) / 8;
    const uint32_t t = (g & 7) * per + (g >> 3);
    if (t >= sv.ntiles) return;
    const SortSeg& sg = sv.segs[sv.tile_seg[t]];
    const uint32_t i0 = (t - sg.tile0) * SORT_TILE;
    const uint32_t* I = inv + sg.base;
    const PRec* R = rs + sg.base;
    PRec* O = prs + sg.base;
    uint32_t q[SORT_ITEMS];
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) q[r] = I[i0 + threadIdx.x + r * SORT_THREADS];   // (pads included)
#pragma unroll
    for (int r = 0; r < SORT_ITEMS; r++) {
        const uint32_t i = i0 + threadIdx.x + r * SORT_THREADS;
        if (i < sg.count) O[i] = R[q[r]];
    }
}

// ---------------------------------------------------------------------------
// AUX model replay: SIMPLE_MODEL<N> (kModelEncode@0x42ccb0 and every inlined
// copy), one model run = the symbols of one (block, model) in stream order.
//   k_replay_aux_short: one lane per run start; runs of >= LONG_RUN symbols are
//     appended to a list instead.  Model in LDS, one RP_STRIDE region per lane.
//   k_replay_aux_long: one wave per long run.  The wave loads 64 keys/positions
//     per step coalesced; the serial model update runs on wave-uniform values
//     (scalar unit), each lane collects the record of "its" symbol with
//     writelane, and the 64 records are stored once per step.
// ---------------------------------------------------------------------------
constexpr int RP_THREADS = 64;
constexpr int RP_STRIDE = 253;   // >= 256 - RP_REG entries, odd -> conflict-free
constexpr uint32_t LONG_RUN = 512;

constexpr uint32_t HUGE_RUN = 1u << 16;   // long runs replayed first
constexpr uint32_t FIND_ITEMS = 16;        // sorted keys per thread in k_find_runs

// Run lists of the AUX space (RunLists in sa_device.h terms):
//   short: run starts (< LONG_RUN symbols), replayed one lane each;
//   long:  LongRun entries, the runs of >= HUGE_RUN symbols from the front of
//          the array, the others from the back, so that the long-run kernel
//          (a work queue) takes the longest first.
struct RunLists {
    uint64_t* short_at;
    uint32_t* n_short;
    LongRun* longs;
    uint32_t* n_huge;
    uint32_t* n_long;
    uint64_t cap_long;
    uint32_t* next;        // work-queue counter of k_replay_aux_long
    LongRun* huge_sorted;  // the huge runs, longest first (k_sort_huge)
};

// The same run lists when the AUX space was sorted by ONE dense pass (§4.2):
// the runs are then exactly the digit buckets, so their starts and lengths are
// the scan's per-segment digit bases (hist row of the segment's first tile)
// and no sorted key is read but each run's first (for its model id).  One
// thread per (segment, digit); the pad keys sort into the last digit, after
// the segment's symbols, and are cut off by the segment's count.
template <int DB>
__global__ __launch_bounds__(256) void k_runs_dense(const SortView sv, const uint32_t* __restrict__ keys,
                                                    const RunLists rl)
{
    constexpr uint32_t ND = 1u << DB;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t seg = gid / ND, d = gid % ND;
    if (seg >= sv.nsegs) return;
    const SortSeg& sg = sv.segs[seg];
    if (!sg.ntiles) return;
    const uint32_t* H = sv.hist + (size_t)sg.tile0 * ND;
    const uint32_t s = H[d];
    uint32_t e = d + 1 < ND ? H[d + 1] : sg.ntiles * SORT_TILE;
    if (e > sg.count) e = sg.count;
    if (e <= s) return;
    const size_t i = sg.base + s;
    if (e - s >= LONG_RUN) {
        const LongRun lr{i, sg.base + e, sg.base, keys[i] >> AUX_SYM_BITS, 0};
        if (e - s >= HUGE_RUN) rl.longs[atomicAdd(rl.n_huge, 1u)] = lr;
        else rl.longs[rl.cap_long - 1 - atomicAdd(rl.n_long, 1u)] = lr;
    } else {
        rl.short_at[atomicAdd(rl.n_short, 1u)] = i;
    }
}

__global__ __launch_bounds__(256) void k_find_runs(const SortView sv, const uint32_t* __restrict__ keys,
                                                   const RunLists rl)
{
    const size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * FIND_ITEMS;
    if (i0 >= sv.total) return;
    const SortSeg& sg = sv.segs[sv.tile_seg[i0 / SORT_TILE]];   // FIND_ITEMS divides SORT_TILE
    const size_t end = sg.base + sg.count;
    uint32_t k[FIND_ITEMS];
    const uint4* K4 = reinterpret_cast<const uint4*>(keys + i0);
#pragma unroll
    for (uint32_t q = 0; q < FIND_ITEMS / 4; q++) {
        const uint4 a = K4[q];
        k[4 * q] = a.x; k[4 * q + 1] = a.y; k[4 * q + 2] = a.z; k[4 * q + 3] = a.w;
    }
    uint32_t prev = i0 > sg.base ? keys[i0 - 1] >> AUX_SYM_BITS : 0xffffffffu;
#pragma unroll
    for (uint32_t e = 0; e < FIND_ITEMS; e++) {
        const size_t i = i0 + e;
        const uint32_t model = k[e] >> AUX_SYM_BITS;
        const bool start = i < end && k[e] != SORT_PAD && model != prev;
        prev = model;
        if (!start) continue;
        if (i + LONG_RUN <= end && (keys[i + LONG_RUN - 1] >> AUX_SYM_BITS) == model) {
            // run end: galloping then binary search over the sorted keys
            size_t lo = i + LONG_RUN - 1, step = LONG_RUN, hi;
            for (;;) {
                hi = lo + step;
                if (hi >= end || (keys[hi] >> AUX_SYM_BITS) != model) break;
                lo = hi;
                step *= 2;
            }
            if (hi > end) hi = end;
            while (hi - lo > 1) {   // keys[lo] in the run, hi past it (or end)
                const size_t mid = lo + (hi - lo) / 2;
                if ((keys[mid] >> AUX_SYM_BITS) == model) lo = mid;
                else hi = mid;
            }
            const LongRun lr{i, hi, sg.base, model, 0};
            if (hi - i >= HUGE_RUN) rl.longs[atomicAdd(rl.n_huge, 1u)] = lr;
            else rl.longs[rl.cap_long - 1 - atomicAdd(rl.n_long, 1u)] = lr;
        } else {
            rl.short_at[atomicAdd(rl.n_short, 1u)] = i;
        }
    }
}

// The huge runs, longest first (ties by list position), into huge_sorted: one
// workgroup, rank by counting (up to HUGE_SORT_MAX runs; beyond that the list is
// copied unsorted).
constexpr uint32_t HUGE_SORT_MAX = 4096;

__global__ __launch_bounds__(1024) void k_sort_huge(const RunLists rl)
{
    __shared__ uint32_t len[HUGE_SORT_MAX];
    const uint32_t n = *rl.n_huge;
    if (n > HUGE_SORT_MAX) {
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) rl.huge_sorted[i] = rl.longs[i];
        return;
    }
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) len[i] = (uint32_t)(rl.longs[i].end - rl.longs[i].start);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t li = len[i];
        uint32_t rank = 0;
        for (uint32_t j = 0; j < n; j++) {
            const uint32_t lj = len[j];
            rank += (lj > li || (lj == li && j < i)) ? 1u : 0u;
        }
        rl.huge_sorted[rank] = rl.longs[i];
    }
}

// Short runs: a grid of lanes strides over the list; model in LDS, one
// RP_STRIDE region per lane.
constexpr uint32_t SHORT_GRID = 1024;

__global__ __launch_bounds__(RP_THREADS) void k_replay_aux_short(const SortView sv, const uint32_t* __restrict__ keys,
                                                                 const uint32_t* __restrict__ vals,
                                                                 const SymSink rec, const RunLists rl,
                                                                 uint32_t* __restrict__ err)
{
    __shared__ uint32_t lds[RP_THREADS * RP_STRIDE];
    uint32_t* F = lds + threadIdx.x * RP_STRIDE;
    const uint32_t n = *rl.n_short;
    uint32_t e = 0;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const size_t i = rl.short_at[k];
        const SortSeg& sg = sv.segs[sv.tile_seg[i / SORT_TILE]];
        e |= replay_simple_run(keys, vals, i, sg.base + sg.count, keys[i] >> AUX_SYM_BITS,
                               SymSink{rec.prs + sg.base, rec.cum + sg.base}, F);
    }
    if (e) atomicOr(err, e);
}

// k_replay_aux_long: one wave per long model run, 64 symbols per step.
// Within a step the symbol order of the model only changes by the bubble swaps
// (every 16th update of the model) and the frequencies only by +8 per
// occurrence (a halving is made to fall on a step's last update), so for lane i
// holding symbol s_i at position p_i:
//     freq_i = F[s_i] + 8 * #{j < i : s_j = s_i}
//     cum_i  = C[s_i] + 8 * #{j < i : p_j < p_i}   (+ bubble corrections)
//     tot_i  = Tot + 8 i
// One pass over the distinct symbols of the step (one ballot each) gives the
// counts; the frequency increments are LDS atomics by position.  A bubble event
// swaps at most one adjacent pair (x ahead of y); lanes after it that hold y
// gain freq_x, lanes that hold x lose freq_y.  Only events whose symbol is not
// already in front are visited.  Model state (RunModel) lives in LDS; the
// prefix of the freqs by position is a DPP scan.

// Orders this wave's LDS accesses for the compiler only: one wave's LDS
// operations are performed in issue order, so no s_waitcnt is needed (a
// workgroup fence would also wait for the outstanding global loads and stores).
__device__ inline void lds_order() { asm volatile("" ::: "memory"); }


// LDS ring of a long run's sorted (key, value) pairs, filled ahead of the
// replaying wave by a loader wave of the same workgroup.
constexpr uint32_t RING_WIN = 32;                 // windows of 64 pairs
constexpr uint32_t RING_LEN = RING_WIN * 64;
constexpr uint32_t RING_BATCH = 8;                // windows per loader batch
struct RunRing {
    uint32_t key[RING_LEN];
    uint32_t val[RING_LEN];
    uint32_t filled;     // windows published by the loader
    uint32_t consumed;   // first window the replaying wave still needs
    uint32_t done;       // replaying wave finished
};

// Relaxed workgroup-scope atomics keep these on the LDS path (a volatile access
// through the reference becomes a flat access that waits for every outstanding
// global store), and readfirstlane tells the compiler the polled value is
// uniform (a loop exit on a "divergent" LDS load makes the whole step loop
// divergent: waterfalled, exec-masked code).
__device__ inline uint32_t lds_poll(const uint32_t* p)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ inline void lds_publish(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Loader wave: windows w = 0, 1, ... of [lr.start, lr.end) into the ring, a
// batch of RING_BATCH windows per round trip, until the batch after the one
// that leaves the run (or the block's end) is published -- the replaying wave
// reads up to 63 pairs past its position -- or the replaying wave is done.
// `shift`: a pair belongs to the run while key >> shift == lr.model.
__device__ void run_loader(const LongRun& lr, const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                           RunRing& rg, uint32_t shift)
{
    const uint32_t lane = threadIdx.x & 63;
    bool last = false;
    for (uint32_t w = 0;; w += RING_BATCH) {
        uint32_t spins = 0;
        while (w + RING_BATCH > lds_poll(&rg.consumed) + RING_WIN) {
            if (lds_poll(&rg.done) || ++spins > (1u << 24)) return;
            __builtin_amdgcn_s_sleep(2);
        }
        uint32_t k[RING_BATCH], v[RING_BATCH];
#pragma unroll
        for (uint32_t j = 0; j < RING_BATCH; j++) {
            const size_t at = lr.start + (size_t)(w + j) * 64 + lane;
            k[j] = SORT_PAD;
            v[j] = 0;
            if (at < lr.end) {
                k[j] = keys[at];
                v[j] = vals[at];
            }
        }
        bool out = false;
#pragma unroll
        for (uint32_t j = 0; j < RING_BATCH; j++) {
            const uint32_t slot = ((w + j) % RING_WIN) * 64 + lane;
            rg.key[slot] = k[j];
            rg.val[slot] = v[j];
            out |= (k[j] >> shift) != lr.model;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the windows are in LDS
        lds_order();
        if (lane == 0) lds_publish(&rg.filled, w + RING_BATCH);
        if (last) return;
        last = __ballot(out) != 0;
    }
}

#ifdef SA_PROF   // scripts/micro/replay_long.hip: per-section cycle counts of one run
__device__ unsigned long long g_prof[8];
#define PROF_T(i) const uint64_t pt##i = __builtin_amdgcn_s_memtime()
#define PROF_ACC(k, a, b) acc[k] += pt##b - pt##a
#else
#define PROF_T(i)
#define PROF_ACC(k, a, b)
#endif

// The model state of one long run, in LDS (N <= 256 entries).
struct RunModel {
    uint32_t ent[256];    // symbol at position
    uint32_t posr[256];   // position of symbol
    uint32_t fpos[256];   // freq of the entry at position
    uint32_t cpos[256];   // exclusive prefix of fpos
};

__device__ inline uint32_t uread(const uint32_t* p)   // wave-uniform LDS read
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)*p);
}

__device__ inline uint32_t bytesum(uint32_t x) { return (x * 0x01010101u) >> 24; }   // sum < 256
__device__ inline uint32_t bytes_below(uint32_t k) { return k ? 0xffffffffu >> (32 - 8 * k) : 0u; }   // k < 4

// counts by position q < 8 packed one byte each in (lo, hi)
__device__ inline uint32_t pos_count(uint32_t lo, uint32_t hi, uint32_t q)
{
    return q < 8 ? ((q < 4 ? lo : hi) >> (8 * (q & 3))) & 0xffu : 0u;
}
__device__ inline uint32_t pos_below(uint32_t lo, uint32_t hi, uint32_t q)   // sum of the counts below q < 8
{
    const uint32_t bm = bytes_below(q & 3);
    return q < 4 ? bytesum(lo & bm) : bytesum(lo) + bytesum(hi & bm);
}

// One long SIMPLE_MODEL run, 64 symbols per step (see above).  Fast steps --
// every symbol of the step at a position < 8, no bubble swap, no halving --
// run on registers: the counts by position are packed bytes scanned over the
// wave, the freqs and prefixes of positions < 8 live in lanes 0..7 (f8, c8;
// written through to LDS), the prefixes of positions >= 8 are stored without
// cadd, and the end-of-step bubble event is checked on registers.  Other steps
// take the general path.
template <int NR>
__device__ __forceinline__ void replay_long_run(const LongRun& lr, const SymSink& rec, uint32_t* __restrict__ err,
                                                RunModel& md, RunRing& rg)
{
#ifdef SA_PROF
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    const uint32_t lane = threadIdx.x;
    const uint32_t N = model_nsym(lr.model);
#pragma unroll
    for (int j = 0; j < NR; j++) {
        const uint32_t k = 64u * j + lane;
        md.ent[k] = k;
        md.posr[k] = k;
        md.fpos[k] = k < N ? 1u : 0u;
        md.cpos[k] = k < N ? k : N;
    }
    lds_order();
    uint32_t f8 = lane < 8 ? md.fpos[lane] : 0u, c8 = lane < 8 ? md.cpos[lane] : 0u;
    uint32_t tot = N, bub = 0, cadd = 0;
    bool bad = false;
    size_t base = lr.start;
    uint32_t avail = 0;                                          // windows known published
    uint32_t nxt_rel = 0xffffffffu, nxt_key = 0, nxt_pos = 0;   // next window, read ahead
    uint32_t tlo = 0, thi = 0;   // the step's counts by position (fast steps)
    auto swap_at = [&](uint32_t P, uint32_t x, uint32_t y) __attribute__((always_inline)) {
        // x at P moves ahead of y at P - 1 (the freqs travel with the symbols)
        if (lane == 0) {
            const uint32_t fx = md.fpos[P], fy = md.fpos[P - 1];
            md.ent[P - 1] = x;
            md.ent[P] = y;
            md.fpos[P - 1] = fx;
            md.fpos[P] = fy;
            md.posr[x] = P - 1;
            md.posr[y] = P;
        }
        lds_order();
    };
    for (;;) {
        PROF_T(0);
        const uint32_t rel = (uint32_t)(base - lr.start);
        const uint32_t need = (rel + 63) / 64 + 1;   // windows that must be published
        if (avail < need) {
            uint32_t spins = 0;   // bounded: a stalled loader fails the batch instead of hanging
            while ((avail = lds_poll(&rg.filled)) < need && ++spins < (1u << 24)) __builtin_amdgcn_s_sleep(1);
            if (spins >= (1u << 24)) {
                bad = true;
                break;
            }
            lds_order();
            nxt_rel = 0xffffffffu;
        }
        PROF_T(1);
        uint32_t key, pos;
        if (nxt_rel == rel) {
            key = nxt_key;
            pos = nxt_pos;
        } else {
            const uint32_t slot = (rel + lane) % RING_LEN;
            key = rg.key[slot];
            pos = rg.val[slot];
        }
        // read the following window ahead when it is published (a step takes 64
        // symbols except at a halving cut)
        nxt_rel = 0xffffffffu;
        if ((rel + 127) / 64 < avail) {
            const uint32_t slot = (rel + 64 + lane) % RING_LEN;
            nxt_key = rg.key[slot];
            nxt_pos = rg.val[slot];
            nxt_rel = rel + 64;
        }
        const bool in_run = (key >> AUX_SYM_BITS) == lr.model;
        // symbols of the run in this window: the leading in-run lanes
        const uint64_t outm = ~__ballot(in_run);
        uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane(outm ? (int)__builtin_ctzll(outm) : 64);
        if (c == 0) break;
        tot = (uint32_t)__builtin_amdgcn_readfirstlane((int)tot);
        const uint32_t to_halve = (0xffe0u - tot) / 8u + 1u;
        bool halve = false;
        if (to_halve <= c) {   // cut the step so that a halving falls on its last update
            c = to_halve;
            halve = true;
        }
        const bool act = lane < c;
        const uint64_t amask = c == 64 ? ~0ull : ((1ull << c) - 1ull);
        const uint32_t sym = act ? (key & 0xffu) : 0u;
        if (act && sym >= N) bad = true;
        uint32_t p = md.posr[sym];
        const uint32_t f0 = md.fpos[p], c0 = md.cpos[p] + (p >= 8 ? cadd : 0u);
        uint32_t fprev = p ? md.fpos[p - 1] : 0u;
        // Counts.  Fast: every symbol of the step sits at a position < 8 -- one
        // byte counter per position, packed 4 to a dword, scanned over the wave.
        // Otherwise one ballot per distinct symbol of the step.
        const uint64_t hi8 = __ballot(act && p >= 8);
        uint32_t same = 0, less = 0, inlo = 0, inhi = 0;
        if (!hi8) {
            const uint32_t ohlo = act && p < 4 ? 1u << (8 * p) : 0u;
            const uint32_t ohhi = act && p >= 4 ? 1u << (8 * (p - 4)) : 0u;
            inlo = wave_incl_scan_dpp(ohlo);
            inhi = wave_incl_scan_dpp(ohhi);
            const uint32_t exlo = inlo - ohlo, exhi = inhi - ohhi;
            same = pos_count(exlo, exhi, p);
            less = pos_below(exlo, exhi, p);
        } else {
            uint64_t rem = amask;
            while (rem) {
                const int fl = (int)__builtin_ctzll(rem);
                const uint32_t x = __builtin_amdgcn_readlane(sym, fl), px = __builtin_amdgcn_readlane(p, fl);
                const uint64_t m = __ballot(act && sym == x);
                const uint32_t below = lanes_below(m);
                if (sym == x) same = below;
                less += px < p ? below : 0u;
                rem &= ~m;
            }
        }
        int32_t cum = (int32_t)(c0 + 8u * less);
        PROF_T(2);
        // bubble events inside the step whose symbol is not in front
        // updates b0, b0 + 16, ... before the last one (that one comes after the
        // state update)
        const uint32_t b0 = 15u - (bub & 15u);
        const uint64_t emask = (0x0001000100010001ull << b0) & ((1ull << (c - 1)) - 1ull);
        uint64_t cand = __ballot(p != 0) & emask;
        bool swapped = false;
        if (cand && !hi8) {
            // fast check of every event against the step-start order: x (this
            // lane's symbol) after its update vs y (position p - 1) at that time
            const bool sw = p != 0 && f0 + 8u * (same + 1u) > fprev + 8u * pos_count(inlo, inhi, p - 1u);
            if (!(__ballot(sw) & cand)) cand = 0;
        }
        // (LDS fpos holds the step-start freqs until the increments below; the
        // per-lane copies p / fprev / yprev are refreshed after a swap)
        uint32_t yprev = 0;
        if (cand) yprev = p ? md.ent[p - 1] : 0u;
        while (cand) {
            const uint32_t b = (uint32_t)__builtin_ctzll(cand);
            cand &= cand - 1;
            const uint32_t x = __builtin_amdgcn_readlane(sym, (int)b);
            const uint32_t P = __builtin_amdgcn_readlane(p, (int)b);
            const uint32_t y = __builtin_amdgcn_readlane(yprev, (int)b);
            const uint32_t fx0 = __builtin_amdgcn_readlane(f0, (int)b), fy0 = __builtin_amdgcn_readlane(fprev, (int)b);
            const uint64_t upto = (2ull << b) - 1ull;
            const uint64_t mx = __ballot(act && sym == x), my = __ballot(act && sym == y);
            if (fx0 + 8u * (uint32_t)__popcll(mx & upto) > fy0 + 8u * (uint32_t)__popcll(my & upto)) {
                swap_at(P, x, y);
                swapped = true;
                if (lane > b) {
                    const uint32_t bx = lanes_below(mx), by = lanes_below(my);
                    if (sym == y) cum += (int32_t)(fx0 + 8u * bx);
                    else if (sym == x) cum -= (int32_t)(fy0 + 8u * by);
                }
                p = md.posr[sym];
                fprev = p ? md.fpos[p - 1] : 0u;
                yprev = p ? md.ent[p - 1] : 0u;
                cand = __ballot(p != 0) & emask & ~upto;
            }
        }
        PROF_T(3);
        if (act) {
            const uint32_t f = f0 + 8u * same;
            const uint32_t t = tot + 8u * lane;
            if (cum < 0 || (uint32_t)cum + f > t || f == 0) bad = true;
            rec.prs[pos] = PRec{t | (f << 16)};
            rec.cum[pos] = (uint16_t)cum;
        }
        PROF_T(4);
        // frequency increments: fast steps from the position counts (the prefixes
        // of positions >= 8 via cadd), else at the symbols' current positions with
        // a full prefix recompute below
        bool full = hi8 || swapped;
        if (!full) {
            tlo = __builtin_amdgcn_readlane(inlo, (int)(c - 1));
            thi = __builtin_amdgcn_readlane(inhi, (int)(c - 1));
            if (lane < 8) {
                f8 += 8u * pos_count(tlo, thi, lane);
                c8 += 8u * pos_below(tlo, thi, lane);
                md.fpos[lane] = f8;
                md.cpos[lane] = c8;
            }
            cadd += 8u * c;
        } else if (act) {
            __hip_atomic_fetch_add(&md.fpos[p], 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        lds_order();
        tot += 8u * c;
        bub += c;
        if (halve) {
            uint32_t part = 0;
#pragma unroll
            for (int j = 0; j < NR; j++) {
                const uint32_t v = md.fpos[64u * j + lane];
                md.fpos[64u * j + lane] = v - (v >> 1);
                part += v - (v >> 1);
            }
            tot = __builtin_amdgcn_readlane(wave_incl_scan_dpp(part), 63);
            lds_order();
            full = true;
        }
        if ((bub & 15u) == 0) {   // the step's last update was a bubble event
            const uint32_t x = __builtin_amdgcn_readlane(sym, (int)(c - 1));
            if (!full) {   // from registers: x after the step vs y after the step
                const uint32_t P = __builtin_amdgcn_readlane(p, (int)(c - 1));
                const uint32_t fx = __builtin_amdgcn_readlane(f0 + 8u * (same + 1u), (int)(c - 1));
                const uint32_t fy = __builtin_amdgcn_readlane(fprev, (int)(c - 1)) + 8u * pos_count(tlo, thi, P - 1u);
                if (P > 0 && fx > fy) {
                    swap_at(P, x, uread(&md.ent[P - 1]));
                    full = true;
                }
            } else {
                const uint32_t P = uread(&md.posr[x]);
                if (P > 0 && uread(&md.fpos[P]) > uread(&md.fpos[P - 1])) swap_at(P, x, uread(&md.ent[P - 1]));
            }
        }
        if (full) {   // prefix of the freqs by position
            uint32_t carry = 0;
#pragma unroll
            for (int j = 0; j < NR; j++) {
                const uint32_t fv = md.fpos[64u * j + lane];
                const uint32_t inc = wave_incl_scan_dpp(fv);
                md.cpos[64u * j + lane] = carry + inc - fv;
                carry += __builtin_amdgcn_readlane(inc, 63);
            }
            lds_order();
            cadd = 0;
            f8 = lane < 8 ? md.fpos[lane] : 0u;
            c8 = lane < 8 ? md.cpos[lane] : 0u;
        }
        base += c;
        if (lane == 0) lds_publish(&rg.consumed, (uint32_t)(base - lr.start) / 64);
        lds_order();
        PROF_T(5);
        PROF_ACC(0, 0, 1);
        PROF_ACC(1, 1, 2);
        PROF_ACC(2, 2, 3);
        PROF_ACC(3, 3, 4);
        PROF_ACC(4, 4, 5);
    }
    if (lane == 0) lds_publish(&rg.done, 1u);
    if (__ballot(bad) && lane == 0) atomicOr(err, (uint32_t)E_CODER);
#ifdef SA_PROF
    if (lane == 0 && blockIdx.x == 0)
        for (int k = 0; k < 5; k++) g_prof[k] = acc[k];
#endif
}

// Workgroups of two waves (wave 0 replays, wave 1 loads) take long runs from
// a work queue, the runs of >= HUGE_RUN symbols first.
// (k_replay_aux_long's grid is sized to what its CUs hold at once -- sa_engine
// long_grid: it is a work queue, and workgroups beyond that waited for slots
// until the queue was empty, holding up the kernels queued behind the launch
// on its hardware queue: 100-200 ms stalls of single front kernels, round 3)

__global__ __launch_bounds__(128) void k_replay_aux_long(const RunLists rl, const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ vals, const SymSink rec_all,
                                                         uint32_t* __restrict__ err, uint32_t prio)
{
    set_chain_prio(prio);
    __shared__ RunModel md;
    __shared__ RunRing rg;
    __shared__ uint32_t job;
    const uint32_t nh = *rl.n_huge, n = nh + *rl.n_long;
    for (;;) {
        if (threadIdx.x == 0) {
            job = atomicAdd(rl.next, 1u);
            rg.filled = 0;
            rg.consumed = 0;
            rg.done = 0;
        }
        __syncthreads();
        const uint32_t r = job;
        if (r >= n) break;
        const LongRun lr = r < nh ? rl.huge_sorted[r] : rl.longs[rl.cap_long - 1 - (r - nh)];
        if (threadIdx.x >= 64) {
            run_loader(lr, keys, vals, rg, AUX_SYM_BITS);
        } else {
            const SymSink rec{rec_all.prs + lr.rec_base, rec_all.cum + lr.rec_base};
            const uint32_t N = model_nsym(lr.model);
            if (N <= 64) replay_long_run<1>(lr, rec, err, md, rg);
            else if (N <= 128) replay_long_run<2>(lr, rec, err, md, rg);
            else replay_long_run<4>(lr, rec, err, md, rg);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// k_replay_seq_long: BASE_MODEL context runs that reach the first halving
// (queued by k_replay_seq), one wave per run, 64 symbols per step.  Within a
// step the four counts only grow by one per occurrence, so lane i's counts are
// the step-start counts plus the occurrences in lanes below it (one ballot per
// base).  A step is cut so that it ends right before the symbol whose total
// exceeds 253 (that symbol halves first, at the start of the next step).  Only
// the in-run indices >= SEQ_HALVE_J are written (k_replay_seq wrote the rest).
// ---------------------------------------------------------------------------
__device__ void replay_seq_long_run(const LongRun& lr, const SymSink& rec, RunRing& rg, bool& bad, uint32_t sh)
{
    const uint32_t lane = threadIdx.x;
    uint32_t c0 = 3, c1 = 3, c2 = 3, c3 = 3;   // wave-uniform model state
    size_t base = lr.start;
    uint32_t avail = 0;
    for (;;) {
        const uint32_t rel = (uint32_t)(base - lr.start);
        const uint32_t need = (rel + 63) / 64 + 1;   // windows that must be published
        if (avail < need) {
            uint32_t spins = 0;   // bounded: a stalled loader fails the batch instead of hanging
            while ((avail = lds_poll(&rg.filled)) < need && ++spins < (1u << 24)) __builtin_amdgcn_s_sleep(1);
            if (spins >= (1u << 24)) {
                bad = true;
                break;
            }
            lds_order();
        }
        const uint32_t slot = (rel + lane) % RING_LEN;
        const uint32_t key = rg.key[slot], val = rg.val[slot];
        const uint64_t outm = ~__ballot((key >> sh) == lr.model);
        uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane(outm ? (int)__builtin_ctzll(outm) : 64);
        if (c == 0) break;
        uint32_t T = c0 + c1 + c2 + c3;
        if (T > 253u) {
            c0 -= c0 >> 1;
            c1 -= c1 >> 1;
            c2 -= c2 >> 1;
            c3 -= c3 >> 1;
            T = c0 + c1 + c2 + c3;
        }
        if (c > 254u - T) c = 254u - T;
        const bool act = lane < c;
        const uint32_t b = (sh ? key : val) & 3u;
        const uint64_t m0 = __ballot(act && b == 0), m1 = __ballot(act && b == 1), m2 = __ballot(act && b == 2),
                       m3 = __ballot(act && b == 3);
        const uint32_t n0 = c0 + lanes_below(m0), n1 = c1 + lanes_below(m1), n2 = c2 + lanes_below(m2),
                       n3 = c3 + lanes_below(m3);
        if (act && rel + lane >= SEQ_HALVE_J) {
            const uint32_t cum = (b > 0 ? n0 : 0u) + (b > 1 ? n1 : 0u) + (b > 2 ? n2 : 0u);
            const uint32_t f = b == 0 ? n0 : b == 1 ? n1 : b == 2 ? n2 : n3;
            sink_put(rec, sh ? val : val >> 2, cum, f, T + lane);
        }
        c0 += (uint32_t)__popcll(m0);
        c1 += (uint32_t)__popcll(m1);
        c2 += (uint32_t)__popcll(m2);
        c3 += (uint32_t)__popcll(m3);
        base += c;
        if (lane == 0) lds_publish(&rg.consumed, (uint32_t)(base - lr.start) / 64);
        lds_order();
    }
    if (lane == 0) lds_publish(&rg.done, 1u);
}

// A grid of workgroups (wave 0 replays, wave 1 loads) strides over the queued
// runs (the count is only known on the device).
__global__ __launch_bounds__(128) void k_replay_seq_long(const SortView sv, const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ vals, const SymSink rec_all,
                                                         const uint64_t* __restrict__ long_runs,
                                                         const uint32_t* __restrict__ nlong,
                                                         uint32_t* __restrict__ err, const uint32_t sh)
{
    __shared__ RunRing rg;
    const uint32_t n = *nlong;
    bool bad = false;
    for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
        const size_t i = long_runs[r];
        const SortSeg& sg = sv.segs[sv.tile_seg[i / SORT_TILE]];
        const LongRun lr{i, sg.base + sg.count, sg.base, keys[i] >> sh, 0};
        if (threadIdx.x == 0) {
            rg.filled = 0;
            rg.consumed = 0;
            rg.done = 0;
        }
        __syncthreads();
        if (threadIdx.x >= 64) run_loader(lr, keys, vals, rg, sh);
        else replay_seq_long_run(lr, SymSink{rec_all.prs + sg.base, nullptr}, rg, bad, sh);
        __syncthreads();
    }
    if (threadIdx.x < 64 && __ballot(bad) && threadIdx.x == 0) atomicOr(err, (uint32_t)E_CODER);
}

// ---------------------------------------------------------------------------
// Range coder, decomposed (sa_logic.h "decomposed range coder").
//
// k_coder_rv: pass R, one wave per stream.  The range chain runs on the scalar
// unit (a hand-scheduled 10-instruction SALU step per symbol); the records are
// fed to it through VGPRs (below).  One range checkpoint per segment is
// collected in a VGPR (lane = segment mod 64) and stored 64 at a time.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void rc_range_salu(uint32_t& r, uint32_t m, uint32_t tf, uint32_t tmask)
{
    uint32_t t, f, q, p;
    asm volatile(
        "s_and_b32 %1, %5, %7\n\t"
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
        : "s"(tf), "s"(m), "s"(tmask)
        : "scc");
}

// Pass R may start before the model replays have written every record (the
// long runs are replayed concurrently): the record arrays are zeroed first, a
// written record has tot >= 1, and an unwritten one (tot = 0, m = 0) sends the
// range to 0, where it stays -- a range chain never reaches 0 otherwise
// (q >= 1, f >= 1).  So a segment that ends with r == 0 is re-coded from its
// start once its records are in, read through L2.
// (round 5) The wait is bounded in time, on the constant 100 MHz clock:
// `wait_ticks` per segment, and after one timeout the wave waits no more -- a
// long-run kernel that never ran (tests/test_gpu_parity.py::
// test_pass_r_starved_long_runs) ends the batch with E_CODER in about that
// time, not after 2^22 polls for every segment it left unwritten.
__device__ uint32_t seg_retry(const PRec* __restrict__ P, uint32_t r0, uint32_t tmask, uint32_t& bad,
                              uint32_t wait_ticks)
{
    const uint32_t lane = threadIdx.x & 63;
    if (bad) return r0;
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + (wait_ticks ? wait_ticks : 2000000000u);
    for (;;) {
        const uint32_t tf = __hip_atomic_load(reinterpret_cast<const uint32_t*>(P + lane), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t m = recip32z(tf & tmask);
        uint32_t r = r0;
#pragma unroll 8
        for (int k = 0; k < 64; k++)
            rc_range_salu(r, __builtin_amdgcn_readlane(m, k), __builtin_amdgcn_readlane(tf, k), tmask);
        if (r != 0) return r;
        if (__builtin_amdgcn_s_memrealtime() > t_end) break;
        __builtin_amdgcn_s_sleep(32);
    }
    bad = 1;
    return r0;
}

// Chains are listed longest first, in workgroups of `coder_waves` (1, 2 or 4)
// waves.  Chain placement is what the hardware dispatcher makes of it; two
// knobs steer it: waves per workgroup (the waves of a workgroup share a CU, one
// per SIMD) and unused dynamic LDS per workgroup (`coder_lds`, limiting pass-R
// workgroups per CU).  Two chains on one SIMD run at half speed each (DESIGN.md
// section 4.4).
constexpr uint32_t CODER_MAX_WAVES = 4;

// Records through VGPRs: one lane-parallel global load per 64-record segment,
// CODER_LA segments ahead of the chain (vector loads return in order, so the
// compiler's counted vmcnt waits keep all of them in flight); each lane derives
// its record's reciprocal, and per symbol two v_readlane move m and tf into the
// SGPRs of the SALU step.  (A scalar-load variant -- s_load chunks of 16
// records -- can keep only one chunk in flight, since SMEM returns out of order,
// and needed an L2 touch-prefetch that other batches' traffic evicts; DESIGN.md
// section 4.4.)
constexpr uint32_t CODER_LA = 6;

// Eight steps of the chain per asm block.  Each step reads the record of the
// step after it out of its lanes first (readlane -> SGPR; used one step later,
// so the SALU never waits on it): reciprocal, total and frequency, split per
// segment in the VALU (11 instructions a step; with the record read whole and
// split in the SALU, 12); two register triples alternate, so there are no
// copies.  (One block per step made the compiler put an s_nop between the
// blocks: a ninth of the issue slots.)
#define SA_RV_STEP8 \
        "v_readlane_b32 %[mb], %[cm], %[l0]\n\t" \
        "v_readlane_b32 %[tb], %[vt], %[l0]\n\t" \
        "v_readlane_b32 %[fb], %[vf], %[l0]\n\t" \
        "s_mul_hi_u32 %[q], %[r], %[ma]\n\t" \
        "s_mul_i32 %[p], %[q], %[ta]\n\t" \
        "s_cmp_lt_u32 %[r], %[p]\n\t" \
        "s_subb_u32 %[q], %[q], 0\n\t" \
        "s_mul_i32 %[q], %[q], %[fa]\n\t" \
        "s_flbit_i32_b32 %[p], %[q]\n\t" \
        "s_and_b32 %[p], %[p], 24\n\t" \
        "s_lshl_b32 %[r], %[q], %[p]\n\t" \
        "v_readlane_b32 %[ma], %[cm], %[l1]\n\t" \
        "v_readlane_b32 %[ta], %[vt], %[l1]\n\t" \
        "v_readlane_b32 %[fa], %[vf], %[l1]\n\t" \
        "s_mul_hi_u32 %[q], %[r], %[mb]\n\t" \
        "s_mul_i32 %[p], %[q], %[tb]\n\t" \
        "s_cmp_lt_u32 %[r], %[p]\n\t" \
        "s_subb_u32 %[q], %[q], 0\n\t" \
        "s_mul_i32 %[q], %[q], %[fb]\n\t" \
        "s_flbit_i32_b32 %[p], %[q]\n\t" \
        "s_and_b32 %[p], %[p], 24\n\t" \
        "s_lshl_b32 %[r], %[q], %[p]\n\t" \
        "v_readlane_b32 %[mb], %[cm], %[l2]\n\t" \
        "v_readlane_b32 %[tb], %[vt], %[l2]\n\t" \
        "v_readlane_b32 %[fb], %[vf], %[l2]\n\t" \
        "s_mul_hi_u32 %[q], %[r], %[ma]\n\t" \
        "s_mul_i32 %[p], %[q], %[ta]\n\t" \
        "s_cmp_lt_u32 %[r], %[p]\n\t" \
        "s_subb_u32 %[q], %[q], 0\n\t" \
        "s_mul_i32 %[q], %[q], %[fa]\n\t" \
        "s_flbit_i32_b32 %[p], %[q]\n\t" \
        "s_and_b32 %[p], %[p], 24\n\t" \
        "s_lshl_b32 %[r], %[q], %[p]\n\t" \
        "v_readlane_b32 %[ma], %[cm], %[l3]\n\t" \
        "v_readlane_b32 %[ta], %[vt], %[l3]\n\t" \
        "v_readlane_b32 %[fa], %[vf], %[l3]\n\t" \
        "s_mul_hi_u32 %[q], %[r], %[mb]\n\t" \
        "s_mul_i32 %[p], %[q], %[tb]\n\t" \
        "s_cmp_lt_u32 %[r], %[p]\n\t" \
        "s_subb_u32 %[q], %[q], 0\n\t" \
        "s_mul_i32 %[q], %[q], %[fb]\n\t" \
        "s_flbit_i32_b32 %[p], %[q]\n\t" \
        "s_and_b32 %[p], %[p], 24\n\t" \
        "s_lshl_b32 %[r], %[q], %[p]\n\t" \
        "v_readlane_b32 %[mb], %[cm], %[l4]\n\t" \
        "v_readlane_b32 %[tb], %[vt], %[l4]\n\t" \
        "v_readlane_b32 %[fb], %[vf], %[l4]\n\t" \
        "s_mul_hi_u32 %[q], %[r], %[ma]\n\t" \
        "s_mul_i32 %[p], %[q], %[ta]\n\t" \
        "s_cmp_lt_u32 %[r], %[p]\n\t" \
        "s_subb_u32 %[q], %[q], 0\n\t" \
        "s_mul_i32 %[q], %[q], %[fa]\n\t" \
        "s_flbit_i32_b32 %[p], %[q]\n\t" \
        "s_and_b32 %[p], %[p], 24\n\t" \
        "s_lshl_b32 %[r], %[q], %[p]\n\t" \
        "v_readlane_b32 %[ma], %[cm], %[l5]\n\t" \
        "v_readlane_b32 %[ta], %[vt], %[l5]\n\t" \
        "v_readlane_b32 %[fa], %[vf], %[l5]\n\t" \
        "s_mul_hi_u32 %[q], %[r], %[mb]\n\t" \
        "s_mul_i32 %[p], %[q], %[tb]\n\t" \
        "s_cmp_lt_u32 %[r], %[p]\n\t" \
        "s_subb_u32 %[q], %[q], 0\n\t" \
        "s_mul_i32 %[q], %[q], %[fb]\n\t" \
        "s_flbit_i32_b32 %[p], %[q]\n\t" \
        "s_and_b32 %[p], %[p], 24\n\t" \
        "s_lshl_b32 %[r], %[q], %[p]\n\t" \
        "v_readlane_b32 %[mb], %[cm], %[l6]\n\t" \
        "v_readlane_b32 %[tb], %[vt], %[l6]\n\t" \
        "v_readlane_b32 %[fb], %[vf], %[l6]\n\t" \
        "s_mul_hi_u32 %[q], %[r], %[ma]\n\t" \
        "s_mul_i32 %[p], %[q], %[ta]\n\t" \
        "s_cmp_lt_u32 %[r], %[p]\n\t" \
        "s_subb_u32 %[q], %[q], 0\n\t" \
        "s_mul_i32 %[q], %[q], %[fa]\n\t" \
        "s_flbit_i32_b32 %[p], %[q]\n\t" \
        "s_and_b32 %[p], %[p], 24\n\t" \
        "s_lshl_b32 %[r], %[q], %[p]\n\t" \
        "v_readlane_b32 %[ma], %[cm], %[l7]\n\t" \
        "v_readlane_b32 %[ta], %[vt], %[l7]\n\t" \
        "v_readlane_b32 %[fa], %[vf], %[l7]\n\t" \
        "s_mul_hi_u32 %[q], %[r], %[mb]\n\t" \
        "s_mul_i32 %[p], %[q], %[tb]\n\t" \
        "s_cmp_lt_u32 %[r], %[p]\n\t" \
        "s_subb_u32 %[q], %[q], 0\n\t" \
        "s_mul_i32 %[q], %[q], %[fb]\n\t" \
        "s_flbit_i32_b32 %[p], %[q]\n\t" \
        "s_and_b32 %[p], %[p], 24\n\t" \
        "s_lshl_b32 %[r], %[q], %[p]\n\t" \
        ""

// (A/B, SA_RV_VARIANT=5) the eight steps' 24 v_readlane issued together ahead
// of their 64 SALU instructions: one switch from the vector to the scalar unit
// per eight steps instead of one per step.
#define SA_RV_RL(k)                                                                                           \
    "v_readlane_b32 %[m" #k "], %[cm], %[l" #k "]\n\tv_readlane_b32 %[t" #k "], %[vt], %[l" #k "]\n\t" \
    "v_readlane_b32 %[f" #k "], %[vf], %[l" #k "]\n\t"
#define SA_RV_ST(k)                                                                                           \
    "s_mul_hi_u32 %[q], %[r], %[m" #k "]\n\ts_mul_i32 %[p], %[q], %[t" #k "]\n\ts_cmp_lt_u32 %[r], %[p]\n\t"   \
    "s_subb_u32 %[q], %[q], 0\n\ts_mul_i32 %[q], %[q], %[f" #k "]\n\ts_flbit_i32_b32 %[p], %[q]\n\t"           \
    "s_and_b32 %[p], %[p], 24\n\ts_lshl_b32 %[r], %[q], %[p]\n\t"

template <int J>
__device__ __forceinline__ void rv_step8_batched(uint32_t& r, uint32_t cm, uint32_t vt, uint32_t vf)
{
    uint32_t q, p, m0, m1, m2, m3, m4, m5, m6, m7, t0, t1, t2, t3, t4, t5, t6, t7, f0, f1, f2, f3, f4, f5, f6, f7;
    asm volatile(SA_RV_RL(0) SA_RV_RL(1) SA_RV_RL(2) SA_RV_RL(3) SA_RV_RL(4) SA_RV_RL(5) SA_RV_RL(6) SA_RV_RL(7)
                 SA_RV_ST(0) SA_RV_ST(1) SA_RV_ST(2) SA_RV_ST(3) SA_RV_ST(4) SA_RV_ST(5) SA_RV_ST(6) SA_RV_ST(7)
                 : [r] "+s"(r), [q] "=&s"(q), [p] "=&s"(p), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2),
                   [m3] "=&s"(m3), [m4] "=&s"(m4), [m5] "=&s"(m5), [m6] "=&s"(m6), [m7] "=&s"(m7), [t0] "=&s"(t0),
                   [t1] "=&s"(t1), [t2] "=&s"(t2), [t3] "=&s"(t3), [t4] "=&s"(t4), [t5] "=&s"(t5), [t6] "=&s"(t6),
                   [t7] "=&s"(t7), [f0] "=&s"(f0), [f1] "=&s"(f1), [f2] "=&s"(f2), [f3] "=&s"(f3), [f4] "=&s"(f4),
                   [f5] "=&s"(f5), [f6] "=&s"(f6), [f7] "=&s"(f7)
                 : [cm] "v"(cm), [vt] "v"(vt), [vf] "v"(vf), [l0] "i"(J), [l1] "i"(J + 1), [l2] "i"(J + 2),
                   [l3] "i"(J + 3), [l4] "i"(J + 4), [l5] "i"(J + 5), [l6] "i"(J + 6), [l7] "i"(J + 7)
                 : "scc");
}
#undef SA_RV_RL
#undef SA_RV_ST

template <int J>
__device__ __forceinline__ void rv_step8(uint32_t& r, uint32_t& ma, uint32_t& ta, uint32_t& fa, uint32_t& mb,
                                         uint32_t& tb, uint32_t& fb, uint32_t cm, uint32_t vt, uint32_t vf)
{
    uint32_t q, p;
#define SA_RV_OPERANDS                                                                                            \
    : [r] "+s"(r), [ma] "+s"(ma), [ta] "+s"(ta), [fa] "+s"(fa), [mb] "+s"(mb), [tb] "+s"(tb), [fb] "+s"(fb),     \
      [q] "=&s"(q), [p] "=&s"(p)                                                                                  \
    : [cm] "v"(cm), [vt] "v"(vt), [vf] "v"(vf), [l0] "i"((J + 1) & 63), [l1] "i"((J + 2) & 63),                  \
      [l2] "i"((J + 3) & 63), [l3] "i"((J + 4) & 63), [l4] "i"((J + 5) & 63), [l5] "i"((J + 6) & 63),             \
      [l6] "i"((J + 7) & 63), [l7] "i"((J + 8) & 63)                                                             \
    : "scc"
    asm volatile(SA_RV_STEP8 SA_RV_OPERANDS);
#undef SA_RV_OPERANDS
}
#undef SA_RV_STEP8

// the 64 steps of one segment (records in lanes 0..63 of cm / ctf)
template <int V, int... P>
__device__ __forceinline__ void rv_segment(uint32_t& r, uint32_t cm, uint32_t vt, uint32_t vf,
                                           std::integer_sequence<int, P...>)
{
    if constexpr (V == 5) {
        (rv_step8_batched<8 * P>(r, cm, vt, vf), ...);
    } else {
        uint32_t ma = __builtin_amdgcn_readlane(cm, 0), ta = __builtin_amdgcn_readlane(vt, 0),
                 fa = __builtin_amdgcn_readlane(vf, 0), mb = 0, tb = 0, fb = 0;
        (rv_step8<8 * P>(r, ma, ta, fa, mb, tb, fb, cm, vt, vf), ...);
    }
}

// ---------------------------------------------------------------------------
// (round 6) V = 6: the operands reach the scalar unit through SMEM instead of
// v_readlane.  The lanes derive (m, tf) of segment g+2 from its records and
// store them to the wave's ring in global memory (4 segment slots, 2 KiB); the
// chain reads 16 symbols' pairs per group with two s_load_dwordx16 (glc: the
// scalar cache does not see the vector stores), the next group's loads issued
// at the start of the current group's steps, so a load has one group's steps
// (~700 cycles) to return (SMEM returns out of order: every wait is
// lgkmcnt(0)).  Per symbol the scalar unit issues the step's eight
// instructions plus the split of tf into t and f: 10 SALU and 1/8 of a load
// against 8 SALU and three v_readlane (scripts/micro/feed_probe.hip, r6a: 44-45
// against 50-63 cycles per symbol; the step alone 39).  The two buffers live
// at fixed SGPRs (A = s[36:67], B = s[68:99]); no code between the groups uses
// them (tests/test_isa.py checks the compiled kernel).
constexpr uint32_t RING_SLOT = 2 * SEG_SYMS;   // dwords per segment slot
constexpr uint32_t RING_DW = 4 * RING_SLOT;    // dwords per wave

#define SA_RG_STEP(M, TF)                                                                                     \
    "s_and_b32 %[t], " TF ", %[mk]\n\ts_lshr_b32 %[f], " TF ", 16\n\ts_mul_hi_u32 %[q], %[r], " M "\n\t"      \
    "s_mul_i32 %[p], %[q], %[t]\n\ts_cmp_lt_u32 %[r], %[p]\n\ts_subb_u32 %[q], %[q], 0\n\t"                    \
    "s_mul_i32 %[q], %[q], %[f]\n\ts_flbit_i32_b32 %[p], %[q]\n\ts_and_b32 %[p], %[p], 24\n\t"                 \
    "s_lshl_b32 %[r], %[q], %[p]\n\t"
#define SA_RG_A                                                                                               \
    SA_RG_STEP("s36", "s37") SA_RG_STEP("s38", "s39") SA_RG_STEP("s40", "s41") SA_RG_STEP("s42", "s43")         \
    SA_RG_STEP("s44", "s45") SA_RG_STEP("s46", "s47") SA_RG_STEP("s48", "s49") SA_RG_STEP("s50", "s51")         \
    SA_RG_STEP("s52", "s53") SA_RG_STEP("s54", "s55") SA_RG_STEP("s56", "s57") SA_RG_STEP("s58", "s59")         \
    SA_RG_STEP("s60", "s61") SA_RG_STEP("s62", "s63") SA_RG_STEP("s64", "s65") SA_RG_STEP("s66", "s67")
#define SA_RG_B                                                                                               \
    SA_RG_STEP("s68", "s69") SA_RG_STEP("s70", "s71") SA_RG_STEP("s72", "s73") SA_RG_STEP("s74", "s75")         \
    SA_RG_STEP("s76", "s77") SA_RG_STEP("s78", "s79") SA_RG_STEP("s80", "s81") SA_RG_STEP("s82", "s83")         \
    SA_RG_STEP("s84", "s85") SA_RG_STEP("s86", "s87") SA_RG_STEP("s88", "s89") SA_RG_STEP("s90", "s91")         \
    SA_RG_STEP("s92", "s93") SA_RG_STEP("s94", "s95") SA_RG_STEP("s96", "s97") SA_RG_STEP("s98", "s99")
#define SA_RG_LOAD_A "s_load_dwordx16 s[36:51], %[nx], 0x0 glc\n\ts_load_dwordx16 s[52:67], %[nx], 0x40 glc\n\t"
#define SA_RG_LOAD_B "s_load_dwordx16 s[68:83], %[nx], 0x0 glc\n\ts_load_dwordx16 s[84:99], %[nx], 0x40 glc\n\t"
#define SA_RG_CLOBBER                                                                                         \
    "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50",   \
        "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", \
        "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", \
        "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95", \
        "s96", "s97", "s98", "s99"

__device__ __forceinline__ const uint32_t* wave_ptr(const uint32_t* p)
{
    const uint64_t x = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x), hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return (const uint32_t*)((uint64_t)hi << 32 | lo);
}
// the first group of a segment into buffer A
__device__ __forceinline__ void rg_first(const uint32_t* p)
{
    asm volatile("; sa_rg_first\n\t" SA_RG_LOAD_A ::[nx] "s"(wave_ptr(p)) : "memory", SA_RG_CLOBBER);
}
// every load in (before code that may use the buffers' registers)
__device__ __forceinline__ void rg_drain()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\t; sa_rg_drained" ::: "memory", SA_RG_CLOBBER);
}
// one group: buffer A (ODD = 0) or B coded while the other one loads from nx
template <int ODD>
__device__ __forceinline__ void rg_group(uint32_t& r, const uint32_t* nx, const uint32_t tmask)
{
    uint32_t q, p, t, f;
    if constexpr (ODD == 0)
        asm volatile("s_waitcnt lgkmcnt(0)\n\t" SA_RG_LOAD_B SA_RG_A
                     : [r] "+s"(r), [q] "=&s"(q), [p] "=&s"(p), [t] "=&s"(t), [f] "=&s"(f)
                     : [nx] "s"(wave_ptr(nx)), [mk] "s"(tmask)
                     : "scc", SA_RG_CLOBBER);
    else
        asm volatile("s_waitcnt lgkmcnt(0)\n\t" SA_RG_LOAD_A SA_RG_B
                     : [r] "+s"(r), [q] "=&s"(q), [p] "=&s"(p), [t] "=&s"(t), [f] "=&s"(f)
                     : [nx] "s"(wave_ptr(nx)), [mk] "s"(tmask)
                     : "scc", SA_RG_CLOBBER);
}
#undef SA_RG_STEP
#undef SA_RG_A
#undef SA_RG_B
#undef SA_RG_LOAD_A
#undef SA_RG_LOAD_B

// the lanes' part: segment g's (m, tf) pairs into its slot
__device__ __forceinline__ void rg_put(uint32_t* R, uint32_t g, uint32_t ctf, uint32_t tmask)
{
    const uint32_t lane = threadIdx.x & 63;
    *reinterpret_cast<uint2*>(R + (g & 3) * RING_SLOT + 2 * lane) = make_uint2(recip32z(ctf & tmask), ctf);
}

__device__ __forceinline__ void coder_rg_chain(const uint32_t li, const CoderTask* __restrict__ tasks,
                                               const TaskList& tl, const PRec* __restrict__ prs0,
                                               const PRec* __restrict__ prs1, uint32_t* __restrict__ ck_r,
                                               uint32_t* __restrict__ err, const uint32_t prio, uint32_t* R)
{
    typedef const __attribute__((address_space(1))) uint32_t g_u32;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t t = tl.ids[li];
    const CoderTask tk = tasks[t];
    const CoderRun run = tl.run[li];
    const PRec* P = (tk.space ? prs1 : prs0) + tk.rec_base;
    g_u32* G = (g_u32*)(P) + lane;
    const uint32_t tmask = tk.space ? 0xffffu : 0xffu;   // wide AUX / packed SEQ records
    uint32_t* ck = ck_r + tk.seg_base;
    const uint32_t first = run.start_seg, last = tk.nseg - 1;
    uint32_t r = run.r0;
    uint32_t g = first;
    uint32_t kv = 0;
    set_chain_prio(prio);
    if (g < last) {
        uint32_t bad = 0;
        // buf[j] holds the records of a segment = j (mod CODER_LA), loaded
        // CODER_LA - 2 segments before the lanes put it into the ring
        uint32_t buf[CODER_LA];
#pragma unroll
        for (uint32_t k = 0; k < CODER_LA; k++) buf[k] = G[(size_t)min(g + k, last) * SEG_SYMS];
        rg_put(R, g, buf[0], tmask);
        rg_put(R, g + 1, buf[1], tmask);
        buf[0] = G[(size_t)min(g + CODER_LA, last) * SEG_SYMS];
        buf[1] = G[(size_t)min(g + CODER_LA + 1, last) * SEG_SYMS];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        rg_first(R + (g & 3) * RING_SLOT);
        for (; g < last;) {
#pragma unroll
            for (uint32_t k = 0; k < CODER_LA; k++) {
                if (g >= last) break;
                const uint32_t kk = (k + 2) % CODER_LA;
                rg_put(R, g + 2, buf[kk], tmask);
                buf[kk] = G[(size_t)min(g + 2 + CODER_LA, last) * SEG_SYMS];
                kv = lane == (g & 63) ? r : kv;
                if ((g & 63) == 63) {
                    const uint32_t s = g - 63 + lane;
                    if (s >= first) ck[s] = kv;
                }
                r = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
                const uint32_t r_seg = r;
                // segment g+1's slot (stored one segment ago) is in L2 before its
                // first group is loaded at the end of this segment: younger than
                // that store are at least this segment's store and load
                asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                const uint32_t* cur = R + (g & 3) * RING_SLOT;
                rg_group<0>(r, cur + 32, tmask);
                rg_group<1>(r, cur + 64, tmask);
                rg_group<0>(r, cur + 96, tmask);
                rg_group<1>(r, R + ((g + 1) & 3) * RING_SLOT, tmask);
                if (r == 0) {   // (records not in yet: seg_retry's own code may use the buffers' registers)
                    rg_drain();
                    r = seg_retry(P + (size_t)g * SEG_SYMS, r_seg, tmask, bad, tl.wait_ticks);
                    rg_first(R + ((g + 1) & 3) * RING_SLOT);
                }
                g++;
            }
        }
        rg_drain();
        if (bad && lane == 0) atomicOr(err, (uint32_t)E_CODER);
    }
    kv = lane == (g & 63) ? r : kv;
    const uint32_t s = (g & ~63u) + lane;
    if (s >= first && s <= g) ck[s] = kv;
}

template <int V>
__device__ __forceinline__ void coder_rv_chain(const uint32_t li, const CoderTask* __restrict__ tasks,
                                               const TaskList& tl, const PRec* __restrict__ prs0,
                                               const PRec* __restrict__ prs1, uint32_t* __restrict__ ck_r,
                                               uint32_t* __restrict__ err, const uint32_t prio)
{
    typedef const __attribute__((address_space(1))) uint32_t g_u32;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t t = tl.ids[li];
    const CoderTask tk = tasks[t];
    const CoderRun run = tl.run[li];
    const PRec* P = (tk.space ? prs1 : prs0) + tk.rec_base;
    g_u32* G = (g_u32*)(P) + lane;
    const uint32_t tmask = tk.space ? 0xffffu : 0xffu;   // wide AUX / packed SEQ records
    uint32_t* ck = ck_r + tk.seg_base;
    const uint32_t first = run.start_seg, last = tk.nseg - 1;
    uint32_t r = run.r0;
    uint32_t g = first;
    uint32_t kv = 0;
    set_chain_prio(prio);
    if (g < last) {
        uint32_t bad = 0;
        // segment loads at or past the last segment read the last one (the
        // record arrays hold >= 64 records of slack past every stream's end)
        uint32_t buf[CODER_LA];
#pragma unroll
        for (uint32_t k = 0; k < CODER_LA; k++) buf[k] = G[(size_t)min(g + k, last) * SEG_SYMS];
        for (; g < last;) {
#pragma unroll
            for (uint32_t k = 0; k < CODER_LA; k++) {
                if (g >= last) break;
                const uint32_t ctf = buf[k];
                buf[k] = G[(size_t)min(g + CODER_LA, last) * SEG_SYMS];
                kv = lane == (g & 63) ? r : kv;
                if ((g & 63) == 63) {
                    const uint32_t s = g - 63 + lane;
                    if (s >= first) ck[s] = kv;
                }
                r = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);   // (scalar for the asm: see k_coder_rv)
                const uint32_t r_seg = r;
                const uint32_t vt = ctf & tmask, cm = recip32z(vt);
                rv_segment<V>(r, cm, vt, ctf >> 16, std::make_integer_sequence<int, 8>{});
                if (r == 0) r = seg_retry(P + (size_t)g * SEG_SYMS, r_seg, tmask, bad, tl.wait_ticks);
                g++;
            }
        }
        if (bad && lane == 0) atomicOr(err, (uint32_t)E_CODER);
    }
    kv = lane == (g & 63) ? r : kv;
    const uint32_t s = (g & ~63u) + lane;
    if (s >= first && s <= g) ck[s] = kv;
}

// Waves [0, nlong) take one (long) chain each; the waves after them share the
// remaining (short) chains round robin, longest first.  A launch then asks for
// one pass-R workgroup slot (one per CU) per four long chains plus a few,
// instead of one per four chains: with three or four batches' pass R in flight
// the excess waited for slots, and a launch that cannot place all its
// workgroups holds up the kernels queued behind it on its hardware queue.
// probe (SA_RV_PROBE, diagnostics): per wave its start / end on the constant
// 100 MHz clock (s_memrealtime), the shader-clock cycles between them
// (s_memtime), and where it ran (HW_ID: wave slot, SIMD, CU, SE; XCC_ID) with
// the number of chains it coded
template <int V>
__global__ __launch_bounds__(64 * CODER_MAX_WAVES) void k_coder_rv(
    const CoderTask* __restrict__ tasks, const TaskList tl, const PRec* __restrict__ prs0,
    const PRec* __restrict__ prs1, uint32_t* __restrict__ ck_r, uint32_t* __restrict__ err, const uint32_t prio,
    uint64_t* __restrict__ probe, uint32_t* __restrict__ ring)
{
    const uint32_t wpg = blockDim.x >> 6;
    const uint32_t wi = blockIdx.x * wpg + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t nl = tl.nlong < tl.count ? tl.nlong : tl.count;
    uint64_t t0 = 0, c0 = 0;
    if (probe) {
        t0 = __builtin_amdgcn_s_memrealtime();
        c0 = __builtin_amdgcn_s_memtime();
    }
    // (one call site: two inlined copies of the chain's asm made the compiler
    // move its scalar operands through VGPRs)
    const uint32_t step = wi < nl ? 0u : gridDim.x * wpg - nl;
    uint32_t chains = 0;
    for (uint32_t li = wi; li < tl.count;) {
        if constexpr (V == 6) coder_rg_chain(li, tasks, tl, prs0, prs1, ck_r, err, prio, ring + (size_t)wi * RING_DW);
        else coder_rv_chain<V>(li, tasks, tl, prs0, prs1, ck_r, err, prio);
        chains++;
        if (!step) break;
        li += step;
    }
    if (probe) {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if ((threadIdx.x & 63) == 0) {
            probe[4 * wi + 0] = t0;
            probe[4 * wi + 1] = t1;
            probe[4 * wi + 2] = c1 - c0;
            probe[4 * wi + 3] = hw | (uint64_t)(xcc & 0xffu) << 32 | (uint64_t)chains << 40;
        }
    }
}

// ---------------------------------------------------------------------------
// k_coder_rl (round 5): pass R with one chain per LANE.  k_coder_rv runs a
// chain per wave on the scalar unit -- one scalar unit per CU, so its ~600
// waves in flight (three to four batches of 172) held the scalar issue of
// three quarters of the CUs, and the front kernels beside them, whose loops
// and address arithmetic are scalar instructions, ran 2.5-6x slower than alone
// (k_prep_sq16 4.4 -> 26.5 ms, k_emit_sq16 17 -> 43 ms; profiles/round5_r5e_*).
// Here the same step runs in the VALU, 64 chains per workgroup (a batch's ~760
// chains in ~12 workgroups, longest first).  Wave 4 codes: lane c is chain c,
// one ds_read_b64 of (m, record) and the step per symbol.  Waves 0-3 feed it
// through a two-half LDS ring, one 64-record segment of every chain per
// round: for chain c (c = w, w + 4, ...) the wave loads the segment whole --
// lane k its record k, 256 contiguous bytes -- derives m (BASE_MODEL totals
// < 256 from an LDS table; wider totals by an exact double division), and
// writes the pairs transposed, at [k][c] of a 65-wide row (2-way bank
// conflicts at most).  The first version had each lane load its own chain's
// records and look m up in a 2^16-entry table in memory: 128 gathers of 64
// lines per round, pass R 1,835-1,864 ms under the bench's load (r5k).  The
// loads of round j + 1 are issued before round j is converted; one barrier per
// round hands the halves over.  Records the long model runs have not written
// yet (total 0) are waited for as in seg_retry (agent-scope loads, bounded by
// tl.wait_ticks, then E_CODER).  Checkpoints (ck_r): each lane stores its
// range at the start of every segment of its chain, first..last, as
// k_coder_rv does.
// ---------------------------------------------------------------------------
constexpr uint32_t RL_FEEDERS = 4, RL_WAVES = RL_FEEDERS + 1, RL_ROW = SEG_SYMS + 1;
constexpr uint32_t RL_PER_FEEDER = 64 / RL_FEEDERS;

// The ring hand-over: LDS writes done, then the barrier -- without
// __syncthreads' release fence, which waits for every outstanding global
// access of the wave (vmcnt(0)): the feeders' loads of the next round and the
// chain's checkpoint store would each cost a memory round trip per round.
__device__ __forceinline__ void rl_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// m for a record of one chain (tmask wave-uniform): recip32z of its total
__device__ __forceinline__ uint32_t rl_recip(uint32_t v, uint32_t tmask, const uint32_t* tab)
{
    if (tmask == 0xffu) return tab[v & 0xffu];
    const uint32_t t = v & 0xffffu;
    // (2^32 - 1) / t rounded to nearest in double truncates to the integer
    // quotient: below 2^32 a double's spacing is <= 2^-21, a non-integer
    // quotient is >= 1/t >= 2^-16 from the next integer (recip32 for t >= 1;
    // t = 1 wraps to 0 as recip32 does)
    return t ? (uint32_t)(4294967295.0 / (double)t) + 1u : 0u;
}

__global__ __launch_bounds__(64 * RL_WAVES) void k_coder_rl(const CoderTask* __restrict__ tasks, const TaskList tl,
                                                            const PRec* __restrict__ prs0,
                                                            const PRec* __restrict__ prs1,
                                                            uint32_t* __restrict__ ck_r, uint32_t* __restrict__ err,
                                                            const uint32_t prio)
{
    __shared__ uint2 ring[2][SEG_SYMS * RL_ROW];   // 66,560 B: (m, tf) at [step][chain]
    __shared__ uint32_t tab[256];                  // recip32z(t), t < 256
    typedef const __attribute__((address_space(1))) uint32_t g_u32;   // (global loads: vmcnt only, not lgkmcnt)
    __shared__ g_u32* cbase[64];                   // chain c's first coded segment
    __shared__ uint32_t cnj[64], cmask[64], cmax;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint32_t t = threadIdx.x; t < 256; t += blockDim.x) tab[t] = recip32z(t);
    const uint32_t li = blockIdx.x * 64 + lane;
    uint32_t first = 0, nj = 0, r = 0, tmask = 0xffu;
    uint64_t seg_base = 0;
    if (wave == RL_FEEDERS) {
        uint32_t last = 0;
        const PRec* P = prs0;
        if (li < tl.count) {
            const CoderTask tk = tasks[tl.ids[li]];
            const CoderRun run = tl.run[li];
            P = (tk.space ? prs1 : prs0) + tk.rec_base;
            tmask = tk.space ? 0xffffu : 0xffu;
            first = run.start_seg;
            last = tk.nseg - 1;
            r = run.r0;
            seg_base = tk.seg_base;
        }
        // segments coded by this lane: first .. last - 1 (the last is L3's alone)
        nj = li < tl.count && last > first ? last - first : 0u;
        cbase[lane] = (g_u32*)(P + (size_t)first * SEG_SYMS);
        cnj[lane] = nj;
        cmask[lane] = tmask;
        uint32_t J = nj;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t o = (uint32_t)__shfl_xor((int)J, d, 64);
            J = J > o ? J : o;
        }
        if (lane == 0) cmax = J;
    }
    __syncthreads();
    const uint32_t J = cmax;
    if (wave < RL_FEEDERS) {
        uint32_t bad = 0;
        const uint64_t wait = tl.wait_ticks ? tl.wait_ticks : 2000000000u;
        // this wave's chains c = wave + RL_FEEDERS i: their record bases, segment
        // counts and total masks in registers (the LDS copies are read once)
        g_u32* base[RL_PER_FEEDER];
        uint32_t cn[RL_PER_FEEDER], cm[RL_PER_FEEDER];
#pragma unroll
        for (uint32_t i = 0; i < RL_PER_FEEDER; i++) {
            const uint32_t c = wave + RL_FEEDERS * i;
            base[i] = cbase[c] + lane;
            cn[i] = cnj[c];
            cm[i] = cmask[c];
        }
        // a round's loads of segment j (clamped to the chain's last coded
        // segment: branch-free)
        auto load = [&](uint32_t j, uint32_t (&v)[RL_PER_FEEDER]) __attribute__((always_inline)) {
#pragma unroll
            for (uint32_t i = 0; i < RL_PER_FEEDER; i++) {
                const uint32_t jj = j < cn[i] ? j : (cn[i] ? cn[i] - 1 : 0u);
                v[i] = base[i][(size_t)jj * SEG_SYMS];
            }
        };
        // round j's records (in v) waited for where the long model runs have
        // not written them yet (total 0; replayed concurrently) -- before the
        // next round's loads are issued, so the wait for v is the only one
        auto check = [&](uint32_t j, uint32_t (&v)[RL_PER_FEEDER]) __attribute__((always_inline)) {
            bool zero = false;
#pragma unroll
            for (uint32_t i = 0; i < RL_PER_FEEDER; i++) zero |= j < cn[i] && (v[i] & cm[i]) == 0;
            if (__ballot(zero) && !bad) {
                const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + wait;
#pragma unroll
                for (uint32_t i = 0; i < RL_PER_FEEDER; i++) {   // (unrolled: v, cn, cm stay in registers)
                    if (j < cn[i] && !bad) {
                        g_u32* S = base[i] + (size_t)j * SEG_SYMS;
                        while (__ballot((v[i] & cm[i]) == 0)) {
                            if (__builtin_amdgcn_s_memrealtime() > t_end) {
                                bad = 1;
                                break;
                            }
                            __builtin_amdgcn_s_sleep(32);
                            v[i] = __hip_atomic_load((const uint32_t*)S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                }
            }
        };
        // round j's records converted into ring half j & 1 (pairs of chains
        // past their end are written too: their lanes do not read them)
        auto put = [&](uint32_t j, const uint32_t (&v)[RL_PER_FEEDER]) __attribute__((always_inline)) {
            uint2* R = ring[j & 1] + lane * RL_ROW + wave;
#pragma unroll
            for (uint32_t i = 0; i < RL_PER_FEEDER; i++)
                R[RL_FEEDERS * i] = make_uint2(rl_recip(v[i], cm[i], tab), v[i]);
        };
        uint32_t va[RL_PER_FEEDER], vb[RL_PER_FEEDER];
        load(0, va);
        check(0, va);
        load(1, vb);
        put(0, va);
        rl_barrier();
        for (uint32_t j = 1; j <= J; j += 2) {   // round j into its half while the chain codes round j - 1
            check(j, vb);
            load(j + 1, va);
            put(j, vb);
            rl_barrier();
            if (j + 1 <= J) {
                check(j + 1, va);
                load(j + 2, vb);
                put(j + 1, va);
                rl_barrier();
            }
        }
        if (bad && lane == 0) atomicOr(err, (uint32_t)E_CODER);
    } else {
        set_chain_prio(prio);
        uint32_t* ck = ck_r + seg_base;
        rl_barrier();
        for (uint32_t j = 0; j < J; j++) {
            if (j < nj) {
                ck[first + j] = r;
                const uint2* R = ring[j & 1] + lane;
                uint32_t rr = r;
#pragma unroll 16
                for (uint32_t k = 0; k < SEG_SYMS; k++) {
                    const uint2 e = R[k * RL_ROW];
                    const uint32_t t = e.y & tmask, f = e.y >> 16;
                    uint32_t q = __umulhi(rr, e.x);
                    q -= rr < q * t ? 1u : 0u;
                    const uint32_t x = q * f;
                    rr = x << (__builtin_clz(x) & 24);   // (x > 0: records are written)
                }
                r = rr;
            }
            rl_barrier();
        }
        if (li < tl.count) ck[first + nj] = r;   // (the range entering segment `last`)
    }
}

// Locate list entry and segment of global coder-lane gi (gbase ascending).
__device__ inline uint32_t list_find(const TaskList& tl, uint64_t gi)
{
    uint32_t lo = 0, hi = tl.count;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tl.gbase[mid] <= gi) lo = mid;
        else hi = mid;
    }
    return lo;
}

// L1: one lane per segment -> its LowMap.
template <uint32_t CH>
__global__ __launch_bounds__(256) void k_coder_l1(const CoderView cv, const TaskList tl)
{
    set_l_prio(cv.lprio);
    const uint64_t gi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= tl.total_segs) return;
    const uint32_t li = list_find(tl, gi);
    const CoderTask& tk = cv.tasks[tl.ids[li]];
    const uint32_t g = tl.run[li].start_seg + (uint32_t)(gi - tl.gbase[li]);
    const size_t at = tk.rec_base + (size_t)g * SEG_SYMS;
    cv.maps[tk.seg_base + g] =
        seg_lowmap<CH>(cv.prs[tk.space] + at, cv.cum[tk.space] ? cv.cum[tk.space] + at : nullptr,
                   cv.ck_r[tk.seg_base + g], seg_count(tk.n, g));
}

// L2: one workgroup per listed stream: exclusive scan of the segment maps from
// the stream's start state -> low and output offset at every segment.  Each
// thread composes L2_PER consecutive maps first, so a 22 M-symbol stream
// (344 K segments) takes 84 workgroup steps instead of 1,344 (round 3: one map
// per thread, 8.7 ms per batch on the tail's critical path).
constexpr int L2_THREADS = 256;
constexpr uint32_t L2_PER = 16;

__device__ inline LowMap shfl_up_map(const LowMap& m, int d)
{
    LowMap o;
    o.B = __shfl_up(m.B, d, 64);
    o.s = __shfl_up(m.s, d, 64);
    o.nbytes = __shfl_up(m.nbytes, d, 64);
    return o;
}

__global__ __launch_bounds__(L2_THREADS) void k_coder_l2(const CoderView cv, const TaskList tl)
{
    __shared__ LowMap wtot[L2_THREADS / 64];
    __shared__ uint64_t carry_low;
    __shared__ uint32_t carry_off;
    const uint32_t li = blockIdx.x;
    const CoderTask tk = cv.tasks[tl.ids[li]];
    const CoderRun run = tl.run[li];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        carry_low = run.low0;
        carry_off = run.off0;
    }
    __syncthreads();
    const LowMap id{0ull, 0u, 0u};
    for (uint32_t base = run.start_seg; base < tk.nseg; base += L2_THREADS * L2_PER) {
        const uint32_t g0 = base + threadIdx.x * L2_PER;
        LowMap m[L2_PER];
        LowMap x = id;
#pragma unroll
        for (uint32_t k = 0; k < L2_PER; k++) {
            m[k] = g0 + k < tk.nseg ? cv.maps[tk.seg_base + g0 + k] : id;
            x = lowmap_compose(x, m[k]);
        }
        // inclusive wave scan of the threads' compositions (earlier then later)
        LowMap inc = x;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const LowMap y = shfl_up_map(inc, d);
            if (lane >= (uint32_t)d) inc = lowmap_compose(y, inc);
        }
        if (lane == 63) wtot[w] = inc;
        __syncthreads();
        LowMap pre = id;
        for (uint32_t k = 0; k < w; k++) pre = lowmap_compose(pre, wtot[k]);
        LowMap e = shfl_up_map(inc, 1);
        if (lane == 0) e = id;
        e = lowmap_compose(pre, e);
        const uint64_t cl = carry_low;
        const uint32_t co = carry_off;
#pragma unroll
        for (uint32_t k = 0; k < L2_PER; k++) {
            if (g0 + k < tk.nseg) {
                cv.low_at[tk.seg_base + g0 + k] = shl64(cl, e.s) + e.B;
                cv.off_at[tk.seg_base + g0 + k] = co + e.nbytes;
            }
            e = lowmap_compose(e, m[k]);
        }
        __syncthreads();
        if (threadIdx.x == L2_THREADS - 1) {   // (e: the composition through this thread's last map)
            carry_low = shl64(cl, e.s) + e.B;
            carry_off = co + e.nbytes;
        }
        __syncthreads();
    }
}

// Bytes of every listed stream up to its last segment's flush (L1 maps + L2
// offsets): the host sizes the payload arena from them before L3 writes it.
__global__ __launch_bounds__(256) void k_task_ends(const CoderView cv, const TaskList tl, uint32_t* __restrict__ ends)
{
    const uint32_t li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= tl.count) return;
    const uint32_t t = tl.ids[li];
    const CoderTask& tk = cv.tasks[t];
    const uint64_t sg = tk.seg_base + tk.nseg - 1;
    ends[t] = cv.off_at[sg] + cv.maps[sg].nbytes;
}

// L3: one lane per segment: the exact coder from (range, low) at its offset.
template <uint32_t CH>
__global__ __launch_bounds__(256) void k_coder_l3(const CoderView cv, const TaskList tl)
{
    set_l_prio(cv.lprio);
    const uint64_t gi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= tl.total_segs) return;
    const uint32_t li = list_find(tl, gi);
    const uint32_t t = tl.ids[li];
    const CoderTask& tk = cv.tasks[t];
    const uint32_t g = tl.run[li].start_seg + (uint32_t)(gi - tl.gbase[li]);
    const size_t at = tk.rec_base + (size_t)g * SEG_SYMS;
    const uint64_t sg = tk.seg_base + g;
    const uint32_t off = cv.off_at[sg];
    const bool last = g + 1 == tk.nseg;
    const SegEnd e = seg_code<CH>(cv.prs[tk.space] + at, cv.cum[tk.space] ? cv.cum[tk.space] + at : nullptr,
                              cv.ck_r[sg], cv.low_at[sg],
                              seg_count(tk.n, g), cv.out + tk.out_base + off, tk.out_cap > off ? tk.out_cap - off : 0,
                              last);
    if (last) cv.out_len[t] = off + e.nbytes;
    if (e.squeezed) {
        cv.maps[sg] = LowMap{e.low, e.r, e.nbytes};
        atomicMin(&cv.first_sq[t], g);
    }
}

// ---------------------------------------------------------------------------
// MD5 (RFC 1321; MDString@0x4058f0): one lane per message.  Messages start at
// 16-byte aligned offsets (the host aligns every block's name/seq/qual base).
// ---------------------------------------------------------------------------
__device__ inline uint32_t rotl(uint32_t x, int c) { return __builtin_amdgcn_alignbit(x, x, 32 - c); }

// One MD5 step.  mk = M[g] + K[i], prepared off the chain by the loader wave,
// so the chain is F (one v_bitop3), v_add3, v_alignbit, v_add.
#define MD5_STEP(F, a, b, c, d, mk, s) \
    a = b + rotl(a + F(b, c, d) + mk, s)
// the round functions as one v_bitop3 each (truth table over b = 0xf0,
// c = 0xcc, d = 0xaa): F = b ? c : d, G = d ? b : c, H = b ^ c ^ d, I = c ^ (b | ~d)
#define MD5_F(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0xca)
#define MD5_G(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0xe4)
#define MD5_H(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0x96)
#define MD5_I(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0x39)

__device__ const uint32_t kMd5K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

// message word of step i (RFC 1321 3.4)
__device__ inline uint32_t md5_word_of_step(uint32_t i)
{
    return i < 16 ? i : i < 32 ? (5 * i + 1) & 15 : i < 48 ? (3 * i + 5) & 15 : (7 * i) & 15;
}

// One 64-byte block from its 64 prepared words (read from LDS as 16 x 16 bytes).
__device__ inline void md5_block_q(uint32_t h[4], const uint4 (&q)[16])
{
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#define R4(F, i, s0, s1, s2, s3)                 \
    MD5_STEP(F, a, b, c, d, q[i].x, s0);         \
    MD5_STEP(F, d, a, b, c, q[i].y, s1);         \
    MD5_STEP(F, c, d, a, b, q[i].z, s2);         \
    MD5_STEP(F, b, c, d, a, q[i].w, s3)
    R4(MD5_F, 0, 7, 12, 17, 22);
    R4(MD5_F, 1, 7, 12, 17, 22);
    R4(MD5_F, 2, 7, 12, 17, 22);
    R4(MD5_F, 3, 7, 12, 17, 22);
    R4(MD5_G, 4, 5, 9, 14, 20);
    R4(MD5_G, 5, 5, 9, 14, 20);
    R4(MD5_G, 6, 5, 9, 14, 20);
    R4(MD5_G, 7, 5, 9, 14, 20);
    R4(MD5_H, 8, 4, 11, 16, 23);
    R4(MD5_H, 9, 4, 11, 16, 23);
    R4(MD5_H, 10, 4, 11, 16, 23);
    R4(MD5_H, 11, 4, 11, 16, 23);
    R4(MD5_I, 12, 6, 10, 15, 21);
    R4(MD5_I, 13, 6, 10, 15, 21);
    R4(MD5_I, 14, 6, 10, 15, 21);
    R4(MD5_I, 15, 6, 10, 15, 21);
#undef R4
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

__device__ inline void md5_block_mk(uint32_t h[4], const uint4* __restrict__ w4)
{
    uint4 q[16];
#pragma unroll
    for (int i = 0; i < 16; i++) q[i] = w4[i];
    md5_block_q(h, q);
}

// One workgroup of two waves per message.  MD5 is one dependent chain per
// message: wave 0 runs it (every lane the same chain, so no lane masking), and
// wave 1 streams the message a chunk of 16 blocks ahead: lane i loads the
// message word of step i of each block and adds K[i], so the chain reads its
// 64 step words with 16 LDS reads per block and does no other work -- four
// dependent VALU ops per step (round 1 spent six issue slots per step: the
// word moves to an SGPR and the add of K rode the chain wave).
constexpr uint32_t MD5_CHUNK_BLOCKS = 16;

template <bool PIPE>
__global__ __launch_bounds__(128) void k_md5(const Md5Task* __restrict__ tasks, uint32_t ntasks,
                                             uint32_t* __restrict__ digests, uint32_t prio)
{
    __shared__ uint4 mk[2][MD5_CHUNK_BLOCKS][16];   // prepared words: [slot][block][step / 4]
    __shared__ uint32_t tb32[32];                   // the last one or two blocks (tail + padding)
    const uint32_t t = blockIdx.x;
    if (t >= ntasks) return;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave == 0) set_chain_prio(prio);
    const Md5Task tk = tasks[t];
    const uint32_t g = md5_word_of_step(lane);
    const uint32_t kk = kMd5K[lane];
    typedef const __attribute__((address_space(1))) uint32_t g_u32;
    g_u32* w = (g_u32*)(tk.ptr);
    const uint64_t nfull = tk.len / 64;
    const uint64_t nck = (nfull + MD5_CHUNK_BLOCKS - 1) / MD5_CHUNK_BLOCKS;
    auto produce = [&](uint64_t c) __attribute__((always_inline)) {
        uint32_t* slot = reinterpret_cast<uint32_t*>(mk[c & 1]);
        const uint64_t b0 = c * MD5_CHUNK_BLOCKS;
        uint32_t v[MD5_CHUNK_BLOCKS];   // (past the last full block: its words again, unused)
#pragma unroll
        for (uint32_t k = 0; k < MD5_CHUNK_BLOCKS; k++) v[k] = w[min(b0 + k, nfull - 1) * 16 + g];
#pragma unroll
        for (uint32_t k = 0; k < MD5_CHUNK_BLOCKS; k++) slot[k * 64 + lane] = v[k] + kk;
    };
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    if (wave == 1 && nck) produce(0);
    __syncthreads();
    for (uint64_t c = 0; c < nck; c++) {
        if (wave == 1) {
            if (c + 1 < nck) produce(c + 1);
        } else {
            const uint64_t left = nfull - c * MD5_CHUNK_BLOCKS;
            const uint32_t nb = left < MD5_CHUNK_BLOCKS ? (uint32_t)left : MD5_CHUNK_BLOCKS;
            // the next block's words are read while this block's chain runs (two
            // register sets; the scheduler barriers keep the reads ahead)
            const uint4(*blk)[16] = mk[c & 1];
            if (!PIPE) {   // (SA_MD5_PIPE=0: one block's reads at a time, for A/B)
                for (uint32_t k = 0; k < nb; k++) md5_block_mk(h, blk[k]);
            } else {
                uint4 qa[16], qb[16];
#pragma unroll
                for (int i = 0; i < 16; i++) qa[i] = blk[0][i];
                for (uint32_t k = 0; k < nb; k += 2) {
                    const uint32_t k1 = min(k + 1, nb - 1), k2 = min(k + 2, nb - 1);
#pragma unroll
                    for (int i = 0; i < 16; i++) qb[i] = blk[k1][i];
                    __builtin_amdgcn_sched_barrier(0);
                    md5_block_q(h, qa);
                    __builtin_amdgcn_sched_barrier(0);
                    if (k + 1 >= nb) break;
#pragma unroll
                    for (int i = 0; i < 16; i++) qa[i] = blk[k2][i];
                    __builtin_amdgcn_sched_barrier(0);
                    md5_block_q(h, qb);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        __syncthreads();
    }
    if (wave == 1) return;
    // tail + padding (bit length of the u32 length, as the RSA MDString): the
    // wave writes the last one or two 64-byte blocks into LDS, two bytes a lane
    const uint32_t rem = (uint32_t)(tk.len - nfull * 64);
    const uint8_t* tail = tk.ptr + nfull * 64;
    const uint32_t tl = rem < 56 ? 64 : 128;
    const uint64_t bits = (uint64_t)(uint32_t)tk.len << 3;
    uint8_t* tb = reinterpret_cast<uint8_t*>(tb32);
#pragma unroll
    for (uint32_t j = lane; j < 128; j += 64) {
        uint8_t v = 0;
        if (j < rem) v = tail[j];
        else if (j == rem) v = 0x80;
        else if (j >= tl - 8 && j < tl) v = (uint8_t)(bits >> (8 * (j - (tl - 8))));
        tb[j] = v;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    uint32_t* slot = reinterpret_cast<uint32_t*>(mk[0]);
    for (uint32_t o = 0; o < tl / 64; o++) {
        slot[o * 64 + lane] = tb32[o * 16 + g] + kk;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    for (uint32_t o = 0; o < tl / 64; o++) md5_block_mk(h, mk[0][o]);
    if (lane == 0)
        for (int k = 0; k < 4; k++) digests[(size_t)t * 4 + k] = h[k];
}

// ---------------------------------------------------------------------------
// Block assembly (doFqzEncode@0x42d2d0): one workgroup per block.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_assemble(const BatchView bv, const AsmView av,
                                                 const uint32_t* __restrict__ out_len,
                                                 const uint32_t* __restrict__ digests,
                                                 uint8_t* __restrict__ final_out,
                                                 uint64_t* __restrict__ final_len)
{
    // one lane per block: headers, MD5s, ID-bin payload and the list of coder
    // payloads to copy (k_assemble_copy)
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= bv.nblocks) return;
    const AsmBlock& ab = av.blocks[b];
    uint32_t* cp = av.copies + (size_t)b * ASM_COPY_WORDS;
    uint32_t ns = 0;
    final_len[b] = assemble_plan(bv, b, ab, out_len, digests, final_out + ab.out_base, cp + 1,
                                 cp + 1 + ASM_MAX_COPIES, cp + 1 + 2 * ASM_MAX_COPIES, ns);
    cp[0] = ns;
}

// Coder payloads into place: ASM_SLICES workgroups per block, consecutive threads
// copy consecutive bytes.
constexpr uint32_t ASM_SLICES = 32;

__global__ __launch_bounds__(256) void k_assemble_copy(const AsmView av, const uint8_t* __restrict__ payload,
                                                       uint8_t* __restrict__ final_out)
{
    const uint32_t b = blockIdx.x / ASM_SLICES, slice = blockIdx.x % ASM_SLICES;
    const uint32_t* cp = av.copies + (size_t)b * ASM_COPY_WORDS;
    const uint32_t ns = cp[0];
    uint8_t* o = final_out + av.blocks[b].out_base;
    for (uint32_t sgi = 0; sgi < ns; sgi++) {
        const uint8_t* src = payload + av.task_out_base[cp[1 + ASM_MAX_COPIES + sgi]];
        uint8_t* dst = o + cp[1 + sgi];
        const uint32_t L = cp[1 + 2 * ASM_MAX_COPIES + sgi];
        for (uint32_t k = slice * blockDim.x + threadIdx.x; k < L; k += ASM_SLICES * blockDim.x) dst[k] = src[k];
    }
}

}  // namespace sa
