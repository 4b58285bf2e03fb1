// sa_align_host.h -- the serial bookkeeping of the reference (HASH index) path
// per block, on the host: which reads get aligned, the align_info state the
// encode thread carries from read to read, the 5 % probe and bail-out, the PE
// insert window.  Shared by the engine (sa_align.hip) and the CPU decomposition
// test (tests/cpu_emu).
//
// The reference runs, per block (AlignEncodeSEJob::doAlign@0x411910 /
// AlignEncodePEJob::doAlign@0x413580):
//   SE: per read, DegeInfoProcess@0x433a10; a read with more N / IUPAC bases
//       than maxmis is not aligned (the aligner is not called); otherwise
//       getHashAlignInfo@0x4113c0 on the thread's align_info.
//   PE: per pair, both mates (align_info +0x8 / +0x50, never skipped).
//   After read (pair) i, once i exceeds 5 % of the block's reads: if fewer
//   than half of the reads so far aligned, the rest of the block is not
//   aligned at all (no order bytes: the order count ends there); PE computes
//   its insert window there first (CaclInsertSize@0x413270) from the pairs so
//   far that both aligned within 20000, unless -I gave it.
// The aligner's outcome depends on the carried align_info only through "was
// the last aligned read's mismatch count within maxmis" (hashAligner@0x410f50
// consults it before a read's first candidate is verified).  The GPU aligns
// every read with the state "no" and the reads that consulted it again with
// "yes"; this pass follows the chain and picks per read.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

namespace sa {

// per read, from the GPU pass (k_hash_align_batch)
enum : uint8_t {
    AL_OK0 = 1,      // aligned with the carried state "not aligned"
    AL_CONS = 2,     // the search consulted the carried state
    AL_NSKIP = 4,    // more N / IUPAC bases than maxmis
    AL_OK1 = 8,      // aligned with the carried state "aligned" (AL_CONS reads)
};

struct AlignChainState {
    bool c[2] = {true, true};   // mate 1 (SE) / mate 2 align_info "aligned" (nmis in [0, maxmis])
};

struct AlignBlockPlan {
    uint32_t order_count = 0, win = 0, ibits = 0, insert_bits = 0, aligned = 0;
};

// AlignEncodePEJob::CaclInsertSize@0x413270 over the distances: the median,
// then the narrowest window med +- 2^e (e = 2, 3, ...) holding more than 90 %
// of them; no distances: 512 (9 bits)
inline void insert_window(std::vector<int>& v, uint32_t& win, uint32_t& bits)
{
    if (v.empty()) {
        win = 0x200;
        bits = 9;
        return;
    }
    std::sort(v.begin(), v.end());
    const int n = (int)v.size();
    int lo, hi, med;
    if (n & 1) {
        lo = hi = (n - 1) / 2;
        med = v[(size_t)lo];
    } else {
        lo = (n - 2) / 2;
        hi = lo + 1;
        med = (v[(size_t)lo] + v[(size_t)hi]) / 2;
    }
    const int thr = (int)(0.9 * (double)n);   // @0x44a2b8
    for (int e = 2;; e++) {
        const int w = 1 << e, a = med - w, b = med + w;
        while (lo >= 0 && v[(size_t)lo] > a) lo--;
        while (hi < n && v[(size_t)hi] < b) hi++;
        if (thr < hi - lo) {
            win = (uint32_t)(b - a);
            bits = (uint32_t)e + 1;
            return;
        }
    }
}

inline uint32_t host_bits(uint64_t v)   // getbitnum@0x40d470
{
    uint32_t n = 0;
    while (v) { n++; v >>= 1; }
    return n;
}

// One block: st[i] the AL_* flags of its reads, pos0 / pos1 their positions in
// the two variants (PE insert sizes).  Appends to `sel` the block-local reads
// that take the "aligned" variant; advances the chain.
inline AlignBlockPlan align_plan_block(bool paired, uint32_t n, const uint8_t* st, const uint32_t* pos0,
                                       const uint32_t* pos1, uint32_t insert_size, AlignChainState& ch,
                                       std::vector<uint32_t>& sel)
{
    AlignBlockPlan bp;
    const int limit = (int)((double)(int)n * 0.05);   // @0x44a218
    bool checking = true;
    auto take = [&](uint32_t i, bool& carried, bool& ok, uint32_t& pos) {
        const bool v1 = carried && (st[i] & AL_CONS);
        ok = v1 ? (st[i] & AL_OK1) != 0 : (st[i] & AL_OK0) != 0;
        pos = v1 ? pos1[i] : pos0[i];
        if (v1) sel.push_back(i);
        carried = ok;
    };
    if (!paired) {
        uint32_t i = 0;
        while (i < n) {
            if (!(st[i] & AL_NSKIP)) {
                bool ok;
                uint32_t p;
                take(i, ch.c[0], ok, p);
                bp.aligned += ok;
            }
            i++;
            if ((uint32_t)limit < i && checking) {
                if ((double)i * 0.5 > (double)bp.aligned) break;   // bail out
                checking = false;
            }
        }
        bp.order_count = i;
        return bp;
    }
    uint32_t win = insert_size, ibits = insert_size ? host_bits(insert_size) : 0;   // job ctor @0x412e4b
    std::vector<int> ins;
    uint32_t r = 0;
    while (r + 1 < n) {
        bool ok1, ok2;
        uint32_t p1, p2;
        take(r, ch.c[0], ok1, p1);
        take(r + 1, ch.c[1], ok2, p2);
        bp.aligned += (uint32_t)ok1 + (uint32_t)ok2;
        if (!win && ok1 && ok2) {
            const int64_t d = p1 > p2 ? (int64_t)p1 - p2 : (int64_t)p2 - p1;
            if (d <= 0x4e1f) ins.push_back((int)d);
        }
        r += 2;
        if ((int)r > limit && checking) {
            if (!insert_size) {
                insert_window(ins, win, ibits);
                bp.insert_bits = ibits;
            }
            if ((double)(int)r * 0.5 > (double)bp.aligned) break;
            checking = false;
        }
    }
    bp.order_count = r;
    bp.win = win;
    bp.ibits = ibits;
    return bp;
}

}  // namespace sa
