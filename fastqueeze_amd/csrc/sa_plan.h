// sa_plan.h -- host-side layout of a batch after the per-read count scan:
// symbol spaces, sort segments, coder tasks and the final output arena.
// Shared by the engine (sa_engine.hip) and the CPU decomposition test.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

#include "sa_device.h"

namespace sa {

inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

struct SortPlan {
    std::vector<SortSeg> segs;
    std::vector<uint32_t> tile_seg;
    uint64_t total = 0;
};

inline SortPlan plan_sort(const std::vector<uint64_t>& counts)
{
    SortPlan p;
    uint64_t base = 0;
    uint32_t tile = 0;
    for (size_t s = 0; s < counts.size(); s++) {
        SortSeg g{};
        g.base = base;
        g.count = (uint32_t)counts[s];
        g.ntiles = (uint32_t)((counts[s] + SORT_TILE - 1) / SORT_TILE);
        g.tile0 = tile;
        for (uint32_t t = 0; t < g.ntiles; t++) p.tile_seg.push_back((uint32_t)s);
        tile += g.ntiles;
        base += (uint64_t)g.ntiles * SORT_TILE;
        p.segs.push_back(g);
    }
    p.total = base;
    return p;
}

struct BatchPlan {
    SortPlan seq, aux;
    std::vector<CoderTask> tasks;
    std::vector<uint64_t> task_out_base;
    std::vector<AsmBlock> asmb;
    uint64_t total_segs = 0;
    uint64_t payload_bytes = 0;
    uint64_t final_bytes = 0;
};

constexpr uint32_t NO_TASK = 0xffffffffu;   // AsmBlock::task of a stream the layout does not have

// totals: per block, the NCOL column sums of k_scan_reads.  atot (reference
// path only): per block the NACOL sums of the alignment columns, whose streams
// follow the others in the AUX space; mis_model: the Mis stream's model (0: no
// symbols).  Fills the symbol space fields of every DevBlock.  Returns false if
// a block is too large.
inline bool plan_batch(std::vector<DevBlock>& blocks, const std::vector<uint32_t>& totals, BatchPlan& bp,
                       const std::vector<uint32_t>* atot = nullptr, uint32_t mis_model = 0)
{
    const size_t nbk = blocks.size();
    std::vector<uint64_t> seq_counts(nbk), aux_counts(nbk);
    for (size_t b = 0; b < nbk; b++) {
        DevBlock& d = blocks[b];
        const uint32_t* t = &totals[b * NCOL];
        const uint32_t sc[NAUX] = {t[C_LEN], t[C_NAME], t[C_QUAL], t[C_TIP], t[C_CH], t[C_MAXQ], t[C_NCNT], t[C_NPOS]};
        uint64_t a = 0;
        for (int s = 0; s < NSTREAM; s++) d.sbase[s] = d.scount[s] = 0;
        for (int s = 0; s < NAUX; s++) {
            d.sbase[s] = (uint32_t)a;
            d.scount[s] = sc[s];
            a += sc[s];
        }
        if (atot) {
            const uint32_t* at = &(*atot)[b * NACOL];
            for (int k = 0; k < NACOL; k++) {
                const int s = ST_ORD + k;
                d.sbase[s] = (uint32_t)a;
                d.scount[s] = (k == A_MIS && !mis_model) ? 0u : at[k];
                a += d.scount[s];
            }
            d.align_count = at[A_REV];
        }
        // (< 2^30 keys per space: the sort scatter's 32-bit byte offsets in a segment)
        if (a >= (1ull << 30) || t[C_SEQ] >= (1u << 30)) return false;
        d.n_aux = (uint32_t)a;
        d.n_seq = t[C_SEQ];
        for (int s = 0; s < NSTREAM; s++) d.vcount[s] = 0;
        d.vcount[ST_TIP] = d.nreads;
        d.vcount[ST_CH] = t[C_CH];
        d.vcount[ST_MAXQ] = t[C_MAXQ];
        d.vcount[ST_NCNT] = t[C_MAXQ];
        d.vcount[ST_NPOS] = t[C_NPOSV];
        seq_counts[b] = d.n_seq;
        aux_counts[b] = d.n_aux;
    }
    bp.seq = plan_sort(seq_counts);
    bp.aux = plan_sort(aux_counts);
    bp.tasks.clear();
    bp.task_out_base.clear();
    AsmBlock none{};
    for (int s = 0; s < NSTREAM; s++) none.task[s] = NO_TASK;
    bp.asmb.assign(nbk, none);
    uint64_t payload = 0, fin = 0, segs = 0;
    // coder tasks: every block's SEQ stream first (tasks [0, nbk)), then the AUX
    // streams (tasks [nbk, 9 nbk)), so the two groups can be coded on two streams
    auto add_task = [&](size_t b, int s) {
        const DevBlock& d = blocks[b];
        CoderTask tk{};
        if (s == ST_SEQ) {
            tk.space = 0;
            tk.rec_base = d.seq_sym_base;
            tk.n = d.n_seq;
        } else {
            tk.space = 1;
            tk.rec_base = d.aux_sym_base + d.sbase[s];
            tk.n = d.scount[s];
        }
        tk.nseg = tk.n ? (tk.n + SEG_SYMS - 1) / SEG_SYMS : 1;
        tk.seg_base = segs;
        segs += tk.nseg;
        // each symbol narrows the range by at most 2^16 (tot <= 0xffe0):
        // <= 2 output bytes per symbol, plus the 8-byte flush
        const uint64_t cap = 2ull * tk.n + 64;
        tk.out_cap = (uint32_t)std::min<uint64_t>(cap, 0xffffffffull);
        tk.out_base = payload;
        payload = align_up(payload + tk.out_cap, 16);
        bp.asmb[b].task[s] = (uint32_t)bp.tasks.size();
        bp.tasks.push_back(tk);
        bp.task_out_base.push_back(tk.out_base);
    };
    for (size_t b = 0; b < nbk; b++) {
        DevBlock& d = blocks[b];
        d.seq_sym_base = bp.seq.segs[b].base;
        d.aux_sym_base = bp.aux.segs[b].base;
        add_task(b, ST_SEQ);
    }
    const int nst = atot ? NSTREAM : ST_SEQ + 1;   // (the alignment streams: reference path only)
    for (size_t b = 0; b < nbk; b++)
        for (int s = 0; s < nst; s++)
            if (s != ST_SEQ) add_task(b, s);
    for (size_t b = 0; b < nbk; b++) {
        const DevBlock& d = blocks[b];
        uint64_t blk_out = 64 + 2 + d.name_bytes + (atot ? 96 : 0);   // headers, counts, MD5s, ID-bin first ID
        for (int s = 0; s < NSTREAM; s++)
            if (bp.asmb[b].task[s] != NO_TASK) blk_out += bp.tasks[bp.asmb[b].task[s]].out_cap + 32;
        for (int f = 0; f < 3; f++) bp.asmb[b].md5_task[f] = (uint32_t)(3 * b + f);
        bp.asmb[b].out_base = fin;
        fin = align_up(fin + blk_out, 16);
    }
    bp.total_segs = segs;
    bp.payload_bytes = payload;
    bp.final_bytes = fin;
    return true;
}

}  // namespace sa
