// sa_device.h -- device-side views of a batch of blocks (POD, passed by value
// to kernels).  Filled by the host engine (sa_engine.hip).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "sa_common.h"

namespace sa {

constexpr int SORT_THREADS = 256;
constexpr int SORT_ITEMS = 16;
constexpr uint32_t SORT_TILE = SORT_THREADS * SORT_ITEMS;   // 4096 keys per tile
constexpr uint32_t SORT_PAD = 0xffffffffu;

// One block of the batch.  Read-level arrays are indexed by the global read id.
struct DevBlock {
    uint32_t nreads;
    uint32_t read0;            // global id of the block's first read
    uint64_t name_base;        // byte offset of the block's IDs in BatchView::names (16-aligned)
    uint64_t seq_base;         // byte offset of the block's bases/quals (16-aligned)
    uint64_t name_bytes;
    uint64_t seq_bytes;
    uint64_t seq_sym_base;     // element offset of the block's SEQ symbol space (tile-aligned)
    uint64_t aux_sym_base;     // element offset of the block's AUX symbol space (tile-aligned)
    uint32_t sbase[NSTREAM];   // start of each AUX stream inside the AUX space (ST_SEQ unused)
    uint32_t scount[NSTREAM];  // symbols of each AUX stream
    uint32_t vcount[NSTREAM];  // value counts written in the dege encaps
    uint32_t n_seq;
    uint32_t n_aux;
    uint32_t len_long;         // a read > 0xffff bp: compressLen_long@0x423710 (SeqArcMemBuf+0x2)
    // reference path (SeqArcMemBuf fields the block's doAlign leaves):
    uint32_t order_count;      // +0x34: reads with an order byte (the rest after a bail-out)
    uint32_t align_count;      // +0x30: aligned reads
    uint32_t insert_bits;      // +0x28: PE insert-window bits (CaclInsertSize@0x413270)
    uint32_t win;              // AlignEncodePEJob+0xa8: insert window
    uint32_t ibits;            // AlignEncodePEJob+0xac: bits of a distance inside it
};

struct BatchView {
    const DevBlock* blocks;
    uint32_t nblocks;
    uint32_t nreads_total;
    const uint32_t* read_block;   // block index of every read
    const uint8_t* names;
    const uint8_t* seq;
    const uint8_t* qual;
    const uint8_t* qual_q;        // qualities the QUAL stream codes: qual, or the rblock output (-l)
    const uint32_t* name_off;     // within the block
    const uint16_t* name_len;
    const uint32_t* seq_off;      // within the block
    const uint32_t* seq_len;
    uint32_t seq_mask;            // NS - 1, NS = 1u << ((2k) & 31)
    int32_t qlevel;
    int32_t bin_mode;
    int32_t md5;
    int32_t lossy;                // -l: QUAL codes qual_q, no quality MD5 (compressQual@0x426eca)
    // reference (HASH index) path, doAlignEncode@0x42d4c0
    int32_t aligned;              // blocks in the doAlignEncode layout
    int32_t paired;               // PE (param+0x1b38 == 0): the PE relation streams
    const uint8_t* seq_skip;      // per read: aligned, not in the SEQ stream (compressSeq@0x4249b3)
};

// Per-read alignment of the reference path (getHashAlignInfo@0x4113c0 after the
// carried-state choice) and the constants of the position split
// (HashAlignment::loadRefIndex@0x40fe9b: shift = bits(genome) - 2).
struct AlignView {
    const int32_t* ret;       // mismatches, -1 = not aligned
    const uint8_t* rev;       // reverse-complement strand
    const uint32_t* pos;      // 1-based reference position
    const int32_t* mispos;    // per read `stride` slots, offsets along the aligned strand
    const int32_t* mistype;   // per read `stride` slots (type @0x44a0c0; 3: N / IUPAC in the read)
    uint32_t stride;          // maxmis + 1
    uint32_t shift;           // param+0x1858
    uint64_t mask;            // param+0x1860 = 2^shift - 1
    uint64_t glen;            // param+0x1868: genome bases
    int32_t paired;
    uint32_t mis_model;       // M_MIS8 / M_MIS9, 0 = no Mis symbols (maxmis 0 or > 8)
};

// R-Block lossy pre-pass (rblock@0x426c10): a block's quality bytes are cut
// into RB_CHUNK-byte chunks (the last one of a block may be shorter).
struct RbChunk {
    uint64_t base;       // byte offset of the chunk in BatchView::qual
    uint32_t len;
    uint32_t flags;      // RB_FIRST: the block's first chunk, RB_LAST: its last
};
constexpr uint32_t RB_FIRST = 1u, RB_LAST = 2u;
// one open run of rblock: start position (byte offset in BatchView::qual), min, max
struct RbRun {
    uint64_t start;
    uint32_t mn, mx;
};

// A sort segment = one block's symbol space.
struct SortSeg {
    uint64_t base;       // element offset (multiple of SORT_TILE)
    uint32_t count;      // real symbols (the rest of the last tile is padding)
    uint32_t tile0;      // global index of the segment's first tile
    uint32_t ntiles;
};

struct SortView {
    const SortSeg* segs;
    const uint32_t* tile_seg;   // segment of every global tile
    uint32_t* hist;
    uint64_t total;             // padded elements over all segments
    uint32_t ntiles;
    uint32_t nsegs;
    // AUX space, dense model ids (k_aux_dense): per segment AUX_DENSE_WORDS
    // entries {models present in the 32 ids, bits; models below them, << 32};
    // the digits of a DENSE sort pass are digits of the dense id
    const uint64_t* dense = nullptr;
};

// A model run long enough for its own wave (k_replay_aux_long).
struct LongRun {
    uint64_t start, end;   // run start; end of its block's sorted AUX keys (the run ends earlier)
    uint64_t rec_base;     // the block's first AUX record
    uint32_t model, pad_;
};

// One range-coder stream (block, stream) and its segments (SEG_SYMS symbols
// each; at least one, so that an empty stream still flushes its 8 bytes).
struct CoderTask {
    uint64_t rec_base;   // first record (element offset into the space's record arrays)
    uint64_t out_base;   // byte offset into the payload arena
    uint64_t seg_base;   // first global segment
    uint32_t n;          // symbols
    uint32_t out_cap;    // payload capacity in bytes
    uint32_t space;      // 0 = SEQ records, 1 = AUX records
    uint32_t nseg;
};

// Where a (re)started stream begins: segment, range, low and output offset there.
struct CoderRun {
    uint64_t low0;
    uint32_t r0;
    uint32_t start_seg;
    uint32_t off0;
    uint32_t pad_;
};

// The streams of one coder launch: ids into the task table, per listed task
// the prefix of its segment counts from start_seg, and its start state.
struct TaskList {
    const uint32_t* ids;
    const uint64_t* gbase;   // count + 1 entries
    const CoderRun* run;
    uint32_t count;
    uint32_t nlong;          // pass R: entries [0, nlong) get a wave each, the rest are shared (k_coder_rv)
    uint64_t total_segs;
    uint32_t wait_ticks;     // pass R: how long a wave waits for unwritten records (100 MHz ticks; 0: 20 s)
};

struct CoderView {
    const CoderTask* tasks;
    const PRec* prs[2];        // [space]
    const uint16_t* cum[2];
    uint8_t* out;              // payload arena
    uint32_t* ck_r;            // per segment: range at its first symbol (pass R)
    LowMap* maps;              // per segment: L1 map; end state of a squeezed segment (L3)
    uint64_t* low_at;          // per segment: low at its first symbol (L2)
    uint32_t* off_at;          // per segment: output offset of its first byte (L2)
    uint32_t* out_len;         // per task
    uint32_t* first_sq;        // per task: first segment whose exact coding squeezed
    uint32_t lprio;            // the L passes at s_setprio 2 (SA_L_PRIO=1, A/B)
};

struct Md5Task {
    const uint8_t* ptr;   // 16-byte aligned
    uint64_t len;
};

struct AsmBlock {
    uint64_t out_base;          // byte offset of the block's final bytes
    uint32_t task[NSTREAM];     // coder task of each stream
    uint32_t md5_task[3];       // names, seq, qual
};

struct AsmView {
    const AsmBlock* blocks;
    const uint64_t* task_out_base;
    uint32_t* copies;   // per block: count, then (dst offset, source task, length) x ASM_MAX_COPIES
};
constexpr uint32_t ASM_MAX_COPIES = 20;
constexpr uint32_t ASM_COPY_WORDS = 1 + 3 * ASM_MAX_COPIES;

}  // namespace sa
