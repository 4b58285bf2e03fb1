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
    uint32_t sbase[NAUX];      // start of each AUX stream inside the AUX space
    uint32_t scount[NAUX];     // symbols of each AUX stream
    uint32_t vcount[NSTREAM];  // value counts written in the dege encaps
    uint32_t n_seq;
    uint32_t n_aux;
};

struct BatchView {
    const DevBlock* blocks;
    uint32_t nblocks;
    uint32_t nreads_total;
    const uint32_t* read_block;   // block index of every read
    const uint8_t* names;
    const uint8_t* seq;
    const uint8_t* qual;
    const uint32_t* name_off;     // within the block
    const uint16_t* name_len;
    const uint32_t* seq_off;      // within the block
    const uint32_t* seq_len;
    uint32_t seq_mask;            // NS - 1, NS = 1u << ((2k) & 31)
    int32_t qlevel;
    int32_t bin_mode;
    int32_t md5;
};

// A sort segment = one block's symbol space.
struct SortSeg {
    uint64_t base;       // element offset (multiple of SORT_TILE)
    uint64_t hist_base;  // offset of the segment's 256 x ntiles digit counts
    uint32_t count;      // real symbols (the rest of the last tile is padding)
    uint32_t tile0;      // global index of the segment's first tile
    uint32_t ntiles;
    uint32_t pad_;
};

struct SortView {
    const SortSeg* segs;
    const uint32_t* tile_seg;   // segment of every global tile
    uint32_t* hist;
    uint64_t total;             // padded elements over all segments
    uint32_t ntiles;
    uint32_t nsegs;
};

// A model run long enough for its own wave (k_replay_aux_long).
struct LongRun {
    uint64_t start, end;   // run start; end of its block's sorted AUX keys (the run ends earlier)
    uint64_t rec_base;     // the block's first AUX record
    uint32_t model, pad_;
};

struct CoderTask {
    uint64_t rec_base;   // first record (element offset into the space's record array)
    uint64_t out_base;   // byte offset into the payload arena
    uint32_t n;          // symbols
    uint32_t out_cap;    // payload capacity in bytes
    uint32_t space;      // 0 = SEQ records, 1 = AUX records
    uint32_t pad_;
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
};

}  // namespace sa
