// sa_engine.hip -- host orchestration of the gfx950 block encoder and the C-ABI
// (include/seqarc_amd.h).  Replaces EncapFqzComp::doFqzEncode@0x42d2d0 for a
// batch of blocks: all blocks of a batch are encoded concurrently, every
// stream of every block on its own range-coder lane.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <memory>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <optional>
#include <sys/mman.h>
#include <unistd.h>
#include <cerrno>
#include <string>
#include <thread>
#include <vector>

#include "../../include/seqarc_amd.h"
#include "sa_align_host.h"
#include "sa_kernels.hip"
#include "sa_plan.h"

using namespace sa;

namespace {

std::atomic<uint32_t> g_grows{0};   // buffer re-allocations (each hipFree synchronises the device)
std::atomic<uint64_t> g_alloc_ns{0};  // host time in hipMalloc / hipFree (SA_TRACE)
// (sa_set_reserve) a context whose batches grow -- the command line's ramp of
// first batches -- allocates for its full batch from the first one: a
// re-allocation's hipFree would synchronise the device under the other contexts
thread_local double g_reserve_scale = 1.0;

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes)
    {
        if (bytes <= cap && p) return hipSuccess;
        const auto t0 = std::chrono::steady_clock::now();
        if (p) {
            (void)hipFree(p);
            g_grows++;
        }
        p = nullptr;
        // slack for the next, slightly larger batch: a re-allocation's hipFree
        // synchronises the whole device, stalling every other context on it
        // (the reserve scale gets the same slack on top: a full batch of the
        // command line's ramp can need a little more than scale x a ramp batch,
        // e.g. the exact payload arena, and a grow then stalled every context
        // for 1.5 s, round 3 g3m)
        const size_t scaled = g_reserve_scale > 1.0 ? (size_t)((double)bytes * g_reserve_scale) : bytes;
        size_t want = std::max(scaled + scaled / 16, cap + cap / 16);
        want = std::max<size_t>(want, 256);
        hipError_t e = hipMalloc(&p, want);
        cap = e == hipSuccess ? want : 0;
        g_alloc_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now() - t0).count();
        return e;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct ReserveScope {   // g_reserve_scale for one call on a batch of nbk blocks
    explicit ReserveScope(uint32_t reserve_blocks, uint32_t nbk)
    {
        g_reserve_scale = reserve_blocks > nbk && nbk ? (double)reserve_blocks / nbk : 1.0;
    }
    ~ReserveScope() { g_reserve_scale = 1.0; }
};

// Device time of each phase of the last sa_run, from HIP events on the stream
// the phase runs on.  MD5 runs on its own stream concurrently with the
// others; "total" is the wall time of the whole batch.
const char* kPhaseNames[] = {"prep+scan", "emit", "sort_seq", "sort_aux", "replay_seq", "replay_aux", "coder_r",
                             "coder_l", "md5", "assemble", "total"};
enum { PH_PREP, PH_EMIT, PH_SORT_SEQ, PH_SORT_AUX, PH_REPLAY_SEQ, PH_REPLAY_AUX, PH_CODER_R, PH_CODER_L, PH_MD5,
       PH_ASM, PH_TOTAL, PH_N };

}  // namespace

// The front scratch of a device: buffers only the throughput-bound front of a
// batch uses (count columns, name prefix/suffix, the SEQ sort's key/value ping
// pong, one half of the AUX sort's, histograms, run lists of the front), shared
// by the contexts of one device that are created together (sa_create_shared).
// Their fronts run one at a time -- they are throughput-bound, two at once only
// slow each other -- while each context's latency-bound part (long model runs,
// range-coder chains, MD5) overlaps the next context's front.  `mu` is held
// while a context enqueues its front; its stream first waits for `ev_free`,
// recorded after the previous front's last kernel.
struct FrontShare {
    int refs = 0;
    // the front is taken in arrival order (a ticket lock): std::mutex lets a
    // returning thread barge in, and in the command line's pipeline some
    // contexts waited 2+ s for their turn while others went again (r3b trace)
    std::mutex mu;
    std::condition_variable turn_cv;
    uint64_t next_ticket = 0, serving = 0;
    hipEvent_t ev_free = nullptr;
    bool have_ev = false;
    std::atomic<int> tails{0};   // contexts of the device inside coder_run (pass R in flight)
    DBuf d_seq_k[2], d_seq_v[2], d_auxs_k, d_auxs_v;
    DBuf d_bkt_spare;   // (k_replay_seq_bkt: the inactive lanes' record stores)
    DBuf d_bkt_order;   // (k_bkt_order: the digits, largest first)
    DBuf d_hist_seq, d_hist_aux, d_segs_seq, d_segs_aux, d_tile_seq, d_tile_aux, d_seq_longs, d_nseq_long, d_short_at;
    std::vector<DBuf*> buffers()
    {
        return {&d_seq_k[0], &d_seq_k[1], &d_seq_v[0], &d_seq_v[1], &d_auxs_k, &d_auxs_v, &d_hist_seq, &d_hist_aux,
                &d_segs_seq, &d_segs_aux, &d_tile_seq, &d_tile_aux, &d_seq_longs, &d_nseq_long, &d_short_at,
                &d_bkt_spare, &d_bkt_order};
    }
    uint64_t held_bytes()
    {
        uint64_t h = 0;
        for (DBuf* b : buffers()) h += b->cap;
        return h;
    }
};
std::mutex g_share_mu;   // FrontShare::refs

// RAII turn on a FrontShare's front (FIFO)
struct FrontTurn {
    FrontShare* F = nullptr;
    hipStream_t st = nullptr;   // the stream the holder enqueues its front on
    bool held = false;
    bool freed = false;         // F->ev_free recorded after this front's last kernel
    FrontTurn(FrontShare* f, hipStream_t s) : F(f), st(s)
    {
        std::unique_lock<std::mutex> lk(F->mu);
        const uint64_t t = F->next_ticket++;
        F->turn_cv.wait(lk, [&] { return F->serving == t; });
        held = true;
    }
    void unlock()
    {
        if (!held) return;
        // an early exit (error) after front kernels were queued: the next front
        // must still wait for them before it reuses the shared scratch
        if (!freed && hipEventRecord(F->ev_free, st) == hipSuccess) {
            F->have_ev = true;
            freed = true;
        }
        {
            std::lock_guard<std::mutex> g(F->mu);
            F->serving++;
        }
        F->turn_cv.notify_all();
        held = false;
    }
    ~FrontTurn() { unlock(); }
};

// A batch of parsed blocks resident in HBM (names, bases, qualities and the
// per-read offsets), read-only while it is encoded: any number of contexts of
// its device may encode it, one after the other or concurrently.
struct sa_input {
    int device = 0;
    std::vector<DevBlock> blocks;   // layout fields only (the symbol spaces are per run)
    uint32_t nblocks = 0, nreads = 0;
    uint64_t names_bytes = 0, seq_bytes = 0, text_bytes = 0;
    DBuf d_names, d_seq, d_qual, d_read_block, d_name_off, d_name_len, d_seq_off, d_seq_len;
    std::vector<uint32_t> h_read_block, h_name_off, h_seq_off, h_seq_len;
    std::vector<uint16_t> h_name_len;
    // sa_stage_text: the texts and the device parse's scratch (sa_parse.hip)
    DBuf d_text, d_tile_text, d_tile_cnt, d_tile_base, d_ptexts, d_ntiles, d_text_nl, d_pblocks, d_btot, d_perr, d_nl,
        d_src;
    DBuf d_text_b;   // (round 6) the second text arena of sa_text_upload / sa_text_parse (slot 1)
    ~sa_input()
    {
        for (DBuf* b : {&d_names, &d_seq, &d_qual, &d_read_block, &d_name_off, &d_name_len, &d_seq_off, &d_seq_len,
                        &d_text, &d_tile_text, &d_tile_cnt, &d_tile_base, &d_ptexts, &d_ntiles, &d_text_nl, &d_pblocks,
                        &d_btot, &d_perr, &d_nl, &d_src, &d_text_b})
            b->release();
    }
};

struct sa_ctx {
    int device = 0;
    // main/AUX, MD5, SEQ path (CU-masked), long AUX runs (CU-masked, disjoint)
    hipStream_t st = nullptr, st2 = nullptr, st3 = nullptr, st4 = nullptr;
    // SA_L_CU_EVERY=N (N >= 2): the L passes of the coder (L1 / L2 / L3) on a
    // stream of their own, masked to every N-th CU, after the host has seen
    // pass R end (the L passes are throughput kernels: on pass R's CUs they
    // take the whole GPU for ~40 ms per batch and the other batches' front
    // kernels beside them run ~3x slower, round 4 r4c trace).  0: after pass R
    // on its stream (st3).
    hipStream_t st5 = nullptr;
    hipEvent_t ev_r_done = nullptr;
    // (round 6) sa_text_upload's copies: a stream of their own, made on first
    // use (from whichever thread uploads), so the next batch's texts go to the
    // device while this context's kernels run
    hipStream_t st_copy = nullptr;
    std::mutex copy_mu;
    // the dense AUX sort (k_aux_presence / k_aux_dense: one 9-bit pass over the
    // blocks' dense model ids instead of two over the 17-bit ids).  The emit's
    // target buffer depends on the number of passes, so the batch follows this
    // context's previous one: a batch with more than 512 models in a block sorts
    // in two dense passes and a copy, and turns it off.  SA_AUX_DENSE=0: off.
    bool aux_dense = !(std::getenv("SA_AUX_DENSE") && std::atoi(std::getenv("SA_AUX_DENSE")) == 0);
    DBuf d_aux_bm, d_aux_tab, d_aux_nmod;
    uint32_t* h_aux_nmod = nullptr;   // (pinned)
    size_t h_aux_nmod_cap = 0;
    hipEvent_t ev_dense = nullptr;
    hipEvent_t ev_fork = nullptr, ev_fork_seq = nullptr, ev_md5_done = nullptr, ev_r[2] = {nullptr, nullptr};
    hipEvent_t ev_seq_done = nullptr, ev_long_done = nullptr;
    // the AUX record array is all zero between batches (pass R's unwritten-record
    // test): zeroed in the tail of the batch that used it (st3, after the L
    // passes), not in the front turn; prs_zero_cap = its bytes known zero,
    // ev_prs_zero = that tail memset
    hipEvent_t ev_prs_zero = nullptr;
    size_t prs_zero_cap = 0;
    void* prs_zero_p = nullptr;
    bool prs_zero_pending = false;
    uint32_t long_lds = 0;
    bool serial_seq = false;
    uint32_t chain_prio = 1;   // s_setprio 3 in the latency-bound chain kernels (SA_CHAIN_PRIO=0: off)
    uint32_t md5_prio = 1;     // ... and in k_md5 (SA_MD5_PRIO; off the critical path)
    bool prep_fused = std::getenv("SA_PREP_FUSED") != nullptr;   // name columns in k_prep_sq16 (A/B)
    bool prep_wave = std::getenv("SA_PREP_WAVE") != nullptr;   // k_prep_sq instead of k_prep_sq16
    bool emit_wave = std::getenv("SA_EMIT_WAVE") != nullptr;
    uint32_t reserve_blocks = 0;   // sa_set_reserve: the batch size to allocate for
    bool front_warm = false;       // a batch ran: its buffers exist (run_input's `early`)
    // records per chunk in the L passes (SA_L_CHUNK=16: 56 VGPRs, 8 waves per
    // SIMD, half a line per chunk; 32: 88 VGPRs, 5 waves, a whole line)
    uint32_t l_chunk = std::getenv("SA_L_CHUNK") && std::atoi(std::getenv("SA_L_CHUNK")) == 16 ? 16u : 32u;
    // the L passes at issue priority 2 (they are on the batch's critical path,
    // the other contexts' fronts beside them are not always; SA_L_PRIO=1, A/B)
    uint32_t l_prio = std::getenv("SA_L_PRIO") && std::atoi(std::getenv("SA_L_PRIO")) != 0 ? 1u : 0u;
    bool seq_unpacked = std::getenv("SA_SEQ_PACK") && std::atoi(std::getenv("SA_SEQ_PACK")) == 0;
    // k_prep_sq16 / k_emit_sq16 with the round-4 static grid stride instead of
    // reads taken from a counter (WaveReads; SA_FRONT_STATIC=1, A/B)
    bool front_static = std::getenv("SA_FRONT_STATIC") && std::atoi(std::getenv("SA_FRONT_STATIC")) != 0;
    // reads a front wave takes from the counter at a time (WaveReads): 0 = by the
    // batch's mean read length (front_wq_chunk), SA_WQ_CHUNK=n to fix it (A/B;
    // 64 was the only value until round 6)
    uint32_t wq_chunk_env = std::getenv("SA_WQ_CHUNK") ? (uint32_t)std::atoi(std::getenv("SA_WQ_CHUNK")) : 0u;
    // pass R with one chain per lane in the VALU (k_coder_rl: the scalar units
    // stay free for the front kernels of the other batches) instead of one
    // chain per wave on the scalar unit (k_coder_rv); SA_RV_LANES=1 / 0.  Off:
    // pass R 1,835-1,864 against 679-689 ms under the bench's load, the bench
    // 7,971-8,064 against 16,849-16,908 MB/s (r5k)
    bool rv_lanes = std::getenv("SA_RV_LANES") && std::atoi(std::getenv("SA_RV_LANES")) != 0;
    // the SEQ space sorted by the context's low 8-9 bits only and replayed per
    // bucket with the models in LDS (k_replay_seq_bkt, contexts of <= 22 bits);
    // SA_SEQ_BUCKET=0: the full sort and k_replay_seq.  By the low bits the
    // bench gained 1-3 % (r5k: 17,039 / 17,349 against 16,908 / 16,849 MB/s,
    // SEQ sort + replay 84 against 88-98 ms); by the top bits it had lost
    // (r5e-r5h: 14.9-15.4 against 15.9-16.8 GB/s)
    bool seq_bucket = !(std::getenv("SA_SEQ_BUCKET") && std::atoi(std::getenv("SA_SEQ_BUCKET")) == 0);
    // the bucket replay's records in sorted order (coalesced stores), then put
    // in stream order by a gather through the sort's inverse permutation, which
    // the bucket pass writes in stream order instead of the positions
    // (k_seq_unpermute); SA_SEQ_INV=0: one scattered 4-byte store per symbol
    bool seq_inv = !(std::getenv("SA_SEQ_INV") && std::atoi(std::getenv("SA_SEQ_INV")) == 0);
    // SA_BKT_DB=8 / 9 / 10: the bucket pass's digit bits (default 8 for contexts
    // of <= 20 bits, 9 above; 10 with the inverse-permutation pass only)
    int bkt_db_env = std::getenv("SA_BKT_DB") ? std::atoi(std::getenv("SA_BKT_DB")) : 0;
    int prep_row = std::getenv("SA_PREP_ROW") ? std::atoi(std::getenv("SA_PREP_ROW")) : 0;
    // the bucket replay's largest digits first (k_bkt_order); SA_BKT_LPT=0: digit order
    bool bkt_lpt = !(std::getenv("SA_BKT_LPT") && std::atoi(std::getenv("SA_BKT_LPT")) == 0);
    // SA_BKT_PROBE=file: per bucket-replay wave its clocks and steps, appended
    // to file (the front waits for the replay to read them back: diagnostics)
    const char* bkt_probe = std::getenv("SA_BKT_PROBE");
    DBuf d_bkt_probe;
    // workgroups per CU of the grid-stride wave-per-read kernels (SA_WAVE_GRID)
    uint32_t wg_per_cu = std::getenv("SA_WAVE_GRID") ? (uint32_t)std::max(1, std::atoi(std::getenv("SA_WAVE_GRID"))) : 8u;
    // k_md5<true> reads the next block's words while the chain runs: 148 VGPRs instead
    // of 60, which costs the co-resident front kernels more than it saves (r2x:
    // 11.6 vs 12.9 GB/s), so SA_MD5_PIPE=1 only
    bool md5_pipe = std::getenv("SA_MD5_PIPE") && std::atoi(std::getenv("SA_MD5_PIPE")) != 0;
    // pass-R placement (k_coder_rv): four chains per workgroup, one per SIMD, and
    // enough unused LDS that a CU holds one pass-R workgroup (SA_CODER_WAVES /
    // SA_CODER_LDS)
    // The waits between this context's streams happen on the host thread (which
    // has nothing else to do then) instead of as barrier packets: the boxes run
    // with four hardware queues per process (GPU_MAX_HW_QUEUES=4), so the
    // contexts' streams share queues, and a barrier waiting for this batch's
    // front or long runs held up every other context's work queued behind it
    // (pass R, L passes).  SA_HOST_WAITS=0: device-side waits, for A/B.
    bool host_waits = !(std::getenv("SA_HOST_WAITS") && std::atoi(std::getenv("SA_HOST_WAITS")) == 0);
    uint32_t coder_waves = 4;
    // the pass-R step order (k_coder_rv<V>): 5 = the 24 v_readlane of eight steps
    // issued together ahead of their SALU steps (r4z3: pass R 671-675 against
    // 767-776 ms, the bench +3-5 %); 0 = a step's three v_readlane ahead of it.
    // The batched moves hold the vector unit of their SIMD longer, and batches
    // of long reads (mean > 1000 bp), whose fronts are VALU-heavy and set the
    // pace, ran 11 % slower with them (r4z5: ONT shape 7,187 / 7,281 against
    // 8,081 / 8,260 MB/s), so those keep 0.  SA_RV_VARIANT=0 / 5: one for all.
    // Round 6: 6 = the operands through SMEM from a per-wave ring the lanes fill
    // (k_coder_rv<6>, coder_rg_chain): the chain itself is faster (r6b: one
    // context alone 504 against 630 ms; under the bench's load 626-644 against
    // 665-691) but it issues 10 SALU per symbol instead of 8 and holds its SIMD's
    // scalar issue ~90 % of the time, so the kernels that share those SIMDs
    // slow (L passes 89 against 52 ms, prep 16 against 10) and the bench lost
    // 3 % (r6b / r6c: 16,623-16,904 against 17,281-17,493 MB/s).  On the tree
    // with the full-segment L passes the bench is level (r6m: 19,301 / 19,237
    // against 19,437 / 19,279) and the command line, whose batches' latency
    // sets its pace, faster: 42.8 GB in 3.47 / 3.53 s against 4.22 / 3.89 s
    // (r6o); and in r6q the bench too (19,339 / 19,422 against 18,386 /
    // 18,851 MB/s), so 6 is the default for short-read batches since round 6.
    int rv_variant = std::getenv("SA_RV_VARIANT") ? std::atoi(std::getenv("SA_RV_VARIANT")) : -1;
    // (default variant, A/B) 6 only while at most SA_RV_V6_MAX other contexts of
    // the device are in pass R, else 5; -1: 5 always.  Unset: 6 always -- the
    // limit measured no better (r6q: bench 19,106 / 19,264 with 2, 18,386 /
    // 18,851 with -1, 19,339 / 19,422 without; 42.8 GB in 5.02 / 4.28 s with 2,
    // 4.44 / 4.11 with -1, 4.35 / 4.17 without)
    int rv_v6_max = std::getenv("SA_RV_V6_MAX") ? std::atoi(std::getenv("SA_RV_V6_MAX")) : 1 << 30;
    int rv_batch = 5;   // the current batch's (run_input)
    // pass R's wait for records the long runs have not written (SA_RV_WAIT_MS, default 20 s: the
    // long runs take ~0.4 s; a wave that waits longer gives up and the batch fails with E_CODER)
    uint32_t rv_wait_ticks = std::getenv("SA_RV_WAIT_MS")
                                 ? (uint32_t)std::min<uint64_t>(100000ull * (uint64_t)std::max(1, std::atoi(std::getenv("SA_RV_WAIT_MS"))),
                                                                4000000000ull)
                                 : 2000000000u;
    bool test_skip_long = std::getenv("SA_TEST_SKIP_LONG") != nullptr;   // (tests: starve pass R)
    uint32_t rv_short_waves = std::getenv("SA_RV_SHORT_WAVES") ? (uint32_t)std::atoi(std::getenv("SA_RV_SHORT_WAVES")) : 32u;
    // k_replay_aux_long workgroups: what the long-run CUs hold at once (6 per CU;
    // SA_LONG_GRID overrides, round 2 used 2048)
    uint32_t long_grid = 0;
    uint32_t coder_lds = 82 * 1024;
    std::string err;
    bool timing = false;
    bool trace = std::getenv("SA_TRACE") != nullptr;
    // pinned host mailbox for the run's small copies (plans, task lists, count
    // and length read-backs): a pageable copy goes through the runtime's
    // staging path, which the other contexts' bulk copies hold up; bump
    // allocation, reset at the start of a run (no copy of the previous run is
    // in flight then); D2H copies land in it and reach their destination at the
    // next sync_d2h
    uint8_t* mail = nullptr;
    size_t mail_cap = 0, mail_used = 0, mail_high = 16u << 20;   // (16 MiB from the first run on)
    std::vector<uint8_t*> mail_retired;   // outgrown mailboxes, freed in the destructor
    struct Pending {
        void* dst;
        const void* src;
        size_t n;
    };
    std::vector<Pending> pending;
    uint32_t n_cu = 256;
    uint32_t coder_restarts = 0;
    uint64_t max_stream_syms = 0, total_stream_syms = 0;
    hipEvent_t ev_beg[PH_N] = {}, ev_end[PH_N] = {};
    float ph_ms[PH_N];
    float align_kernel_ms = 0.f;   // sa_hash_align: the aligner kernel of the last call (variant 0)
    // SA_RV_PROBE=file: per pass-R wave its timing and placement, appended to
    // the file per batch (diagnostics, k_coder_rv)
    const char* rv_probe = std::getenv("SA_RV_PROBE");
    DBuf d_probe;
    uint32_t probe_waves = 0;
    DBuf d_ring;   // pass R's per-wave operand rings (k_coder_rv<6>)

    // the batch sa_stage uploads (sa_run encodes it); blocks = the working copy
    // of the batch being encoded (its symbol spaces filled by plan_batch)
    sa_input own;
    std::vector<DevBlock> blocks;

    // work
    FrontShare* fs = nullptr;   // front scratch, possibly shared with other contexts of the device
    DBuf d_blocks, d_totals, d_err;
    DBuf d_auxp_k, d_auxp_v, d_prs_seq, d_prs_aux, d_cum_seq, d_cum_aux;   // d_auxp: the sorted AUX keys/values
    DBuf d_task_ends;
    DBuf d_tasks, d_out_len, d_payload, d_md5tasks, d_digests, d_asm, d_asm_copies, d_task_out_base, d_final, d_final_len;
    DBuf d_longs, d_huge_sorted, d_nlong;
    DBuf d_ck, d_maps, d_low_at, d_off_at, d_first_sq;
    DBuf d_list_ids[2], d_list_gbase[2], d_list_run[2];
    DBuf d_dege_list;   // the reads with N / IUPAC bases (k_dege_list -> k_emit_sq)
    DBuf d_qual_q, d_rb_chunks, d_rb_ck0, d_rb_opens, d_rb_spec, d_rb_entry, d_rb_guess, d_rb_tab;   // -l (rblock)
    DBuf d_rb_vals, d_rb_info;   // (round 5: run values per chunk byte, RbInfo per chunk)
    // SA_RB_APPLY=1: the round-4 second full walk (k_rb_apply) instead of k_rb_true + k_rb_fill (A/B)
    bool rb_apply_walk = std::getenv("SA_RB_APPLY") && std::atoi(std::getenv("SA_RB_APPLY")) != 0;
    // SA_RB_FIX_SERIAL=1: the entries by k_rb_fix (a lane per block, chunk by
    // chunk) instead of k_rb_fix_w (a wave per block, 64 chunks a step; A/B)
    bool rb_fix_serial = std::getenv("SA_RB_FIX_SERIAL") && std::atoi(std::getenv("SA_RB_FIX_SERIAL")) != 0;
    // k_rb_spec on n workgroups per CU taking 64 chunks at a time from a
    // counter (round 6: n = 2, the ONT batch's prep+scan 25.0 / 26.4 against
    // 28.6 / 29.7 ms with one grid of a lane per chunk, r6z8; 4: no gain);
    // SA_RB_SPEC_WG=n to change, 0 = the one grid
    uint32_t rb_spec_wg = std::getenv("SA_RB_SPEC_WG") ? (uint32_t)std::max(0, std::atoi(std::getenv("SA_RB_SPEC_WG"))) : 2u;
    // R-Block chunk length, also the stride of the per-chunk arrays (opens,
    // vals): SA_RB_CHUNK=n, a multiple of 32 up to RB_CHUNK.  Not a power of
    // two: the lanes of k_rb_spec walk their chunks in step, so at 8192 every
    // lane's load and store of a step fell on addresses 8 KiB apart (round 6)
    uint32_t rb_chunk = [] {
        const char* e = std::getenv("SA_RB_CHUNK");
        const uint32_t n = e ? (uint32_t)std::atoi(e) : RB_CHUNK_DEFAULT;
        return n >= 32 && n <= RB_CHUNK && n % 32 == 0 ? n : RB_CHUNK;
    }();
    std::vector<uint32_t> rb_tab_host;   // the R decision tables (RbTab) of rb_tab_r
    double rb_tab_r = -1.0;
    bool rb_tab_sent = false;
    // reference path: per read the alignment of both carried states, status, the
    // alignment columns, the SEQ skip flags (sa_hash.hip, align_front)
    // per-read counts of every column (k_prep, k_prep_sq16 -> k_scan_reads ->
    // the emitters), name prefix / suffix, the per-block running name maximum,
    // the N / IUPAC maxq: this context's own (the prep runs before its front turn)
    DBuf d_counts, d_name_p, d_name_s, d_maxlen, d_dege_maxq;
    DBuf d_al_ret[2], d_al_rev[2], d_al_pos[2], d_al_mp[2], d_al_mt[2], d_al_st, d_al_sel, d_al_scr, d_acounts, d_atot,
        d_seq_skip;
    // the last aligned batch's block plans (a re-run of the same batch -- the
    // exact-payload fallback -- reuses them instead of passing the chain again)
    const sa_input* al_input = nullptr;
    uint64_t al_batch = 0;
    std::vector<uint32_t> al_plan;   // per block: order count, win, ibits, insert bits

    // last run
    std::vector<uint64_t> final_base, final_len;
    bool have_output = false;

    std::vector<DBuf*> work_buffers()
    {
        return {&d_blocks, &d_totals, &d_err, &d_auxp_k, &d_auxp_v, &d_prs_seq, &d_prs_aux, &d_cum_seq, &d_cum_aux,
                &d_task_ends, &d_tasks, &d_out_len, &d_payload, &d_md5tasks, &d_digests, &d_asm, &d_asm_copies, &d_task_out_base,
                &d_final, &d_final_len, &d_longs, &d_huge_sorted, &d_nlong, &d_ck, &d_maps, &d_low_at, &d_off_at,
                &d_dege_list, &d_qual_q, &d_rb_chunks, &d_rb_ck0, &d_rb_opens, &d_rb_spec, &d_rb_entry, &d_rb_guess, &d_rb_tab, &d_rb_vals, &d_rb_info, &d_first_sq,
                &d_list_ids[0], &d_list_gbase[0], &d_list_run[0], &d_list_ids[1], &d_list_gbase[1], &d_list_run[1],
                &d_al_ret[0], &d_al_rev[0], &d_al_pos[0], &d_al_mp[0], &d_al_mt[0], &d_al_ret[1], &d_al_rev[1],
                &d_al_pos[1], &d_al_mp[1], &d_al_mt[1], &d_al_st, &d_al_sel, &d_al_scr, &d_acounts, &d_atot,
                &d_seq_skip, &d_counts, &d_name_p, &d_name_s, &d_maxlen, &d_dege_maxq, &d_probe, &d_bkt_probe, &d_ring, &d_aux_bm,
                &d_aux_tab, &d_aux_nmod};
    }
    uint64_t held_bytes()
    {
        uint64_t h = own.d_names.cap + own.d_seq.cap + own.d_qual.cap;
        for (DBuf* b : work_buffers()) h += b->cap;
        return h;   // (the front scratch: front_bytes)
    }

    ~sa_ctx()
    {
        if (fs) {
            std::lock_guard<std::mutex> g(g_share_mu);
            if (--fs->refs == 0) {
                for (DBuf* b : fs->buffers()) b->release();
                if (fs->ev_free) (void)hipEventDestroy(fs->ev_free);
                delete fs;
            }
            fs = nullptr;
        }
        std::vector<DBuf*> all = work_buffers();
        for (DBuf* b : all) b->release();
        for (int i = 0; i < PH_N; i++) {
            if (ev_beg[i]) (void)hipEventDestroy(ev_beg[i]);
            if (ev_end[i]) (void)hipEventDestroy(ev_end[i]);
        }
        for (hipEvent_t e : {ev_fork, ev_fork_seq, ev_md5_done, ev_r[0], ev_r[1], ev_seq_done, ev_long_done, ev_prs_zero})
            if (e) (void)hipEventDestroy(e);
        if (mail) (void)hipHostFree(mail);
        for (uint8_t* m : mail_retired) (void)hipHostFree(m);
        if (st) (void)hipStreamDestroy(st);
        if (st2) (void)hipStreamDestroy(st2);
        if (st3) (void)hipStreamDestroy(st3);
        if (st4) (void)hipStreamDestroy(st4);
        if (st5) (void)hipStreamDestroy(st5);
        if (st_copy) (void)hipStreamDestroy(st_copy);
        if (ev_r_done) (void)hipEventDestroy(ev_r_done);
        if (ev_dense) (void)hipEventDestroy(ev_dense);
        if (h_aux_nmod) (void)hipHostFree(h_aux_nmod);
    }
};

#define SA_CHECK(ctx, expr)                                                              \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);              \
            return -1;                                                                   \
        }                                                                                \
    } while (0)

namespace {

// ---- the pinned mailbox (sa_ctx::mail) ----
// Starts a run's use of the mailbox: grows it (to the previous runs' high-water
// mark) while nothing of this context is in flight.
int mail_reset(sa_ctx* c)
{
    c->pending.clear();
    c->mail_used = 0;
    const size_t want = std::max<size_t>(c->mail_high + c->mail_high / 8, 1u << 20);
    if (want > c->mail_cap) {
        // the old one is retired, not freed: hipHostFree waits for the whole
        // device, i.e. for every other context's work in flight
        if (c->mail) c->mail_retired.push_back(c->mail);
        c->mail = nullptr;
        c->mail_cap = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&c->mail), want, hipHostMallocDefault) != hipSuccess) {
            c->mail = nullptr;
            return 0;   // (copies fall back to pageable memory)
        }
        c->mail_cap = want;
    }
    return 0;
}

uint8_t* mail_take(sa_ctx* c, size_t n)
{
    const size_t at = align_up(c->mail_used, 64);
    c->mail_high = std::max(c->mail_high, at + n);
    if (!c->mail || at + n > c->mail_cap) return nullptr;
    c->mail_used = at + n;
    return c->mail + at;
}

// host -> device through the mailbox (the source may be reused at once)
hipError_t h2d(sa_ctx* c, void* dst, const void* src, size_t n, hipStream_t st)
{
    if (!n) return hipSuccess;
    uint8_t* m = mail_take(c, n);
    if (!m) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
    std::memcpy(m, src, n);
    return hipMemcpyAsync(dst, m, n, hipMemcpyHostToDevice, st);
}

// device -> host through the mailbox: `dst` holds the bytes after sync_d2h
hipError_t d2h(sa_ctx* c, void* dst, const void* src, size_t n, hipStream_t st)
{
    if (!n) return hipSuccess;
    uint8_t* m = mail_take(c, n);
    if (!m) return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, st);
    c->pending.push_back(sa_ctx::Pending{dst, m, n});
    return hipMemcpyAsync(m, src, n, hipMemcpyDeviceToHost, st);
}

hipError_t sync_d2h(sa_ctx* c, hipStream_t st)
{
    const hipError_t e = hipStreamSynchronize(st);
    for (const sa_ctx::Pending& p : c->pending) std::memcpy(p.dst, p.src, p.n);
    c->pending.clear();
    return e;
}

// Reads per take of the front kernels' read counter: ~64 reads' worth of
// 150 bp (about 10 KB of bases) a take, so short-read batches keep WQ_CHUNK
// and long-read batches take one wave's four reads at a time; a multiple of
// four (the rows of a wave).
uint32_t front_wq_chunk(const sa_ctx* c, uint64_t seq_bytes, uint32_t nreads)
{
    if (c->wq_chunk_env) return std::max<uint32_t>(4, std::min<uint32_t>(1024, c->wq_chunk_env & ~3u));
    const uint64_t mean = nreads ? std::max<uint64_t>(1, seq_bytes / nreads) : 1;
    const uint64_t k = (uint64_t)WQ_CHUNK * 150 / mean;
    return (uint32_t)std::max<uint64_t>(4, std::min<uint64_t>(WQ_CHUNK, k) & ~3ull);
}

// grid of a wave-per-read, grid-stride kernel (EMIT_WAVES waves per workgroup):
// 8 workgroups per CU, fewer for a small batch
uint32_t wave_grid(const sa_ctx* c, uint32_t nreads)
{
    return std::max<uint32_t>(1, std::min<uint32_t>((nreads + EMIT_WAVES - 1) / EMIT_WAVES, c->wg_per_cu * c->n_cu));
}

// Digit widths of a sort over bits [lo, hi): the fewest passes of at most
// SORT_MAX_DB bits, widths as even as possible and at least SORT_MIN_DB (a
// digit may reach above hi: those key bits are 0, or 1 in the pad keys, which
// sort last anyway).
std::vector<int> sort_digits(int lo, int hi, int max_db = SORT_MAX_DB)
{
    std::vector<int> w;
    if (hi <= lo) return w;
    static const int min_db = std::getenv("SA_SORT_MIN_DB") ? std::max(7, std::min(9, std::atoi(std::getenv("SA_SORT_MIN_DB"))))
                                                           : SORT_MIN_DB;
    const int bits = hi - lo, passes = (bits + max_db - 1) / max_db;
    for (int p = 0, done = 0; p < passes; p++) {
        const int d = (bits - done + (passes - p) - 1) / (passes - p);
        w.push_back(std::max(d, min_db));
        done += d;
    }
    return w;
}

// histogram words per tile of a sort over bits [lo, hi)
uint64_t sort_hist_per_tile(int lo, int hi, int max_db = SORT_MAX_DB)
{
    int m = 0;
    for (int d : sort_digits(lo, hi, max_db)) m = std::max(m, d);
    return 1ull << m;
}

template <int DB>
void sort_pass(hipStream_t st, const SortView& sv, const uint32_t* kin, const uint32_t* vin, uint32_t* kout,
               uint32_t* vout, uint32_t shift, bool wide, bool inv = false)
{
    const dim3 hgrid((sv.ntiles + HIST_TILES - 1) / HIST_TILES);
    if (sv.dense)
        hipLaunchKernelGGL((k_sort_hist<DB, true>), hgrid, dim3(SORT_THREADS), 0, st, sv, kin, shift);
    else
        hipLaunchKernelGGL((k_sort_hist<DB, false>), hgrid, dim3(SORT_THREADS), 0, st, sv, kin, shift);
    hipLaunchKernelGGL(k_sort_scan<DB>, dim3(sv.nsegs), dim3(1024), 0, st, sv);
    // (vin = nullptr: the values are the elements' index, IDX)
    auto scatter = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(sv.ntiles), dim3(SORT_THREADS), 0, st, sv, kin, vin, kout, vout, shift); };
    if (wide) {
        if (vin) scatter(k_sort_scatter<DB, true, false, false>);
        else scatter(k_sort_scatter<DB, true, false, true>);
    } else if (sv.dense) {
        if (vin) scatter(k_sort_scatter<DB, false, true, false>);
        else scatter(k_sort_scatter<DB, false, true, true>);
    } else if (inv) {   // (one pass over implicit values: run_sort checks)
        scatter(k_sort_scatter<DB, false, false, true, true>);
    } else {
        if (vin) scatter(k_sort_scatter<DB, false, false, false>);
        else scatter(k_sort_scatter<DB, false, false, true>);
    }
}

// sorts keys by bits [lo, hi) (bits below lo ride along); the result is in
// keys[result_buf] / vals[result_buf]
// index_vals: the input values are each element's index in its segment and are
// not read (the first pass computes them)
// dense: the AUX space by dense model ids (k_aux_dense's tables; bits
// [lo, hi) of the dense id)
int run_sort(sa_ctx* c, hipStream_t st, const SortPlan& plan, DBuf& segs, DBuf& tiles, DBuf& hist,
             DBuf* const* keys, DBuf* const* vals, int lo, int hi, int& result_buf, bool index_vals = false,
             const uint64_t* dense = nullptr, bool inv_vals = false, int max_db = SORT_MAX_DB)
{
    result_buf = 0;
    if (plan.total && hi <= lo && index_vals) {
        c->err = "internal: a sort without passes over implicit values";
        return -1;
    }
    if (plan.total == 0 || hi <= lo) return 0;
    SortView sv{};
    sv.segs = segs.as<SortSeg>();
    sv.tile_seg = tiles.as<uint32_t>();
    sv.hist = hist.as<uint32_t>();
    sv.total = plan.total;
    sv.ntiles = (uint32_t)plan.tile_seg.size();
    sv.nsegs = (uint32_t)plan.segs.size();
    sv.dense = dense;
    // a segment of >= 2^30 keys needs 64-bit offsets in the scatter (the HASH
    // index of a genome > 2^31 bases: one segment of all its seeds)
    bool wide = false;
    for (const SortSeg& g : plan.segs) {
        wide |= (uint64_t)g.ntiles * SORT_TILE >= (1ull << 30);
        if ((uint64_t)g.ntiles * SORT_TILE >= (1ull << 32)) {
            c->err = "sort segment of 2^32 keys or more";
            return -1;
        }
    }
    if (inv_vals && (!index_vals || wide || dense || sort_digits(lo, hi, max_db).size() != 1)) {
        c->err = "internal: an inverse-permutation sort that is not one plain pass over implicit values";
        return -1;
    }
    if (wide && dense) {
        c->err = "internal: a dense sort of a segment of 2^30 keys or more";
        return -1;
    }
    int cur = 0, shift = lo;
    for (const int db : sort_digits(lo, hi, max_db)) {
        const uint32_t* kin = keys[cur]->as<uint32_t>();
        const uint32_t* vin = index_vals && shift == lo ? nullptr : vals[cur]->as<uint32_t>();
        uint32_t* kout = keys[cur ^ 1]->as<uint32_t>();
        uint32_t* vout = vals[cur ^ 1]->as<uint32_t>();
        if (db == 7) sort_pass<7>(st, sv, kin, vin, kout, vout, (uint32_t)shift, wide, inv_vals);
        else if (db == 8) sort_pass<8>(st, sv, kin, vin, kout, vout, (uint32_t)shift, wide, inv_vals);
        else if (db == 9) sort_pass<9>(st, sv, kin, vin, kout, vout, (uint32_t)shift, wide, inv_vals);
        else if (db == 10 && inv_vals) sort_pass<10>(st, sv, kin, vin, kout, vout, (uint32_t)shift, false, true);
        else {
            c->err = "internal: no sort pass of this digit width";
            return -1;
        }
        shift += db;
        cur ^= 1;
    }
    SA_CHECK(c, hipGetLastError());
    result_buf = cur;
    return 0;
}

void ev_begin(sa_ctx* c, int ph, hipStream_t st);
void ev_finish(sa_ctx* c, int ph, hipStream_t st);

// -l R: the R-Block pre-pass (rblock@0x426c10) of every block's qualities into
// d_qual_q, which the QUAL stream then codes (speculative chunks, one carry
// lane per block, chunk replay; sa_logic.h).  The staged qualities stay
// untouched: the N/IUPAC side streams use them, and the batch can be re-run.
int run_rblock(sa_ctx* c, double ratio, uint64_t seq_bytes, BatchView& bv)
{
    hipStream_t st = c->st;
    std::vector<RbChunk> ck;
    std::vector<uint32_t> ck0;
    for (const DevBlock& d : c->blocks) {
        ck0.push_back((uint32_t)ck.size());
        for (uint64_t o = 0; o < d.seq_bytes; o += c->rb_chunk) {
            const uint32_t len = (uint32_t)std::min<uint64_t>(c->rb_chunk, d.seq_bytes - o);
            uint32_t fl = (o == 0 ? RB_FIRST : 0u) | (o + len == d.seq_bytes ? RB_LAST : 0u);
            ck.push_back(RbChunk{d.seq_base + o, len, fl});
        }
    }
    ck0.push_back((uint32_t)ck.size());
    const uint32_t nck = (uint32_t)ck.size(), nbk = (uint32_t)c->blocks.size();
    SA_CHECK(c, c->d_qual_q.ensure(seq_bytes + 64));
    bv.qual_q = c->d_qual_q.as<uint8_t>();
    if (!nck) return 0;
    SA_CHECK(c, c->d_rb_chunks.ensure(sizeof(RbChunk) * nck));
    SA_CHECK(c, c->d_rb_ck0.ensure(4ull * (nbk + 1)));
    SA_CHECK(c, c->d_rb_opens.ensure(4ull * RB_WORDS * nck));
    SA_CHECK(c, c->d_rb_spec.ensure(sizeof(RbRun) * nck));
    SA_CHECK(c, c->d_rb_entry.ensure(sizeof(RbRun) * nck));
    SA_CHECK(c, c->d_rb_guess.ensure(sizeof(RbRun) * nck));
    SA_CHECK(c, h2d(c, c->d_rb_chunks.p, ck.data(), sizeof(RbChunk) * nck, st));
    SA_CHECK(c, h2d(c, c->d_rb_ck0.p, ck0.data(), 4ull * (nbk + 1), st));
    // the decision tables of this R (rebuilt when R changes)
    if (c->rb_tab_r != ratio || c->rb_tab_host.empty()) {
        c->rb_tab_host.assign(2 * RB_TAB_WORDS, 0u);
        rb_tab_build(ratio, c->rb_tab_host.data(), c->rb_tab_host.data() + RB_TAB_WORDS);
        c->rb_tab_r = ratio;
        c->rb_tab_sent = false;
    }
    if (!c->d_rb_tab.p) c->rb_tab_sent = false;
    SA_CHECK(c, c->d_rb_tab.ensure(8ull * RB_TAB_WORDS));
    if (!c->rb_tab_sent) {   // (through the mailbox, once per R)
        SA_CHECK(c, h2d(c, c->d_rb_tab.p, c->rb_tab_host.data(), 8ull * RB_TAB_WORDS, st));
        c->rb_tab_sent = true;
    }
    const uint32_t* tab = c->d_rb_tab.as<uint32_t>();
    const RbChunk* dck = c->d_rb_chunks.as<RbChunk>();
    const uint32_t rgrid = (nck + RB_THREADS - 1) / RB_THREADS;
    const bool walk = c->rb_apply_walk;
    if (!walk) {
        SA_CHECK(c, c->d_rb_vals.ensure((uint64_t)RB_CHUNK * nck));
        SA_CHECK(c, c->d_rb_info.ensure(sizeof(RbInfo) * nck));
    }
    uint8_t* vals = walk ? nullptr : c->d_rb_vals.as<uint8_t>();
    RbInfo* info = walk ? nullptr : c->d_rb_info.as<RbInfo>();
    const uint32_t cs = c->rb_chunk;   // (the arrays' stride per chunk: bytes, opens words * 32)
    // (rb_spec_wg workgroups per CU taking chunks from a counter; 0: one grid)
    uint32_t* wq_spec = c->rb_spec_wg > 0 ? c->d_err.as<uint32_t>() + 11 : nullptr;
    const uint32_t sgrid = wq_spec ? std::max<uint32_t>(1, std::min<uint32_t>(rgrid, c->rb_spec_wg * c->n_cu)) : rgrid;
    hipLaunchKernelGGL(k_rb_spec, dim3(sgrid), dim3(RB_THREADS), 0, st, bv.qual, dck, nck, tab,
                       c->d_rb_opens.as<uint32_t>(), c->d_rb_spec.as<RbRun>(), vals, info, cs, wq_spec);
    hipLaunchKernelGGL(k_rb_guess, dim3(rgrid), dim3(RB_THREADS), 0, st, bv.qual, dck, nck, tab,
                       c->d_rb_opens.as<uint32_t>(), c->d_rb_spec.as<RbRun>(), c->d_rb_guess.as<RbRun>(), cs);
    if (c->rb_fix_serial)
        hipLaunchKernelGGL(k_rb_fix, dim3((nbk + 63) / 64), dim3(64), 0, st, bv.qual, dck, c->d_rb_ck0.as<uint32_t>(),
                           nbk, tab, c->d_rb_opens.as<uint32_t>(), c->d_rb_spec.as<RbRun>(),
                           c->d_rb_guess.as<RbRun>(), c->d_rb_entry.as<RbRun>(), cs);
    else
        hipLaunchKernelGGL(k_rb_fix_w, dim3(nbk), dim3(64), 0, st, bv.qual, dck, c->d_rb_ck0.as<uint32_t>(), nbk, tab,
                           c->d_rb_opens.as<uint32_t>(), c->d_rb_spec.as<RbRun>(), c->d_rb_guess.as<RbRun>(),
                           c->d_rb_entry.as<RbRun>(), cs);
    if (walk) {
        hipLaunchKernelGGL(k_rb_apply, dim3(rgrid), dim3(RB_THREADS), 0, st, bv.qual, c->d_qual_q.as<uint8_t>(), dck,
                           nck, tab, c->d_rb_entry.as<RbRun>());
    } else {
        hipLaunchKernelGGL(k_rb_true, dim3(rgrid), dim3(RB_THREADS), 0, st, bv.qual, dck, nck, tab,
                           c->d_rb_opens.as<uint32_t>(), vals, info, c->d_rb_entry.as<RbRun>(), cs);
        hipLaunchKernelGGL(k_rb_fill, dim3(nck), dim3(RB_WORDS), 0, st, c->d_qual_q.as<uint8_t>(), dck,
                           c->d_rb_opens.as<uint32_t>(), vals, info, cs);
    }
    SA_CHECK(c, hipGetLastError());
    return 0;
}

int coder_buffers(sa_ctx* c, size_t ntasks, uint64_t total_segs, CoderView& cv)
{
    const uint64_t nsegs = std::max<uint64_t>(total_segs, 1);
    SA_CHECK(c, c->d_ck.ensure(nsegs * 4));
    SA_CHECK(c, c->d_maps.ensure(nsegs * sizeof(LowMap)));
    SA_CHECK(c, c->d_low_at.ensure(nsegs * 8));
    SA_CHECK(c, c->d_off_at.ensure(nsegs * 4));
    SA_CHECK(c, c->d_first_sq.ensure(4 * std::max<size_t>(ntasks, 1)));
    for (int g = 0; g < 2; g++) {
        SA_CHECK(c, c->d_list_ids[g].ensure(4 * std::max<size_t>(ntasks, 1)));
        SA_CHECK(c, c->d_list_gbase[g].ensure(8 * (ntasks + 1)));
        SA_CHECK(c, c->d_list_run[g].ensure(sizeof(CoderRun) * std::max<size_t>(ntasks, 1)));
    }
    cv.ck_r = c->d_ck.as<uint32_t>();
    cv.maps = c->d_maps.as<LowMap>();
    cv.low_at = c->d_low_at.as<uint64_t>();
    cv.off_at = c->d_off_at.as<uint32_t>();
    cv.first_sq = c->d_first_sq.as<uint32_t>();
    return 0;
}

// Uploads the list of one round (tasks ids + start states) into list slot `slot`.
int coder_list(sa_ctx* c, hipStream_t st, int slot, const std::vector<CoderTask>& tasks,
               const std::vector<uint32_t>& ids, const std::vector<CoderRun>& runs, std::vector<uint64_t>& gbase,
               TaskList& tl)
{
    const size_t cnt = ids.size();
    gbase.assign(cnt + 1, 0);
    for (size_t i = 0; i < cnt; i++) gbase[i + 1] = gbase[i] + (tasks[ids[i]].nseg - runs[i].start_seg);
    if (cnt) {
        SA_CHECK(c, h2d(c, c->d_list_ids[slot].p, ids.data(), 4 * cnt, st));
        SA_CHECK(c, h2d(c, c->d_list_gbase[slot].p, gbase.data(), 8 * (cnt + 1), st));
        SA_CHECK(c, h2d(c, c->d_list_run[slot].p, runs.data(), sizeof(CoderRun) * cnt, st));
    }
    tl = TaskList{c->d_list_ids[slot].as<uint32_t>(), c->d_list_gbase[slot].as<uint64_t>(),
                  c->d_list_run[slot].as<CoderRun>(), (uint32_t)cnt, 0u, gbase[cnt]};
    return 0;
}

// pass R: chains of at least RV_LONG_SYMS symbols get a wave each; the others
// share rv_short_waves waves (k_coder_rv; SA_RV_SHORT_WAVES=0: a wave per chain)
constexpr uint32_t RV_LONG_SYMS = 1u << 21;

int coder_launch_r(sa_ctx* c, hipStream_t st, TaskList tl, const CoderView& cv, int ph, uint32_t nlong)
{
    if (!tl.count) return 0;
    uint32_t waves = tl.count;
    tl.nlong = tl.count;
    if (c->rv_short_waves && nlong + c->rv_short_waves < tl.count) {
        tl.nlong = nlong;
        waves = nlong + c->rv_short_waves;
    }
    if (ph >= 0) ev_begin(c, ph, st);
    tl.wait_ticks = c->rv_wait_ticks;
    if (c->rv_lanes) {   // a chain per lane, 64 per workgroup, longest first
        hipLaunchKernelGGL(k_coder_rl, dim3((tl.count + 63) / 64), dim3(64 * RL_WAVES), 0, st, cv.tasks, tl, cv.prs[0],
                           cv.prs[1], cv.ck_r, c->d_err.as<uint32_t>(), c->chain_prio);
        if (ph >= 0) ev_finish(c, ph, st);
        return 0;
    }
    const uint32_t grid = (waves + c->coder_waves - 1) / c->coder_waves;
    uint64_t* probe = nullptr;
    if (c->rv_probe && ph >= 0 && c->d_probe.ensure(32ull * grid * c->coder_waves) == hipSuccess) {
        probe = c->d_probe.as<uint64_t>();
        c->probe_waves = grid * c->coder_waves;
        (void)hipMemsetAsync(probe, 0, 32ull * c->probe_waves, st);
    }
    // (V = 6) a 2 KiB ring per wave, sized for 1024 waves from the start (a
    // re-allocation's hipFree would synchronise the device)
    if (c->rv_batch == 6 &&
        c->d_ring.ensure(4ull * RING_DW * std::max<uint32_t>(1024u, grid * c->coder_waves)) != hipSuccess) {
        c->err = "pass R: cannot allocate the operand ring";
        return -1;
    }
    hipLaunchKernelGGL(c->rv_batch == 6   ? k_coder_rv<6>
                       : c->rv_batch == 5 ? k_coder_rv<5>
                                          : k_coder_rv<0>,
                       dim3(grid), dim3(64 * c->coder_waves), c->coder_lds, st, cv.tasks, tl, cv.prs[0], cv.prs[1],
                       cv.ck_r, c->d_err.as<uint32_t>(), c->chain_prio, probe, c->d_ring.as<uint32_t>());
    if (ph >= 0) ev_finish(c, ph, st);
    return 0;
}

// SA_RV_PROBE: one line per pass-R wave of this batch: context, batch, wave,
// start / end (us on the 100 MHz clock, absolute), shader MHz over the wave,
// XCC, SE, CU, SIMD, wave slot, chains
void write_rv_probe(sa_ctx* c, const std::vector<uint64_t>& p)
{
    static std::mutex mu;
    static uint64_t batch = 0;
    std::lock_guard<std::mutex> g(mu);
    FILE* f = std::fopen(c->rv_probe, "a");
    if (!f) return;
    const uint64_t b = batch++;
    for (size_t w = 0; w + 3 < p.size(); w += 4) {
        const uint64_t t0 = p[w], t1 = p[w + 1], cyc = p[w + 2], id = p[w + 3];
        if (!t1) continue;
        const uint32_t hw = (uint32_t)id;
        const double us = (double)(t1 - t0) / 100.0;
        std::fprintf(f, "%p %llu %zu %.1f %.1f %.0f xcc %u se %u cu %u simd %u slot %u chains %u sh %u hwid %08x\n",
                     (void*)c, (unsigned long long)b, w / 4, (double)t0 / 100.0, (double)t1 / 100.0,
                     us > 0 ? (double)cyc / us : 0.0, (unsigned)((id >> 32) & 0xff), (hw >> 13) & 7u,
                     (hw >> 8) & 15u, (hw >> 4) & 3u, hw & 15u, (unsigned)(id >> 40), (hw >> 12) & 1u, hw);
    }
    std::fclose(f);
}

void coder_launch_l12(sa_ctx* c, hipStream_t st, const TaskList& tl, const CoderView& cv)
{
    if (!tl.count) return;
    const uint32_t lgrid = (uint32_t)((tl.total_segs + 255) / 256);
    hipLaunchKernelGGL(c->l_chunk == 16 ? k_coder_l1<16> : k_coder_l1<32>, dim3(lgrid), dim3(256), 0, st, cv, tl);
    hipLaunchKernelGGL(k_coder_l2, dim3(tl.count), dim3(L2_THREADS), 0, st, cv, tl);
}

void coder_launch_l3(sa_ctx* c, hipStream_t st, const TaskList& tl, const CoderView& cv)
{
    if (!tl.count) return;
    const uint32_t lgrid = (uint32_t)((tl.total_segs + 255) / 256);
    hipLaunchKernelGGL(c->l_chunk == 16 ? k_coder_l3<16> : k_coder_l3<32>, dim3(lgrid), dim3(256), 0, st, cv, tl);
}

// Range coder driver (DESIGN.md "Coder"): pass R of every listed chain (on st,
// longest first), then -- once `before_l` (the long model runs) is done -- L1
// and L2.  With `exact`, the payload arena is then sized from the streams'
// real byte counts (k_task_ends; a stream's out_cap gets 1/64 + 4 KiB of slack
// for squeeze restarts) instead of the 2-bytes-per-symbol bound the plan
// carries: tasks' out_base / out_cap, d_tasks and the payload are set here.
// Then L3, and the streams whose exact coding squeezed before their last
// segment restart after that segment from the state L3 computed, until none
// does.  out_len: every stream's bytes.  Returns 0, -1 on error, 2 when a
// stream outgrew its slack (the caller re-runs with exact = false).
int coder_run(sa_ctx* c, std::vector<CoderTask>& tasks, CoderView& cv, hipStream_t st, int ph_r, int ph_l,
              hipEvent_t before_l, bool exact, std::vector<uint32_t>& out_len, uint64_t& payload_bytes)
{
    out_len.assign(tasks.size(), 0);
    if (tasks.empty()) return 0;
    c->coder_restarts = 0;
    std::vector<uint64_t> gb;
    TaskList tl;
    uint32_t nlong = 0;
    {
        std::vector<uint32_t> ids;
        for (uint32_t t = 0; t < (uint32_t)tasks.size(); t++) ids.push_back(t);
        // longest streams first: a pass-R workgroup's chains are of similar length
        std::stable_sort(ids.begin(), ids.end(), [&](uint32_t a, uint32_t b) { return tasks[a].n > tasks[b].n; });
        std::vector<CoderRun> runs(ids.size(), CoderRun{0ull, 0xffffffffu, 0u, 0u, 0u});
        if (coder_list(c, st, 0, tasks, ids, runs, gb, tl)) return -1;
        for (const uint32_t t : ids) nlong += tasks[t].n >= RV_LONG_SYMS ? 1u : 0u;
    }
    if (coder_launch_r(c, st, tl, cv, c->timing ? ph_r : -1, nlong)) return -1;
    if (c->st5) {   // (SA_L_CU_EVERY) the L passes on their own CUs once pass R is done
        SA_CHECK(c, hipEventRecord(c->ev_r_done, st));
        SA_CHECK(c, hipEventSynchronize(c->ev_r_done));
        st = c->st5;
    }
    if (before_l) {
        if (c->host_waits) SA_CHECK(c, hipEventSynchronize(before_l));   // (see host_waits)
        else SA_CHECK(c, hipStreamWaitEvent(st, before_l, 0));
    }
    if (c->timing && ph_l >= 0) ev_begin(c, ph_l, st);
    coder_launch_l12(c, st, tl, cv);
    SA_CHECK(c, hipGetLastError());
    if (exact) {
        SA_CHECK(c, c->d_task_ends.ensure(4 * tasks.size()));
        hipLaunchKernelGGL(k_task_ends, dim3((tl.count + 255) / 256), dim3(256), 0, st, cv, tl,
                           c->d_task_ends.as<uint32_t>());
        std::vector<uint32_t> ends(tasks.size());
        uint32_t perr[4] = {0, 0, 0, 0};
        SA_CHECK(c, d2h(c, ends.data(), c->d_task_ends.p, 4 * tasks.size(), st));
        SA_CHECK(c, d2h(c, perr, c->d_err.p, 16, st));
        std::vector<uint64_t> probe;
        if (c->rv_probe && c->probe_waves) {
            probe.resize(4ull * c->probe_waves);
            SA_CHECK(c, d2h(c, probe.data(), c->d_probe.p, 32ull * c->probe_waves, st));
        }
        SA_CHECK(c, sync_d2h(c, st));
        if (!probe.empty()) write_rv_probe(c, probe);
        if (perr[0] & E_CODER) {   // (pass R gave up on unwritten records: L3 is not run on them)
            c->err = "range coder: pass R timed out waiting for model records (E_CODER)";
            return -1;
        }
        uint64_t payload = 0, slack = 4096;
        if (const char* e = std::getenv("SA_PAYLOAD_SLACK")) slack = std::strtoull(e, nullptr, 10);   // (tests)
        for (size_t t = 0; t < tasks.size(); t++) {
            const uint64_t cap = (uint64_t)ends[t] + ends[t] / 64 + slack;
            tasks[t].out_cap = (uint32_t)std::min<uint64_t>(cap, tasks[t].out_cap);
            tasks[t].out_base = payload;
            payload = align_up(payload + tasks[t].out_cap, 16);
        }
        payload_bytes = payload;
        SA_CHECK(c, c->d_payload.ensure(std::max<uint64_t>(payload, 16)));
        cv.out = c->d_payload.as<uint8_t>();
        SA_CHECK(c, h2d(c, c->d_tasks.p, tasks.data(), sizeof(CoderTask) * tasks.size(), st));
    }
    coder_launch_l3(c, st, tl, cv);
    if (c->timing && ph_l >= 0) ev_finish(c, ph_l, st);
    SA_CHECK(c, hipGetLastError());
    std::vector<uint32_t> first_sq(tasks.size());
    for (int round = 0;; round++) {
        SA_CHECK(c, d2h(c, first_sq.data(), cv.first_sq, 4 * tasks.size(), st));
        SA_CHECK(c, d2h(c, out_len.data(), cv.out_len, 4 * tasks.size(), st));
        SA_CHECK(c, sync_d2h(c, st));
        std::vector<uint32_t> ids;
        for (size_t t = 0; t < tasks.size(); t++) {
            const uint32_t k = first_sq[t];
            if (k != 0xffffffffu && k + 1 < tasks[t].nseg) ids.push_back((uint32_t)t);
        }
        if (ids.empty()) break;
        // the exact end state L3 left at each restarted stream's squeezed
        // segment: all copies queued on st, one wait
        std::vector<LowMap> endst(ids.size());
        std::vector<uint32_t> off(ids.size());
        for (size_t i = 0; i < ids.size(); i++) {
            const uint64_t sg = tasks[ids[i]].seg_base + first_sq[ids[i]];
            SA_CHECK(c, d2h(c, &endst[i], cv.maps + sg, sizeof(LowMap), st));
            SA_CHECK(c, d2h(c, &off[i], cv.off_at + sg, 4, st));
        }
        SA_CHECK(c, hipMemsetAsync(cv.first_sq, 0xff, 4 * tasks.size(), st));
        SA_CHECK(c, sync_d2h(c, st));
        std::vector<CoderRun> runs;
        for (size_t i = 0; i < ids.size(); i++)
            runs.push_back(CoderRun{endst[i].B, endst[i].s, first_sq[ids[i]] + 1, off[i] + endst[i].nbytes, 0u});
        if (round > 1000) {
            c->err = "range coder: too many restarts";
            return -1;
        }
        c->coder_restarts += (uint32_t)ids.size();
        if (coder_list(c, st, 0, tasks, ids, runs, gb, tl)) return -1;
        if (coder_launch_r(c, st, tl, cv, -1, 0)) return -1;
        coder_launch_l12(c, st, tl, cv);
        coder_launch_l3(c, st, tl, cv);
        SA_CHECK(c, hipGetLastError());
    }
    for (size_t t = 0; t < tasks.size(); t++)
        if (out_len[t] > tasks[t].out_cap) {
            if (exact) return 2;
            c->err = "range coder output overflowed its buffer";
            return -1;
        }
    return 0;
}

void ev_begin(sa_ctx* c, int ph, hipStream_t st)
{
    if (c->timing) (void)hipEventRecord(c->ev_beg[ph], st);
}
void ev_finish(sa_ctx* c, int ph, hipStream_t st)
{
    if (c->timing) (void)hipEventRecord(c->ev_end[ph], st);
}

}  // namespace

extern "C" {

const char* sa_version(void) { return "seqarc_amd 0.1 (gfx950)"; }

sa_ctx* sa_create(int device)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return nullptr;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        std::fprintf(stderr, "seqarc_amd: device %d is %s, this library is built for gfx950 only\n", device,
                     prop.gcnArchName);
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    // SA_SYNC=block: host waits sleep instead of spinning (the command line sets
    // it: five encoder threads spinning on their streams took the CPU share the
    // reader needs); only effective before the device's first use in the process
    if (const char* e = std::getenv("SA_SYNC")) {
        if (!std::strcmp(e, "block")) (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
        else if (!std::strcmp(e, "spin")) (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
        (void)hipGetLastError();   // (hipErrorSetOnActiveProcess when the device is in use already)
    }
    sa_ctx* c = new sa_ctx();
    // pass-R placement knobs (k_coder_rv): waves per workgroup, unused LDS per workgroup
    if (const char* e = std::getenv("SA_CODER_WAVES")) {
        const int w = std::atoi(e);
        c->coder_waves = (w == 1 || w == 2) ? (uint32_t)w : 4u;
    }
    if (const char* e = std::getenv("SA_CODER_LDS")) c->coder_lds = (uint32_t)std::min(std::max(std::atoi(e), 0), 160 * 1024);
    if (c->coder_lds > 64 * 1024 &&
        (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_coder_rv<0>), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)c->coder_lds) != hipSuccess ||
         hipFuncSetAttribute(reinterpret_cast<const void*>(&k_coder_rv<5>), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)c->coder_lds) != hipSuccess ||
         hipFuncSetAttribute(reinterpret_cast<const void*>(&k_coder_rv<6>), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)c->coder_lds) != hipSuccess)) {
        std::fprintf(stderr, "seqarc_amd: cannot reserve %u B of LDS for pass R\n", c->coder_lds);
        delete c;
        return nullptr;
    }
    c->device = device;
    c->timing = c->trace;
    c->n_cu = (uint32_t)prop.multiProcessorCount;
    for (int i = 0; i < PH_N; i++) c->ev_beg[i] = c->ev_end[i] = nullptr;
    // st carries the critical path (AUX symbols -> QUAL coder chain).  While the
    // long AUX model runs replay (latency-bound, st4: every 4th CU), the SEQ path
    // (throughput, st3: the other CUs) runs beside them without sharing a SIMD.
    // (SA_LONG_CU_EVERY / SA_LONG_LDS: tuning overrides of the split and of the
    //  LDS per long-run workgroup, i.e. how many share a CU)
    const char* ev = std::getenv("SA_LONG_CU_EVERY");
    const int every = ev ? std::max(1, std::atoi(ev)) : 4;
    const char* el = std::getenv("SA_LONG_LDS");
    c->long_lds = el ? (uint32_t)std::atoi(el) : 0u;
    c->serial_seq = std::getenv("SA_SERIAL_SEQ") != nullptr;
    if (const char* cp = std::getenv("SA_CHAIN_PRIO")) c->chain_prio = std::atoi(cp) != 0;
    c->md5_prio = c->chain_prio;
    if (const char* cp = std::getenv("SA_MD5_PRIO")) c->md5_prio = std::atoi(cp) != 0;
    std::vector<uint32_t> m_long((prop.multiProcessorCount + 31) / 32, 0u), m_seq(m_long.size(), 0u);
    for (int cu = 0; cu < prop.multiProcessorCount; cu++)
        ((cu % every) == 0 || every == 1 ? m_long : m_seq)[cu / 32] |= 1u << (cu % 32);
    if (every == 1) m_seq = m_long;   // (st3: the coder chains; st4: the long model runs)
    // (A/B, round 5) SA_RV_CUS=n (1..5, with every = 4): pass R and the L passes
    // (st3) on n of each 8 CUs only, the front (st) on the others -- the scalar
    // units of the front's CUs free of chain waves (k_coder_rl showed the
    // fronts 2-3x faster beside a pass R that leaves the scalar units alone)
    std::vector<uint32_t> m_front;
    if (const char* rc = std::getenv("SA_RV_CUS")) {
        const int n = std::atoi(rc);
        if (every == 4 && n >= 1 && n <= 5) {
            m_front.assign(m_long.size(), 0u);
            std::fill(m_seq.begin(), m_seq.end(), 0u);
            static const int order[6] = {1, 5, 2, 6, 3, 7};   // (the non-long CUs of each 8, spread)
            for (int cu = 0; cu < prop.multiProcessorCount; cu++) {
                bool r = false;
                for (int k = 0; k < n; k++) r |= (cu % 8) == order[k];
                (r ? m_seq : m_front)[cu / 32] |= 1u << (cu % 32);
            }
        }
    }
    {
        uint32_t ncu_long = 0;
        for (uint32_t w : m_long) ncu_long += (uint32_t)__builtin_popcount(w);
        c->long_grid = std::max(1u, 6u * ncu_long);
        if (const char* lg = std::getenv("SA_LONG_GRID")) c->long_grid = (uint32_t)std::max(1, std::atoi(lg));
    }
    if ((m_front.empty() ? hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking)
                         : hipExtStreamCreateWithCUMask(&c->st, (uint32_t)m_front.size(), m_front.data())) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&c->st2, (uint32_t)m_long.size(), m_long.data()) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&c->st3, (uint32_t)m_seq.size(), m_seq.data()) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&c->st4, (uint32_t)m_long.size(), m_long.data()) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_seq_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_long_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_prs_zero, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork_seq, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_md5_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_r[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_r[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_dense, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return nullptr;
    }
    if (const char* le = std::getenv("SA_L_CU_EVERY")) {
        const int n = std::atoi(le);
        if (n == 1) {   // (A/B, round 6) the L passes on the front's CUs (all of them without SA_RV_CUS)
            if ((m_front.empty() ? hipStreamCreateWithFlags(&c->st5, hipStreamNonBlocking)
                                 : hipExtStreamCreateWithCUMask(&c->st5, (uint32_t)m_front.size(), m_front.data())) !=
                    hipSuccess ||
                hipEventCreateWithFlags(&c->ev_r_done, hipEventDisableTiming) != hipSuccess) {
                delete c;
                return nullptr;
            }
        } else if (n >= 2) {
            std::vector<uint32_t> m_l(m_long.size(), 0u);
            for (int cu = 0; cu < prop.multiProcessorCount; cu++)
                if (cu % n == n / 2) m_l[cu / 32] |= 1u << (cu % 32);   // (offset: not the long runs' CUs when n = 4)
            if (hipExtStreamCreateWithCUMask(&c->st5, (uint32_t)m_l.size(), m_l.data()) != hipSuccess ||
                hipEventCreateWithFlags(&c->ev_r_done, hipEventDisableTiming) != hipSuccess) {
                delete c;
                return nullptr;
            }
        }
    }
    for (int i = 0; i < PH_N; i++) {
        if (hipEventCreate(&c->ev_beg[i]) != hipSuccess || hipEventCreate(&c->ev_end[i]) != hipSuccess) {
            delete c;
            return nullptr;
        }
    }
    c->fs = new FrontShare();
    c->fs->refs = 1;
    if (hipEventCreateWithFlags(&c->fs->ev_free, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return nullptr;
    }
    return c;
}

sa_ctx* sa_create_shared(int device, sa_ctx* peer)
{
    if (!peer || peer->device != device) return nullptr;
    sa_ctx* c = sa_create(device);
    if (!c) return nullptr;
    std::lock_guard<std::mutex> g(g_share_mu);
    FrontShare* own = c->fs;
    c->fs = peer->fs;
    c->fs->refs++;
    for (DBuf* b : own->buffers()) b->release();
    if (own->ev_free) (void)hipEventDestroy(own->ev_free);
    delete own;
    return c;
}

uint64_t sa_front_bytes(const sa_ctx* c) { return c && c->fs ? c->fs->held_bytes() : 0; }

void sa_destroy(sa_ctx* ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    delete ctx;
}

const char* sa_last_error(const sa_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

void sa_set_timing(sa_ctx* ctx, int on)
{
    if (ctx) ctx->timing = on != 0;
}

int sa_host_register(void* p, uint64_t bytes)
{
    if (!p || !bytes) return -1;
    return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? 0 : -1;
}

int sa_host_unregister(void* p)
{
    if (!p) return -1;
    return hipHostUnregister(p) == hipSuccess ? 0 : -1;
}

uint64_t sa_output_bound(const sa_block* b)
{
    uint64_t nb = 0, nn = 0;
    for (uint32_t r = 0; r < b->nreads; r++) {
        nb += (uint64_t)(b->seq_lens[r] > 0 ? b->seq_lens[r] : 0);
        nn += b->name_lens[r];
    }
    // coded symbols per stream: len <= 5 per read, names <= 3 per read + the
    // name bytes, quals <= bases + 1 per read, tip / max-qual 1 per read, N/IUPAC
    // chars <= bases, exception counts <= 33 per read (kModel), gaps <= bases
    // (1 + bits(g) symbols per g + 1 bases), bases; each symbol narrows the
    // range by < 2^16 (<= 2 bytes); + per stream flush and header, the MD5s and
    // the ID-bin first ID
    // (+ 140 per read: the reference path's alignment symbols, <= 64 position
    // bits, <= 63 x 17 mismatch bits and types at maxmis 7 ...)
    const uint64_t syms = 3 * nb + nn + (45ull + 140ull) * b->nreads;
    return 2 * syms + 9 * 96 + 4096 + 0x10000;
}

}  // extern "C"

namespace {

// Uploads a batch of parsed blocks into `in` (its buffers grow as needed) on
// stream st and waits for the copies.  Returns 0 or -1 with err set.
int input_upload(sa_input* I, const sa_block* in, int n, hipStream_t st, std::string& err)
{
#define IN_CHECK(expr)                                                                   \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            err = std::string(#expr) + ": " + hipGetErrorString(e_);                     \
            return -1;                                                                   \
        }                                                                                \
    } while (0)
    if (n < 0 || (n > 0 && !in)) {
        err = "invalid block list";
        return -1;
    }
    I->nblocks = (uint32_t)n;
    I->blocks.assign((size_t)n, DevBlock{});
    uint64_t nb = 0, sb = 0, tb = 0;
    uint32_t nr = 0;
    for (int b = 0; b < n; b++) {
        DevBlock& d = I->blocks[(size_t)b];
        d.nreads = in[b].nreads;
        d.read0 = nr;
        uint64_t ln = 0, ls = 0;
        for (uint32_t r = 0; r < in[b].nreads; r++) {
            if (in[b].seq_lens[r] < 0) {
                err = "negative read length";
                return -1;
            }
            ln += in[b].name_lens[r];
            ls += (uint64_t)in[b].seq_lens[r];
            if (in[b].seq_lens[r] > 0xffff) d.len_long = 1;   // getBlockRead@0x411d2a
        }
        if (ls >= (1ull << 30) || ln >= (1ull << 32)) {
            err = "block too large (a reference block is 50 MiB of FASTQ)";
            return -1;
        }
        if ((uint64_t)nr + in[b].nreads >= (1ull << 31)) {
            err = "too many reads in one batch";
            return -1;
        }
        d.name_base = nb;
        d.seq_base = sb;
        d.name_bytes = ln;
        d.seq_bytes = ls;
        nb = align_up(nb + ln, 16);
        sb = align_up(sb + ls, 16);
        tb += ln + 2 * ls;
        nr += in[b].nreads;
    }
    I->nreads = nr;
    I->names_bytes = nb;
    I->seq_bytes = sb;
    I->text_bytes = tb;
    I->h_read_block.resize(nr);
    I->h_name_off.resize(nr);
    I->h_name_len.resize(nr);
    I->h_seq_off.resize(nr);
    I->h_seq_len.resize(nr);
    for (int b = 0; b < n; b++) {
        const DevBlock& d = I->blocks[(size_t)b];
        uint32_t no = 0, so = 0;
        for (uint32_t r = 0; r < d.nreads; r++) {
            const uint32_t g = d.read0 + r;
            I->h_read_block[g] = (uint32_t)b;
            I->h_name_off[g] = no;
            I->h_name_len[g] = in[b].name_lens[r];
            I->h_seq_off[g] = so;
            I->h_seq_len[g] = (uint32_t)in[b].seq_lens[r];
            no += in[b].name_lens[r];
            so += (uint32_t)in[b].seq_lens[r];
        }
    }
    IN_CHECK(I->d_names.ensure(nb + 64));   // (k_prep_sq16 reads whole dwords past a name)
    IN_CHECK(I->d_seq.ensure(sb + 64));   // (k_prep_sq16 reads whole dwords past a read)
    IN_CHECK(I->d_qual.ensure(sb + 64));
    const size_t nr4 = (size_t)std::max<uint32_t>(nr, 1) * 4;
    IN_CHECK(I->d_read_block.ensure(nr4));
    IN_CHECK(I->d_name_off.ensure(nr4));
    IN_CHECK(I->d_name_len.ensure(nr4));
    IN_CHECK(I->d_seq_off.ensure(nr4));
    IN_CHECK(I->d_seq_len.ensure(nr4));
    for (int b = 0; b < n; b++) {
        const DevBlock& d = I->blocks[(size_t)b];
        if (d.name_bytes)
            IN_CHECK(hipMemcpyAsync(I->d_names.as<uint8_t>() + d.name_base, in[b].names, d.name_bytes,
                                    hipMemcpyHostToDevice, st));
        if (d.seq_bytes) {
            IN_CHECK(hipMemcpyAsync(I->d_seq.as<uint8_t>() + d.seq_base, in[b].seq, d.seq_bytes,
                                    hipMemcpyHostToDevice, st));
            IN_CHECK(hipMemcpyAsync(I->d_qual.as<uint8_t>() + d.seq_base, in[b].qual, d.seq_bytes,
                                    hipMemcpyHostToDevice, st));
        }
    }
    if (nr) {
        IN_CHECK(hipMemcpyAsync(I->d_read_block.p, I->h_read_block.data(), nr * 4ull, hipMemcpyHostToDevice, st));
        IN_CHECK(hipMemcpyAsync(I->d_name_off.p, I->h_name_off.data(), nr * 4ull, hipMemcpyHostToDevice, st));
        IN_CHECK(hipMemcpyAsync(I->d_name_len.p, I->h_name_len.data(), nr * 2ull, hipMemcpyHostToDevice, st));
        IN_CHECK(hipMemcpyAsync(I->d_seq_off.p, I->h_seq_off.data(), nr * 4ull, hipMemcpyHostToDevice, st));
        IN_CHECK(hipMemcpyAsync(I->d_seq_len.p, I->h_seq_len.data(), nr * 4ull, hipMemcpyHostToDevice, st));
    }
    IN_CHECK(hipStreamSynchronize(st));
#undef IN_CHECK
    return 0;
}

}  // namespace

extern "C" {

void sa_alloc_stats(uint32_t* grows, double* alloc_ms)
{
    if (grows) *grows = g_grows.load();
    if (alloc_ms) *alloc_ms = g_alloc_ns.load() / 1e6;
}

void sa_set_reserve(sa_ctx* c, uint32_t blocks)
{
    if (c) c->reserve_blocks = blocks;
}

int sa_stage(sa_ctx* c, const sa_block* in, int n)
{
    const ReserveScope reserve(c ? c->reserve_blocks : 0, n > 0 ? (uint32_t)n : 0);
    if (!c) return -1;
    SA_CHECK(c, hipSetDevice(c->device));
    c->have_output = false;
    return input_upload(&c->own, in, n, c->st, c->err);
}

sa_input* sa_input_create(int device, const sa_block* in, int n)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return nullptr;
    sa_input* I = new sa_input();
    I->device = device;
    std::string err;
    const int rc = input_upload(I, in, n, st, err);
    (void)hipStreamDestroy(st);
    if (rc) {
        std::fprintf(stderr, "seqarc_amd: sa_input_create: %s\n", err.c_str());
        delete I;
        return nullptr;
    }
    return I;
}

void sa_input_destroy(sa_input* in)
{
    if (!in) return;
    (void)hipSetDevice(in->device);
    delete in;
}

int sa_run(sa_ctx* c, const sa_cfg* cfg)
{
    if (!c) return -1;
    return sa_run_input(c, &c->own, cfg);
}

}  // extern "C"

// The reference (HASH index) path of a batch: doAlignEncode@0x42d4c0 instead of
// doFqzEncode@0x42d2d0 (sa_run_input_aligned).
struct AlignReq {
    const sa_hash_index* ix;
    sa_align_cfg cfg;
    sa_align_chain* chain;
    uint64_t batch;   // the batch's place in the chain (UINT64_MAX: the chain's next)
};
// sa_hash.hip: aligns the batch, follows the carried state through it (after
// the chain's previous batch), plans its blocks (c->blocks: order count, insert
// window), counts and scans the alignment columns (atot: per block NACOL sums)
// and sets the BatchView / AlignView fields of the path
int align_front(sa_ctx* c, const sa_input* I, BatchView& bv, const AlignReq& rq, std::vector<uint32_t>& atot,
                AlignView& av);
void align_chain_fail(sa_align_chain* ch);

namespace {

// One encode of a resident batch; exact: the payload arena sized from the
// streams' real byte counts after L2 (else the 2-bytes-per-symbol bound).
// al: the reference path (nullptr: no reference).
// Returns 0, -1, or 2 when a stream outgrew its exact cap.
int run_input(sa_ctx* c, const sa_input* I, const sa_cfg* cfg, bool exact, const AlignReq* al = nullptr)
{
    if (!c) return -1;
    if (!I || !cfg || I->device != c->device) {
        c->err = "sa_run_input: no input, no config, or an input of another device";
        return -1;
    }
    const ReserveScope reserve(c->reserve_blocks, I->nblocks);
    SA_CHECK(c, hipSetDevice(c->device));
    c->have_output = false;
    if (mail_reset(c)) return -1;
    c->blocks = I->blocks;
    const uint32_t nbk = I->nblocks;
    if (nbk == 0) {
        c->final_base.clear();
        c->final_len.clear();
        c->have_output = true;
        return 0;
    }
    if (cfg->slevel < 0 || cfg->slevel > 9 || cfg->qlevel < 0 || cfg->qlevel > 3) {
        c->err = "unsupported slevel/qlevel";
        return -1;
    }
    const bool lossy = cfg->lossy > 0.0;   // -l R: param+0x1870 / +0x1878
    const int k = cfg->slevel + 7;
    const uint32_t ns = 1u << ((2 * k) & 31);
    const int seq_bits = (2 * k) & 31;   // NS = 1 << seq_bits (x86 shl masks the count)
    // k <= 14: the SEQ key carries the base in its low two bits and the values
    // are the stream position, i.e. the index (the emitter writes no values, the
    // first sort pass computes them); k = 15 fills all 32 key bits (a key could
    // equal the sort pad) and order 0 has no sort pass, so they keep values
    // position << 2 | base (SA_SEQ_PACK=0: always)
    const uint32_t seq_sh = (ns > 1 && seq_bits <= 28 && !c->seq_unpacked) ? 2u : 0u;
    // contexts of <= 22 bits (Slevel <= 4): one sort pass over the context's low
    // 8 (9) bits, the high bkt_sb bits replayed per bucket with the models in LDS
    // (k_replay_seq_bkt); longer contexts: the full sort and k_replay_seq
    const bool seq_bkt = c->seq_bucket && seq_sh == 2 && seq_bits >= 12 && seq_bits <= 22;
    // (SA_BKT_DB: one more digit bit halves the models a replay wave holds in
    // LDS -- 2^12 contexts in 20 KB instead of 2^13 in 40 KB at 22 bits --
    // for twice the waves per CU; 10 bits with the inverse-permutation pass only)
    const int bkt_db = c->bkt_db_env >= 8 && c->bkt_db_env <= (c->seq_inv ? 10 : 9) && seq_bits - c->bkt_db_env >= 4
                           ? c->bkt_db_env
                           : (seq_bits <= 20 ? 8 : 9);
    const int bkt_sb = seq_bits - bkt_db;
    const int seq_max_db = seq_bkt ? std::max(bkt_db, (int)SORT_MAX_DB) : (int)SORT_MAX_DB;
    // (the bucket pass sorts by the context's LOW bits: k_replay_seq_bkt)
    const int seq_lo = (int)seq_sh,
              seq_hi = ns > 1 ? (int)seq_sh + (seq_bkt ? seq_bits - bkt_sb : seq_bits) : 0;
    const int aux_bits = cfg->qlevel > 2 ? 21 : 17;
    hipStream_t st = c->st;
    const uint32_t nr = I->nreads;
    FrontShare* F = c->fs;
    c->rv_batch = c->rv_variant == 0 || c->rv_variant == 5 || c->rv_variant == 6
                      ? c->rv_variant
                      : (nr && I->seq_bytes / nr > 1000 ? 0 : 6);   // (see rv_variant)

    SA_CHECK(c, c->d_blocks.ensure(sizeof(DevBlock) * nbk));
    SA_CHECK(c, h2d(c, c->d_blocks.p, c->blocks.data(), sizeof(DevBlock) * nbk, st));
    BatchView bv{};
    bv.blocks = c->d_blocks.as<DevBlock>();
    bv.nblocks = nbk;
    bv.nreads_total = nr;
    bv.read_block = I->d_read_block.as<uint32_t>();
    bv.names = I->d_names.as<uint8_t>();
    bv.seq = I->d_seq.as<uint8_t>();
    bv.qual = I->d_qual.as<uint8_t>();
    bv.qual_q = bv.qual;
    bv.lossy = lossy ? 1 : 0;
    bv.name_off = I->d_name_off.as<uint32_t>();
    bv.name_len = I->d_name_len.as<uint16_t>();
    bv.seq_off = I->d_seq_off.as<uint32_t>();
    bv.seq_len = I->d_seq_len.as<uint32_t>();
    bv.seq_mask = ns - 1;
    bv.qlevel = cfg->qlevel;
    bv.bin_mode = cfg->bin_mode ? 1 : 0;
    bv.md5 = cfg->md5 ? 1 : 0;
    // reference path: the reads are aligned (and the batch placed in the
    // align_info chain) before the front is taken: the chain may wait for
    // the batch before this one, which another context runs
    std::vector<uint32_t> aln_tot;
    AlignView alv{};
    if (al && align_front(c, I, bv, *al, aln_tot, alv)) {
        align_chain_fail(al->chain);
        return -1;
    }
    const bool trace = al && std::getenv("SA_ALN_TRACE");
    // the front (prep up to the short model runs) holds the device's front
    // scratch.  (The prep before the turn, overlapping another context's
    // front, measured slower: 12.6 vs 13.9 GB/s, round 3 g3i -- the front
    // kernels are throughput-bound together.)  A context's first batch is the
    // exception: its prep touches no front scratch, and its own buffers (~34
    // GB for a 69-block batch) are allocated from the plan -- hipMalloc of
    // tens of GB takes ~0.3 s, which inside the turn held up every other
    // context (the command line's first batches: 1.4 s of allocations in
    // series, round 4 r4c).  So the first batch preps, plans and allocates
    // first, then takes its turn.
    const bool early = !c->front_warm;
    std::optional<FrontTurn> front_lock;
    if (!early) front_lock.emplace(F, st);
    if (trace && !early) fprintf(stderr, "[align] front turn taken\n");
    SA_CHECK(c, c->d_counts.ensure((size_t)std::max<uint32_t>(nr, 1) * NCOL * 4));
    SA_CHECK(c, c->d_dege_maxq.ensure((size_t)std::max<uint32_t>(nr, 1)));
    uint8_t* dege_maxq = c->prep_wave ? nullptr : c->d_dege_maxq.as<uint8_t>();   // (k_prep_sq: k_emit's serial path)
    SA_CHECK(c, c->d_totals.ensure((size_t)nbk * NCOL * 4));
    SA_CHECK(c, c->d_name_p.ensure((size_t)std::max<uint32_t>(nr, 1) * 2));
    SA_CHECK(c, c->d_name_s.ensure((size_t)std::max<uint32_t>(nr, 1) * 2));
    SA_CHECK(c, c->d_maxlen.ensure((size_t)std::max<uint32_t>(nr, 1) * 2));
    SA_CHECK(c, c->d_err.ensure(64));   // error words 0-3, the front kernels' read counters (WaveReads) 8-9
    SA_CHECK(c, hipMemsetAsync(c->d_err.p, 0, 64, st));

    uint32_t* d_err = c->d_err.as<uint32_t>();
    // the front kernels' dynamic read counters (nullptr: the static grid stride)
    uint32_t* wq_prep = c->front_static ? nullptr : d_err + 8;
    uint32_t* wq_emit = c->front_static ? nullptr : d_err + 9;
    const uint32_t wqc = front_wq_chunk(c, I->seq_bytes, nr);
    // k_emit_sq's listed reads from a counter (one a take) for long-read batches
    uint32_t* wq_dege = c->front_static || wqc >= WQ_CHUNK ? nullptr : d_err + 10;

    ev_begin(c, PH_TOTAL, st);
    // ---- MD5 of every block's IDs/bases/quals (calcBlockMd5@0x414d90) on st2,
    //      concurrent with everything up to the assembly ----
    std::vector<Md5Task> md5t;
    for (uint32_t b = 0; b < nbk; b++) {
        const DevBlock& d = c->blocks[b];
        md5t.push_back(Md5Task{I->d_names.as<uint8_t>() + d.name_base, d.name_bytes});
        md5t.push_back(Md5Task{I->d_seq.as<uint8_t>() + d.seq_base, d.seq_bytes});
        md5t.push_back(Md5Task{I->d_qual.as<uint8_t>() + d.seq_base, d.seq_bytes});
    }
    if (cfg->md5) {
        SA_CHECK(c, c->d_md5tasks.ensure(sizeof(Md5Task) * md5t.size()));
        SA_CHECK(c, c->d_digests.ensure(16 * md5t.size()));
        SA_CHECK(c, hipEventRecord(c->ev_fork, st));
        SA_CHECK(c, hipStreamWaitEvent(c->st2, c->ev_fork, 0));
        SA_CHECK(c, h2d(c, c->d_md5tasks.p, md5t.data(), sizeof(Md5Task) * md5t.size(), c->st2));
        ev_begin(c, PH_MD5, c->st2);
        hipLaunchKernelGGL(c->md5_pipe ? k_md5<true> : k_md5<false>, dim3((uint32_t)md5t.size()), dim3(128), 0, c->st2,
                           c->d_md5tasks.as<Md5Task>(),
                           (uint32_t)md5t.size(), c->d_digests.as<uint32_t>(), c->md5_prio);
        ev_finish(c, PH_MD5, c->st2);
        SA_CHECK(c, hipGetLastError());
        SA_CHECK(c, hipEventRecord(c->ev_md5_done, c->st2));
    } else {
        SA_CHECK(c, c->d_digests.ensure(16 * md5t.size()));
    }
    if (!early && F->have_ev) SA_CHECK(c, hipStreamWaitEvent(st, F->ev_free, 0));   // the previous front is done with it
    ev_begin(c, PH_PREP, st);
    if (lossy && run_rblock(c, cfg->lossy, I->seq_bytes, bv)) return -1;
    // thread-per-read kernels: one thread per read (a grid-stride variant with
    // 8 workgroups per CU measured slower: k_prep 1.2 -> 1.7 ms, k_emit 6.8 -> 9.4)
    const uint32_t rgrid = (nr + 255) / 256;
    // SA_PREP_ROW=64: a whole wave per read (round 6; for long reads the ONT
    // batch's prep+scan measured the same as with 16-lane rows under load, r6l:
    // 44.2 / 46.4 against 44.9 / 41.4 ms, so 16 stays the default)
    const bool prep_wide = c->prep_row == 64;
    if (nr) {
        // k_prep (names, lengths: lane per read) and k_prep_sq16 (SEQ / QUAL /
        // N-IUPAC columns: a row per read).  SA_PREP_FUSED=1: k_prep_sq16 takes
        // the name columns too (row-parallel prefix / suffix) -- measured no
        // faster under load (prep 38 vs 32 ms, same GB/s, round 3 g3r / g3s);
        // SA_PREP_WAVE=1: round 2's wave-per-read k_prep_sq
        if (c->prep_fused) {
            hipLaunchKernelGGL(wq_prep ? k_prep_sq16<true> : k_prep_sq16<false>, dim3(wave_grid(c, (nr + 3) / 4)),
                               dim3(256), 0, st, bv, c->d_counts.as<uint32_t>(), d_err, c->d_dege_maxq.as<uint8_t>(),
                               c->d_name_p.as<int16_t>(), c->d_name_s.as<int16_t>(), wq_prep, wqc);
        } else {
            hipLaunchKernelGGL(k_prep, dim3(rgrid), dim3(256), 0, st, bv, c->d_counts.as<uint32_t>(),
                               c->d_name_p.as<int16_t>(), c->d_name_s.as<int16_t>(), d_err);
            if (c->prep_wave)
                hipLaunchKernelGGL(k_prep_sq, dim3(wave_grid(c, nr)), dim3(64 * EMIT_WAVES), 0, st, bv,
                                   c->d_counts.as<uint32_t>(), d_err);
            else if (prep_wide)
                hipLaunchKernelGGL((wq_prep ? k_prep_sq16<true, 64> : k_prep_sq16<false, 64>), dim3(wave_grid(c, nr)),
                                   dim3(256), 0, st, bv, c->d_counts.as<uint32_t>(), d_err,
                                   c->d_dege_maxq.as<uint8_t>(), nullptr, nullptr, wq_prep, wqc);
            else
                hipLaunchKernelGGL(wq_prep ? k_prep_sq16<true> : k_prep_sq16<false>,
                                   dim3(wave_grid(c, (nr + 3) / 4)), dim3(256), 0, st, bv, c->d_counts.as<uint32_t>(),
                                   d_err, c->d_dege_maxq.as<uint8_t>(), nullptr, nullptr, wq_prep, wqc);
        }
    }
    hipLaunchKernelGGL(k_scan_reads, dim3(nbk), dim3(1024), 0, st, bv, c->d_counts.as<uint32_t>(),
                       c->d_totals.as<uint32_t>(), c->d_maxlen.as<uint16_t>());
    SA_CHECK(c, hipGetLastError());
    ev_finish(c, PH_PREP, st);
    std::vector<uint32_t> tot((size_t)nbk * NCOL);
    uint32_t herr[4];
    SA_CHECK(c, d2h(c, tot.data(), c->d_totals.p, tot.size() * 4, st));
    SA_CHECK(c, d2h(c, herr, c->d_err.p, 16, st));
    SA_CHECK(c, sync_d2h(c, st));
    if (herr[0]) {
        char buf[128];
        std::snprintf(buf, sizeof buf, "input rejected (error bits 0x%x)", herr[0]);
        c->err = buf;
        return -1;
    }

    uint64_t n_ch = 0;   // N / IUPAC bases in the batch
    for (uint32_t b = 0; b < nbk; b++) n_ch += tot[(size_t)b * NCOL + C_CH];

    // ---- layout of the symbol spaces, coder tasks, md5 tasks, outputs ----
    BatchPlan bp;
    if (!plan_batch(c->blocks, tot, bp, al ? &aln_tot : nullptr, alv.mis_model)) {
        c->err = "block symbol space too large";
        return -1;
    }
    const SortPlan& ps = bp.seq;
    const SortPlan& pa = bp.aux;
    std::vector<CoderTask> tasks = bp.tasks;
    c->max_stream_syms = c->total_stream_syms = 0;
    for (const CoderTask& tk : tasks) {
        c->max_stream_syms = std::max<uint64_t>(c->max_stream_syms, tk.n);
        c->total_stream_syms += tk.n;
    }
    std::vector<AsmBlock> asmb = bp.asmb;

    // ---- device buffers ----
    // slack: the replay loops read up to 2 chunks past a run's end, pass R one
    // 16-record chunk past a stream's last full segment
    const uint64_t stot = ps.total + KEY_SLACK, atot = pa.total + KEY_SLACK;
    // AUX sort ping-pong: the sorted keys/values must land in this context's
    // buffers (the long model runs read them after the front scratch is released)
    const bool dense = c->aux_dense && aux_bits == (int)AUX_DENSE_BITS && pa.total;
    const int aux_passes = dense ? 1 : (int)sort_digits(AUX_SYM_BITS, AUX_SYM_BITS + aux_bits).size();
    const uint64_t max_long = pa.total / LONG_RUN + 1;
    const uint64_t max_seq_long = ps.total / (SEQ_HALVE_J + 1) + 1;
    // at most one run per (block, model) and per symbol
    const uint64_t max_short = std::max<uint64_t>(std::min<uint64_t>(pa.total, (uint64_t)nbk << aux_bits), 1);
    uint64_t payload = bp.payload_bytes;
    CoderView cv{};
    auto ensure_ctx = [&]() -> int {   // this context's own buffers
        SA_CHECK(c, c->d_auxp_k.ensure(atot * 4));
        SA_CHECK(c, c->d_auxp_v.ensure(atot * 4));
        SA_CHECK(c, c->d_prs_seq.ensure(stot * sizeof(PRec)));
        SA_CHECK(c, c->d_prs_aux.ensure(atot * sizeof(PRec)));
        SA_CHECK(c, c->d_cum_aux.ensure(atot * 2));
        SA_CHECK(c, c->d_longs.ensure(max_long * sizeof(LongRun)));
        SA_CHECK(c, c->d_huge_sorted.ensure((pa.total / HUGE_RUN + 1) * sizeof(LongRun)));
        SA_CHECK(c, c->d_nlong.ensure(16));   // RunLists counters: short, huge, long, queue
        SA_CHECK(c, c->d_tasks.ensure(sizeof(CoderTask) * tasks.size()));
        SA_CHECK(c, c->d_out_len.ensure(4 * tasks.size()));
        if (!exact) SA_CHECK(c, c->d_payload.ensure(std::max<uint64_t>(payload, 16)));
        SA_CHECK(c, c->d_asm.ensure(sizeof(AsmBlock) * nbk));
        SA_CHECK(c, c->d_asm_copies.ensure(4ull * ASM_COPY_WORDS * nbk));
        SA_CHECK(c, c->d_task_out_base.ensure(8 * tasks.size()));
        SA_CHECK(c, c->d_final_len.ensure(8 * nbk));
        return coder_buffers(c, tasks.size(), bp.total_segs, cv);
    };
    if (ensure_ctx()) return -1;
    if (early) {   // (see `early`): now the turn, and the previous front's end on the device
        front_lock.emplace(F, st);
        if (trace) fprintf(stderr, "[align] front turn taken\n");
        if (F->have_ev) SA_CHECK(c, hipStreamWaitEvent(st, F->ev_free, 0));
    }
    // the device's front scratch (shared by its contexts: inside the turn)
    for (int i = 0; i < 2; i++) {
        SA_CHECK(c, F->d_seq_k[i].ensure(stot * 4));
        SA_CHECK(c, F->d_seq_v[i].ensure(stot * 4));
    }
    SA_CHECK(c, F->d_auxs_k.ensure(atot * 4));
    SA_CHECK(c, F->d_auxs_v.ensure(atot * 4));
    DBuf* akb[2] = {aux_passes % 2 ? &F->d_auxs_k : &c->d_auxp_k, aux_passes % 2 ? &c->d_auxp_k : &F->d_auxs_k};
    DBuf* avb[2] = {aux_passes % 2 ? &F->d_auxs_v : &c->d_auxp_v, aux_passes % 2 ? &c->d_auxp_v : &F->d_auxs_v};
    DBuf* skb[2] = {&F->d_seq_k[0], &F->d_seq_k[1]};
    DBuf* svb[2] = {&F->d_seq_v[0], &F->d_seq_v[1]};
    int seq_sorted_buf = 0, aux_sorted_buf = 0;
    SA_CHECK(c, F->d_seq_longs.ensure(max_seq_long * 8));
    SA_CHECK(c, F->d_nseq_long.ensure(4));
    SA_CHECK(c, F->d_short_at.ensure(max_short * 8));
    SA_CHECK(c, F->d_hist_seq.ensure(std::max<uint64_t>(ps.tile_seg.size(), 1) * 4 *
                                     sort_hist_per_tile(seq_lo, seq_hi, seq_max_db)));
    SA_CHECK(c, F->d_hist_aux.ensure(std::max<uint64_t>(pa.tile_seg.size(), 1) * 4 *
                                     sort_hist_per_tile(AUX_SYM_BITS, AUX_SYM_BITS + aux_bits)));
    SA_CHECK(c, F->d_segs_seq.ensure(sizeof(SortSeg) * nbk));
    SA_CHECK(c, F->d_segs_aux.ensure(sizeof(SortSeg) * nbk));
    SA_CHECK(c, F->d_tile_seq.ensure(std::max<size_t>(ps.tile_seg.size(), 1) * 4));
    SA_CHECK(c, F->d_tile_aux.ensure(std::max<size_t>(pa.tile_seg.size(), 1) * 4));

    SA_CHECK(c, h2d(c, c->d_blocks.p, c->blocks.data(), sizeof(DevBlock) * nbk, st));
    SA_CHECK(c, h2d(c, F->d_segs_seq.p, ps.segs.data(), sizeof(SortSeg) * nbk, st));
    SA_CHECK(c, h2d(c, F->d_segs_aux.p, pa.segs.data(), sizeof(SortSeg) * nbk, st));
    if (!ps.tile_seg.empty())
        SA_CHECK(c, h2d(c, F->d_tile_seq.p, ps.tile_seg.data(), ps.tile_seg.size() * 4, st));
    if (!pa.tile_seg.empty())
        SA_CHECK(c, h2d(c, F->d_tile_aux.p, pa.tile_seg.data(), pa.tile_seg.size() * 4, st));
    SA_CHECK(c, h2d(c, c->d_tasks.p, tasks.data(), sizeof(CoderTask) * tasks.size(), st));


    cv.tasks = c->d_tasks.as<CoderTask>();
    cv.prs[0] = c->d_prs_seq.as<PRec>();
    cv.prs[1] = c->d_prs_aux.as<PRec>();
    cv.cum[0] = nullptr;   // packed SEQ records
    cv.cum[1] = c->d_cum_aux.as<uint16_t>();
    cv.out = c->d_payload.as<uint8_t>();
    cv.out_len = c->d_out_len.as<uint32_t>();
    cv.lprio = c->l_prio;

    // ---- emit (main stream) ----
    ev_begin(c, PH_EMIT, st);
    {
        const SortView pv_s{F->d_segs_seq.as<SortSeg>(), nullptr, nullptr, ps.total, 0u, nbk};
        const SortView pv_a{F->d_segs_aux.as<SortSeg>(), nullptr, nullptr, pa.total, 0u, nbk};
        const uint32_t pgrid = (uint32_t)(((uint64_t)(nbk + 1) * SORT_TILE + 255) / 256);
        hipLaunchKernelGGL(k_pad_keys, dim3(pgrid), dim3(256), 0, st, pv_s, F->d_seq_k[0].as<uint32_t>(),
                           F->d_seq_k[1].as<uint32_t>());
        hipLaunchKernelGGL(k_pad_keys, dim3(pgrid), dim3(256), 0, st, pv_a, akb[0]->as<uint32_t>(),
                           akb[1]->as<uint32_t>());
    }
    SA_CHECK(c, hipMemsetAsync(c->d_first_sq.p, 0xff, 4 * tasks.size(), st));
    if (nr) {
        hipLaunchKernelGGL(k_emit, dim3(rgrid), dim3(256), 0, st, bv, c->d_counts.as<uint32_t>(),
                           c->d_totals.as<uint32_t>(), c->d_name_p.as<int16_t>(), c->d_name_s.as<int16_t>(),
                           c->d_maxlen.as<uint16_t>(), F->d_seq_k[0].as<uint32_t>(), F->d_seq_v[0].as<uint32_t>(),
                           akb[0]->as<uint32_t>(), nullptr, d_err, dege_maxq);   // (AUX values: the index, run_sort)
        if (c->emit_wave) {   // (SA_EMIT_WAVE=1: round 2's wave-per-read SEQ / QUAL, for A/B)
            hipLaunchKernelGGL(k_emit_sq, dim3(wave_grid(c, nr)), dim3(64 * EMIT_WAVES), 0, st, bv,
                               c->d_counts.as<uint32_t>(), F->d_seq_k[0].as<uint32_t>(), F->d_seq_v[0].as<uint32_t>(),
                               akb[0]->as<uint32_t>(), nullptr, c->d_totals.as<uint32_t>(), dege_maxq, seq_sh,
                               (uint32_t)(EMIT_SEQ | EMIT_QUAL | EMIT_DEGE), nullptr, nullptr);
        } else {
            hipLaunchKernelGGL(seq_sh ? (wq_emit ? k_emit_sq16<2, true> : k_emit_sq16<2, false>)
                                      : (wq_emit ? k_emit_sq16<0, true> : k_emit_sq16<0, false>),
                               dim3(wave_grid(c, (nr + 3) / 4)), dim3(256), 0,
                               st, bv, c->d_counts.as<uint32_t>(), F->d_seq_k[0].as<uint32_t>(),
                               F->d_seq_v[0].as<uint32_t>(), akb[0]->as<uint32_t>(), nullptr, wq_emit, wqc);
            if (dege_maxq && n_ch) {   // the N / IUPAC side streams of the reads that have such bases
                SA_CHECK(c, c->d_dege_list.ensure(4ull * ((uint64_t)nr + 1)));
                SA_CHECK(c, hipMemsetAsync(c->d_dege_list.p, 0, 4, st));
                hipLaunchKernelGGL(k_dege_list, dim3(std::max<uint32_t>(1, std::min<uint32_t>((nr + 255) / 256, c->n_cu * 4))),
                                   dim3(256), 0, st, bv, c->d_counts.as<uint32_t>(), c->d_totals.as<uint32_t>(),
                                   c->d_dege_list.as<uint32_t>());
                hipLaunchKernelGGL(k_emit_sq, dim3(wave_grid(c, nr)), dim3(64 * EMIT_WAVES), 0, st, bv,
                                   c->d_counts.as<uint32_t>(), F->d_seq_k[0].as<uint32_t>(),
                                   F->d_seq_v[0].as<uint32_t>(), akb[0]->as<uint32_t>(), nullptr,
                                   c->d_totals.as<uint32_t>(), dege_maxq, seq_sh, (uint32_t)EMIT_DEGE,
                                   c->d_dege_list.as<uint32_t>(), wq_dege);
            }
        }
        if (al)   // the alignment streams (AlignInfoProcess[PE], decomposeAlignInfo)
            hipLaunchKernelGGL(k_align_emit, dim3(rgrid), dim3(256), 0, st, bv, alv, c->d_acounts.as<uint32_t>(),
                               akb[0]->as<uint32_t>());
    }
    SA_CHECK(c, hipGetLastError());
    ev_finish(c, PH_EMIT, st);
    SortView svs{F->d_segs_seq.as<SortSeg>(), F->d_tile_seq.as<uint32_t>(), F->d_hist_seq.as<uint32_t>(),
                 ps.total, (uint32_t)ps.tile_seg.size(), nbk};
    SortView sva{F->d_segs_aux.as<SortSeg>(), F->d_tile_aux.as<uint32_t>(), F->d_hist_aux.as<uint32_t>(),
                 pa.total, (uint32_t)pa.tile_seg.size(), nbk};
    const SymSink sink_seq{c->d_prs_seq.as<PRec>(), nullptr};   // packed
    const SymSink sink_aux{c->d_prs_aux.as<PRec>(), c->d_cum_aux.as<uint16_t>()};
    if (dense) {   // the blocks' model bitmaps and rank tables; the model counts to the host
        SA_CHECK(c, c->d_aux_bm.ensure(4ull * AUX_DENSE_WORDS * nbk));
        SA_CHECK(c, c->d_aux_tab.ensure(8ull * AUX_DENSE_WORDS * nbk));
        SA_CHECK(c, c->d_aux_nmod.ensure(4ull * nbk));
        if (c->h_aux_nmod_cap < nbk) {
            if (c->h_aux_nmod) SA_CHECK(c, hipHostFree(c->h_aux_nmod));
            c->h_aux_nmod = nullptr;
            c->h_aux_nmod_cap = 0;
            SA_CHECK(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_aux_nmod), 4ull * nbk * 2, 0));
            c->h_aux_nmod_cap = 2ull * nbk;
        }
        SA_CHECK(c, hipMemsetAsync(c->d_aux_bm.p, 0, 4ull * AUX_DENSE_WORDS * nbk, st));
        hipLaunchKernelGGL(k_aux_presence, dim3((uint32_t)((pa.tile_seg.size() + PRESENCE_TILES - 1) / PRESENCE_TILES)),
                           dim3(SORT_THREADS), 0, st, sva,
                           akb[0]->as<uint32_t>(), c->d_aux_bm.as<uint32_t>());
        hipLaunchKernelGGL(k_aux_dense, dim3(nbk), dim3(256), 0, st, c->d_aux_bm.as<uint32_t>(),
                           c->d_aux_tab.as<uint64_t>(), c->d_aux_nmod.as<uint32_t>());
        SA_CHECK(c, hipGetLastError());
        SA_CHECK(c, hipMemcpyAsync(c->h_aux_nmod, c->d_aux_nmod.p, 4ull * nbk, hipMemcpyDeviceToHost, st));
        SA_CHECK(c, hipEventRecord(c->ev_dense, st));
    }

    // ---- throughput phases on st (each fills the GPU): SEQ sort and BASE_MODEL
    //      replay, AUX sort and short SIMPLE_MODEL runs.  Then the long SIMPLE_MODEL
    //      runs (latency-bound, st4: CU set B) and pass R of every coder chain
    //      (st3: the other CUs) start together: pass R waits per segment for
    //      records the long runs have not written yet (k_coder_r) ----
    if (c->prs_zero_p != c->d_prs_aux.p || c->prs_zero_cap < atot * sizeof(PRec)) {
        // (a new buffer, or the last batch did not end normally: zeroed here, all of it)
        SA_CHECK(c, hipMemsetAsync(c->d_prs_aux.p, 0, c->d_prs_aux.cap, st));
    } else if (c->prs_zero_pending) {   // (the previous batch's tail memset: long done by now)
        SA_CHECK(c, hipStreamWaitEvent(st, c->ev_prs_zero, 0));
    }
    c->prs_zero_p = c->d_prs_aux.p;
    c->prs_zero_cap = 0;   // (until this batch's tail zeroes what it wrote)
    c->prs_zero_pending = false;
    ev_begin(c, PH_SORT_SEQ, st);
    const bool seq_inv = seq_bkt && c->seq_inv;   // (see sa_ctx::seq_inv)
    if (run_sort(c, st, ps, F->d_segs_seq, F->d_tile_seq, F->d_hist_seq, skb, svb, seq_lo, seq_hi, seq_sorted_buf,
                 seq_sh != 0, nullptr, seq_inv, seq_max_db))
        return -1;
    ev_finish(c, PH_SORT_SEQ, st);
    ev_begin(c, PH_REPLAY_SEQ, st);
    if (ps.total && seq_bkt) {
        const std::vector<int> dg = sort_digits(seq_lo, seq_hi, seq_max_db);   // (one pass: its digit width)
        if (dg.size() != 1) {
            c->err = "internal: the SEQ bucket sort is not one pass";
            return -1;
        }
        const uint32_t bgrid = nbk << dg[0];
        SA_CHECK(c, F->d_bkt_spare.ensure(256ull * bgrid));
        PRec* spare = F->d_bkt_spare.as<PRec>();
        const uint32_t* border = nullptr;
        if (c->bkt_lpt) {
            SA_CHECK(c, F->d_bkt_order.ensure(4ull << dg[0]));
            hipLaunchKernelGGL(k_bkt_order, dim3(1), dim3(1u << dg[0]), 0, st, svs, 1u << dg[0],
                               F->d_bkt_order.as<uint32_t>());
            border = F->d_bkt_order.as<uint32_t>();
        }
        uint64_t* bprobe = nullptr;
        if (c->bkt_probe) {
            SA_CHECK(c, c->d_bkt_probe.ensure(32ull * bgrid));
            SA_CHECK(c, hipMemsetAsync(c->d_bkt_probe.p, 0, 32ull * bgrid, st));
            bprobe = c->d_bkt_probe.as<uint64_t>();
        }
        if (seq_inv) {
            // records in sorted order into the other value buffer (the bucket
            // pass over implicit values never read it), then gathered through
            // the inverse permutation the pass left in d_seq_v[sorted]
            PRec* rs = F->d_seq_v[seq_sorted_buf ^ 1].as<PRec>();
            hipLaunchKernelGGL(k_replay_seq_bkt<true>, dim3(nbk << dg[0]), dim3(64), (size_t)5 * ((1u << bkt_sb) + 64), st, svs,
                               F->d_seq_k[seq_sorted_buf].as<uint32_t>(), nullptr, SymSink{rs, nullptr},
                               (uint32_t)dg[0], (uint32_t)bkt_sb, (uint32_t)(seq_sh + dg[0]), spare, bprobe, border);
            hipLaunchKernelGGL(k_seq_unpermute, dim3(8 * (uint32_t)((ps.tile_seg.size() + 7) / 8)),
                               dim3(SORT_THREADS), 0, st, svs, F->d_seq_v[seq_sorted_buf].as<uint32_t>(), rs,
                               c->d_prs_seq.as<PRec>());
        } else {
            hipLaunchKernelGGL(k_replay_seq_bkt<false>, dim3(nbk << dg[0]), dim3(64), (size_t)5 * ((1u << bkt_sb) + 64), st, svs,
                               F->d_seq_k[seq_sorted_buf].as<uint32_t>(), F->d_seq_v[seq_sorted_buf].as<uint32_t>(),
                               sink_seq, (uint32_t)dg[0], (uint32_t)bkt_sb, (uint32_t)(seq_sh + dg[0]), spare, bprobe, border);
        }
        if (bprobe) {   // one line per wave: block, digit (its rank with k_bkt_order), start / end (us, 100 MHz), cycles, steps, shared steps, xcc
            std::vector<uint64_t> pr(4ull * bgrid);
            SA_CHECK(c, hipMemcpyAsync(pr.data(), bprobe, 32ull * bgrid, hipMemcpyDeviceToHost, st));
            SA_CHECK(c, hipStreamSynchronize(st));
            if (FILE* f = std::fopen(c->bkt_probe, "a")) {
                for (uint32_t w = 0; w < bgrid; w++) {
                    const uint64_t* q = &pr[4ull * w];
                    if (!q[1]) continue;
                    std::fprintf(f, "%u %u %.2f %.2f %llu %llu %llu %llu\n", border ? w % nbk : w >> dg[0],
                                 border ? w / nbk : w & ((1u << dg[0]) - 1),   // (k_bkt_order: the digit's rank)
                                 (double)q[0] / 100.0, (double)q[1] / 100.0, (unsigned long long)q[2],
                                 (unsigned long long)(q[3] & 0xffffff), (unsigned long long)((q[3] >> 24) & 0xffffff),
                                 (unsigned long long)(q[3] >> 48));
                }
                std::fclose(f);
            }
        }
    } else if (ps.total) {
        SA_CHECK(c, hipMemsetAsync(F->d_nseq_long.p, 0, 4, st));
        hipLaunchKernelGGL(k_replay_seq, dim3((uint32_t)ps.tile_seg.size()), dim3(SORT_THREADS), 0, st, svs,
                           F->d_seq_k[seq_sorted_buf].as<uint32_t>(), F->d_seq_v[seq_sorted_buf].as<uint32_t>(),
                           sink_seq, F->d_seq_longs.as<uint64_t>(), F->d_nseq_long.as<uint32_t>(), seq_sh);
        hipLaunchKernelGGL(k_replay_seq_long, dim3((uint32_t)std::min<uint64_t>(max_seq_long, 2048)), dim3(128), 0,
                           st, svs, F->d_seq_k[seq_sorted_buf].as<uint32_t>(),
                           F->d_seq_v[seq_sorted_buf].as<uint32_t>(), sink_seq, F->d_seq_longs.as<uint64_t>(),
                           F->d_nseq_long.as<uint32_t>(), d_err, seq_sh);
    }
    SA_CHECK(c, hipGetLastError());
    ev_finish(c, PH_REPLAY_SEQ, st);
    ev_begin(c, PH_SORT_AUX, st);
    bool runs_from_hist = false;   // one dense pass: the run lists from the scan (k_runs_dense)
    if (dense) {
        // (the counts were read back right after the emit: the SEQ sort and
        // replay queued above keep the device busy while the host waits here)
        SA_CHECK(c, hipEventSynchronize(c->ev_dense));
        uint32_t dmax = 0;
        for (uint32_t b = 0; b < nbk; b++) dmax = std::max(dmax, c->h_aux_nmod[b]);
        const int dbits = dmax > 512 ? (int)AUX_DENSE_BITS : 9;
        runs_from_hist = dbits == 9 && !std::getenv("SA_FIND_RUNS");   // (SA_FIND_RUNS=1: k_find_runs, A/B)
        if (run_sort(c, st, pa, F->d_segs_aux, F->d_tile_aux, F->d_hist_aux, akb, avb, 0, dbits, aux_sorted_buf, true,
                     c->d_aux_tab.as<uint64_t>()))
            return -1;
        if (aux_sorted_buf != 1) {   // (two dense passes: the result is in the front scratch)
            SA_CHECK(c, hipMemcpyAsync(c->d_auxp_k.p, F->d_auxs_k.p, atot * 4, hipMemcpyDeviceToDevice, st));
            SA_CHECK(c, hipMemcpyAsync(c->d_auxp_v.p, F->d_auxs_v.p, atot * 4, hipMemcpyDeviceToDevice, st));
            aux_sorted_buf = 1;
            c->aux_dense = false;   // (this input has too many models per block for one pass)
        }
    } else if (run_sort(c, st, pa, F->d_segs_aux, F->d_tile_aux, F->d_hist_aux, akb, avb, AUX_SYM_BITS,
                        AUX_SYM_BITS + aux_bits, aux_sorted_buf, true)) {
        return -1;
    }
    ev_finish(c, PH_SORT_AUX, st);
    ev_begin(c, PH_REPLAY_AUX, st);
    if (pa.total && akb[aux_sorted_buf] != &c->d_auxp_k) {
        c->err = "internal: sorted AUX keys not in the context's buffer";
        return -1;
    }
    const uint32_t* ak = akb[aux_sorted_buf]->as<uint32_t>();
    const uint32_t* av = avb[aux_sorted_buf]->as<uint32_t>();
    uint32_t* ctr = c->d_nlong.as<uint32_t>();
    const RunLists rl{F->d_short_at.as<uint64_t>(), ctr, c->d_longs.as<LongRun>(), ctr + 1, ctr + 2, max_long, ctr + 3,
                      c->d_huge_sorted.as<LongRun>()};
    SA_CHECK(c, hipMemsetAsync(ctr, 0, 16, st));
    if (pa.total) {
        if (runs_from_hist)
            hipLaunchKernelGGL(k_runs_dense<9>, dim3((nbk * 512u + 255) / 256), dim3(256), 0, st, sva, ak, rl);
        else
            hipLaunchKernelGGL(k_find_runs, dim3((uint32_t)((pa.total / FIND_ITEMS + 255) / 256)), dim3(256), 0, st,
                               sva, ak, rl);
        hipLaunchKernelGGL(k_sort_huge, dim3(1), dim3(1024), 0, st, rl);
        hipLaunchKernelGGL(k_replay_aux_short, dim3(SHORT_GRID), dim3(RP_THREADS), 0, st, sva, ak, av, sink_aux, rl,
                           d_err);
    }
    SA_CHECK(c, hipGetLastError());
    SA_CHECK(c, hipEventRecord(c->ev_fork_seq, st));
    // the front scratch is free once the kernels enqueued so far on st are done
    SA_CHECK(c, hipEventRecord(F->ev_free, st));
    F->have_ev = true;
    front_lock->freed = true;
    front_lock->unlock();
    hipStream_t st3 = c->st3, st4 = c->st4;
    if (c->host_waits) SA_CHECK(c, hipEventSynchronize(c->ev_fork_seq));
    else SA_CHECK(c, hipStreamWaitEvent(st4, c->ev_fork_seq, 0));
    if (pa.total && !c->test_skip_long)
        hipLaunchKernelGGL(k_replay_aux_long, dim3(c->long_grid), dim3(128), c->long_lds, st4, rl, ak, av, sink_aux,
                           d_err, c->chain_prio);
    SA_CHECK(c, hipGetLastError());
    SA_CHECK(c, hipEventRecord(c->ev_long_done, st4));
    ev_finish(c, PH_REPLAY_AUX, st4);

    // ---- range coders: every chain in one launch on st3, longest first
    //      (concurrent latency-bound launches land on shared SIMDs); the L passes
    //      after the long runs are done ----
    if (!c->host_waits) SA_CHECK(c, hipStreamWaitEvent(st3, c->ev_fork_seq, 0));
    std::vector<uint32_t> out_len;
    {
        // (SA_RV_V6_MAX, see rv_v6_max) the SMEM-fed chain only when few other
        // contexts' chains are in flight
        if (c->rv_variant < 0 && c->rv_batch == 6 && F->tails.load() > c->rv_v6_max) c->rv_batch = 5;
        F->tails++;
        const int rc = coder_run(c, tasks, cv, st3, PH_CODER_R, PH_CODER_L, c->ev_long_done, exact, out_len, payload);
        F->tails--;
        if (rc) return rc;
    }
    // the records this batch wrote back to zero, in its tail (after the L passes on st3)
    SA_CHECK(c, hipMemsetAsync(c->d_prs_aux.p, 0, atot * sizeof(PRec), st3));
    SA_CHECK(c, hipEventRecord(c->ev_prs_zero, st3));
    c->prs_zero_cap = c->d_prs_aux.cap;
    c->prs_zero_pending = true;
    // the final arena from the streams' real sizes: per block its encaps
    // (<= 32 header bytes each), count / MD5s, and the ID-bin first ID
    uint64_t final_bytes = 0;
    std::vector<uint64_t> task_out_base(tasks.size());
    for (size_t t = 0; t < tasks.size(); t++) task_out_base[t] = tasks[t].out_base;
    c->final_base.assign(nbk, 0);
    for (uint32_t b = 0; b < nbk; b++) {
        uint64_t blk = 64 + 2 + 0x10000 + 96;
        for (int s = 0; s < NSTREAM; s++)
            if (asmb[b].task[s] != NO_TASK) blk += out_len[asmb[b].task[s]] + 32;
        asmb[b].out_base = final_bytes;
        c->final_base[b] = final_bytes;
        final_bytes = align_up(final_bytes + blk, 16);
    }
    SA_CHECK(c, c->d_final.ensure(std::max<uint64_t>(final_bytes, 16)));
    SA_CHECK(c, h2d(c, c->d_asm.p, asmb.data(), sizeof(AsmBlock) * nbk, st));
    SA_CHECK(c, h2d(c, c->d_task_out_base.p, task_out_base.data(), 8 * tasks.size(), st));

    // ---- assembly (after MD5) ----
    if (cfg->md5) SA_CHECK(c, hipStreamWaitEvent(st, c->ev_md5_done, 0));
    ev_begin(c, PH_ASM, st);
    AsmView asv{c->d_asm.as<AsmBlock>(), c->d_task_out_base.as<uint64_t>(), c->d_asm_copies.as<uint32_t>()};
    hipLaunchKernelGGL(k_assemble, dim3((nbk + 63) / 64), dim3(64), 0, st, bv, asv, c->d_out_len.as<uint32_t>(),
                       c->d_digests.as<uint32_t>(), c->d_final.as<uint8_t>(), c->d_final_len.as<uint64_t>());
    hipLaunchKernelGGL(k_assemble_copy, dim3(nbk * ASM_SLICES), dim3(256), 0, st, asv, c->d_payload.as<uint8_t>(),
                       c->d_final.as<uint8_t>());
    SA_CHECK(c, hipGetLastError());
    ev_finish(c, PH_ASM, st);
    ev_finish(c, PH_TOTAL, st);

    c->final_len.assign(nbk, 0);
    SA_CHECK(c, d2h(c, c->final_len.data(), c->d_final_len.p, 8ull * nbk, st));
    SA_CHECK(c, d2h(c, herr, c->d_err.p, 16, st));
    SA_CHECK(c, sync_d2h(c, st));
    if (herr[0]) {
        char buf[128];
        std::snprintf(buf, sizeof buf, "device error bits 0x%x", herr[0]);
        c->err = buf;
        return -1;
    }
    if (c->timing) {
        for (int i = 0; i < PH_N; i++) {
            c->ph_ms[i] = 0.f;
            if (i == PH_MD5 && !cfg->md5) continue;
            (void)hipEventElapsedTime(&c->ph_ms[i], c->ev_beg[i], c->ev_end[i]);
        }
    }
    if (trace) fprintf(stderr, "[align] batch queued\n");
    c->have_output = true;
    c->front_warm = true;
    return 0;
}

// A batch that failed part-way (E_CODER, a device error bit, a failed call)
// may still have work in flight on the context's streams -- e.g. the long-run
// replay writing d_prs_aux after pass R gave up: the next batch's full memset
// of that buffer (prs_zero_cap is 0 after a failure) must not race it.
void drain_after_error(sa_ctx* c)
{
    for (hipStream_t s : {c->st, c->st2, c->st3, c->st4, c->st5})
        if (s) (void)hipStreamSynchronize(s);
    c->prs_zero_cap = 0;
    c->prs_zero_pending = false;
}

}  // namespace

extern "C" {

int sa_run_input(sa_ctx* c, const sa_input* I, const sa_cfg* cfg)
{
    if (!c) return -1;
    int rc = run_input(c, I, cfg, true);
    if (rc == 2) {   // a stream outgrew its exact payload cap (rare): drain, re-run with the bound
        for (hipStream_t s : {c->st, c->st2, c->st3, c->st4}) SA_CHECK(c, hipStreamSynchronize(s));
        rc = run_input(c, I, cfg, false);
    }
    if (rc) drain_after_error(c);
    return rc ? -1 : 0;
}

int sa_phase_times(const sa_ctx* c, const char** names, float* ms, int max)
{
    if (!c || !c->timing) return 0;
    int n = std::min(max, (int)PH_N);
    for (int i = 0; i < n; i++) {
        if (names) names[i] = kPhaseNames[i];
        if (ms) ms[i] = c->ph_ms[i];
    }
    return n;
}

int sa_fetch(sa_ctx* c, sa_out* out, int n)
{
    if (!c || !c->have_output) return -1;
    if ((uint32_t)n != c->final_len.size()) {
        c->err = "sa_fetch: block count mismatch";
        return -1;
    }
    SA_CHECK(c, hipSetDevice(c->device));
    for (int b = 0; b < n; b++) {
        if (c->final_len[(size_t)b] > out[b].cap) {
            c->err = "sa_fetch: output buffer too small";
            return -1;
        }
        SA_CHECK(c, hipMemcpyAsync(out[b].data, c->d_final.as<uint8_t>() + c->final_base[(size_t)b],
                                   c->final_len[(size_t)b], hipMemcpyDeviceToHost, c->st));
        out[b].size = c->final_len[(size_t)b];
    }
    SA_CHECK(c, hipStreamSynchronize(c->st));
    return 0;
}

int sa_fetch_sizes(const sa_ctx* c, uint64_t* sizes, int n)
{
    if (!c || !c->have_output || (n && !sizes) || (uint32_t)n != c->final_len.size()) return -1;
    for (int b = 0; b < n; b++) sizes[b] = c->final_len[(size_t)b];
    return 0;
}

int sa_code_records(sa_ctx* c, int nstreams, const uint32_t* lens, const uint16_t* cum, const uint16_t* freq,
                    const uint16_t* tot, uint8_t* out, uint64_t out_cap, uint64_t* out_lens)
{
    if (!c || nstreams < 0 || (nstreams && (!lens || !out || !out_lens))) return -1;
    SA_CHECK(c, hipSetDevice(c->device));
    std::vector<CoderTask> tasks((size_t)nstreams);
    uint64_t nsym = 0, payload = 0, segs = 0;
    for (int s = 0; s < nstreams; s++) {
        CoderTask& tk = tasks[(size_t)s];
        tk.rec_base = nsym;
        tk.n = lens[s];
        tk.space = 1;   // wide records
        tk.nseg = tk.n ? (tk.n + SEG_SYMS - 1) / SEG_SYMS : 1;
        tk.seg_base = segs;
        tk.out_base = payload;
        const uint64_t cap = 2ull * tk.n + 64;
        if (cap > 0xffffffffull) {
            c->err = "sa_code_records: stream too long";
            return -1;
        }
        tk.out_cap = (uint32_t)cap;
        nsym += tk.n;
        segs += tk.nseg;
        payload = align_up(payload + cap, 16);
    }
    std::vector<PRec> prs(nsym + 128, PRec{0});
    std::vector<uint16_t> cm(nsym + 128, 0);
    for (uint64_t i = 0; i < nsym; i++) {
        const uint32_t t = tot[i], f = freq[i], cu = cum[i];
        if (t < 2 || f < 1 || cu + f > t) {
            c->err = "sa_code_records: invalid (cum, freq, tot)";   // the reference abort()s
            return -1;
        }
        prs[i] = PRec{t | (f << 16)};
        cm[i] = (uint16_t)cu;
    }
    hipStream_t st = c->st;
    SA_CHECK(c, c->d_prs_seq.ensure(prs.size() * sizeof(PRec)));
    SA_CHECK(c, c->d_cum_seq.ensure(cm.size() * 2));
    SA_CHECK(c, c->d_tasks.ensure(sizeof(CoderTask) * std::max<size_t>(tasks.size(), 1)));
    SA_CHECK(c, c->d_out_len.ensure(4 * std::max<size_t>(tasks.size(), 1)));
    SA_CHECK(c, c->d_payload.ensure(std::max<uint64_t>(payload, 16)));
    SA_CHECK(c, hipMemcpyAsync(c->d_prs_seq.p, prs.data(), prs.size() * sizeof(PRec), hipMemcpyHostToDevice, st));
    SA_CHECK(c, hipMemcpyAsync(c->d_cum_seq.p, cm.data(), cm.size() * 2, hipMemcpyHostToDevice, st));
    if (!tasks.empty())
        SA_CHECK(c, hipMemcpyAsync(c->d_tasks.p, tasks.data(), sizeof(CoderTask) * tasks.size(), hipMemcpyHostToDevice, st));
    CoderView cv{};
    cv.tasks = c->d_tasks.as<CoderTask>();
    cv.prs[0] = cv.prs[1] = c->d_prs_seq.as<PRec>();
    cv.cum[0] = cv.cum[1] = c->d_cum_seq.as<uint16_t>();
    cv.out = c->d_payload.as<uint8_t>();
    cv.out_len = c->d_out_len.as<uint32_t>();
    c->have_output = false;
    if (coder_buffers(c, tasks.size(), segs, cv)) return -1;
    SA_CHECK(c, hipMemsetAsync(c->d_first_sq.p, 0xff, 4 * std::max<size_t>(tasks.size(), 1), st));
    std::vector<uint32_t> out_len;
    if (coder_run(c, tasks, cv, st, -1, -1, nullptr, false, out_len, payload)) return -1;
    std::vector<uint32_t> ol(tasks.size());
    if (!tasks.empty())
        SA_CHECK(c, hipMemcpyAsync(ol.data(), c->d_out_len.p, 4 * tasks.size(), hipMemcpyDeviceToHost, st));
    SA_CHECK(c, hipStreamSynchronize(st));
    uint64_t o = 0;
    for (size_t s = 0; s < tasks.size(); s++) {
        if (o + ol[s] > out_cap) {
            c->err = "sa_code_records: output buffer too small";
            return -1;
        }
        SA_CHECK(c, hipMemcpyAsync(out + o, c->d_payload.as<uint8_t>() + tasks[s].out_base, ol[s], hipMemcpyDeviceToHost, st));
        out_lens[s] = ol[s];
        o += ol[s];
    }
    SA_CHECK(c, hipStreamSynchronize(st));
    return 0;
}

uint32_t sa_coder_restarts(const sa_ctx* c) { return c ? c->coder_restarts : 0; }

uint64_t sa_device_bytes(const sa_ctx* c) { return c ? const_cast<sa_ctx*>(c)->held_bytes() : 0; }

void sa_stream_stats(const sa_ctx* c, uint64_t* max_symbols, uint64_t* total_symbols)
{
    if (max_symbols) *max_symbols = c ? c->max_stream_syms : 0;
    if (total_symbols) *total_symbols = c ? c->total_stream_syms : 0;
}

// HBM a block needs while its batch is encoded: per SEQ symbol the
// double-buffered u32 keys and values plus the 4-byte record (20 B); per AUX
// symbol the same plus its u16 cum (22 B); per symbol up to 2 payload and 2
// final bytes; per read the count columns and the read arrays; the input.
// AUX symbols ~ qualities + name bytes + 8 per read (len, name tokens, dege).
static uint64_t block_footprint(const sa_block& b)
{
    uint64_t bases = 0, nb = 0;
    for (uint32_t r = 0; r < b.nreads; r++) {
        bases += (uint64_t)std::max(b.seq_lens[r], 0);
        nb += b.name_lens[r];
    }
    const uint64_t aux = bases + nb + 8ull * b.nreads;
    return (20 + 4) * bases + (22 + 4) * aux + (nb + 2 * bases + 16) + 64ull * b.nreads;
}

int sa_encode_blocks(sa_ctx* ctx, const sa_block* in, int n, const sa_cfg* cfg, sa_out* out)
{
    if (!ctx || !cfg || (n > 0 && (!in || !out))) return -1;
    if (n == 0) return 0;
    SA_CHECK(ctx, hipSetDevice(ctx->device));
    // Blocks are independent, so a batch larger than the HBM this context can
    // use is encoded as consecutive sub-batches (outputs keep the input order).
    // Budget: 85 % of what is free plus what this context already holds (its
    // buffers are reused).  SA_BATCH_BASES caps the bases per sub-batch (tests).
    size_t free_b = 0, total_b = 0;
    SA_CHECK(ctx, hipMemGetInfo(&free_b, &total_b));
    const uint64_t budget = (uint64_t)((double)(free_b + ctx->held_bytes()) * 0.85);
    uint64_t cap_bases = ~0ull;
    if (const char* e = std::getenv("SA_BATCH_BASES")) {
        const unsigned long long v = std::strtoull(e, nullptr, 10);
        if (v > 0) cap_bases = v;
    }
    int b0 = 0;
    while (b0 < n) {
        int b1 = b0;
        uint64_t bases = 0, bytes = 0;
        while (b1 < n) {
            uint64_t ls = 0;
            for (uint32_t r = 0; r < in[b1].nreads; r++) ls += (uint64_t)std::max(in[b1].seq_lens[r], 0);
            const uint64_t fb = block_footprint(in[b1]);
            if (b1 > b0 && (bases + ls > cap_bases || bytes + fb > budget)) break;
            bases += ls;
            bytes += fb;
            b1++;
        }
        const auto t0 = std::chrono::steady_clock::now();
        if (sa_stage(ctx, in + b0, b1 - b0)) return -1;
        const auto t1 = std::chrono::steady_clock::now();
        if (sa_run(ctx, cfg)) return -1;
        const auto t2 = std::chrono::steady_clock::now();
        if (sa_fetch(ctx, out + b0, b1 - b0)) return -1;
        if (ctx->trace) {   // SA_TRACE: per sub-batch host-side stage timings
            const auto t3 = std::chrono::steady_clock::now();
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            std::string ph;
            for (int i = 0; i < PH_N; i++) {
                char pb[48];
                std::snprintf(pb, sizeof pb, " %s %.0f", kPhaseNames[i], ctx->ph_ms[i]);
                ph += pb;
            }
            std::fprintf(stderr,
                         "seqarc_amd[%p]: %d blocks: stage %.1f ms, run %.1f ms, fetch %.1f ms, grows %u, "
                         "alloc %.1f ms (all contexts); phases ms:%s\n",
                         (void*)ctx, b1 - b0, ms(t0, t1), ms(t1, t2), ms(t2, t3), g_grows.load(),
                         g_alloc_ns.load() / 1e6, ph.c_str());
        }
        b0 = b1;
    }
    return 0;
}

}  // extern "C"

// FASTQ text parsed on the device (sa_stage_text)
#include "sa_parse.hip"

// the HASH reference-index path
#include "sa_hash.hip"
