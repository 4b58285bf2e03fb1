/*
 * seqarc_amd.h -- C-ABI of the MI355X SeqArc block encoder (libseqarc_amd.so).
 *
 * Plain pointers and sizes only.  The reference (SeqArc-1.6) is one monolithic
 * executable with no plugin API; the seam this library replaces is the per-block
 * encoder call inside the encode thread:
 *
 *   int EncapFqzComp::doFqzEncode(SeqArcMemBuf*, DebugInfo*)   SeqArc-1.6@0x42d2d0
 *     called from ISeqArcEncodeThread::doTask                   SeqArc-1.6@0x433dd0
 *     after SeqArcMemBuf::calcBlockMd5@0x414d90 and DegeInfoProcess@0x433a10
 *
 * sa_encode_blocks() takes a batch of parsed blocks (the SeqArcMemBuf SoA:
 * IDs + u16 lengths, bases + i32 lengths, qualities; PE reads interleaved
 * r1,r2) and returns, per block, exactly the bytes doFqzEncode writes
 * ("81 <size4> ..." : count, len, ID, qual, dege streams, seq).
 *
 * Errors: a non-zero return and sa_last_error(); the reference abort()s on a
 * coder invariant violation -- here the batch fails and no output is produced.
 * Thread-safety: one sa_ctx per host thread / device; contexts are independent.
 */
#ifndef SEQARC_AMD_H
#define SEQARC_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sa_ctx sa_ctx;

/* One parsed block (SeqArcMemBuf fields +0x80/+0xc0, +0x88/+0xd0, +0x90, +0x4). */
typedef struct {
    const uint8_t *names;       /* concatenated IDs without '@'            */
    const uint16_t *name_lens;  /* nreads entries                           */
    const uint8_t *seq;         /* concatenated bases                       */
    const int32_t *seq_lens;    /* nreads entries                           */
    const uint8_t *qual;        /* concatenated quals (same lengths)        */
    uint32_t nreads;
} sa_block;

/* Encoder parameters (SeqArcParam fields of the no-reference path). */
typedef struct {
    int32_t slevel;    /* param+0x1b54 (default 3): seq order k = slevel + 7      */
    int32_t qlevel;    /* param+0x1b58 (default 2)                                */
    int32_t md5;       /* param+0x1880 (default 1): per-block MD5 of ID/seq/qual  */
    int32_t bin_mode;  /* param+0x18a4 (ID template byte 0, see sa_analyze_ids)   */
    double lossy;      /* -l R (param+0x1878; param+0x1870 set iff R > 0): R-Block
                          quality pre-pass rblock@0x426c10, no quality MD5; 0 = off */
} sa_cfg;

typedef struct {
    uint8_t *data;     /* caller-allocated, >= sa_output_bound() bytes  */
    uint64_t cap;
    uint64_t size;     /* written                                     */
} sa_out;

/* ---- lifecycle ------------------------------------------------------- */
sa_ctx *sa_create(int device);               /* NULL if no usable gfx950 device */
/* A context of the same device sharing `peer`'s front scratch: the contexts'
 * throughput-bound fronts (symbol extraction, sorts, short model runs) run one
 * at a time on it while each one's latency-bound range coder chains overlap the
 * next front (the pipeline of encoder lanes on one GPU). */
sa_ctx *sa_create_shared(int device, sa_ctx *peer);
void sa_destroy(sa_ctx *ctx);
const char *sa_last_error(const sa_ctx *ctx);
const char *sa_version(void);

/* ---- one-shot batch: replaces doFqzEncode@0x42d2d0 per block ---------- */
uint64_t sa_output_bound(const sa_block *blk);
/* page-locks host memory the caller hands to the encoder (block SoA buffers)
 * so that staging is a DMA instead of a pageable copy through the runtime's
 * bounce buffer (4.9 vs 56 GB/s H2D on MI355X); unregister before freeing it.
 * 0 on success.  (The reader/parser buffers of seqarc_amd -c.) */
int sa_host_register(void *p, uint64_t bytes);
int sa_host_unregister(void *p);
/* Batches above 3 Gi bases (env SA_BATCH_BASES lowers the cap) are encoded as
 * consecutive sub-batches; outputs keep the input order. */
int sa_encode_blocks(sa_ctx *ctx, const sa_block *in, int n, const sa_cfg *cfg, sa_out *out);

/* ---- staged API (inputs resident in HBM; used by bench.py) ------------ */
/* the batch size (blocks) the context's buffers are sized for from its first
 * batch on, when its first batches are smaller (a re-allocation synchronises
 * the device); 0: as each batch needs */
void sa_set_reserve(sa_ctx *ctx, uint32_t blocks);
/* device buffer re-allocations in this process so far (each one's hipFree
 * synchronises the device) and the host time spent allocating, in ms */
void sa_alloc_stats(uint32_t *grows, double *alloc_ms);
int sa_stage(sa_ctx *ctx, const sa_block *in, int n);     /* H2D copy of a batch   */
/* FASTQ text of one block as the reader cut it (doReadPEJob@0x432d10 /
 * cultPEbuf@0x432180 hand these to getBlockRead[PE]): file 1 and, for PE,
 * file 2 (text2 = NULL: single-end). */
typedef struct sa_text_block {
    const uint8_t *text1;
    uint64_t len1;
    const uint8_t *text2;
    uint64_t len2;
} sa_text_block;
typedef struct sa_text_info {   /* per block, written by sa_stage_text */
    uint32_t nreads;
    uint32_t len_long;          /* a read > 65535 bp (SeqArcMemBuf+0x2)     */
    uint64_t name_bytes;
    uint64_t seq_bytes;
    uint64_t out_bound;         /* sa_output_bound of the parsed block      */
} sa_text_info;
/* Stages a batch given as FASTQ text: the texts are copied to HBM (a DMA when
 * they are in sa_host_alloc memory) and parsed there into the batch sa_stage
 * would upload -- getBlockRead@0x411b60 (SE) / getBlockReadPE@0x412920 (PE),
 * byte for byte the blocks sa_parse_se / sa_parse_pe give.  info (optional, n
 * entries) gets each block's counts.  Then sa_run / sa_fetch.  -1 and
 * sa_last_error where sa_parse_* fail.  The texts may be reused on return. */
int sa_stage_text(sa_ctx *ctx, const sa_text_block *in, int n, sa_text_info *info);
/* page-locked host memory for the reader's text windows (2 MiB-aligned, huge pages
 * asked for, registered portable with the runtime); free with sa_host_free */
void *sa_host_alloc(uint64_t bytes);
void sa_host_free(void *p);
int sa_run(sa_ctx *ctx, const sa_cfg *cfg);                /* encode the staged batch */
int sa_fetch(sa_ctx *ctx, sa_out *out, int n);             /* D2H of the encaps     */
/* the encoded size of each of the last run's n blocks (what sa_fetch will
 * copy), so a caller can size its output buffers before the fetch instead of
 * reserving sa_output_bound for every block; -1 on a count mismatch */
int sa_fetch_sizes(const sa_ctx *ctx, uint64_t *sizes, int n);
/* per-phase device time (ms) of the last sa_run, measured with HIP events on
 * the stream each phase runs on; returns the number of phases written */
int sa_phase_times(const sa_ctx *ctx, const char **names, float *ms, int max);
void sa_set_timing(sa_ctx *ctx, int on);
/* HBM bytes the context's work buffers hold (they grow to the largest batch) */
uint64_t sa_device_bytes(const sa_ctx *ctx);
/* HBM bytes of the (possibly shared) front scratch */
uint64_t sa_front_bytes(const sa_ctx *ctx);

/* ---- resident inputs: a batch uploaded once, encoded by any context ----
 * The reference keeps a pool of parsed blocks between its reader and its
 * encode threads (ReadBufPool::getEmptybuf/getFullbuf@0x4341e0/0x4343d0); an
 * sa_input is such a batch resident in HBM.  Several contexts of one device
 * (one host thread each) encode their batches concurrently: one batch's
 * throughput-bound front overlaps another's latency-bound range coder. */
typedef struct sa_input sa_input;
sa_input *sa_input_create(int device, const sa_block *in, int n);   /* NULL on error */
void sa_input_destroy(sa_input *in);
int sa_run_input(sa_ctx *ctx, const sa_input *in, const sa_cfg *cfg);   /* then sa_fetch */
/* an empty input of a device, filled by sa_stage_text_input: FASTQ text staged
 * and parsed on the device with ctx's stream (ctx may be another context than
 * the one that later runs the input: the command line stages a context's next
 * batch while the context encodes the current one) */
sa_input *sa_input_empty(int device);
int sa_stage_text_input(sa_ctx *ctx, sa_input *in, const sa_text_block *blocks, int n, sa_text_info *info);
/* Streaming form of sa_stage_text (round 6): the reader hands each block's text
 * over as it cuts it (doReadPEJob@0x432d10 / ReadBufPool::addFullbuf@0x434900),
 * and its bytes go to the device at once, so the reader's buffer is free again
 * before the rest of the batch is cut.  in = NULL: the context's own input.
 * Each input has two text arenas (slot 0 / 1): a thread of its own may fill one
 * while the context encodes the batch parsed from the other.  Block `index` of
 * a batch of at most nmax blocks lands at 2 x index x stride (file 1) and
 * (2 x index + 1) x stride (file 2); stride >= every text length (the reader's
 * window).  Block 0 of a batch first.  Returns once the copy is done. */
int sa_text_upload(sa_ctx *ctx, sa_input *in, int slot, int index, int nmax, const sa_text_block *blk,
                   uint64_t stride);
/* Parses the n blocks uploaded into arena `slot` (lens: their lengths; text2
 * non-NULL for PE) into the input, byte for byte what sa_stage_text gives.
 * The input must not be in use (its previous sa_run* returned). */
int sa_text_parse(sa_ctx *ctx, sa_input *in, int slot, const sa_text_block *lens, int n, uint64_t stride,
                  sa_text_info *info);

/* ---- range coder over pre-modelled symbols ---------------------------- */
/* The carry-less range coder inlined in every EncapFqzComp::encode_* (e.g.
 * encode_seq@0x422010-0x422085, finish @0x424a1c), applied to nstreams streams
 * of (cum, freq, tot) triples laid out back to back (stream s has lens[s]
 * symbols).  Writes the streams' coded bytes back to back into out and their
 * lengths into out_lens.  Rejects cum + freq > tot (the reference abort()s). */
int sa_code_records(sa_ctx *ctx, int nstreams, const uint32_t *lens, const uint16_t *cum,
                    const uint16_t *freq, const uint16_t *tot, uint8_t *out, uint64_t out_cap,
                    uint64_t *out_lens);
/* streams restarted after a carry-less squeeze in the last sa_run / sa_code_records */
uint32_t sa_coder_restarts(const sa_ctx *ctx);
/* symbols of the longest coder stream and of all streams in the last sa_run
 * (the serial range chain of the longest stream bounds the batch) */
void sa_stream_stats(const sa_ctx *ctx, uint64_t *max_symbols, uint64_t *total_symbols);

/* ---- host-side mirrors of the reference's block plumbing -------------- */
/* Block cut: SeqArcRead::doReadJob@0x432a80 / cultbuf@0x432530 / getEndPos@0x4320c0
 * (SE) and doReadPEJob@0x432d10 / cultPEbuf@0x432180 (PE).  Returns #blocks. */
int64_t sa_cut_se(const uint8_t *text, uint64_t len, uint64_t block_size,
                  uint64_t *ends, uint64_t max_blocks);
int64_t sa_cut_pe(const uint8_t *t1, uint64_t len1, const uint8_t *t2, uint64_t len2,
                  uint64_t block_size, uint64_t *ends1, uint64_t *ends2, uint64_t max_blocks);
/* Streaming forms (the reader thread's view, doReadJob / doReadPEJob): the end of
 * the next block in a window of the input that starts at a block boundary.
 * first/flen: the input's first line, '\n' included (getFirstLine@0x431eb0);
 * eof: the window holds the rest of that input.  SE: returns the block's
 * bytes, or -1 when the window is too short (read more) or no cut exists.  PE:
 * 0 and the block's bytes of each file in end1/end2, or -1 likewise. */
int64_t sa_cut_next_se(const uint8_t *win, uint64_t avail, int eof, uint64_t block_size,
                       const uint8_t *first, uint64_t flen);
int sa_cut_next_pe(const uint8_t *w1, uint64_t avail1, int eof1, const uint8_t *w2, uint64_t avail2, int eof2,
                   uint64_t block_size, const uint8_t *first, uint64_t flen, uint64_t *end1, uint64_t *end2);
/* sa_cut_next_pe with the newline counts of both windows given: k1 / k2 =
 * newlines in the first min(avail, block_size / 2) bytes of each window (the
 * command line's reader threads count them as they read the input). */
int sa_cut_next_pe_nl(const uint8_t *w1, uint64_t avail1, int eof1, uint64_t k1, const uint8_t *w2,
                      uint64_t avail2, int eof2, uint64_t k2, uint64_t block_size, const uint8_t *first,
                      uint64_t flen, uint64_t *end1, uint64_t *end2);
/* Block parse: getBlockRead@0x411b60 (SE) / getBlockReadPE@0x412920 (PE).
 * Output arrays sized >= text bytes (names/seq/qual) and text/4+1 (lens). */
int64_t sa_parse_se(const uint8_t *text, uint64_t len, uint8_t *names, uint16_t *name_lens,
                    uint8_t *seq, int32_t *seq_lens, uint8_t *qual);
int64_t sa_parse_pe(const uint8_t *t1, uint64_t len1, const uint8_t *t2, uint64_t len2,
                    uint8_t *names, uint16_t *name_lens, uint8_t *seq, int32_t *seq_lens,
                    uint8_t *qual);
/* ID template ("adaptive binning") detection on the first block:
 * IDProcess::analysisIDBinType@0x4310a0.  tmpl = the 512-byte param+0x18a4
 * area, caller zero-initialised; tmpl[0] is sa_cfg.bin_mode. */
int sa_analyze_ids(const sa_block *first, int single_end, uint8_t tmpl[512]);

/* ---- .arc container (SeqArcFile, host) ---------------------------------- */
/* Archive = 16-byte header + the encoded blocks back to back (input order,
 * the reference's -t 1 order) + trailer.  Restated from
 * SeqArcFile::writeFileInfo@0x4171b0, writeParam@0x416450 and
 * writeBlockLenArry{SE,PE}@0x416d60/0x416e90 (fastqueeze_amd/csrc/arc_file.cpp). */
typedef struct {
    uint32_t size;         /* encoded block bytes (sa_out.size of the block)           */
    uint32_t long_reads;   /* a read > 65535 bp (SeqArcMemBuf+0x2; compressLen_long)   */
    uint64_t text1;        /* FASTQ text bytes of the block in input 1 (ReadBuf+0xc)   */
    uint64_t text2;        /* ... in input 2 (ReadBuf+0x10; 0 for single-end)          */
} sa_arc_block;

typedef struct {
    const char *file1;             /* input paths as given (basename stored, ".gz" cut) */
    const char *file2;             /* NULL / "" for single-end                          */
    int32_t paired;
    int32_t gz1;                   /* param+0x6: input 1 is gzip (getFileType@0x40d9f0)  */
    int32_t bare_plus;             /* '+' lines carry no ID (getFirstLine@0x431eb0)      */
    int32_t md5;                   /* param+0x1880                                       */
    int32_t lossy;                 /* param+0x1870 (-l)                                  */
    const uint8_t *id_template;    /* 512 B, param+0x18a4 (sa_analyze_ids)               */
    /* reference path (-c ref.fa): param+0x3 clear, -I in field 10, and the
     * index MD5 encap writeMd5@0x416b10 (ID 8: the 16 bytes of "<ref.fa>.md5",
     * the MD5 of the FASTA file, getMd5@0x416810) */
    const uint8_t *ref_md5;        /* NULL: no reference                                 */
    uint32_t insert_size;          /* param+0x28 (-I)                                    */
} sa_arc_info;   /* (layout unchanged since round 1: maxmis is sa_arc_trailer2's argument) */

/* ---- block decoder (SeqArc -d; host) ------------------------------------ */
/* The inverse of sa_encode_blocks for one block: EncapFqzComp::doFqzDecode@0x42c680
 * and, in ID-bin mode, IDProcess::decodeIDS@0x430610 (fastqueeze_amd/csrc/arc_decode.cpp).
 * Caller-owned arrays; PE reads come back interleaved r1, r2. */
typedef struct {
    uint8_t *names;        /* >= name_cap bytes     */
    uint16_t *name_lens;   /* >= max_reads entries  */
    uint8_t *seq;          /* >= seq_cap bytes      */
    int32_t *seq_lens;     /* >= max_reads entries  */
    uint8_t *qual;         /* >= seq_cap bytes      */
    uint64_t name_cap, seq_cap;
    uint32_t max_reads;
    uint32_t nreads;       /* out */
    int32_t md5_ok;        /* out: stored digests match (blockMd5Verify@0x414e00), 1 if MD5 off */
} sa_decoded;
/* Returns nreads, or -1 on a malformed block / too small arrays.  tmpl: the
 * archive's 512-byte ID template (trailer field 15); long_reads: the block
 * record's flag bit (compressLen_long). */
int64_t sa_decode_block(const uint8_t *in, uint64_t len, const sa_cfg *cfg, const uint8_t tmpl[512],
                        int32_t long_reads, sa_decoded *out);

/* The reference path's blocks (doAlignEncode@0x42d4c0 layout): aligned reads are
 * rebuilt from the genome (EncapFqzComp::decompressSeq@0x42e390 ->
 * getRealPos@0x42de30, AlignInfoToSeq@0x42e020). */
typedef struct {
    const uint32_t *genome;   /* packed bases: sa_hash_packed / the .hash file's words */
    uint64_t bases;           /* genome length (param+0x1868)                          */
    int32_t paired;           /* the archive is PE (the mate relation streams)         */
    int32_t maxmis;           /* param+0x1b60 the archive was made with (Mis model)    */
    uint32_t insert_size;     /* -I (trailer field 10): the mate distances' bits when  */
                              /* the block's insert-bits count is 0 (the reference's   */
                              /* own decoder reads 0 bits there)                       */
} sa_ref;
int64_t sa_decode_block_ref(const uint8_t *in, uint64_t len, const sa_cfg *cfg, const uint8_t tmpl[512],
                            int32_t long_reads, const sa_ref *ref, sa_decoded *out);

/* RFC 1321 MD5 (MD5File@0x405950 of the reference FASTA, the block digests) */
void sa_md5(const uint8_t *data, uint64_t len, uint8_t digest[16]);

/* 16-byte header; block_bytes = sum of the blocks' sizes. Returns 0. */
int sa_arc_header(uint64_t block_bytes, uint8_t out[16]);
/* Trailer bytes written to out (written at offset 16 + block_bytes), or -1
 * (writeParam@0x416450 + writeMd5@0x416b10 + writeBlockLenArry{SE,PE}@0x416d60/0x416e90). */
int64_t sa_arc_trailer(const sa_arc_info *info, const sa_arc_block *blocks, uint32_t nblocks,
                       uint8_t *out, uint64_t cap);
/* The same with the reference path's maxmis (param+0x1b60, 0..8).  SeqArc reads it
 * from ./seqarc.config and stores none; a value other than its default 7 is
 * written as params field 19 so that -d rebuilds the same Mis model.
 * sa_arc_trailer(...) == sa_arc_trailer2(info, 7, ...). */
int64_t sa_arc_trailer2(const sa_arc_info *info, int32_t maxmis, const sa_arc_block *blocks, uint32_t nblocks,
                        uint8_t *out, uint64_t cap);

/* ---- HASH reference index and gapless seed alignment ----
 * The index `SeqArc -i ref.fa` builds (HashAlignment::buildRefIndex@0x410190
 * with HashRefIndex32: FASTA < 5 GiB), built on ctx's device and kept there;
 * K / step / maxcount = param+0x1b64 / +0x1b70 / 2^(+0x1b6c) (14, 2, 65536).
 * NULL on error (sa_last_error(ctx)). */
typedef struct sa_hash_index sa_hash_index;
sa_hash_index *sa_hash_build(sa_ctx *ctx, const char *fasta, uint64_t bytes, uint32_t K, uint32_t step,
                             uint32_t maxcount);
/* the "<ref.fa>.hash" file (HashRefIndex32::writeIndexFile@0x41ed00): K, bases,
 * words, positions (u32), packed bases, per-K-mer counts, starts, positions */
uint64_t sa_hash_file_bytes(const sa_hash_index *ix);
int sa_hash_serialize(sa_ctx *ctx, const sa_hash_index *ix, uint8_t *out, uint64_t cap);
uint32_t sa_hash_genome_length(const sa_hash_index *ix);
void sa_hash_destroy(sa_hash_index *ix);
/* getHashAlignInfo@0x4113c0 for n reads in order (HashAlignment::doSEAlign@
 * 0x4117b0; doPEAlign@0x4117d0 aligns each mate the same way): per read the
 * mismatch count or -1 (unaligned), strand (1: reverse complement), 1-based
 * reference position, and maxmis + 1 slots of mismatch offsets and types (-1
 * past the read's mismatches).  maxmis = param+0x1b60 (7), good = +0x1b74 (1).
 * *ai_nmis is the align_info state the reference carries from read to read
 * (AlignParam+0xc, never reset by doAlign@0x411910): in, before the first
 * read; out, after the last. */
int sa_hash_align(sa_ctx *ctx, const sa_hash_index *ix, const char *seq, const uint64_t *off, const int32_t *lens,
                  int64_t n, int32_t maxmis, int32_t good, int32_t *ai_nmis, int32_t *ret, uint8_t *rev,
                  uint64_t *pos, int32_t *mispos, int32_t *mistype);

/* ---- reference path: the block encoder with a HASH index ---------------
 * Replaces, per block, EncapFqzComp::doAlignEncode@0x42d4c0 together with the
 * per-block alignment driver ISeqArcEncodeThread::doTask@0x433ed8 runs before
 * it (AlignEncodeSEJob::doAlign@0x411910 / AlignEncodePEJob::doAlign@0x413580):
 * every read aligned (getHashAlignInfo@0x4113c0), aligned reads coded as order /
 * position / mismatch / strand streams (and the PE mate relation), the rest
 * through the SEQ stream.  The encode thread carries one align_info per mate
 * from read to read and from block to block; an sa_align_chain is that state,
 * and batches of one input pass it on in order. */
typedef struct {
    const sa_hash_index *index;   /* on the encoding context's device              */
    int32_t paired;               /* PE, reads interleaved r1, r2 (-2 given)       */
    int32_t maxmis;               /* param+0x1b60 (7), 0..8 (the Mis model's range) */
    int32_t good;                 /* param+0x1b74 (1)                              */
    uint32_t insert_size;         /* -I (param+0x28); 0: estimated per block       */
} sa_align_cfg;
typedef struct sa_align_chain sa_align_chain;
/* the align_info mismatch counts before the first batch (AlignParam+0xc / +0x54;
 * 0 for a fresh encode thread) */
sa_align_chain *sa_align_chain_create(int32_t nmis_mate1, int32_t nmis_mate2);
void sa_align_chain_destroy(sa_align_chain *ch);
/* marks the chain failed: every call waiting on it (and every later one)
 * returns an error.  For a caller whose batch cannot reach the chain (e.g. its
 * staging failed), so that the batches after it do not wait forever. */
void sa_align_chain_fail(sa_align_chain *ch);
/* encodes the resident batch in the doAlignEncode layout; batch = its place in
 * the chain (0, 1, 2, ...: a call waits until the previous batch has passed
 * its alignment), or UINT64_MAX for the chain's next.  Then sa_fetch. */
int sa_run_input_aligned(sa_ctx *ctx, const sa_input *in, const sa_cfg *cfg, const sa_align_cfg *acfg,
                         sa_align_chain *chain, uint64_t batch);
int sa_run_aligned(sa_ctx *ctx, const sa_cfg *cfg, const sa_align_cfg *acfg, sa_align_chain *chain, uint64_t batch);
/* one-shot form of the above (sub-batches in order through the chain) */
int sa_encode_blocks_aligned(sa_ctx *ctx, const sa_block *in, int n, const sa_cfg *cfg, const sa_align_cfg *acfg,
                             sa_align_chain *chain, sa_out *out);
/* device time (ms, HIP events) of sa_hash_align's aligner kernel over all the
 * reads of the last call (the first pass: the carried state "not aligned") */
float sa_hash_align_kernel_ms(const sa_ctx *ctx);
/* the ".hash" file back onto ctx's device (HashRefIndex32::readIndexFile) */
sa_hash_index *sa_hash_load(sa_ctx *ctx, const uint8_t *file, uint64_t bytes);
/* the genome's packed bases (16 a word, 2 bits, first base in the top bits,
 * N as A): what decoding an aligned read reads (HashAlignment::doGetSeq@0x40ff90);
 * out has room for (bases + 15) / 16 words */
int sa_hash_packed(sa_ctx *ctx, const sa_hash_index *ix, uint32_t *out, uint64_t words);

#ifdef __cplusplus
}
#endif
#endif
