/*
 * fqz_oracle.h -- CPU restatement of the SeqArc-1.6 no-reference block encoder.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (fastqueeze_amd/, the
 * C-ABI library, the CLI) may link, load or call this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / the timed CPU baseline.
 *
 * The reference (/root/reference) ships a single prebuilt executable
 * (SeqArc-1.6) and no sources; this file restates its algorithm from static
 * disassembly (objdump -d of the binary, read as text -- never executed).
 * Every function cites SeqArc-1.6@0xADDR of the routine it restates.
 *
 * Parity pinning: the reference ships no output fixtures and its binary may not
 * be run here, so byte-level parity is anchored on (1) the reference's own
 * input files (test/ERR2755197_test_{1,2}.fq) together with the per-stream
 * encoded sizes recorded in SURVEY.md section 6 from a reference run, and
 * (2) exact restatement of the disassembly.  See DESIGN.md "Oracle".
 */
#ifndef FQZ_ORACLE_H
#define FQZ_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Encoder parameters (SeqArcParam fields used by the no-ref path). */
typedef struct {
    int slevel;        /* param+0x1b54, default 3; seq order k = slevel + 7   */
    int qlevel;        /* param+0x1b58, default 2                             */
    int md5;           /* param+0x1880, default 1                             */
    int bin_mode;      /* param+0x18a4 (ID template byte 0): encodeIDS path   */
    double lossy;      /* -l R: param+0x1878 (R), param+0x1870 set iff R > 0  */
} orc_cfg;

/* One parsed block (SeqArcMemBuf SoA; PE reads interleaved r1,r2). */
typedef struct {
    const uint8_t  *names;      /* concatenated IDs without '@'              */
    const uint16_t *name_lens;
    const uint8_t  *seq;        /* concatenated bases                        */
    const int32_t  *seq_lens;
    const uint8_t  *qual;       /* concatenated quals (same lengths as seq)  */
    uint32_t        nreads;
} orc_block;

/* Encode one block exactly as EncapFqzComp::doFqzEncode@0x42d2d0 (after
 * SeqArcMemBuf::calcBlockMd5@0x414d90 and DegeInfoProcess@0x433a10).
 * Returns bytes written, or -1 on error / insufficient capacity. */
int64_t orc_encode_block(const orc_block *b, const orc_cfg *cfg,
                         uint8_t *out, size_t cap);

/* The per-block arrays the reference path builds in SeqArcMemBuf
 * (AlignEncode{SE,PE}Job::doAlign@0x411910/0x413580, AlignInfoProcess[PE]
 * @0x4118b0/0x412290, decomposeAlignInfo@0x433860) and doAlignEncode@0x42d4c0
 * codes.  Bit arrays hold one bit (0/1) per byte, LSB of the value first. */
typedef struct {
    int paired;                 /* param+0x1b38 == 0                          */
    int maxmis;                 /* param+0x1b60 (Mis model size)              */
    uint32_t order_count;       /* +0xe8 / +0x34: reads with an order byte    */
    uint32_t align_count;       /* +0x30: aligned reads                       */
    uint32_t insert_bits;       /* +0x28 (PE)                                 */
    const uint8_t *order;       /* +0xe0: 0 or (pos >> shift) + 1             */
    const uint8_t *pos;   uint32_t npos;     /* +0xf0 / +0xf8 (bits)        */
    const uint8_t *cigal; uint32_t ncigal;   /* +0x100 / +0x108 (bits)      */
    const uint8_t *mis;   uint32_t nmis;     /* +0x110 / +0x118             */
    const uint8_t *rev;   uint32_t nrev;     /* +0x120 / +0x128             */
    const uint8_t *cigav; uint32_t ncigav;   /* +0x130 / +0x138             */
    const uint8_t *perel; uint32_t nperel;   /* +0x140 / +0x148             */
} orc_align_streams;

/* EncapFqzComp::doAlignEncode@0x42d4c0 over the arrays above. */
int64_t orc_encode_block_aligned(const orc_block *b, const orc_cfg *cfg, const orc_align_streams *a,
                                 uint8_t *out, size_t cap);

/* The whole reference path of one block against the index last built by
 * ho_build (hash_oracle.c): doAlign (the aligner over the read chain, the 5 %
 * probe and bail-out, the PE insert-size estimate CaclInsertSize@0x413270),
 * then doAlignEncode.  carry[0] (SE; PE mate 1) / carry[1] (PE mate 2): the
 * align_info nmis the encode thread carries from read to read and block to
 * block (AlignParam+0xc / +0x54), in and out.  insert_size: -I (param+0x28),
 * 0 = estimated per block.  Returns bytes written or -1. */
int64_t orc_encode_block_hash(const orc_block *b, const orc_cfg *cfg, int paired, int maxmis, int good,
                              uint32_t insert_size, int32_t carry[2], uint8_t *out, size_t cap);

/* Individual streams, each returning the complete encap (ID + size + payload)
 * exactly as the corresponding compressX routine writes it. */
int64_t orc_encap_seq(const orc_block *b, const orc_cfg *cfg, uint8_t *out, size_t cap);
int64_t orc_encap_qual(const orc_block *b, const orc_cfg *cfg, uint8_t *out, size_t cap);
int64_t orc_encap_len(const orc_block *b, uint8_t *out, size_t cap);
int64_t orc_encap_id(const orc_block *b, const orc_cfg *cfg, uint8_t *out, size_t cap);

/* Range-coded payload only (no encap header, no MD5) -- handy for tests. */
int64_t orc_seq_payload(const orc_block *b, int k, uint8_t *out, size_t cap);
int64_t orc_qual_payload(const orc_block *b, int qlevel, uint8_t *out, size_t cap);

/* ID template analysis on the first block, IDProcess::analysisIDBinType@0x4310a0.
 * tmpl is the 512-byte param+0x18a4 area (in/out, caller zero-initialises);
 * se = 1 for single-end input. Returns 0, or -1 if the reference would throw. */
int orc_analyze_idbin(const orc_block *first, int se, uint8_t tmpl[512]);

/* The bare range coder (encode_seq@0x422010-0x422085, finish @0x424a1c) over n
 * given (cum, freq, tot) triples; returns bytes written or -1. */
int64_t orc_rc_encode(const uint16_t *cum, const uint16_t *freq, const uint16_t *tot, size_t n,
                      uint8_t *out, size_t cap);

/* Decoded block (caller-owned arrays; see fqz_decode.c). */
typedef struct {
    uint8_t  *names;      /* >= name_cap bytes */
    uint16_t *name_lens;  /* >= max_reads      */
    uint8_t  *seq;        /* >= seq_cap bytes  */
    int32_t  *seq_lens;   /* >= max_reads      */
    uint8_t  *qual;       /* >= seq_cap bytes  */
    size_t    name_cap, seq_cap;
    uint32_t  max_reads;
    uint32_t  nreads;     /* out */
    int       md5_ok;     /* out: 1 if every stored digest matches (or MD5 off) */
} orc_decoded;

/* Decode one block written by orc_encode_block / the GPU encoder (the inverse
 * of doFqzEncode@0x42d2d0; the reference's decoder is doFqzDecode@0x42c680).
 * Returns nreads, -1 on malformed input, -2 for the ID-bin mode. */
int64_t orc_decode_block(const uint8_t *in, size_t len, const orc_cfg *cfg, orc_decoded *out);

/* R-Block lossy quality pre-pass over one block's concatenated qualities,
 * EncapFqzComp::rblock@0x426c10 (in place; n = bytes before the buffer's '\n'). */
void orc_rblock(uint8_t *q, size_t n, double ratio);

/* RFC1321 MD5 (the vendored RSA implementation, MDString@0x4058f0). */
void orc_md5(const uint8_t *data, size_t len, uint8_t digest[16]);

/* FASTQ block cutting: SeqArcRead::doReadJob@0x432a80 / cultbuf@0x432530 /
 * getEndPos@0x4320c0 (SE) and doReadPEJob@0x432d10 / cultPEbuf@0x432180 (PE).
 * Fills block_ends[] with the end offset (exclusive) of each block in the
 * input text; returns the number of blocks (or -1 if max_blocks too small).
 * For PE, block_ends2[] receives the matching offsets in file 2. */
int64_t orc_cut_se(const uint8_t *text, size_t len, size_t block_size,
                   size_t *block_ends, size_t max_blocks);
int64_t orc_cut_pe(const uint8_t *t1, size_t len1, const uint8_t *t2, size_t len2,
                   size_t block_size, size_t *ends1, size_t *ends2, size_t max_blocks);

/* Parse one block of FASTQ text into SoA: getBlockRead@0x411b60 (SE) and
 * getBlockReadPE@0x412920 (PE, interleaving r1,r2).  The arrays must be large
 * enough: names/seq/qual >= text length, lens >= text length / 4 + 1.
 * Returns nreads or -1. */
int64_t orc_parse_se(const uint8_t *text, size_t len,
                     uint8_t *names, uint16_t *name_lens,
                     uint8_t *seq, int32_t *seq_lens, uint8_t *qual);
int64_t orc_parse_pe(const uint8_t *t1, size_t len1, const uint8_t *t2, size_t len2,
                     uint8_t *names, uint16_t *name_lens,
                     uint8_t *seq, int32_t *seq_lens, uint8_t *qual);

#ifdef __cplusplus
}
#endif
#endif
