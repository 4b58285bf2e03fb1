/*
 * orc_cli.c -- command-line driver for the CPU restatement (test infrastructure).
 *
 *   orc_cli [-b block_bytes] [-s slevel] [-q qlevel] [-o blocks.bin] [-t] in1.fq [in2.fq]
 *
 * Cuts the input into blocks (SeqArcRead::doReadJob@0x432a80 / doReadPEJob@0x432d10),
 * parses each (getBlockRead@0x411b60 / getBlockReadPE@0x412920), runs the ID template
 * analysis on the first block (analysisIDBinType@0x4310a0), encodes every block
 * (doFqzEncode@0x42d2d0) and writes the concatenated block encaps to -o.
 * Prints one line per block with the per-stream encap sizes; -t prints timing.
 */
#define _POSIX_C_SOURCE 199309L
#include "fqz_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static uint8_t *slurp(const char *p, size_t *n)
{
    FILE *f = fopen(p, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = (uint8_t *)malloc((size_t)sz + 1);
    if (b && fread(b, 1, (size_t)sz, f) != (size_t)sz) { free(b); b = NULL; }
    fclose(f);
    *n = (size_t)sz;
    return b;
}

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char **argv)
{
    size_t bs = 50u << 20;
    int slevel = 3, qlevel = 2, timing = 0;
    const char *outp = NULL;
    const char *in[2] = {NULL, NULL};
    int nin = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-b") && i + 1 < argc) bs = (size_t)strtoull(argv[++i], NULL, 10);
        else if (!strcmp(argv[i], "-s") && i + 1 < argc) slevel = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-q") && i + 1 < argc) qlevel = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) outp = argv[++i];
        else if (!strcmp(argv[i], "-t")) timing = 1;
        else if (nin < 2) in[nin++] = argv[i];
    }
    if (!nin) {
        fprintf(stderr, "usage: orc_cli [-b bytes] [-s slevel] [-q qlevel] [-o out] [-t] in1 [in2]\n");
        return 2;
    }
    size_t n1 = 0, n2 = 0;
    uint8_t *t1 = slurp(in[0], &n1), *t2 = nin > 1 ? slurp(in[1], &n2) : NULL;
    if (!t1 || (nin > 1 && !t2)) { fprintf(stderr, "cannot read input\n"); return 1; }
    size_t maxb = (n1 + n2) / 1024 + 16;
    size_t *e1 = (size_t *)malloc(maxb * sizeof(size_t)), *e2 = (size_t *)malloc(maxb * sizeof(size_t));
    int64_t nb = nin > 1 ? orc_cut_pe(t1, n1, t2, n2, bs, e1, e2, maxb) : orc_cut_se(t1, n1, bs, e1, maxb);
    if (nb <= 0) { fprintf(stderr, "block cut failed\n"); return 1; }
    FILE *fo = outp ? fopen(outp, "wb") : NULL;
    uint8_t T[512];
    memset(T, 0, sizeof T);
    size_t o1 = 0, o2 = 0;
    double tenc = 0;
    uint64_t total_out = 0;
    for (int64_t b = 0; b < nb; b++) {
        size_t l1 = e1[b] - o1, l2 = nin > 1 ? e2[b] - o2 : 0;
        size_t cap = l1 + l2 + 64;
        uint8_t *names = (uint8_t *)malloc(cap), *seq = (uint8_t *)malloc(cap), *qual = (uint8_t *)malloc(cap);
        uint16_t *nl = (uint16_t *)malloc((cap / 4 + 8) * sizeof(uint16_t));
        int32_t *sl = (int32_t *)malloc((cap / 4 + 8) * sizeof(int32_t));
        int64_t nr = nin > 1 ? orc_parse_pe(t1 + o1, l1, t2 + o2, l2, names, nl, seq, sl, qual)
                             : orc_parse_se(t1 + o1, l1, names, nl, seq, sl, qual);
        if (nr < 0) { fprintf(stderr, "parse failed in block %lld\n", (long long)b); return 1; }
        orc_block blk = {names, nl, seq, sl, qual, (uint32_t)nr};
        if (b == 0 && orc_analyze_idbin(&blk, nin == 1, T)) { fprintf(stderr, "ID analysis failed\n"); return 1; }
        orc_cfg cfg = {slevel, qlevel, 1, T[0], 0.0};
        size_t ocap = 2 * (l1 + l2) + 4096;
        uint8_t *out = (uint8_t *)malloc(ocap);
        double t0 = now();
        int64_t w = orc_encode_block(&blk, &cfg, out, ocap);
        tenc += now() - t0;
        if (w < 0) { fprintf(stderr, "encode failed in block %lld\n", (long long)b); return 1; }
        total_out += (uint64_t)w;
        printf("block %lld reads %lld in %zu out %lld\n", (long long)b, (long long)nr, l1 + l2, (long long)w);
        if (fo && fwrite(out, 1, (size_t)w, fo) != (size_t)w) { fprintf(stderr, "write failed\n"); return 1; }
        free(out); free(names); free(seq); free(qual); free(nl); free(sl);
        o1 = e1[b];
        if (nin > 1) o2 = e2[b];
    }
    if (fo) fclose(fo);
    printf("bin_mode %d petype %d blocks %lld in %zu out %llu\n", T[0], T[1], (long long)nb, n1 + n2,
           (unsigned long long)total_out);
    if (timing) printf("encode_seconds %.6f MBps %.3f\n", tenc, (double)(n1 + n2) / 1e6 / tenc);
    return 0;
}
