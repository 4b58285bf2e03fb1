/* hash_oracle.h -- the CPU restatement of SeqArc 1.6's HASH index and gapless
 * seed aligner (hash_oracle.c), for the reference-path block encoder
 * (align_oracle.c).  TEST INFRASTRUCTURE ONLY (see fqz_oracle.h). */
#ifndef HASH_ORACLE_H
#define HASH_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint32_t K, step, maxcount;
    uint64_t nkmers;
    uint32_t total, nwords, npos;
    uint32_t *seq, *num, *ind, *pos;
} ho_index;

typedef struct {
    uint32_t K;
    int32_t maxmis;
    uint64_t glen;
    int32_t good;
    uint8_t f14, f15;
} ho_args;

#define HO_MAXMIS 64
typedef struct {
    uint8_t rev;
    int32_t nmis;
    int32_t len;
    uint64_t pos;
    int32_t mispos[HO_MAXMIS + 1];
    int32_t mistype[HO_MAXMIS + 1];
} ho_align;

int ho_align_read(const ho_index *ix, const ho_args *a, const char *r, int len, ho_align *ai);
const ho_index *ho_current_index(void);
int64_t ho_build(const char *fa, uint64_t n, uint32_t K, uint32_t step, uint32_t maxcount);

#ifdef __cplusplus
}
#endif

#endif
