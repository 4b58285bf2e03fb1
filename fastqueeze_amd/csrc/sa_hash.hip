// sa_hash.hip -- the HASH reference-index path on gfx950 (SURVEY.md section
// 8(f) 3, configs[3]): the index build of `SeqArc -i ref.fa`
// (HashAlignment::buildRefIndex@0x410190 over HashRefIndex32) and the gapless
// seed alignment of every read (getHashAlignInfo@0x4113c0, which
// doSEAlign@0x4117b0 and, per mate, doPEAlign@0x4117d0 call).
// Included at the end of sa_engine.hip (it sorts with run_sort).
//
// Index build (one FASTA, < 5 GiB: the 32-bit index):
//   host   the base stream (the characters the reference's line loop reads);
//   k_hash_pack   16 bases a word, codes & 3 (N reads as A), last word left-aligned;
//   k_hash_count  per 1-based position p: the K-mer ending at p is a seed if
//                 none of its K characters is N/n and p % step == 0; a global
//                 atomic count per K-mer (4^K counters);
//   k_hash_cap    counts at the cap (2^16) -> 0 (repeats are dropped), then an
//                 exclusive scan of the counts (k_scan_*);
//   k_hash_emit   the seeds of kept K-mers as (K-mer, 1-based start) pairs in
//                 position order (per-chunk counts, scan, write);
//   run_sort      stable LSD radix sort of the pairs by K-mer: the values are
//                 the position table, each K-mer's list ascending, exactly the
//                 order of the reference's second pass.
// Alignment: one lane per read, the restated control flow over the index in
// HBM (random index reads, latency-bound: many reads in flight).
// ---------------------------------------------------------------------------

namespace sa {

constexpr uint32_t HASH_CHUNK = 64;   // positions per thread in count / emit

__device__ __forceinline__ uint32_t hash_code(uint8_t c) { return base_code(c); }   // @0x449fc0 (ASCII)

__global__ __launch_bounds__(256) void k_hash_pack(const uint8_t* __restrict__ b, uint64_t n,
                                                   uint32_t* __restrict__ seq, uint64_t nwords)
{
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint64_t i = w * 16 + j;
        v = (v << 2) | (i < n ? hash_code(b[i]) & 3u : 0u);
    }
    seq[w] = v;
}

// The seed ending at 1-based position p (the K characters p-K .. p-1 of the
// stream): valid when none is N/n ((c & 0xdf) == 'N', buildRefIndex's test)
// and p % step == 0.  A thread walks HASH_CHUNK positions with a rolling
// K-mer and the distance to the last N.
struct SeedWalk {
    uint64_t p;        // 1-based position of the next character
    uint32_t kmer;
    uint32_t since_n;  // characters since the last N (saturating)
};

__device__ __forceinline__ SeedWalk seed_walk_start(const uint8_t* b, uint64_t p0, uint32_t K, uint64_t mask)
{
    SeedWalk s{p0, 0u, 0u};
    const uint64_t from = p0 > K ? p0 - K : 1;   // 1-based
    for (uint64_t q = from; q < p0; q++) {
        const uint8_t c = b[q - 1];
        s.kmer = (uint32_t)((((uint64_t)s.kmer << 2) | (hash_code(c) & 3u)) & mask);
        s.since_n = (c & 0xdf) == 'N' ? 0u : s.since_n + 1u;
    }
    return s;
}

// advances over character p; true if a seed ends there
__device__ __forceinline__ bool seed_walk_step(SeedWalk& s, const uint8_t* b, uint32_t K, uint64_t mask, uint32_t step)
{
    const uint8_t c = b[s.p - 1];
    s.kmer = (uint32_t)((((uint64_t)s.kmer << 2) | (hash_code(c) & 3u)) & mask);
    s.since_n = (c & 0xdf) == 'N' ? 0u : (s.since_n < K ? s.since_n + 1u : K);
    const bool seed = s.since_n >= K && s.p % step == 0;
    s.p++;
    return seed;
}

__global__ __launch_bounds__(256) void k_hash_count(const uint8_t* __restrict__ b, uint64_t n, uint32_t K,
                                                    uint64_t mask, uint32_t step, uint32_t* __restrict__ num)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t p0 = t * HASH_CHUNK + 1;
    if (p0 > n) return;
    SeedWalk s = seed_walk_start(b, p0, K, mask);
    const uint64_t p1 = p0 + HASH_CHUNK <= n + 1 ? p0 + HASH_CHUNK : n + 1;
    while (s.p < p1)
        if (seed_walk_step(s, b, K, mask, step)) atomicAdd(&num[s.kmer], 1u);
}

// setSeedind@0x41e820: a K-mer counted maxcount times or more is dropped
__global__ __launch_bounds__(256) void k_hash_cap(uint32_t* __restrict__ num, uint64_t nk, uint32_t maxcount)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nk && num[i] >= maxcount) num[i] = 0;
}

// ---- exclusive scan of u32 (3 kernels: 4096-element tiles, tile sums, add) ----
constexpr uint32_t SCAN_TILE = 4096;   // 256 threads x 16

__global__ __launch_bounds__(256) void k_scan_tiles(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                    uint64_t n, uint32_t* __restrict__ sums)
{
    __shared__ uint32_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * 16;
    uint32_t v[16], s = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        v[j] = base + j < n ? in[base + j] : 0u;
        s += v[j];
    }
    uint32_t ex;
    wg256_excl_scan(s, ex, sh);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; j++) {
        if (base + j < n) out[base + j] = ex;
        ex += v[j];
    }
    if (threadIdx.x == 255) sums[blockIdx.x] = ex;   // the tile's total
}

__global__ __launch_bounds__(256) void k_scan_add(uint32_t* __restrict__ out, uint64_t n,
                                                  const uint32_t* __restrict__ sums)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] += sums[i / SCAN_TILE];
}

// k_hash_emit: pass 0 counts each thread's kept seeds; pass 1 writes them at
// the thread's scanned offset (position order)
__global__ __launch_bounds__(256) void k_hash_emit(const uint8_t* __restrict__ b, uint64_t n, uint32_t K,
                                                   uint64_t mask, uint32_t step, const uint32_t* __restrict__ num,
                                                   uint32_t* __restrict__ cnt, const uint32_t* __restrict__ at,
                                                   uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, int pass)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t p0 = t * HASH_CHUNK + 1;
    if (p0 > n) return;
    SeedWalk s = seed_walk_start(b, p0, K, mask);
    const uint64_t p1 = p0 + HASH_CHUNK <= n + 1 ? p0 + HASH_CHUNK : n + 1;
    uint32_t k = pass ? at[t] : 0u;
    while (s.p < p1) {
        const uint64_t p = s.p;
        if (seed_walk_step(s, b, K, mask, step) && num[s.kmer]) {
            if (pass) {
                keys[k] = s.kmer;
                vals[k] = (uint32_t)(p - (K - 1));   // setSeedpos@0x41e5f0: 1-based start
            }
            k++;
        }
    }
    if (!pass) cnt[t] = k;
}

// ---------------------------------------------------------------------------
// Alignment (getHashAlignInfo@0x4113c0 and callees; oracle/hash_oracle.c is
// the CPU restatement, every step below mirrors it).
// ---------------------------------------------------------------------------
struct HashView {
    const uint32_t* seq;
    const uint32_t* num;
    const uint32_t* ind;
    const uint32_t* pos;
    uint32_t K;
    uint64_t glen;
};

struct HashArgs {
    int32_t maxmis, good;
};

struct HashRead {   // one read (forward or reverse complement) being aligned
    const uint8_t* r;    // forward bases
    int len;
    bool rc;             // the sequence is the reverse complement of r
    uint32_t* packed;    // its packed words (scratch)
};

__device__ __forceinline__ uint8_t comp_base(uint8_t c)   // rev@0x40d9a0
{
    switch (c) {
    case 'A': case 'a': return 'T';
    case 'C': case 'c': return 'G';
    case 'G': case 'g': return 'C';
    case 'T': case 't': return 'A';
    default: return c;
    }
}

__device__ __forceinline__ uint8_t read_at(const HashRead& h, int i)
{
    return h.rc ? comp_base(h.r[h.len - 1 - i]) : h.r[i];
}

__device__ __forceinline__ uint64_t mask2(uint32_t k) { return k >= 32 ? ~0ull : (1ull << (2 * k)) - 1; }

// getHashSeeds@0x4107f0 (packed words; seeds are read back from them); the
// number of N/IUPAC bases
__device__ int hash_pack_read(const HashRead& h)
{
    int nn = 0;
    const int nw = ((h.len - 1) >> 4) + 1;
    for (int w = 0; w < nw; w++) {
        uint32_t v = 0;
        for (int j = 0; j < 16; j++) {
            const int i = w * 16 + j;
            uint32_t c = 0;
            if (i < h.len) {
                c = hash_code(read_at(h, i));
                nn += c >= 4;
            }
            v = (v << 2) | (c & 3u);
        }
        h.packed[w] = v;
    }
    return nn;
}

// the K-mer ending at read offset i + K - 1 (seed i), from the packed words
__device__ __forceinline__ uint32_t seed_at(const HashRead& h, int i, uint32_t K)
{
    const int e = i + (int)K - 1;             // last base
    const int w = e >> 4, sh = 2 * (15 - (e & 15));
    uint64_t v = (uint64_t)h.packed[w] >> sh;
    if (w > 0) v |= (uint64_t)h.packed[w - 1] << (32 - sh);
    return (uint32_t)(v & mask2(K));
}

__device__ __forceinline__ bool find_seed_d(const HashView& ix, const HashRead& h, int from, int to, uint32_t maxcnt,
                                            bool stop_first, int& out)   // findHashSeeds@0x4108d0
{
    uint32_t best = 100000;
    for (int i = from; i <= to; i += 2) {
        const uint32_t c = ix.num[seed_at(h, i, ix.K)];
        if (c && c < maxcnt && c < best) {
            best = c;
            out = i;
            if (stop_first) return true;
        }
    }
    return best != 100000;
}

__device__ __forceinline__ uint32_t mis2_d(uint32_t x)   // g_mismatch_count@0x65a7c0
{
    const uint32_t y = (x | (x >> 1)) & 0x55555555u;
    return (uint32_t)__popc(y);
}

// mismatch type @0x44a0c0, [ref * 4 + read], 2 bits an entry
__device__ __forceinline__ uint32_t mistype_d(uint32_t rc, uint32_t rb) { return (0xc6b18d87u >> (2 * (rb * 4 + rc))) & 3u; }

// align_info (AlignParam+0x8): nmis is also the state carried from the
// previous read (oracle/hash_oracle.c, ho_align_read): `fresh` once this
// read's first candidate was verified; `consulted` when a search step read the
// carried state before that.
struct HashAlign {
    int nmis;
    uint8_t rev;
    uint64_t pos;
    bool fresh, consulted;
};

// gaplessHashAlignPositions@0x410990
__device__ int align_at_d(uint64_t pos, const HashRead& h, const HashView& ix, const HashArgs& a, HashAlign& ai,
                          int* mp, int* mt, int& best)
{
    const uint64_t p0 = pos - 1;
    const uint32_t off = (uint32_t)(p0 & 15);
    const int lw = (h.len - 1) >> 4, nfull = h.len >> 4;
    int mis = 0;
    ai.fresh = true;
    if (a.maxmis >= 0) {
        uint64_t w = p0 >> 4;
        for (int j = 0;; j++, w++) {
            uint32_t ref = ix.seq[w];
            if (off) {
                const uint32_t nxt = ix.seq[w + 1];
                ref = (uint32_t)(((nxt >> (32 - 2 * off)) & mask2(off)) | (((uint64_t)ref << (2 * off)) & ~mask2(off)));
            }
            uint64_t x = ref ^ h.packed[j];
            if (j >= nfull) x &= ~mask2(16 - (h.len & 15));
            mis += (int)mis2_d((uint32_t)x);
            if (mis > a.maxmis || j + 1 > lw) break;
        }
    }
    int limit;
    if (best > mis) limit = best;
    else if (a.maxmis >= mis) limit = a.maxmis + 1;
    else {
        ai.nmis = -1;
        return 0;
    }
    int n = 0;
    if (p0 >= ix.glen) n = a.maxmis + 1;
    else {
        uint64_t q = p0;
        for (int i = 0;; i++) {
            const uint32_t rb = (ix.seq[q >> 4] >> (30 - 2 * (q & 15))) & 3u;
            const uint32_t rc = hash_code(read_at(h, i));
            if (rb != rc) {
                if (n == a.maxmis) {
                    n++;
                    break;
                }
                mp[n] = i;
                mt[n] = rc > 3 ? 3 : (int)mistype_d(rc, rb);
                n++;
            }
            if (i == h.len - 1) break;
            q++;
            if (q >= ix.glen) {
                n = a.maxmis + 1;
                break;
            }
        }
    }
    if (limit <= n) {
        ai.nmis = -1;
        return 0;
    }
    ai.pos = pos;
    ai.rev = h.rc ? 1 : 0;
    ai.nmis = n;
    if (n < best) best = n;
    return 1;
}

// gaplessSEHashAlign@0x410d80 (mode 0)
__device__ void try_seed_d(int so, const HashRead& h, const HashView& ix, const HashArgs& a, uint32_t kmer,
                           HashAlign& ai, int* mp, int* mt, uint32_t& cnt, int& best, int thr)
{
    const uint32_t n = ix.num[kmer], base = ix.ind[kmer];
    for (uint32_t j = 0; j < n; j++) {
        const uint64_t p = ix.pos[base + j];
        if (p <= (uint64_t)(int64_t)so) continue;
        if (p >= (uint64_t)(int64_t)so + ix.glen - (uint64_t)(int64_t)h.len) continue;
        cnt++;
        align_at_d(p - (uint64_t)(int64_t)so, h, ix, a, ai, mp, mt, best);
        if (thr >= best) return;
        if (ai.nmis >= 0 && ai.nmis <= a.maxmis) return;
        if (cnt > 300) return;
    }
}

__device__ __forceinline__ bool hash_done(HashAlign& ai, const HashArgs& a, uint32_t cnt, int best, int thr)
{
    if (!ai.fresh) ai.consulted = true;
    return thr >= best || cnt > 300 || (ai.nmis >= 0 && ai.nmis <= a.maxmis);
}

// hashAligner@0x410f50
__device__ void aligner_d(const HashRead& h, const HashView& ix, const HashArgs& a, int* sidx, HashAlign& ai, int* mp,
                          int* mt, uint32_t& cnt, int& best, int thr)
{
    for (int par = 0; par < 2; par++) {
        if (find_seed_d(ix, h, par, h.len - (int)ix.K, 100000u, false, sidx[par]))
            try_seed_d(sidx[par], h, ix, a, seed_at(h, sidx[par], ix.K), ai, mp, mt, cnt, best, thr);
        if (hash_done(ai, a, cnt, best, thr)) return;
    }
}

// hashAlignerShortPart@0x411070
__device__ void aligner_parts_d(const HashRead& h, const HashView& ix, const HashArgs& a, int* sidx, HashAlign& ai,
                                int* mp, int* mt, uint32_t& cnt, int& best, int thr)
{
    const int len = h.len, K = (int)ix.K;
    const int np = len > 75 ? 4 : len >= 45 ? 3 : 2;
    const int ovl = len > np * K ? len / np - K : 0;
    bool found = false;
    int b = 0;
    for (int p = 0; p < np; p++) {
        const int e = (len + b) / np, s = b / np;
        b += len;
        for (int par = 0; par < 2; par++) {
            found = find_seed_d(ix, h, s + par, e - K, 620u, false, sidx[par + 2]);
            if (found && sidx[par + 2] != sidx[par]) {
                try_seed_d(sidx[par + 2], h, ix, a, seed_at(h, sidx[par + 2], ix.K), ai, mp, mt, cnt, best, thr);
                if (hash_done(ai, a, cnt, best, thr)) return;
            }
        }
    }
    if (found) return;
    b = 0;
    for (int p = 0; p < np; p++) {
        const int e8 = (len + b) / np - 8, s = b / np + ovl;
        b += len;
        for (int par = 0; par < 2; par++) {
            const int to = e8 < len - K ? e8 : len - K;
            if (find_seed_d(ix, h, s + par, to, 620u, true, sidx[par + 2]) && sidx[par + 2] != sidx[par]) {
                try_seed_d(sidx[par + 2], h, ix, a, seed_at(h, sidx[par + 2], ix.K), ai, mp, mt, cnt, best, thr);
                if (hash_done(ai, a, cnt, best, thr)) return;
            }
        }
    }
}

// getHashAlignInfo@0x4113c0, one lane per read, with the carried align_info
// state taken as `stale` (0: not aligned, 1: aligned).  Outputs per read: ret
// (mismatches, -1 unaligned), strand, 1-based position, maxmis + 1 slots of
// mismatch offsets / types (-1 past the read's mismatches) and whether the
// carried state was consulted (the host then re-runs those reads with the
// other state and picks per read in order, sa_hash_align).  `sel`: the reads
// to do (NULL: all n), outputs at the read's index.
// (k_hash_align, sa_hash_align's kernel, is defined after the row functions)

// ---------------------------------------------------------------------------
// Row-cooperative alignment: one 16-lane row per read (four reads per wave).
// The control flow of getHashAlignInfo@0x4113c0 and its callees is the serial
// one above, row-uniform; the data-parallel steps are spread over the row:
//   * the read is staged in LDS (16-byte loads), both strands packed there, a
//     word per lane, with a mask of its N / IUPAC bases;
//   * findHashSeeds@0x4108d0: the row's lanes look up their seeds' counts
//     together (all loads in flight), then a row minimum of (count, offset):
//     the serial scan's "first strictly smaller" is the smallest count at the
//     smallest offset (stop_first: the smallest qualifying offset);
//   * gaplessSEHashAlign@0x410d80: the next 16 candidate positions are loaded
//     at once, then verified in order;
//   * gaplessHashAlignPositions@0x410990: a word per lane -- the 2-bit XOR
//     count (a row sum: the serial early exit past maxmis changes only the
//     partial count, never the verdict, see align_at_row) and the mismatch
//     list, placed by a row scan of the lanes' mismatch counts.
// Reads longer than AR_MAXW * 16 bases take the serial path on the row's first
// lane (global scratch).
// ---------------------------------------------------------------------------
constexpr int AR = 16;                     // lanes per read
constexpr int AR_MAXW = 32;                // packed words per strand in LDS (reads <= 512 bases)
constexpr int AR_ROWS = 256 / AR;          // rows per 256-thread workgroup
constexpr int AR_BYTES = 16 * AR_MAXW + 32;   // staged read bytes per row (+ the 16-byte loads' slack)

struct RowStrand {
    const uint32_t* pk;   // packed 2-bit codes, 16 bases a word, first base in the top bits (LDS)
    const uint32_t* nm;   // per word: bit j set when base 16 w + j is N / IUPAC (code > 3)
    int len;
    bool rc;
};

__device__ __forceinline__ uint64_t row_min64(uint64_t v)
{
#pragma unroll
    for (int d = AR / 2; d >= 1; d >>= 1) {
        const uint64_t o = __shfl_xor(v, d, AR);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t row_excl_scan(uint32_t v, uint32_t rl)
{
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < AR; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, AR);
        if (rl >= (uint32_t)d) x += y;
    }
    return x - v;
}

// the K-mer ending at offset i + K - 1 (seed i) from the packed words
__device__ __forceinline__ uint32_t seed_at_row(const RowStrand& h, int i, uint32_t K)
{
    const int e = i + (int)K - 1;
    const int w = e >> 4, sh = 2 * (15 - (e & 15));
    uint64_t v = (uint64_t)h.pk[w] >> sh;
    if (w > 0) v |= (uint64_t)h.pk[w - 1] << (32 - sh);
    return (uint32_t)(v & mask2(K));
}

// the row's read (len bytes at rd) into LDS, then both strands packed:
// getHashSeeds@0x4107f0's words (codes & 3) and the N / IUPAC masks.
// Returns the N / IUPAC count (row-uniform).
__device__ int row_stage_pack(const uint8_t* rd, int len, uint8_t* sb, uint32_t* pk, uint32_t* nm, uint32_t* pkr,
                              uint32_t* nmr, const uint8_t* tab, uint32_t rl)
{
    // 16-byte chunks, a lane each (dword loads, funnel-shifted: any start byte);
    // a chunk may read up to 19 bytes past the read, as k_emit_sq16 does
    for (int c = (int)rl; 16 * c < len; c += AR) {
        uint32_t w[4];
        load16(rd + 16 * c, w);
        *reinterpret_cast<uint4*>(sb + 16 * c) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int nw = (len + 15) >> 4;
    int nn = 0;
    for (int wd = (int)rl; wd < nw; wd += AR) {
        uint32_t v = 0, m = 0, vr = 0, mr = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int i = 16 * wd + j;
            uint32_t c = 0, cr = 0;
            if (i < len) {
                c = tab[sb[i]];
                cr = tab[comp_base(sb[len - 1 - i])];   // rev@0x40d9a0 then the code
                if (c > 3) m |= 1u << j;
                if (cr > 3) mr |= 1u << j;
            }
            v = (v << 2) | (c & 3u);
            vr = (vr << 2) | (cr & 3u);
        }
        pk[wd] = v;
        nm[wd] = m;
        pkr[wd] = vr;
        nmr[wd] = mr;
        nn += __popc(m);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    return (int)row_sum<AR>((uint32_t)nn);
}

__device__ __forceinline__ bool find_seed_row(const HashView& ix, const RowStrand& h, int from, int to,
                                              uint32_t maxcnt, bool stop_first, int& out, uint32_t rl)
{
    uint64_t key = ~0ull;
    // every lane's seeds first (loads in flight together), then the reduction
    for (int k0 = from; k0 <= to; k0 += 2 * AR * 4) {
        uint32_t c[4];
        int at[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            at[u] = k0 + 2 * ((int)rl + AR * u);
            c[u] = at[u] <= to ? ix.num[seed_at_row(h, at[u], ix.K)] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (c[u] && c[u] < maxcnt && c[u] < 100000u) {
                const uint64_t kk = stop_first ? (uint64_t)(uint32_t)at[u] : ((uint64_t)c[u] << 32 | (uint32_t)at[u]);
                key = kk < key ? kk : key;
            }
    }
    key = row_min64(key);
    if (key == ~0ull) return false;
    out = (int)(uint32_t)key;
    return true;
}

// gaplessHashAlignPositions@0x410990 for the row.  The serial word loop stops
// once its running count passes maxmis; its verdict depends on the count only
// through "count > maxmis" (then: fail, whether partial or full) or, within
// maxmis, the full count -- so the full count (a row sum) decides identically.
// The base-wise pass: the mismatches are the 2-bit groups that differ plus the
// N / IUPAC bases; it fails (maxmis + 1) past the genome end or past maxmis
// mismatches; a passing candidate lists its mismatches in order.
__device__ void align_at_row(uint64_t pos, const RowStrand& h, const HashView& ix, const HashArgs& a,
                             HashAlign& ai, int* mp, int* mt, int& best, uint32_t rl)
{
    const uint64_t p0 = pos - 1;
    const uint32_t off = (uint32_t)(p0 & 15);
    const int len = h.len, lw = (len - 1) >> 4, nfull = len >> 4;
    ai.fresh = true;
    uint32_t xw[AR_MAXW / AR], rw[AR_MAXW / AR];
    int mis = 0;
#pragma unroll
    for (int k = 0; k < AR_MAXW / AR; k++) {
        const int j = (int)rl + AR * k;
        xw[k] = rw[k] = 0;
        if (j <= lw) {
            const uint64_t w = (p0 >> 4) + (uint64_t)j;
            uint32_t ref = ix.seq[w];
            if (off) {
                const uint32_t nxt = ix.seq[w + 1];
                ref = (uint32_t)(((nxt >> (32 - 2 * off)) & mask2(off)) | (((uint64_t)ref << (2 * off)) & ~mask2(off)));
            }
            uint64_t x = ref ^ h.pk[j];
            if (j >= nfull) x &= ~mask2(16 - (len & 15));
            mis += (int)mis2_d((uint32_t)x);
            xw[k] = (uint32_t)x;
            rw[k] = ref;
        }
    }
    mis = (int)row_sum<AR>((uint32_t)mis);
    int limit;
    if (best > mis) limit = best;
    else if (a.maxmis >= mis) limit = a.maxmis + 1;
    else {
        ai.nmis = -1;
        return;
    }
    int n;
    if (p0 >= ix.glen || (len >= 2 && p0 + (uint64_t)len - 1 >= ix.glen)) {
        n = a.maxmis + 1;
    } else {
        uint32_t mm[AR_MAXW / AR], cnt = 0;
#pragma unroll
        for (int k = 0; k < AR_MAXW / AR; k++) {
            const int j = (int)rl + AR * k;
            mm[k] = 0;
            if (j <= lw) {
                const uint32_t y = (xw[k] | (xw[k] >> 1)) & 0x55555555u;   // a bit per differing 2-bit group
                uint32_t g = 0;   // bit jj = base 16 j + jj (group 15 - jj)
#pragma unroll
                for (int jj = 0; jj < 16; jj++) g |= ((y >> (30 - 2 * jj)) & 1u) << jj;
                g |= h.nm[j];
                const int nb = len - 16 * j;
                if (nb < 16) g &= (1u << nb) - 1u;
                mm[k] = g;
                cnt += (uint32_t)__popc(g);
            }
        }
        const int total = (int)row_sum<AR>(cnt);
        n = total > a.maxmis ? a.maxmis + 1 : total;
        if (n < limit) {   // the candidate passes: its mismatch list, in order
            uint32_t before = 0;
#pragma unroll
            for (int k = 0; k < AR_MAXW / AR; k++) {
                const int j = (int)rl + AR * k;
                if (AR * k > lw) break;   // (row-uniform)
                const uint32_t c = (uint32_t)__popc(mm[k]);
                uint32_t idx = before + row_excl_scan(c, rl);
                for (uint32_t g = mm[k]; g; g &= g - 1) {
                    const int jj = __builtin_ctz(g);
                    if ((int)idx < n) {
                        const uint32_t rb = (rw[k] >> (30 - 2 * jj)) & 3u;
                        const bool isn = (h.nm[j] >> jj) & 1u;
                        const uint32_t code = (h.pk[j] >> (30 - 2 * jj)) & 3u;
                        mp[idx] = 16 * j + jj;
                        mt[idx] = isn ? 3 : (int)mistype_d(code, rb);
                    }
                    idx++;
                }
                before += row_sum<AR>(c);
            }
        }
    }
    if (limit <= n) {
        ai.nmis = -1;
        return;
    }
    ai.pos = pos;
    ai.rev = h.rc ? 1 : 0;
    ai.nmis = n;
    if (n < best) best = n;
}

__device__ void try_seed_row(int so, const RowStrand& h, const HashView& ix, const HashArgs& a, uint32_t kmer,
                             HashAlign& ai, int* mp, int* mt, uint32_t& cnt, int& best, int thr, uint32_t rl)
{
    const uint32_t n = ix.num[kmer], base = ix.ind[kmer];
    for (uint32_t j0 = 0; j0 < n; j0 += AR) {
        const uint32_t mine = j0 + rl < n ? ix.pos[base + j0 + rl] : 0u;   // the next 16 candidates at once
        const uint32_t m = n - j0 < (uint32_t)AR ? n - j0 : (uint32_t)AR;
        for (uint32_t jj = 0; jj < m; jj++) {
            const uint64_t p = __shfl(mine, (int)jj, AR);
            if (p <= (uint64_t)(int64_t)so) continue;
            if (p >= (uint64_t)(int64_t)so + ix.glen - (uint64_t)(int64_t)h.len) continue;
            cnt++;
            align_at_row(p - (uint64_t)(int64_t)so, h, ix, a, ai, mp, mt, best, rl);
            if (thr >= best) return;
            if (ai.nmis >= 0 && ai.nmis <= a.maxmis) return;
            if (cnt > 300) return;
        }
    }
}

__device__ void aligner_row(const RowStrand& h, const HashView& ix, const HashArgs& a, int* sidx, HashAlign& ai,
                            int* mp, int* mt, uint32_t& cnt, int& best, int thr, uint32_t rl)
{
    for (int par = 0; par < 2; par++) {
        if (find_seed_row(ix, h, par, h.len - (int)ix.K, 100000u, false, sidx[par], rl))
            try_seed_row(sidx[par], h, ix, a, seed_at_row(h, sidx[par], ix.K), ai, mp, mt, cnt, best, thr, rl);
        if (hash_done(ai, a, cnt, best, thr)) return;
    }
}

__device__ void aligner_parts_row(const RowStrand& h, const HashView& ix, const HashArgs& a, int* sidx, HashAlign& ai,
                                  int* mp, int* mt, uint32_t& cnt, int& best, int thr, uint32_t rl)
{
    const int len = h.len, K = (int)ix.K;
    const int np = len > 75 ? 4 : len >= 45 ? 3 : 2;
    const int ovl = len > np * K ? len / np - K : 0;
    bool found = false;
    int b = 0;
    for (int p = 0; p < np; p++) {
        const int e = (len + b) / np, s = b / np;
        b += len;
        for (int par = 0; par < 2; par++) {
            found = find_seed_row(ix, h, s + par, e - K, 620u, false, sidx[par + 2], rl);
            if (found && sidx[par + 2] != sidx[par]) {
                try_seed_row(sidx[par + 2], h, ix, a, seed_at_row(h, sidx[par + 2], ix.K), ai, mp, mt, cnt, best, thr,
                             rl);
                if (hash_done(ai, a, cnt, best, thr)) return;
            }
        }
    }
    if (found) return;
    b = 0;
    for (int p = 0; p < np; p++) {
        const int e8 = (len + b) / np - 8, s = b / np + ovl;
        b += len;
        for (int par = 0; par < 2; par++) {
            const int to = e8 < len - K ? e8 : len - K;
            if (find_seed_row(ix, h, s + par, to, 620u, true, sidx[par + 2], rl) && sidx[par + 2] != sidx[par]) {
                try_seed_row(sidx[par + 2], h, ix, a, seed_at_row(h, sidx[par + 2], ix.K), ai, mp, mt, cnt, best, thr,
                             rl);
                if (hash_done(ai, a, cnt, best, thr)) return;
            }
        }
    }
}

// getHashAlignInfo@0x4113c0 for one read on a row (len <= 16 AR_MAXW); the
// results on every lane.  Returns ret (mismatches, -1 unaligned); nn: the N /
// IUPAC count.
__device__ int align_read_row(const uint8_t* rd, int len, const HashView& ix, const HashArgs& a, int stale,
                              HashAlign& ai, int* mp, int* mt, int& nn, uint8_t* sb, uint32_t* lw4, const uint8_t* tab,
                              uint32_t rl)
{
    ai = HashAlign{stale ? 0 : -1, 0, 0, false, false};
    int sidx[4] = {-1, -1, -1, -1};
    int best = -1, r = -1;
    uint32_t cnt = 0;
    nn = 0;
    const int thr = a.good < a.maxmis ? a.good : a.maxmis;
    if (len <= 0) return -1;
    nn = row_stage_pack(rd, len, sb, lw4, lw4 + AR_MAXW, lw4 + 2 * AR_MAXW, lw4 + 3 * AR_MAXW, tab, rl);
    if (nn <= a.maxmis) {
        const RowStrand fw{lw4, lw4 + AR_MAXW, len, false};
        const RowStrand rc{lw4 + 2 * AR_MAXW, lw4 + 3 * AR_MAXW, len, true};
        best = a.maxmis + 1;
        aligner_row(fw, ix, a, sidx, ai, mp, mt, cnt, best, thr, rl);
        if (!(a.maxmis >= best) && cnt <= 299) {
            aligner_row(rc, ix, a, sidx, ai, mp, mt, cnt, best, thr, rl);
            if (!(a.maxmis >= best) && cnt <= 299) {
                aligner_parts_row(fw, ix, a, sidx, ai, mp, mt, cnt, best, thr, rl);
                if (!(a.maxmis >= best) && cnt <= 299) aligner_parts_row(rc, ix, a, sidx, ai, mp, mt, cnt, best, thr, rl);
            }
        }
        if (best <= a.maxmis) r = best;
    }
    return r;
}

// the serial path for one read (the row's first lane): reads longer than the
// rows' LDS staging
__device__ int align_read_serial(const uint8_t* rd, int len, const HashView& ix, const HashArgs& a, int stale,
                                 HashAlign& ai, int* mp, int* mt, int& nn, uint32_t* scr)
{
    const HashRead fw{rd, len, false, scr};
    const HashRead rc{rd, len, true, scr + ((len - 1) >> 4) + 1};
    ai = HashAlign{stale ? 0 : -1, 0, 0, false, false};
    int sidx[4] = {-1, -1, -1, -1};
    int best = -1, r = -1;
    uint32_t cnt = 0;
    const int thr = a.good < a.maxmis ? a.good : a.maxmis;
    nn = 0;
    if (len > 0 && (nn = hash_pack_read(fw)) <= a.maxmis) {
        best = a.maxmis + 1;
        aligner_d(fw, ix, a, sidx, ai, mp, mt, cnt, best, thr);
        if (!(a.maxmis >= best) && cnt <= 299) {
            hash_pack_read(rc);
            aligner_d(rc, ix, a, sidx, ai, mp, mt, cnt, best, thr);
            if (!(a.maxmis >= best) && cnt <= 299) {
                aligner_parts_d(fw, ix, a, sidx, ai, mp, mt, cnt, best, thr);
                if (!(a.maxmis >= best) && cnt <= 299) aligner_parts_d(rc, ix, a, sidx, ai, mp, mt, cnt, best, thr);
            }
        }
        if (best <= a.maxmis) r = best;
    }
    return r;
}

// per workgroup: the base-code table (seq_val_table@0x44b800 / hash_code) and
// each row's staging
struct AlignRowsLds {
    alignas(16) uint8_t bytes[AR_ROWS][AR_BYTES];
    uint32_t words[AR_ROWS][4 * AR_MAXW];
    uint8_t tab[256];
};

__device__ __forceinline__ void align_rows_init(AlignRowsLds& L)
{
    for (uint32_t c = threadIdx.x; c < 256; c += blockDim.x) L.tab[c] = (uint8_t)hash_code((uint8_t)c);
    __syncthreads();
}

// getHashAlignInfo@0x4113c0 over reads given by offset / length (sa_hash_align),
// with the carried align_info state taken as `stale` (0: not aligned, 1:
// aligned).  Outputs per read: ret (mismatches, -1 unaligned), strand, 1-based
// position, maxmis + 1 slots of mismatch offsets / types (-1 past the read's
// mismatches) and whether the carried state was consulted (the host then
// re-runs those reads with the other state and picks per read in order).
// `sel`: the reads to do (NULL: all n), outputs at the read's index.  A row
// per read, grid-stride.
__global__ __launch_bounds__(256) void k_hash_align(const HashView ix, const HashArgs a, const uint8_t* __restrict__ seq,
                                                    const uint64_t* __restrict__ off, const int32_t* __restrict__ lens,
                                                    const uint64_t* __restrict__ woff, uint32_t* __restrict__ scratch,
                                                    const uint32_t* __restrict__ sel, uint64_t n, int stale,
                                                    int32_t* __restrict__ ret, uint8_t* __restrict__ rev,
                                                    uint64_t* __restrict__ pos, int32_t* __restrict__ mispos,
                                                    int32_t* __restrict__ mistype, uint8_t* __restrict__ consulted)
{
    __shared__ AlignRowsLds L;
    align_rows_init(L);
    const uint32_t rl = threadIdx.x % AR, row = threadIdx.x / AR;
    for (uint64_t t = (uint64_t)blockIdx.x * AR_ROWS + row; t < n; t += (uint64_t)gridDim.x * AR_ROWS) {
        const uint64_t i = sel ? sel[t] : t;
        const int len = lens[i];
        const int stride = a.maxmis + 1;
        int* mp = mispos + i * stride;
        int* mt = mistype + i * stride;
        HashAlign ai{-1, 0, 0, false, false};
        int nn = 0, r = -1;
        if (len <= 16 * AR_MAXW) {
            r = align_read_row(seq + off[i], len, ix, a, stale, ai, mp, mt, nn, L.bytes[row], L.words[row], L.tab, rl);
        } else {
            if (rl == 0) r = align_read_serial(seq + off[i], len, ix, a, stale, ai, mp, mt, nn, scratch + 2 * woff[i]);
            __builtin_amdgcn_wave_barrier();
            r = __shfl(rl == 0 ? r : 0, 0, AR);
            ai.nmis = __shfl(rl == 0 ? ai.nmis : 0, 0, AR);
            const uint32_t bits = __shfl(rl == 0 ? (uint32_t)ai.rev | (ai.consulted ? 2u : 0u) : 0u, 0, AR);
            ai.rev = (uint8_t)(bits & 1u);
            ai.consulted = (bits & 2u) != 0;
            ai.pos = __shfl(rl == 0 ? ai.pos : 0ull, 0, AR);
        }
        if (rl == 0) {
            ret[i] = r;
            rev[i] = r >= 0 ? ai.rev : 0;
            pos[i] = r >= 0 ? ai.pos : 0;
            if (consulted) consulted[i] = ai.consulted ? 1 : 0;
        }
        for (int k = (int)rl; k < stride; k += AR)
            if (r < 0 || k >= ai.nmis) {
                mp[k] = -1;
                mt[k] = -1;
            }
    }
}

// ---------------------------------------------------------------------------
// The reference path of a resident batch (doAlignEncode@0x42d4c0's inputs,
// sa_run_input_aligned): every read aligned where it lies in HBM, then the
// alignment streams' per-read columns and keys (sa_logic.h).
// ---------------------------------------------------------------------------
// Scratch words of read r's packed strands: floor(offset / 8) + 2 r (the next
// read's slot starts at least 2 ceil(len / 16) words later).
__device__ __forceinline__ uint64_t align_scratch_word(const BatchView& bv, uint32_t r)
{
    return (bv.blocks[bv.read_block[r]].seq_base + bv.seq_off[r]) / 8 + 2ull * r;
}

// stale = 0: every read (sel == nullptr) with the carried state "not aligned";
// status = AL_OK0 | AL_CONS (the search consulted the carried state) | AL_NSKIP
// (SE: more N / IUPAC bases than maxmis: AlignEncodeSEJob::doAlign@0x411a0b
// does not call the aligner).  stale = 1: the listed reads with "aligned"
// (status |= AL_OK1).  Outputs at the read's index.
__global__ __launch_bounds__(256) void k_hash_align_batch(const HashView ix, const HashArgs a, const BatchView bv,
                                                          uint32_t* __restrict__ scratch, const uint32_t* __restrict__ sel,
                                                          uint32_t n, int stale, int se, int32_t* __restrict__ ret,
                                                          uint8_t* __restrict__ rev, uint32_t* __restrict__ pos,
                                                          int32_t* __restrict__ mispos, int32_t* __restrict__ mistype,
                                                          uint8_t* __restrict__ status)
{
    __shared__ AlignRowsLds L;
    align_rows_init(L);
    const uint32_t rl = threadIdx.x % AR, row = threadIdx.x / AR;
    for (uint32_t t = blockIdx.x * AR_ROWS + row; t < n; t += gridDim.x * AR_ROWS) {
        const uint32_t i = sel ? sel[t] : t;
        const DevBlock& blk = bv.blocks[bv.read_block[i]];
        const uint8_t* rd = bv.seq + blk.seq_base + bv.seq_off[i];
        const int len = (int)bv.seq_len[i];
        const int stride = a.maxmis + 1;
        int* mp = mispos + (size_t)i * stride;
        int* mt = mistype + (size_t)i * stride;
        HashAlign ai{-1, 0, 0, false, false};
        int nn = 0, r = -1;
        if (len <= 16 * AR_MAXW) {
            r = align_read_row(rd, len, ix, a, stale, ai, mp, mt, nn, L.bytes[row], L.words[row], L.tab, rl);
        } else {   // (long reads: the serial path on the row's first lane)
            if (rl == 0) r = align_read_serial(rd, len, ix, a, stale, ai, mp, mt, nn, scratch + align_scratch_word(bv, i));
            __builtin_amdgcn_wave_barrier();
            r = __shfl(rl == 0 ? r : 0, 0, AR);
            nn = __shfl(rl == 0 ? nn : 0, 0, AR);
            ai.nmis = __shfl(rl == 0 ? ai.nmis : 0, 0, AR);
            const uint32_t bits = __shfl(rl == 0 ? (uint32_t)ai.rev | (ai.consulted ? 2u : 0u) : 0u, 0, AR);
            ai.rev = (uint8_t)(bits & 1u);
            ai.consulted = (bits & 2u) != 0;
            ai.pos = __shfl(rl == 0 ? ai.pos : 0ull, 0, AR);
        }
        if (rl == 0) {
            ret[i] = r;
            rev[i] = r >= 0 ? ai.rev : 0;
            pos[i] = r >= 0 ? (uint32_t)ai.pos : 0u;
            if (!stale)
                status[i] = (uint8_t)((r >= 0 ? AL_OK0 : 0) | (ai.consulted ? AL_CONS : 0) |
                                      (se && nn > a.maxmis ? AL_NSKIP : 0));
            else if (r >= 0)
                status[i] |= AL_OK1;
        }
        for (int k = (int)rl; k < stride; k += AR)
            if (r < 0 || k >= ai.nmis) {
                mp[k] = -1;
                mt[k] = -1;
            }
    }
}

// workgroups of the row kernels: a row per read, grid-stride beyond 8192 workgroups
inline uint32_t align_rows_grid(uint64_t reads)
{
    const uint64_t g = (reads + AR_ROWS - 1) / AR_ROWS;
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(g, 8192));
}

// the reads whose carried state was "aligned": variant 1 over variant 0
__global__ __launch_bounds__(256) void k_align_select(const uint32_t* __restrict__ sel, uint32_t n, uint32_t stride,
                                                      const int32_t* __restrict__ ret1, const uint8_t* __restrict__ rev1,
                                                      const uint32_t* __restrict__ pos1, const int32_t* __restrict__ mp1,
                                                      const int32_t* __restrict__ mt1, int32_t* __restrict__ ret,
                                                      uint8_t* __restrict__ rev, uint32_t* __restrict__ pos,
                                                      int32_t* __restrict__ mp, int32_t* __restrict__ mt)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t i = sel[t];
    ret[i] = ret1[i];
    rev[i] = rev1[i];
    pos[i] = pos1[i];
    for (uint32_t k = 0; k < stride; k++) {
        mp[(size_t)i * stride + k] = mp1[(size_t)i * stride + k];
        mt[(size_t)i * stride + k] = mt1[(size_t)i * stride + k];
    }
}

}  // namespace sa

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct sa_hash_index {
    int device = 0;
    uint32_t K = 0, step = 0, maxcount = 0, total = 0, nwords = 0, npos = 0;
    uint64_t nkmers = 0;
    DBuf seq, num, ind, pos;
    ~sa_hash_index()
    {
        for (DBuf* b : {&seq, &num, &ind, &pos}) b->release();
    }
};

namespace {

// a device buffer released when it goes out of scope (DBuf is released by its owner)
struct DTmp : DBuf {
    ~DTmp() { release(); }
};

// exclusive scan of n u32 on the device (tiles of SCAN_TILE, recursing on the
// tile totals); *total (optional) gets the sum
int scan_u32(sa_ctx* c, hipStream_t st, const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* total)
{
    if (n == 0) {
        if (total) *total = 0;
        return 0;
    }
    const uint64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    DTmp sums, sums_x;
    SA_CHECK(c, sums.ensure(tiles * 4));
    hipLaunchKernelGGL(k_scan_tiles, dim3((uint32_t)tiles), dim3(256), 0, st, in, out, n, sums.as<uint32_t>());
    SA_CHECK(c, hipGetLastError());
    if (tiles > 1) {
        SA_CHECK(c, sums_x.ensure(tiles * 4));
        if (scan_u32(c, st, sums.as<uint32_t>(), sums_x.as<uint32_t>(), tiles, nullptr)) return -1;
        hipLaunchKernelGGL(k_scan_add, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, out, n,
                           sums_x.as<uint32_t>());
        SA_CHECK(c, hipGetLastError());
    }
    if (total) {
        uint32_t last_in = 0, last_out = 0;
        SA_CHECK(c, hipMemcpyAsync(&last_in, in + n - 1, 4, hipMemcpyDeviceToHost, st));
        SA_CHECK(c, hipMemcpyAsync(&last_out, out + n - 1, 4, hipMemcpyDeviceToHost, st));
        SA_CHECK(c, hipStreamSynchronize(st));
        *total = last_in + last_out;
    }
    SA_CHECK(c, hipStreamSynchronize(st));   // (sums are freed on return)
    return 0;
}

// The characters buildRefIndex@0x410190 reads: every line that does not start
// with '>', up to strlen(line) - 1 (getdelim keeps the '\n').  Lines before the
// first header are rejected (the reference counts them in one pass only).
bool fasta_bases(const char* fa, uint64_t n, std::vector<uint8_t>& out, std::string& err)
{
    out.clear();
    out.reserve(n);
    bool header = false;
    for (uint64_t at = 0; at < n;) {
        const char* p = fa + at;
        const char* e = static_cast<const char*>(std::memchr(p, '\n', n - at));
        const uint64_t len = e ? (uint64_t)(e - p) + 1 : n - at;
        at += len;
        if (p[0] == '>') {
            header = true;
            continue;
        }
        const char* z = static_cast<const char*>(std::memchr(p, 0, len));
        const uint64_t sl = z ? (uint64_t)(z - p) : len;
        if (sl <= 1) continue;
        if (!header) {
            err = "FASTA: sequence before the first '>' header";
            return false;
        }
        out.insert(out.end(), p, p + sl - 1);
    }
    if (!header) {
        err = "FASTA: no '>' header";
        return false;
    }
    return true;
}

}  // namespace

extern "C" {

sa_hash_index* sa_hash_build(sa_ctx* c, const char* fasta, uint64_t bytes, uint32_t K, uint32_t step,
                             uint32_t maxcount)
{
    if (!c || !fasta) return nullptr;
    if (K < 1 || K > 16 || step < 1 || maxcount < 1) {
        c->err = "sa_hash_build: K must be 1..16, step and maxcount >= 1";
        return nullptr;
    }
    if ((bytes >> 30) > 4) {
        c->err = "sa_hash_build: FASTA of 5 GiB or more (HashRefIndex64) is not supported";
        return nullptr;
    }
    std::vector<uint8_t> b;
    if (!fasta_bases(fasta, bytes, b, c->err)) return nullptr;
    // HashRefIndex32 keeps the genome length and every seed position in 32 bits
    if ((uint64_t)b.size() >= (1ull << 32)) {
        c->err = "sa_hash_build: genome of 2^32 bases or more (HashRefIndex64) is not supported";
        return nullptr;
    }
    std::unique_ptr<sa_hash_index> ix(new sa_hash_index());
    auto fail = [&](int rc) -> sa_hash_index* { return rc ? nullptr : ix.release(); };
    auto body = [&]() -> int {
        SA_CHECK(c, hipSetDevice(c->device));
        hipStream_t st = c->st;
        const uint64_t n = b.size(), mask = K >= 16 ? 0xffffffffull : (1ull << (2 * K)) - 1;
        ix->device = c->device;
        ix->K = K;
        ix->step = step;
        ix->maxcount = maxcount;
        ix->nkmers = mask + 1;
        ix->total = (uint32_t)n;
        ix->nwords = n ? (uint32_t)((n - 1) / 16 + 1) : 1u;   // setEndSeqint@0x41e5a0: last word + 1
        DTmp d_b, cnt, at;
        SA_CHECK(c, d_b.ensure(n + 16));
        if (n) SA_CHECK(c, hipMemcpyAsync(d_b.p, b.data(), n, hipMemcpyHostToDevice, st));
        SA_CHECK(c, ix->seq.ensure(4ull * ix->nwords));
        hipLaunchKernelGGL(k_hash_pack, dim3((uint32_t)((ix->nwords + 255) / 256)), dim3(256), 0, st, d_b.as<uint8_t>(),
                           n, ix->seq.as<uint32_t>(), (uint64_t)ix->nwords);
        SA_CHECK(c, ix->num.ensure(4 * ix->nkmers));
        SA_CHECK(c, ix->ind.ensure(4 * ix->nkmers));
        SA_CHECK(c, hipMemsetAsync(ix->num.p, 0, 4 * ix->nkmers, st));
        const uint64_t nthr = (n + HASH_CHUNK - 1) / HASH_CHUNK;
        const uint32_t grid = (uint32_t)std::max<uint64_t>(1, (nthr + 255) / 256);
        if (n) {
            hipLaunchKernelGGL(k_hash_count, dim3(grid), dim3(256), 0, st, d_b.as<uint8_t>(), n, K, mask, step,
                               ix->num.as<uint32_t>());
            hipLaunchKernelGGL(k_hash_cap, dim3((uint32_t)((ix->nkmers + 255) / 256)), dim3(256), 0, st,
                               ix->num.as<uint32_t>(), ix->nkmers, maxcount);
        }
        SA_CHECK(c, hipGetLastError());
        uint32_t npos = 0;
        if (scan_u32(c, st, ix->num.as<uint32_t>(), ix->ind.as<uint32_t>(), ix->nkmers, &npos)) return -1;
        ix->npos = npos;
        // the kept seeds as (K-mer, start) in position order, then sorted by K-mer
        const SortPlan plan = plan_sort({(uint64_t)npos});
        const uint64_t tot = plan.total + KEY_SLACK;
        DTmp keys[2], vals[2], segs, tiles, hist;
        for (int i = 0; i < 2; i++) {
            SA_CHECK(c, keys[i].ensure(4 * tot));
            SA_CHECK(c, vals[i].ensure(4 * tot));
            SA_CHECK(c, hipMemsetAsync(keys[i].p, 0xff, 4 * tot, st));   // SORT_PAD in the tail tiles
        }
        if (npos && n) {
            SA_CHECK(c, cnt.ensure(4 * nthr));
            SA_CHECK(c, at.ensure(4 * nthr));
            hipLaunchKernelGGL(k_hash_emit, dim3(grid), dim3(256), 0, st, d_b.as<uint8_t>(), n, K, mask, step,
                               ix->num.as<uint32_t>(), cnt.as<uint32_t>(), at.as<uint32_t>(), keys[0].as<uint32_t>(),
                               vals[0].as<uint32_t>(), 0);
            if (scan_u32(c, st, cnt.as<uint32_t>(), at.as<uint32_t>(), nthr, nullptr)) return -1;
            hipLaunchKernelGGL(k_hash_emit, dim3(grid), dim3(256), 0, st, d_b.as<uint8_t>(), n, K, mask, step,
                               ix->num.as<uint32_t>(), cnt.as<uint32_t>(), at.as<uint32_t>(), keys[0].as<uint32_t>(),
                               vals[0].as<uint32_t>(), 1);
            SA_CHECK(c, hipGetLastError());
            SA_CHECK(c, segs.ensure(sizeof(SortSeg) * plan.segs.size()));
            SA_CHECK(c, tiles.ensure(4 * std::max<size_t>(plan.tile_seg.size(), 1)));
            SA_CHECK(c, hist.ensure(4 * std::max<size_t>(plan.tile_seg.size(), 1) * sort_hist_per_tile(0, 2 * (int)K)));
            SA_CHECK(c, hipMemcpyAsync(segs.p, plan.segs.data(), sizeof(SortSeg) * plan.segs.size(),
                                       hipMemcpyHostToDevice, st));
            SA_CHECK(c, hipMemcpyAsync(tiles.p, plan.tile_seg.data(), 4 * plan.tile_seg.size(), hipMemcpyHostToDevice,
                                       st));
            DBuf* kb[2] = {&keys[0], &keys[1]};
            DBuf* vb[2] = {&vals[0], &vals[1]};
            int res = 0;
            if (run_sort(c, st, plan, segs, tiles, hist, kb, vb, 0, 2 * (int)K, res)) return -1;
            std::swap(static_cast<DBuf&>(ix->pos), static_cast<DBuf&>(vals[res]));   // the position table
        } else {
            SA_CHECK(c, ix->pos.ensure(4));
        }
        SA_CHECK(c, hipStreamSynchronize(st));
        return 0;
    };
    return fail(body());
}

uint64_t sa_hash_file_bytes(const sa_hash_index* ix)
{
    return ix ? 16 + 4ull * (ix->nwords + 2 * ix->nkmers + ix->npos) : 0;
}

uint32_t sa_hash_genome_length(const sa_hash_index* ix) { return ix ? ix->total : 0; }

// HashRefIndex32::writeIndexFile@0x41ed00: K, bases, words, positions (u32),
// seq[words], num[4^K], ind[4^K], pos[positions]
int sa_hash_serialize(sa_ctx* c, const sa_hash_index* ix, uint8_t* out, uint64_t cap)
{
    if (!c || !ix || !out) return -1;
    if (cap < sa_hash_file_bytes(ix)) {
        c->err = "sa_hash_serialize: output buffer too small";
        return -1;
    }
    SA_CHECK(c, hipSetDevice(ix->device));
    const uint32_t hdr[4] = {ix->K, ix->total, ix->nwords, ix->npos};
    std::memcpy(out, hdr, 16);
    uint8_t* o = out + 16;
    SA_CHECK(c, hipMemcpy(o, ix->seq.p, 4ull * ix->nwords, hipMemcpyDeviceToHost));
    o += 4ull * ix->nwords;
    SA_CHECK(c, hipMemcpy(o, ix->num.p, 4 * ix->nkmers, hipMemcpyDeviceToHost));
    o += 4 * ix->nkmers;
    SA_CHECK(c, hipMemcpy(o, ix->ind.p, 4 * ix->nkmers, hipMemcpyDeviceToHost));
    o += 4 * ix->nkmers;
    if (ix->npos) SA_CHECK(c, hipMemcpy(o, ix->pos.p, 4ull * ix->npos, hipMemcpyDeviceToHost));
    return 0;
}

void sa_hash_destroy(sa_hash_index* ix)
{
    if (!ix) return;
    (void)hipSetDevice(ix->device);
    delete ix;
}

int sa_hash_align(sa_ctx* c, const sa_hash_index* ix, const char* seq, const uint64_t* off, const int32_t* lens,
                  int64_t n, int32_t maxmis, int32_t good, int32_t* ai_nmis, int32_t* ret, uint8_t* rev,
                  uint64_t* pos, int32_t* mispos, int32_t* mistype)
{
    if (!c || !ix || n < 0 || !ai_nmis ||
        (n && (!seq || !off || !lens || !ret || !rev || !pos || !mispos || !mistype)))
        return -1;
    if (maxmis < 0 || maxmis > 63) {
        c->err = "sa_hash_align: maxmis must be 0..63";
        return -1;
    }
    if (n == 0) return 0;
    SA_CHECK(c, hipSetDevice(c->device));
    if (ix->device != c->device) {
        c->err = "sa_hash_align: index and context on different devices";
        return -1;
    }
    hipStream_t st = c->st;
    uint64_t bytes = 0, words = 0;
    std::vector<uint64_t> woff((size_t)n);
    for (int64_t i = 0; i < n; i++) {
        if (lens[i] < 0) {
            c->err = "sa_hash_align: negative read length";
            return -1;
        }
        bytes = std::max<uint64_t>(bytes, off[i] + (uint64_t)lens[i]);
        woff[(size_t)i] = words;
        words += lens[i] > 0 ? (uint64_t)((lens[i] - 1) >> 4) + 1 : 0;
    }
    const uint64_t N = (uint64_t)n, stride = (uint64_t)maxmis + 1;
    DTmp d_seq, d_off, d_len, d_woff, d_scr, d_sel, d_ret[2], d_rev[2], d_pos[2], d_mp[2], d_mt[2], d_con;
    SA_CHECK(c, d_seq.ensure(bytes + 64));   // (the rows' 16-byte loads read up to 19 bytes past a read)
    SA_CHECK(c, d_off.ensure(8 * N));
    SA_CHECK(c, d_len.ensure(4 * N));
    SA_CHECK(c, d_woff.ensure(8 * N));
    SA_CHECK(c, d_scr.ensure(8 * words + 16));
    SA_CHECK(c, d_con.ensure(N));
    for (int v = 0; v < 2; v++) {
        SA_CHECK(c, d_ret[v].ensure(4 * N));
        SA_CHECK(c, d_rev[v].ensure(N));
        SA_CHECK(c, d_pos[v].ensure(8 * N));
        SA_CHECK(c, d_mp[v].ensure(4 * stride * N));
        SA_CHECK(c, d_mt[v].ensure(4 * stride * N));
    }
    SA_CHECK(c, hipMemcpyAsync(d_seq.p, seq, bytes, hipMemcpyHostToDevice, st));
    SA_CHECK(c, hipMemcpyAsync(d_off.p, off, 8 * N, hipMemcpyHostToDevice, st));
    SA_CHECK(c, hipMemcpyAsync(d_len.p, lens, 4 * N, hipMemcpyHostToDevice, st));
    SA_CHECK(c, hipMemcpyAsync(d_woff.p, woff.data(), 8 * N, hipMemcpyHostToDevice, st));
    const HashView v{ix->seq.as<uint32_t>(), ix->num.as<uint32_t>(), ix->ind.as<uint32_t>(), ix->pos.as<uint32_t>(),
                     ix->K, (uint64_t)ix->total};
    const HashArgs a{maxmis, good};
    // every read with the carried state "not aligned"; then the reads that
    // consulted it again with "aligned"; then the choice, read by read, in order
    hipEvent_t e0 = nullptr, e1 = nullptr;
    SA_CHECK(c, hipEventCreate(&e0));
    SA_CHECK(c, hipEventCreate(&e1));
    SA_CHECK(c, hipEventRecord(e0, st));
    hipLaunchKernelGGL(k_hash_align, dim3(align_rows_grid(N)), dim3(256), 0, st, v, a, d_seq.as<uint8_t>(),
                       d_off.as<uint64_t>(), d_len.as<int32_t>(), d_woff.as<uint64_t>(), d_scr.as<uint32_t>(),
                       nullptr, N, 0, d_ret[0].as<int32_t>(), d_rev[0].as<uint8_t>(), d_pos[0].as<uint64_t>(),
                       d_mp[0].as<int32_t>(), d_mt[0].as<int32_t>(), d_con.as<uint8_t>());
    SA_CHECK(c, hipGetLastError());
    SA_CHECK(c, hipEventRecord(e1, st));
    std::vector<uint8_t> con(N);
    SA_CHECK(c, hipMemcpyAsync(con.data(), d_con.p, N, hipMemcpyDeviceToHost, st));
    SA_CHECK(c, hipStreamSynchronize(st));
    c->align_kernel_ms = 0.f;
    (void)hipEventElapsedTime(&c->align_kernel_ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    std::vector<uint32_t> sel;
    for (uint64_t i = 0; i < N; i++)
        if (con[i]) sel.push_back((uint32_t)i);
    if (!sel.empty()) {
        SA_CHECK(c, d_sel.ensure(4 * sel.size()));
        SA_CHECK(c, hipMemcpyAsync(d_sel.p, sel.data(), 4 * sel.size(), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_hash_align, dim3(align_rows_grid(sel.size())), dim3(256), 0, st, v, a,
                           d_seq.as<uint8_t>(), d_off.as<uint64_t>(), d_len.as<int32_t>(), d_woff.as<uint64_t>(),
                           d_scr.as<uint32_t>(), d_sel.as<uint32_t>(), (uint64_t)sel.size(), 1,
                           d_ret[1].as<int32_t>(), d_rev[1].as<uint8_t>(), d_pos[1].as<uint64_t>(),
                           d_mp[1].as<int32_t>(), d_mt[1].as<int32_t>(), nullptr);
        SA_CHECK(c, hipGetLastError());
    }
    SA_CHECK(c, hipMemcpyAsync(ret, d_ret[0].p, 4 * N, hipMemcpyDeviceToHost, st));
    SA_CHECK(c, hipMemcpyAsync(rev, d_rev[0].p, N, hipMemcpyDeviceToHost, st));
    SA_CHECK(c, hipMemcpyAsync(pos, d_pos[0].p, 8 * N, hipMemcpyDeviceToHost, st));
    SA_CHECK(c, hipMemcpyAsync(mispos, d_mp[0].p, 4 * stride * N, hipMemcpyDeviceToHost, st));
    SA_CHECK(c, hipMemcpyAsync(mistype, d_mt[0].p, 4 * stride * N, hipMemcpyDeviceToHost, st));
    SA_CHECK(c, hipStreamSynchronize(st));
    std::vector<int32_t> r1, m1, t1;
    std::vector<uint8_t> v1;
    std::vector<uint64_t> p1;
    if (!sel.empty()) {
        r1.resize(N);
        v1.resize(N);
        p1.resize(N);
        m1.resize(stride * N);
        t1.resize(stride * N);
        SA_CHECK(c, hipMemcpyAsync(r1.data(), d_ret[1].p, 4 * N, hipMemcpyDeviceToHost, st));
        SA_CHECK(c, hipMemcpyAsync(v1.data(), d_rev[1].p, N, hipMemcpyDeviceToHost, st));
        SA_CHECK(c, hipMemcpyAsync(p1.data(), d_pos[1].p, 8 * N, hipMemcpyDeviceToHost, st));
        SA_CHECK(c, hipMemcpyAsync(m1.data(), d_mp[1].p, 4 * stride * N, hipMemcpyDeviceToHost, st));
        SA_CHECK(c, hipMemcpyAsync(t1.data(), d_mt[1].p, 4 * stride * N, hipMemcpyDeviceToHost, st));
        SA_CHECK(c, hipStreamSynchronize(st));
    }
    bool aligned = *ai_nmis >= 0 && *ai_nmis <= maxmis;
    for (uint64_t i = 0; i < N; i++) {
        if (aligned && con[i]) {   // the "aligned" variant of this read
            ret[i] = r1[i];
            rev[i] = v1[i];
            pos[i] = p1[i];
            std::memcpy(mispos + i * stride, &m1[i * stride], 4 * stride);
            std::memcpy(mistype + i * stride, &t1[i * stride], 4 * stride);
        }
        aligned = ret[i] >= 0;
    }
    *ai_nmis = ret[N - 1];   // getHashAlignInfo leaves nmis = the count, or -1
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// reference path of a resident batch (sa_run_input_aligned)
// ---------------------------------------------------------------------------
// SA_ALN_TRACE=1: the reference path's host steps on stderr
static bool aln_trace()
{
    static const bool on = std::getenv("SA_ALN_TRACE") != nullptr;
    return on;
}
#define ATRACE(...)                                  \
    do {                                             \
        if (aln_trace()) {                           \
            std::fprintf(stderr, "[align] " __VA_ARGS__); \
            std::fflush(stderr);                     \
        }                                            \
    } while (0)

struct sa_align_chain {
    std::mutex mu;
    std::condition_variable cv;
    uint64_t next = 0;            // the batch whose alignment may follow the chain now
    sa::AlignChainState st;
    bool failed = false;
};

void align_chain_fail(sa_align_chain* ch)
{
    if (!ch) return;
    {
        std::lock_guard<std::mutex> g(ch->mu);
        ch->failed = true;
    }
    ch->cv.notify_all();
}

// a batch without blocks passes the chain unchanged (its turn still comes:
// later batches wait for it)
static int align_chain_pass_empty(sa_align_chain* ch, uint64_t batch)
{
    std::unique_lock<std::mutex> lk(ch->mu);
    const uint64_t me = batch == UINT64_MAX ? ch->next : batch;
    ch->cv.wait(lk, [&] { return ch->failed || ch->next == me; });
    if (ch->failed) return -1;
    ch->next = me + 1;
    lk.unlock();
    ch->cv.notify_all();
    return 0;
}

int align_front(sa_ctx* c, const sa_input* I, BatchView& bv, const AlignReq& rq, std::vector<uint32_t>& atot,
                AlignView& av)
{
    const sa_hash_index* ix = rq.ix;
    const sa_align_cfg& a = rq.cfg;
    const uint32_t nr = I->nreads, nbk = I->nblocks;
    if (!ix || !rq.chain || ix->device != c->device) {
        c->err = "sa_run_input_aligned: no index / chain, or an index of another device";
        return -1;
    }
    if (a.maxmis < 0 || a.maxmis > 8 || ix->total < 4) {   // (the Mis model exists for maxmis 1..8)
        c->err = "sa_run_input_aligned: maxmis must be 0..8 and the genome at least 4 bases";
        return -1;
    }
    if (a.paired)
        for (const DevBlock& d : c->blocks)
            if (d.nreads & 1) {
                c->err = "sa_run_input_aligned: a paired block with an odd read count";
                return -1;
            }
    hipStream_t st = c->st;
    const uint32_t stride = (uint32_t)a.maxmis + 1;
    const size_t n1 = std::max<uint32_t>(nr, 1);
    for (int v = 0; v < 2; v++) {
        SA_CHECK(c, c->d_al_ret[v].ensure(4 * n1));
        SA_CHECK(c, c->d_al_rev[v].ensure(n1));
        SA_CHECK(c, c->d_al_pos[v].ensure(4 * n1));
        SA_CHECK(c, c->d_al_mp[v].ensure(4 * stride * n1));
        SA_CHECK(c, c->d_al_mt[v].ensure(4 * stride * n1));
    }
    SA_CHECK(c, c->d_al_st.ensure(n1));
    SA_CHECK(c, c->d_al_scr.ensure(4 * (I->seq_bytes / 8 + 2 * (uint64_t)n1 + 64)));
    SA_CHECK(c, c->d_acounts.ensure(4 * NACOL * n1));
    SA_CHECK(c, c->d_atot.ensure(4 * NACOL * (size_t)std::max<uint32_t>(nbk, 1)));
    SA_CHECK(c, c->d_seq_skip.ensure(n1));
    const HashView hv{ix->seq.as<uint32_t>(), ix->num.as<uint32_t>(), ix->ind.as<uint32_t>(), ix->pos.as<uint32_t>(),
                      ix->K, (uint64_t)ix->total};
    const HashArgs ha{a.maxmis, a.good};
    const bool rerun = c->al_input == I && c->al_plan.size() == 4ull * nbk &&
                       (rq.batch == UINT64_MAX || rq.batch == c->al_batch);
    ATRACE("front: %u reads, %u blocks, rerun %d\n", nr, nbk, (int)rerun);
    if (!rerun) {
        // ---- every read with the carried state "not aligned" ----
        if (nr)
            hipLaunchKernelGGL(k_hash_align_batch, dim3(align_rows_grid(nr)), dim3(256), 0, st, hv, ha, bv,
                               c->d_al_scr.as<uint32_t>(), nullptr, nr, 0, a.paired ? 0 : 1, c->d_al_ret[0].as<int32_t>(),
                               c->d_al_rev[0].as<uint8_t>(), c->d_al_pos[0].as<uint32_t>(), c->d_al_mp[0].as<int32_t>(),
                               c->d_al_mt[0].as<int32_t>(), c->d_al_st.as<uint8_t>());
        SA_CHECK(c, hipGetLastError());
        std::vector<uint8_t> status(n1, 0);
        std::vector<uint32_t> pos0(n1, 0), pos1(n1, 0);
        SA_CHECK(c, d2h(c, status.data(), c->d_al_st.p, nr, st));
        SA_CHECK(c, d2h(c, pos0.data(), c->d_al_pos[0].p, 4ull * nr, st));
        SA_CHECK(c, sync_d2h(c, st));
        ATRACE("variant 0 done\n");
        // ---- the reads that consulted it, again with "aligned" ----
        std::vector<uint32_t> cons;
        for (uint32_t r = 0; r < nr; r++)
            if ((status[r] & AL_CONS) && !(status[r] & AL_NSKIP)) cons.push_back(r);
        if (!cons.empty()) {
            SA_CHECK(c, c->d_al_sel.ensure(4 * cons.size()));
            SA_CHECK(c, h2d(c, c->d_al_sel.p, cons.data(), 4 * cons.size(), st));
            hipLaunchKernelGGL(k_hash_align_batch, dim3(align_rows_grid(cons.size())), dim3(256), 0, st, hv, ha, bv,
                               c->d_al_scr.as<uint32_t>(), c->d_al_sel.as<uint32_t>(), (uint32_t)cons.size(), 1,
                               a.paired ? 0 : 1, c->d_al_ret[1].as<int32_t>(), c->d_al_rev[1].as<uint8_t>(),
                               c->d_al_pos[1].as<uint32_t>(), c->d_al_mp[1].as<int32_t>(), c->d_al_mt[1].as<int32_t>(),
                               c->d_al_st.as<uint8_t>());
            SA_CHECK(c, hipGetLastError());
            SA_CHECK(c, d2h(c, status.data(), c->d_al_st.p, nr, st));
            SA_CHECK(c, d2h(c, pos1.data(), c->d_al_pos[1].p, 4ull * nr, st));
            SA_CHECK(c, sync_d2h(c, st));
        }
        ATRACE("variant 1 done (%zu reads)\n", cons.size());
        // ---- the chain: this batch after the previous one ----
        sa_align_chain* ch = rq.chain;
        std::vector<uint32_t> sel;
        {
            std::unique_lock<std::mutex> lk(ch->mu);
            const uint64_t me = rq.batch == UINT64_MAX ? ch->next : rq.batch;
            ch->cv.wait(lk, [&] { return ch->failed || ch->next == me; });
            if (ch->failed) {
                c->err = "sa_run_input_aligned: an earlier batch of the chain failed";
                return -1;
            }
            c->al_plan.assign(4ull * nbk, 0);
            for (uint32_t b = 0; b < nbk; b++) {
                const DevBlock& d = c->blocks[b];
                std::vector<uint32_t> sl;
                const AlignBlockPlan p = align_plan_block(a.paired != 0, d.nreads, &status[d.read0], &pos0[d.read0],
                                                          &pos1[d.read0], a.insert_size, ch->st, sl);
                for (uint32_t i : sl) sel.push_back(d.read0 + i);
                c->al_plan[4 * b + 0] = p.order_count;
                c->al_plan[4 * b + 1] = p.win;
                c->al_plan[4 * b + 2] = p.ibits;
                c->al_plan[4 * b + 3] = p.insert_bits;
            }
            ch->next = me + 1;
            c->al_batch = me;
        }
        ch->cv.notify_all();
        ATRACE("chain passed, %zu reads take variant 1\n", sel.size());
        c->al_input = I;
        if (!sel.empty()) {
            SA_CHECK(c, c->d_al_sel.ensure(4 * sel.size()));
            SA_CHECK(c, h2d(c, c->d_al_sel.p, sel.data(), 4 * sel.size(), st));
            hipLaunchKernelGGL(k_align_select, dim3((uint32_t)((sel.size() + 255) / 256)), dim3(256), 0, st,
                               c->d_al_sel.as<uint32_t>(), (uint32_t)sel.size(), stride, c->d_al_ret[1].as<int32_t>(),
                               c->d_al_rev[1].as<uint8_t>(), c->d_al_pos[1].as<uint32_t>(), c->d_al_mp[1].as<int32_t>(),
                               c->d_al_mt[1].as<int32_t>(), c->d_al_ret[0].as<int32_t>(), c->d_al_rev[0].as<uint8_t>(),
                               c->d_al_pos[0].as<uint32_t>(), c->d_al_mp[0].as<int32_t>(), c->d_al_mt[0].as<int32_t>());
            SA_CHECK(c, hipGetLastError());
        }
    }
    for (uint32_t b = 0; b < nbk; b++) {
        DevBlock& d = c->blocks[b];
        d.order_count = c->al_plan[4 * b + 0];
        d.win = c->al_plan[4 * b + 1];
        d.ibits = c->al_plan[4 * b + 2];
        d.insert_bits = c->al_plan[4 * b + 3];
    }
    SA_CHECK(c, h2d(c, c->d_blocks.p, c->blocks.data(), sizeof(DevBlock) * nbk, st));
    const uint32_t shift = host_bits(ix->total) - 2;   // HashAlignment::loadRefIndex@0x40fe9b
    av = AlignView{c->d_al_ret[0].as<int32_t>(), c->d_al_rev[0].as<uint8_t>(), c->d_al_pos[0].as<uint32_t>(),
                   c->d_al_mp[0].as<int32_t>(), c->d_al_mt[0].as<int32_t>(), stride, shift, (1ull << shift) - 1,
                   (uint64_t)ix->total, a.paired ? 1 : 0,
                   a.maxmis >= 1 && a.maxmis <= 7 ? M_MIS8 : a.maxmis == 8 ? M_MIS9 : 0u};
    bv.aligned = 1;
    bv.paired = a.paired ? 1 : 0;
    bv.seq_skip = c->d_seq_skip.as<uint8_t>();
    if (nr) {
        hipLaunchKernelGGL(k_align_counts, dim3((nr + 255) / 256), dim3(256), 0, st, bv, av, c->d_acounts.as<uint32_t>(),
                           c->d_seq_skip.as<uint8_t>());
        hipLaunchKernelGGL(k_scan_align, dim3(nbk), dim3(1024), 0, st, bv, c->d_acounts.as<uint32_t>(),
                           c->d_atot.as<uint32_t>());
    } else {
        SA_CHECK(c, hipMemsetAsync(c->d_atot.p, 0, 4ull * NACOL * nbk, st));
    }
    SA_CHECK(c, hipGetLastError());
    atot.assign((size_t)NACOL * nbk, 0);
    SA_CHECK(c, d2h(c, atot.data(), c->d_atot.p, 4ull * NACOL * nbk, st));
    SA_CHECK(c, sync_d2h(c, st));
    for (uint32_t b = 0; b < nbk && aln_trace(); b++)
        ATRACE("block %u: order_count %u win %u ibits %u; columns %u %u %u %u %u %u %u\n", b, c->blocks[b].order_count,
               c->blocks[b].win, c->blocks[b].ibits, atot[NACOL * b], atot[NACOL * b + 1], atot[NACOL * b + 2],
               atot[NACOL * b + 3], atot[NACOL * b + 4], atot[NACOL * b + 5], atot[NACOL * b + 6]);
    return 0;
}

extern "C" {

sa_align_chain* sa_align_chain_create(int32_t nmis_mate1, int32_t nmis_mate2)
{
    sa_align_chain* ch = new sa_align_chain();
    // hashAligner@0x410f50's test: the carried mismatch count within [0, maxmis]
    // (maxmis is not known yet: a fresh thread's 0 and -1 are the cases that arise)
    ch->st.c[0] = nmis_mate1 >= 0;
    ch->st.c[1] = nmis_mate2 >= 0;
    return ch;
}

void sa_align_chain_destroy(sa_align_chain* ch) { delete ch; }

void sa_align_chain_fail(sa_align_chain* ch) { align_chain_fail(ch); }

float sa_hash_align_kernel_ms(const sa_ctx* c) { return c ? c->align_kernel_ms : 0.f; }

int sa_run_input_aligned(sa_ctx* c, const sa_input* I, const sa_cfg* cfg, const sa_align_cfg* acfg,
                         sa_align_chain* chain, uint64_t batch)
{
    if (!c) return -1;
    if (!acfg || !chain) {
        c->err = "sa_run_input_aligned: no alignment config or chain";
        return -1;
    }
    if (acfg->maxmis < 0 || acfg->maxmis > 8) {   // (before anything waits on the chain)
        c->err = "sa_run_input_aligned: maxmis must be 0..8";
        align_chain_fail(chain);
        return -1;
    }
    const AlignReq rq{acfg->index, *acfg, chain, batch};
    c->al_input = nullptr;   // (a new batch: pass the chain)
    int rc = run_input(c, I, cfg, true, &rq);
    if (rc == 2) {   // exact payload outgrown: drain, re-run with the bound (same alignment plan)
        for (hipStream_t s : {c->st, c->st2, c->st3, c->st4}) (void)hipStreamSynchronize(s);
        const AlignReq rq2{acfg->index, *acfg, chain, c->al_batch};
        rc = run_input(c, I, cfg, false, &rq2);
    }
    if (rc == 0 && I && I->nblocks == 0 && align_chain_pass_empty(chain, batch)) {
        c->err = "sa_run_input_aligned: an earlier batch of the chain failed";
        rc = -1;
    }
    // any failure ends the chain: the contexts waiting on later batches return
    // an error instead of waiting for this batch forever
    if (rc) {
        align_chain_fail(chain);
        drain_after_error(c);
    }
    return rc ? -1 : 0;
}

int sa_run_aligned(sa_ctx* c, const sa_cfg* cfg, const sa_align_cfg* acfg, sa_align_chain* chain, uint64_t batch)
{
    if (!c) return -1;
    return sa_run_input_aligned(c, &c->own, cfg, acfg, chain, batch);
}

int sa_encode_blocks_aligned(sa_ctx* ctx, const sa_block* in, int n, const sa_cfg* cfg, const sa_align_cfg* acfg,
                             sa_align_chain* chain, sa_out* out)
{
    if (!ctx || !cfg || !acfg || !chain || (n > 0 && (!in || !out))) return -1;
    SA_CHECK(ctx, hipSetDevice(ctx->device));
    size_t free_b = 0, total_b = 0;
    SA_CHECK(ctx, hipMemGetInfo(&free_b, &total_b));
    // (per read ~2 x (9 + 8 (maxmis + 1)) bytes of alignment on top of the encode)
    const uint64_t budget = (uint64_t)((double)(free_b + ctx->held_bytes()) * 0.75);
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
            const uint64_t fb = block_footprint(in[b1]) + (uint64_t)in[b1].nreads * (40 + 16 * (uint64_t)(acfg->maxmis + 1));
            if (b1 > b0 && (bases + ls > cap_bases || bytes + fb > budget)) break;
            bases += ls;
            bytes += fb;
            b1++;
        }
        if (sa_stage(ctx, in + b0, b1 - b0)) return -1;
        if (sa_run_aligned(ctx, cfg, acfg, chain, UINT64_MAX)) return -1;
        if (sa_fetch(ctx, out + b0, b1 - b0)) return -1;
        b0 = b1;
    }
    return 0;
}

sa_hash_index* sa_hash_load(sa_ctx* c, const uint8_t* file, uint64_t bytes)
{
    if (!c || !file || bytes < 16) return nullptr;
    uint32_t hdr[4];
    std::memcpy(hdr, file, 16);
    const uint32_t K = hdr[0];
    if (K < 1 || K > 16) {
        c->err = "sa_hash_load: not a .hash file (K)";
        return nullptr;
    }
    const uint64_t nk = K >= 16 ? (1ull << 32) : (1ull << (2 * K));
    if (bytes != 16 + 4ull * (hdr[2] + 2 * nk + hdr[3]) || hdr[2] != (hdr[1] ? (hdr[1] - 1) / 16 + 1 : 1u)) {
        c->err = "sa_hash_load: .hash file size does not match its header";
        return nullptr;
    }
    std::unique_ptr<sa_hash_index> ix(new sa_hash_index());
    ix->device = c->device;
    ix->K = K;
    ix->total = hdr[1];
    ix->nwords = hdr[2];
    ix->npos = hdr[3];
    ix->nkmers = nk;
    auto body = [&]() -> int {
        SA_CHECK(c, hipSetDevice(c->device));
        const uint8_t* p = file + 16;
        SA_CHECK(c, ix->seq.ensure(4ull * ix->nwords));
        SA_CHECK(c, hipMemcpy(ix->seq.p, p, 4ull * ix->nwords, hipMemcpyHostToDevice));
        p += 4ull * ix->nwords;
        SA_CHECK(c, ix->num.ensure(4 * nk));
        SA_CHECK(c, hipMemcpy(ix->num.p, p, 4 * nk, hipMemcpyHostToDevice));
        p += 4 * nk;
        SA_CHECK(c, ix->ind.ensure(4 * nk));
        SA_CHECK(c, hipMemcpy(ix->ind.p, p, 4 * nk, hipMemcpyHostToDevice));
        p += 4 * nk;
        SA_CHECK(c, ix->pos.ensure(4ull * std::max<uint32_t>(ix->npos, 1)));
        if (ix->npos) SA_CHECK(c, hipMemcpy(ix->pos.p, p, 4ull * ix->npos, hipMemcpyHostToDevice));
        return 0;
    };
    return body() ? nullptr : ix.release();
}

int sa_hash_packed(sa_ctx* c, const sa_hash_index* ix, uint32_t* out, uint64_t words)
{
    if (!c || !ix || !out || words < ix->nwords) return -1;
    SA_CHECK(c, hipSetDevice(ix->device));
    SA_CHECK(c, hipMemcpy(out, ix->seq.p, 4ull * ix->nwords, hipMemcpyDeviceToHost));
    return 0;
}

}  // extern "C"
