// sa_parse.hip -- FASTQ text -> the resident SoA batch, on the device.
// Included by sa_engine.hip (needs sa_ctx, sa_input, DBuf and the mailbox).
//
// The host reader hands over each block's text exactly as it cut it (file 1
// and, for PE, file 2); the device finds the newlines, takes the records apart
// and copies IDs, bases and qualities into the layout sa_stage would upload,
// with the semantics of the reference's parsers:
//   getBlockRead@0x411b60   (SE): a state machine over '\n'; a header starts
//     two bytes after the previous record's quality newline ('@' skipped by
//     position), the quality copy takes the sequence's length;
//   getBlockReadPE@0x412920 (PE): the newline arrays of both texts, min(k1,k2)
//     lines, reads interleaved r1, r2, the quality line must be as long as the
//     sequence.
// (fastq_host.cpp: sa_parse_se / sa_parse_pe, the host restatement; tests
// compare the two paths block by block.)
//
// Kernels (all on the staging context's stream):
//   k_nl_count   one 4 KiB tile per workgroup: newlines of the tile
//   k_text_scan  one workgroup per text: exclusive scan of its tile counts
//   k_nl_emit    newline positions (u32 within the text), in order
//   k_parse_reads  one lane per read: field offsets / lengths, errors
//   k_block_scan one workgroup per block: per-read offsets inside the block
//   k_copy_reads one wave per read (grid-stride): IDs, bases, qualities
// HBM traffic: the text is read three times (count, emit, copy) and the SoA
// written once -- ~4 B per text byte, ~2 ms per 3.6 GB batch at HBM rate.

namespace {

constexpr uint32_t PARSE_TILE = 4096;   // 256 threads x 16 bytes

struct ParseText {     // one text (file 1 or file 2 of a block) in d_text
    uint64_t off;      // byte offset in d_text (PARSE_TILE-aligned)
    uint64_t nl_base;  // index of its first newline in d_nl
    uint32_t len;
    uint32_t tile0;    // its first tile
};

struct ParseBlock {
    uint32_t text1, text2;   // ParseText indices (text2 = text1 for SE)
    uint32_t read0, nreads;
    uint64_t name_base, seq_base;   // (filled after k_block_scan)
    uint32_t pe, pad_;
};

struct BlockTotals {
    uint64_t name_bytes, seq_bytes;
    uint32_t len_long, pad_;
};

enum : uint32_t { PARSE_ERR_NAME = 1u, PARSE_ERR_QUAL = 2u, PARSE_ERR_QLEN = 4u, PARSE_ERR_LONG = 8u };

__device__ inline uint32_t nl_mask16(uint4 v, uint32_t valid)
{
    uint32_t m = 0;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        // bytes equal to '\n' (0x0a): the zero bytes of w ^ 0x0a0a0a0a
        const uint32_t x = w[k] ^ 0x0a0a0a0au;
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (((x >> (8 * j)) & 0xffu) == 0) m |= 1u << (4 * k + j);
    }
    return valid >= 16 ? m : m & ((1u << valid) - 1u);
}

__global__ __launch_bounds__(256) void k_nl_count(const uint8_t* __restrict__ text, const uint32_t* __restrict__ tile_text,
                                                  const ParseText* __restrict__ texts, uint32_t* __restrict__ tile_cnt)
{
    __shared__ uint32_t sh[4];
    const uint32_t tile = blockIdx.x;
    const ParseText tx = texts[tile_text[tile]];
    const uint64_t at = (uint64_t)(tile - tx.tile0) * PARSE_TILE + threadIdx.x * 16u;
    const uint32_t valid = at < tx.len ? (uint32_t)min<uint64_t>(16, tx.len - at) : 0u;
    uint32_t n = 0;
    if (valid) n = __popc(nl_mask16(*reinterpret_cast<const uint4*>(text + tx.off + at), valid));
    uint32_t ex;
    wg256_excl_scan(n, ex, sh);
    if (threadIdx.x == 255) tile_cnt[tile] = ex + n;
}

// one workgroup per text: its tiles' newline bases (exclusive) and its total
__global__ __launch_bounds__(256) void k_text_scan(const ParseText* __restrict__ texts, const uint32_t* __restrict__ ntiles,
                                                   const uint32_t* __restrict__ tile_cnt, uint32_t* __restrict__ tile_base,
                                                   uint32_t* __restrict__ text_nl)
{
    __shared__ uint32_t sh[4];
    const uint32_t t = blockIdx.x;
    const uint32_t t0 = texts[t].tile0, nt = ntiles[t];
    uint32_t carry = 0;
    for (uint32_t b = 0; b < nt; b += 256) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < nt ? tile_cnt[t0 + i] : 0u;
        uint32_t ex;
        wg256_excl_scan(v, ex, sh);
        if (i < nt) tile_base[t0 + i] = carry + ex;
        __syncthreads();
        carry += sh[0] + sh[1] + sh[2] + sh[3];
        __syncthreads();
    }
    if (threadIdx.x == 0) text_nl[t] = carry;
}

__global__ __launch_bounds__(256) void k_nl_emit(const uint8_t* __restrict__ text, const uint32_t* __restrict__ tile_text,
                                                 const ParseText* __restrict__ texts, const uint32_t* __restrict__ tile_base,
                                                 uint32_t* __restrict__ nl)
{
    __shared__ uint32_t sh[4];
    const uint32_t tile = blockIdx.x;
    const ParseText tx = texts[tile_text[tile]];
    const uint64_t at = (uint64_t)(tile - tx.tile0) * PARSE_TILE + threadIdx.x * 16u;
    const uint32_t valid = at < tx.len ? (uint32_t)min<uint64_t>(16, tx.len - at) : 0u;
    uint32_t m = 0;
    if (valid) m = nl_mask16(*reinterpret_cast<const uint4*>(text + tx.off + at), valid);
    uint32_t ex;
    wg256_excl_scan(__popc(m), ex, sh);
    uint32_t* dst = nl + tx.nl_base + tile_base[tile] + ex;
    while (m) {
        const uint32_t j = __ffs(m) - 1;
        *dst++ = (uint32_t)at + j;
        m &= m - 1;
    }
}

// One lane per read.  src[3 * g + 0/1/2]: name / sequence / quality start
// (within the read's text); name_len, seq_len, read_block as sa_stage writes them.
__global__ __launch_bounds__(256) void k_parse_reads(const ParseBlock* __restrict__ blocks, uint32_t nblocks,
                                                     const ParseText* __restrict__ texts, const uint32_t* __restrict__ nl,
                                                     uint32_t nreads, uint32_t* __restrict__ src,
                                                     uint16_t* __restrict__ name_len, uint32_t* __restrict__ seq_len,
                                                     uint32_t* __restrict__ read_block, uint32_t* __restrict__ err)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nreads) return;
    uint32_t lo = 0, hi = nblocks - 1;   // the block: last read0 <= g
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (blocks[mid].read0 <= g) lo = mid;
        else hi = mid - 1;
    }
    const ParseBlock B = blocks[lo];
    const uint32_t r = g - B.read0;
    const uint32_t rec = B.pe ? r >> 1 : r;
    const ParseText tx = texts[B.pe && (r & 1) ? B.text2 : B.text1];
    const uint32_t* L = nl + tx.nl_base + 4ull * rec;   // this record's four newlines
    const uint64_t start = rec == 0 ? 1ull : (uint64_t)L[-1] + 2;
    const uint64_t ln = (uint64_t)L[0] - start;          // (wraps when the header is empty: > 0xffff)
    const uint32_t s0 = L[0] + 1;
    const uint32_t ls = L[1] - s0;
    const uint32_t q0 = L[2] + 1;
    uint32_t e = 0;
    if (ln > 0xffff) e |= PARSE_ERR_NAME;
    if (B.pe) {
        if (L[3] - q0 != ls) e |= PARSE_ERR_QLEN;       // getBlockReadPE: the quality line's own length
    } else if ((uint64_t)q0 + ls > tx.len) {
        e |= PARSE_ERR_QUAL;                            // getBlockRead copies seqlen bytes from the line start
    }
    if (ls > 0xffff) e |= PARSE_ERR_LONG;                // (not an error: the block's long-read flag)
    if (e & ~PARSE_ERR_LONG) atomicOr(err, e & ~PARSE_ERR_LONG);
    src[3ull * g + 0] = (uint32_t)start;
    src[3ull * g + 1] = s0;
    src[3ull * g + 2] = q0;
    name_len[g] = (uint16_t)ln;
    seq_len[g] = ls;
    read_block[g] = lo;
}

// One workgroup per block: exclusive scans of the name and sequence lengths
// (offsets inside the block) and the block's totals.
__global__ __launch_bounds__(256) void k_block_scan(const ParseBlock* __restrict__ blocks,
                                                    const uint16_t* __restrict__ name_len,
                                                    const uint32_t* __restrict__ seq_len, uint32_t* __restrict__ name_off,
                                                    uint32_t* __restrict__ seq_off, BlockTotals* __restrict__ tot)
{
    __shared__ uint32_t sa[4], sb[4];
    __shared__ uint32_t any_long;
    const ParseBlock B = blocks[blockIdx.x];
    if (threadIdx.x == 0) any_long = 0;
    __syncthreads();
    uint64_t cn = 0, cs = 0;
    uint32_t lng = 0;
    for (uint32_t b = 0; b < B.nreads; b += 256) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t g = B.read0 + i;
        const uint32_t vn = i < B.nreads ? name_len[g] : 0u;
        const uint32_t vs = i < B.nreads ? seq_len[g] : 0u;
        lng |= vs > 0xffff;
        uint32_t en, es;
        wg256_excl_scan(vn, en, sa);
        wg256_excl_scan(vs, es, sb);
        if (i < B.nreads) {
            name_off[g] = (uint32_t)cn + en;
            seq_off[g] = (uint32_t)cs + es;
        }
        __syncthreads();
        cn += (uint64_t)sa[0] + sa[1] + sa[2] + sa[3];
        cs += (uint64_t)sb[0] + sb[1] + sb[2] + sb[3];
        __syncthreads();
    }
    if (lng) atomicOr(&any_long, 1u);
    __syncthreads();
    if (threadIdx.x == 0) tot[blockIdx.x] = BlockTotals{cn, cs, any_long, 0};
}

// One wave per read (grid-stride): the three fields, lane k copying bytes k,
// k + 64, ... (the text offsets are arbitrary, so bytes, not words)
__global__ __launch_bounds__(256) void k_copy_reads(const ParseBlock* __restrict__ blocks,
                                                    const ParseText* __restrict__ texts, const uint8_t* __restrict__ text,
                                                    uint32_t nreads, const uint32_t* __restrict__ src,
                                                    const uint16_t* __restrict__ name_len, const uint32_t* __restrict__ seq_len,
                                                    const uint32_t* __restrict__ read_block,
                                                    const uint32_t* __restrict__ name_off,
                                                    const uint32_t* __restrict__ seq_off, uint8_t* __restrict__ names,
                                                    uint8_t* __restrict__ seq, uint8_t* __restrict__ qual)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t g = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < nreads; g += nw) {
        const ParseBlock B = blocks[read_block[g]];
        const uint32_t r = g - B.read0;
        const ParseText tx = texts[B.pe && (r & 1) ? B.text2 : B.text1];
        const uint8_t* t = text + tx.off;
        const uint32_t ln = name_len[g], ls = seq_len[g];
        const uint32_t sn = src[3ull * g], ss = src[3ull * g + 1], sq = src[3ull * g + 2];
        uint8_t* dn = names + B.name_base + name_off[g];
        uint8_t* ds = seq + B.seq_base + seq_off[g];
        uint8_t* dq = qual + B.seq_base + seq_off[g];
        for (uint32_t k = lane; k < ln; k += 64) dn[k] = t[sn + k];
        for (uint32_t k = lane; k < ls; k += 64) {
            ds[k] = t[ss + k];
            dq[k] = t[sq + k];
        }
    }
}

}  // namespace

extern "C" {

// Page-locked host memory: 2 MiB-aligned, transparent huge pages asked for,
// then registered with the runtime (portable: any device's contexts may stage
// from it, --devices N).  Against hipHostMalloc, pinning 8 GB took 0.61 s
// instead of 1.38 s and the process exit released it in 0.54 s instead of
// 1.27 s (scripts/micro/exit_probe.hip, round 3 g4i); the DMA from it ran at
// the same rate (35 vs 31 GB/s H2D, g3y).
// (A/B knobs, round 5: SA_HOST_THP=0 leaves out the huge-page hint;
// SA_HOST_MALLOC=1 takes hipHostMalloc memory instead of registered memory)
// Round 5: the pages are faulted in first, by up to eight threads, and then
// registered -- hipHostRegister faults an untouched range in itself, one
// thread, at ~23 GB/s; 8 GB of touched huge pages took 0.066 s to touch and
// 0.016 s to register (scripts/micro/pin_probe.hip, r5k; with 4 KiB pages
// touching first saves nothing).  SA_HOST_TOUCH=0: the runtime faults them.
namespace {
bool host_touch()
{
    static const bool t = !(std::getenv("SA_HOST_TOUCH") && std::atoi(std::getenv("SA_HOST_TOUCH")) == 0);
    return t;
}
void touch_pages(void* p, uint64_t n)
{
    const uint64_t nt = std::min<uint64_t>(8, std::max<uint64_t>(1, n >> 27));   // (a thread per 128 MiB, up to 8)
    const uint64_t per = ((n / nt) + 4095) & ~4095ull;
    std::vector<std::thread> th;
    for (uint64_t t = 0; t < nt; t++)
        th.emplace_back([=]() {
            volatile uint8_t* b = static_cast<volatile uint8_t*>(p);
            for (uint64_t o = t * per; o < std::min(n, (t + 1) * per); o += 4096) b[o] = 0;
        });
    for (auto& x : th) x.join();
}
int host_mode()   // 0: register + THP hint, 1: register only, 2: hipHostMalloc
{
    static const int m = std::getenv("SA_HOST_MALLOC") && std::atoi(std::getenv("SA_HOST_MALLOC")) != 0 ? 2
                         : std::getenv("SA_HOST_THP") && std::atoi(std::getenv("SA_HOST_THP")) == 0 ? 1
                                                                                                     : 0;
    return m;
}
}  // namespace

void* sa_host_alloc(uint64_t bytes)
{
    constexpr uint64_t kHuge = 2ull << 20;
    const uint64_t n = ((bytes ? bytes : 1) + kHuge - 1) & ~(kHuge - 1);
    void* p = nullptr;
    if (host_mode() == 2) return hipHostMalloc(&p, n, hipHostMallocPortable) == hipSuccess ? p : nullptr;
    if (posix_memalign(&p, kHuge, n) != 0) return nullptr;
    if (host_mode() == 0) {
        (void)madvise(p, n, MADV_HUGEPAGE);   // (a hint: without THP the pages are 4 KiB)
        if (host_touch()) touch_pages(p, n);
    }
    if (hipHostRegister(p, n, hipHostRegisterPortable) != hipSuccess) {
        free(p);
        return nullptr;
    }
    return p;
}

void sa_host_free(void* p)
{
    if (!p) return;
    if (host_mode() == 2) {
        (void)hipHostFree(p);
        return;
    }
    (void)hipHostUnregister(p);
    free(p);
}

}  // extern "C"

namespace {

// Stages the texts into input I with context c's stream and mailbox
// (sa_stage_text: c's own input; sa_stage_text_input: any input of the device).
// stride = 0: the texts are copied here, packed (a text starts on a tile);
// stride > 0 (sa_text_parse): they are already in I's text arena `slot`, the
// file-1 text of block b at 2b x stride and its file-2 text at (2b + 1) x
// stride (sa_text_upload), and `in` gives only their lengths.
int stage_text(sa_ctx* c, sa_input* I, const sa_text_block* in, int n, sa_text_info* info, uint64_t stride = 0,
               int slot = 0)
{
    const ReserveScope reserve(c ? c->reserve_blocks : 0, n > 0 ? (uint32_t)n : 0);
    if (!c) return -1;
    if (n < 0 || (n > 0 && !in)) {
        c->err = "sa_stage_text: invalid block list";
        return -1;
    }
    if (!I || I->device != c->device) {
        c->err = "sa_stage_text_input: no input, or an input of another device";
        return -1;
    }
    SA_CHECK(c, hipSetDevice(c->device));
    hipStream_t st = c->st;
    if (mail_reset(c)) return -1;
    // (the input is empty until the whole batch is staged: a failed staging
    // leaves nothing for sa_run to encode)
    I->nblocks = 0;
    I->blocks.clear();
    I->nreads = 0;
    I->names_bytes = I->seq_bytes = I->text_bytes = 0;
    if (n == 0) return 0;
    std::vector<DevBlock> dblocks((size_t)n, DevBlock{});

    // ---- text layout: every text starts on a tile ----
    std::vector<ParseText> texts;
    std::vector<ParseBlock> pb((size_t)n);
    std::vector<uint32_t> ntiles;
    uint64_t off = 0;
    uint32_t tiles = 0;
    auto add_text = [&](uint64_t len, uint64_t at) -> int64_t {
        if (len >= (1ull << 32) || (stride && len > stride)) return -1;
        ParseText t{stride ? at : off, 0, (uint32_t)len, tiles};
        const uint32_t nt = (uint32_t)((len + PARSE_TILE - 1) / PARSE_TILE);
        texts.push_back(t);
        ntiles.push_back(nt);
        off += (uint64_t)nt * PARSE_TILE;
        tiles += nt;
        return (int64_t)texts.size() - 1;
    };
    for (int b = 0; b < n; b++) {
        const bool pe = in[b].text2 != nullptr;
        if (!stride && ((!in[b].text1 && in[b].len1) || (pe && !in[b].text2 && in[b].len2))) {
            c->err = "sa_stage_text: missing text";
            return -1;
        }
        const int64_t t1 = add_text(in[b].len1, 2ull * b * stride),
                      t2 = pe ? add_text(in[b].len2, (2ull * b + 1) * stride) : t1;
        if (t1 < 0 || t2 < 0) {
            c->err = stride ? "sa_text_parse: a text longer than the stride" : "sa_stage_text: text of 4 GiB or more";
            return -1;
        }
        pb[(size_t)b] = ParseBlock{(uint32_t)t1, (uint32_t)t2, 0, 0, 0, 0, pe ? 1u : 0u, 0};
    }
    const uint32_t ntext = (uint32_t)texts.size();
    std::vector<uint32_t> tile_text(tiles);
    for (uint32_t t = 0; t < ntext; t++)
        for (uint32_t k = 0; k < ntiles[t]; k++) tile_text[texts[t].tile0 + k] = t;

    DBuf& arena = slot ? I->d_text_b : I->d_text;
    if (!stride) SA_CHECK(c, arena.ensure(std::max<uint64_t>(off, 16)));
    else if (arena.cap < 2ull * n * stride) {
        c->err = "sa_text_parse: the text arena holds fewer blocks (sa_text_upload's nmax)";
        return -1;
    }
    uint8_t* const dtext = arena.as<uint8_t>();
    SA_CHECK(c, I->d_tile_text.ensure((size_t)tiles * 4));
    SA_CHECK(c, I->d_tile_cnt.ensure((size_t)tiles * 4));
    SA_CHECK(c, I->d_tile_base.ensure((size_t)tiles * 4));
    SA_CHECK(c, I->d_ptexts.ensure(sizeof(ParseText) * ntext));
    SA_CHECK(c, I->d_ntiles.ensure((size_t)ntext * 4));
    SA_CHECK(c, I->d_text_nl.ensure((size_t)ntext * 4));
    SA_CHECK(c, I->d_pblocks.ensure(sizeof(ParseBlock) * (size_t)n));
    SA_CHECK(c, I->d_btot.ensure(sizeof(BlockTotals) * (size_t)n));
    SA_CHECK(c, I->d_perr.ensure(4));
    for (int b = 0; b < n && !stride; b++) {   // the texts (a DMA when the host buffer is pinned)
        const ParseBlock& p = pb[(size_t)b];
        if (in[b].len1)
            SA_CHECK(c, hipMemcpyAsync(dtext + texts[p.text1].off, in[b].text1, in[b].len1, hipMemcpyHostToDevice, st));
        if (p.pe && in[b].len2)
            SA_CHECK(c, hipMemcpyAsync(dtext + texts[p.text2].off, in[b].text2, in[b].len2, hipMemcpyHostToDevice, st));
    }
    SA_CHECK(c, h2d(c, I->d_tile_text.p, tile_text.data(), (size_t)tiles * 4, st));
    SA_CHECK(c, h2d(c, I->d_ptexts.p, texts.data(), sizeof(ParseText) * ntext, st));
    SA_CHECK(c, h2d(c, I->d_ntiles.p, ntiles.data(), (size_t)ntext * 4, st));
    SA_CHECK(c, hipMemsetAsync(I->d_perr.p, 0, 4, st));
    if (tiles) {
        hipLaunchKernelGGL(k_nl_count, dim3(tiles), dim3(256), 0, st, dtext,
                           I->d_tile_text.as<uint32_t>(), I->d_ptexts.as<ParseText>(), I->d_tile_cnt.as<uint32_t>());
        SA_CHECK(c, hipGetLastError());
    }
    hipLaunchKernelGGL(k_text_scan, dim3(ntext), dim3(256), 0, st, I->d_ptexts.as<ParseText>(),
                       I->d_ntiles.as<uint32_t>(), I->d_tile_cnt.as<uint32_t>(), I->d_tile_base.as<uint32_t>(),
                       I->d_text_nl.as<uint32_t>());
    SA_CHECK(c, hipGetLastError());
    std::vector<uint32_t> text_nl(ntext);
    SA_CHECK(c, d2h(c, text_nl.data(), I->d_text_nl.p, (size_t)ntext * 4, st));
    SA_CHECK(c, sync_d2h(c, st));

    // ---- records per block (the host parsers' line accounting) ----
    uint64_t nlb = 0;
    for (uint32_t t = 0; t < ntext; t++) {
        texts[t].nl_base = nlb;
        nlb += text_nl[t];
    }
    uint64_t nr = 0;
    for (int b = 0; b < n; b++) {
        ParseBlock& p = pb[(size_t)b];
        uint64_t reads;
        if (p.pe) {
            const uint64_t k = std::min(text_nl[p.text1], text_nl[p.text2]);
            if (k % 4) {
                c->err = "sa_stage_text: PE block of incomplete records (getBlockReadPE)";
                return -1;
            }
            reads = k / 2;
        } else {
            if (text_nl[p.text1] % 4) {
                c->err = "sa_stage_text: SE block of incomplete records (getBlockRead)";
                return -1;
            }
            reads = text_nl[p.text1] / 4;
        }
        p.read0 = (uint32_t)nr;
        p.nreads = (uint32_t)reads;
        nr += reads;
        if (nr >= (1ull << 31)) {
            c->err = "too many reads in one batch";
            return -1;
        }
    }
    const uint32_t nreads = (uint32_t)nr;
    SA_CHECK(c, I->d_nl.ensure(std::max<uint64_t>(nlb, 1) * 4));
    const size_t nr4 = (size_t)std::max<uint32_t>(nreads, 1) * 4;
    SA_CHECK(c, I->d_src.ensure(nr4 * 3));
    SA_CHECK(c, I->d_read_block.ensure(nr4));
    SA_CHECK(c, I->d_name_off.ensure(nr4));
    SA_CHECK(c, I->d_name_len.ensure(nr4));
    SA_CHECK(c, I->d_seq_off.ensure(nr4));
    SA_CHECK(c, I->d_seq_len.ensure(nr4));
    SA_CHECK(c, h2d(c, I->d_ptexts.p, texts.data(), sizeof(ParseText) * ntext, st));
    SA_CHECK(c, h2d(c, I->d_pblocks.p, pb.data(), sizeof(ParseBlock) * (size_t)n, st));
    if (tiles) {
        hipLaunchKernelGGL(k_nl_emit, dim3(tiles), dim3(256), 0, st, dtext,
                           I->d_tile_text.as<uint32_t>(), I->d_ptexts.as<ParseText>(), I->d_tile_base.as<uint32_t>(),
                           I->d_nl.as<uint32_t>());
        SA_CHECK(c, hipGetLastError());
    }
    if (nreads) {
        hipLaunchKernelGGL(k_parse_reads, dim3((nreads + 255) / 256), dim3(256), 0, st, I->d_pblocks.as<ParseBlock>(),
                           (uint32_t)n, I->d_ptexts.as<ParseText>(), I->d_nl.as<uint32_t>(), nreads,
                           I->d_src.as<uint32_t>(), I->d_name_len.as<uint16_t>(), I->d_seq_len.as<uint32_t>(),
                           I->d_read_block.as<uint32_t>(), I->d_perr.as<uint32_t>());
        SA_CHECK(c, hipGetLastError());
    }
    hipLaunchKernelGGL(k_block_scan, dim3((uint32_t)n), dim3(256), 0, st, I->d_pblocks.as<ParseBlock>(),
                       I->d_name_len.as<uint16_t>(), I->d_seq_len.as<uint32_t>(), I->d_name_off.as<uint32_t>(),
                       I->d_seq_off.as<uint32_t>(), I->d_btot.as<BlockTotals>());
    SA_CHECK(c, hipGetLastError());
    std::vector<BlockTotals> tot((size_t)n);
    uint32_t perr = 0;
    SA_CHECK(c, d2h(c, tot.data(), I->d_btot.p, sizeof(BlockTotals) * (size_t)n, st));
    SA_CHECK(c, d2h(c, &perr, I->d_perr.p, 4, st));
    SA_CHECK(c, sync_d2h(c, st));
    if (perr) {
        c->err = std::string("sa_stage_text: malformed FASTQ (") +
                 (perr & PARSE_ERR_NAME ? "ID longer than 65535 bytes" :
                  perr & PARSE_ERR_QLEN ? "quality and sequence lengths differ" : "quality past the end of the block") +
                 ")";
        return -1;
    }

    // ---- layout of the SoA (as input_upload) and the copy ----
    uint64_t nb = 0, sb = 0, tb = 0;
    for (int b = 0; b < n; b++) {
        ParseBlock& p = pb[(size_t)b];
        const BlockTotals& t = tot[(size_t)b];
        if (t.seq_bytes >= (1ull << 30) || t.name_bytes >= (1ull << 32)) {
            c->err = "block too large (a reference block is 50 MiB of FASTQ)";
            return -1;
        }
        DevBlock& d = dblocks[(size_t)b];
        d.nreads = p.nreads;
        d.read0 = p.read0;
        d.name_base = nb;
        d.seq_base = sb;
        d.name_bytes = t.name_bytes;
        d.seq_bytes = t.seq_bytes;
        d.len_long = t.len_long;
        p.name_base = nb;
        p.seq_base = sb;
        nb = align_up(nb + t.name_bytes, 16);
        sb = align_up(sb + t.seq_bytes, 16);
        tb += t.name_bytes + 2 * t.seq_bytes;
        if (info) {
            info[b].nreads = p.nreads;
            info[b].len_long = t.len_long;
            info[b].name_bytes = t.name_bytes;
            info[b].seq_bytes = t.seq_bytes;
            // sa_output_bound of the parsed block
            const uint64_t syms = 3 * t.seq_bytes + t.name_bytes + 45ull * p.nreads;
            info[b].out_bound = 2 * syms + 9 * 96 + 4096 + 0x10000;
        }
    }
    I->nreads = nreads;
    I->names_bytes = nb;
    I->seq_bytes = sb;
    I->text_bytes = tb;
    SA_CHECK(c, I->d_names.ensure(nb + 64));   // (k_prep_sq16 reads whole dwords past a name)
    SA_CHECK(c, I->d_seq.ensure(sb + 64));
    SA_CHECK(c, I->d_qual.ensure(sb + 64));
    SA_CHECK(c, h2d(c, I->d_pblocks.p, pb.data(), sizeof(ParseBlock) * (size_t)n, st));
    if (nreads) {
        hipLaunchKernelGGL(k_copy_reads, dim3(wave_grid(c, nreads)), dim3(256), 0, st, I->d_pblocks.as<ParseBlock>(),
                           I->d_ptexts.as<ParseText>(), dtext, nreads, I->d_src.as<uint32_t>(),
                           I->d_name_len.as<uint16_t>(), I->d_seq_len.as<uint32_t>(), I->d_read_block.as<uint32_t>(),
                           I->d_name_off.as<uint32_t>(), I->d_seq_off.as<uint32_t>(), I->d_names.as<uint8_t>(),
                           I->d_seq.as<uint8_t>(), I->d_qual.as<uint8_t>());
        SA_CHECK(c, hipGetLastError());
    }
    // (sa_run's kernels follow on this stream; the texts on the host are free
    // once this returns)
    SA_CHECK(c, hipStreamSynchronize(st));
    I->blocks = std::move(dblocks);
    I->nblocks = (uint32_t)n;
    return 0;
}

}  // namespace

extern "C" {

int sa_stage_text(sa_ctx* c, const sa_text_block* in, int n, sa_text_info* info)
{
    if (!c) return -1;
    c->have_output = false;
    return stage_text(c, &c->own, in, n, info);
}

sa_input* sa_input_empty(int device)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    sa_input* I = new sa_input();
    I->device = device;
    return I;
}

int sa_stage_text_input(sa_ctx* c, sa_input* I, const sa_text_block* in, int n, sa_text_info* info)
{
    return stage_text(c, I, in, n, info);
}

// (round 6) the streaming form of sa_stage_text: one block's texts to the
// device as the reader cuts it (the host text may be reused on return), into
// text arena `slot` of the input at the fixed stride, on the context's copy
// stream -- a thread of its own may call this while the context encodes from
// its other arena.  Then sa_text_parse.
int sa_text_upload(sa_ctx* c, sa_input* I, int slot, int index, int nmax, const sa_text_block* blk, uint64_t stride)
{
    if (!c) return -1;
    if (!I) I = &c->own;
    stride = (stride + PARSE_TILE - 1) / PARSE_TILE * PARSE_TILE;
    const bool pe = blk && blk->text2 != nullptr;
    if (!blk || slot < 0 || slot > 1 || index < 0 || index >= nmax || !stride || blk->len1 > stride ||
        (pe && blk->len2 > stride) || (!blk->text1 && blk->len1) || I->device != c->device) {
        c->err = "sa_text_upload: invalid block, slot, index or stride";
        return -1;
    }
    std::lock_guard<std::mutex> g(c->copy_mu);   // (one uploader per context at a time)
    SA_CHECK(c, hipSetDevice(c->device));
    if (!c->st_copy) SA_CHECK(c, hipStreamCreateWithFlags(&c->st_copy, hipStreamNonBlocking));
    DBuf& arena = slot ? I->d_text_b : I->d_text;
    // (the whole batch's arena at its first block: a later growth would move
    // the blocks already there)
    if (index == 0 && arena.cap < 2ull * (uint64_t)nmax * stride) SA_CHECK(c, arena.ensure(2ull * (uint64_t)nmax * stride));
    if (arena.cap < 2ull * (uint64_t)(index + 1) * stride) {
        c->err = "sa_text_upload: block 0 of the batch was not uploaded first";
        return -1;
    }
    uint8_t* d = arena.as<uint8_t>() + 2ull * (uint64_t)index * stride;
    if (blk->len1) SA_CHECK(c, hipMemcpyAsync(d, blk->text1, blk->len1, hipMemcpyHostToDevice, c->st_copy));
    if (pe && blk->len2) SA_CHECK(c, hipMemcpyAsync(d + stride, blk->text2, blk->len2, hipMemcpyHostToDevice, c->st_copy));
    SA_CHECK(c, hipStreamSynchronize(c->st_copy));
    return 0;
}

// parses the n blocks sa_text_upload put into text arena `slot` (lens: their
// text lengths; text1 / text2 only tell SE from PE) into the input, as
// sa_stage_text would have
int sa_text_parse(sa_ctx* c, sa_input* I, int slot, const sa_text_block* lens, int n, uint64_t stride,
                  sa_text_info* info)
{
    if (!c) return -1;
    if (!I) {
        I = &c->own;
        c->have_output = false;
    }
    if (slot < 0 || slot > 1 || !stride) {
        c->err = "sa_text_parse: invalid slot or stride";
        return -1;
    }
    return stage_text(c, I, lens, n, info, (stride + PARSE_TILE - 1) / PARSE_TILE * PARSE_TILE, slot);
}

}  // extern "C"
