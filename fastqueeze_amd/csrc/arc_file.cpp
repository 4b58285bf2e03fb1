// arc_file.cpp -- the .arc container around the encoded blocks (host C++).
//
// Restates SeqArcFile (SeqArc-1.6@0x415c20-0x419840) for the no-reference
// encode path, from static disassembly:
//   header   writeFileInfo@0x4171b0 (+0x253..0x2a7): ".arc" 01 06 00, setID(2),
//            8-byte VINT = bytes of the block region; 16 bytes at offset 0
//   blocks   from offset 16, in input order (the reference's -t 1 order)
//   trailer  writeFileInfo@0x4172b9..0x417373: setID(3) + size4 +
//            writeParam@0x416450 (ID 1, size2: fields 1-18) +
//            writeBlockLenArry{SE,PE}@0x416d60/0x416e90 (ID 7, size4, the raw
//            32-byte _tagBlockInfoSE / 40-byte _tagBlockInfoPE records)
// writeMd5@0x416b10 (reference-index MD5, ID 8, when param+0x3 is clear: the
// reference path) follows the params; writeModel (usemodel, param+0x8) and
// writeFileList (-m, param+0xd) are not written.
#include <stdint.h>
#include <string.h>

#include <string>

#include "../../include/seqarc_amd.h"

namespace {

// Encap::setID@0x420720: smallest n with v <= 2^(7n) - 2, v | 2^(7n) big-endian.
int put_id(uint64_t v, uint8_t* o)
{
    int n = 1;
    while (n < 8 && v > (1ull << (7 * n)) - 2) n++;
    const uint64_t x = v | (1ull << (7 * n));
    for (int i = 0; i < n; i++) o[i] = (uint8_t)(x >> (8 * (n - 1 - i)));
    return n;
}

// Encap::setSize@0x420780: fixed width n, v | 2^(7n) big-endian.
void put_size(uint64_t v, int n, uint8_t* o)
{
    const uint64_t x = v | (1ull << (7 * n));
    for (int i = 0; i < n; i++) o[i] = (uint8_t)(x >> (8 * (n - 1 - i)));
}

void put_le(uint64_t v, int n, uint8_t* o)
{
    for (int i = 0; i < n; i++) o[i] = (uint8_t)(v >> (8 * i));
}

struct Out {
    uint8_t* p;
    uint8_t* end;
    bool ok = true;
    uint8_t* take(size_t n)
    {
        if (!ok || (size_t)(end - p) < n) { ok = false; return nullptr; }
        uint8_t* r = p;
        p += n;
        return r;
    }
};

// SeqArcFile::compressBool@0x415f50: setID(id), size 1 (1 byte), the byte.
void field_bool(Out& o, uint32_t id, int v)
{
    uint8_t t[16];
    int n = put_id(id, t);
    put_size(1, 1, t + n);
    t[n + 1] = (uint8_t)(v ? 1 : 0);
    if (uint8_t* d = o.take((size_t)n + 2)) memcpy(d, t, (size_t)n + 2);
}

// compressUInt@0x415fb0: setID(id), 1-byte size = width, width bytes LE.
void field_uint(Out& o, uint32_t id, int width, uint32_t v)
{
    uint8_t t[16];
    int n = put_id(id, t);
    put_size((uint64_t)width, 1, t + n);
    put_le(v, width, t + n + 1);
    if (uint8_t* d = o.take((size_t)n + 1 + (size_t)width)) memcpy(d, t, (size_t)n + 1 + (size_t)width);
}

// compressStr@0x4160f0: nothing for an empty string; else the basename (after
// the last '/'), cut at the last ".gz" (rfind, .rodata 0x44a820), as
// setID(id) + 1-byte size + bytes.
void field_str(Out& o, uint32_t id, const char* path)
{
    if (!path || !*path) return;
    std::string s(path);
    const size_t sl = s.rfind('/');
    if (sl != std::string::npos) s = s.substr(sl + 1);
    const size_t gz = s.rfind(".gz");
    if (gz != std::string::npos) s = s.substr(0, gz);
    uint8_t t[16];
    int n = put_id(id, t);
    put_size(s.size(), 1, t + n);
    if (uint8_t* d = o.take((size_t)n + 1 + s.size())) {
        memcpy(d, t, (size_t)n + 1);
        memcpy(d + n + 1, s.data(), s.size());
    }
}

}  // namespace

extern "C" {

int sa_arc_header(uint64_t block_bytes, uint8_t out[16])
{
    memset(out, 0, 16);
    out[0] = '.'; out[1] = 'a'; out[2] = 'r'; out[3] = 'c';
    out[4] = 1;   // version 1.6 (param+0x10 / +0x14 defaults)
    out[5] = 6;
    const int n = put_id(2, out + 7);
    put_size(block_bytes, 8, out + 7 + n);   // assert headlen == ARCHEADLEN (16)
    return 7 + n + 8 == 16 ? 0 : -1;
}

int64_t sa_arc_trailer2(const sa_arc_info* in, int32_t maxmis, const sa_arc_block* blk, uint32_t n, uint8_t* out,
                        uint64_t cap)
{
    if (!in || (!blk && n) || !out) return -1;
    Out o{out, out + cap};
    uint8_t* top = o.take(1 + 4);   // setID(3) is one byte
    if (!top) return -1;
    put_id(3, top);
    // ---- writeParam@0x416450: ID 1, 2-byte size ----
    uint8_t* ph = o.take(1 + 2);
    if (!ph) return -1;
    put_id(1, ph);
    uint8_t* pbeg = o.p;
    field_bool(o, 1, in->ref_md5 ? 0 : 1);      // param+0x3: no reference index
    field_bool(o, 2, in->bare_plus);            // param+0x4: '+' lines carry no ID (getFirstLine@0x431eb0)
    field_bool(o, 3, in->paired ? 0 : 1);       // param+0x5: single-end (set by -1, cleared by -2: parseOptFromCmd@0x40b460)
    field_bool(o, 4, in->gz1);                  // param+0x6: getFileType@0x40d9f0 of input 1
    field_bool(o, 5, 1);                        // param+0x7 (cleared by -q)
    field_bool(o, 6, 0);                        // param+0x8: usemodel
    field_bool(o, 7, 0);                        // param+0xc
    field_uint(o, 8, 2, 1);                     // param+0x10 (1)
    field_uint(o, 9, 2, 6);                     // param+0x14 (6)
    field_uint(o, 10, 2, in->insert_size);      // param+0x28 (-I)
    field_uint(o, 11, 4, n);                    // param+0x20: block count
    field_uint(o, 12, 4, 0);                    // param+0x24
    field_str(o, 13, in->file1);                // param+0x430
    field_str(o, 14, in->paired ? in->file2 : nullptr);   // param+0x830
    {                                           // compressIDBin@0x4163b0: 512-byte template
        uint8_t* d = o.take(1 + 2 + 512);
        if (d) {
            put_id(15, d);
            put_size(0x200, 2, d + 1);
            if (in->id_template) memcpy(d + 3, in->id_template, 512);
            else memset(d + 3, 0, 512);
        }
    }
    field_bool(o, 16, in->lossy);               // param+0x1870
    field_bool(o, 17, in->md5);                 // param+0x1880
    field_bool(o, 18, 0);                       // param+0xd: file list (-m)
    if (in->ref_md5 && maxmis != 7)             // (ours: a non-default maxmis, see sa_arc_trailer2)
        field_uint(o, 19, 1, (uint32_t)maxmis);
    if (!o.ok) return -1;
    put_size((uint64_t)(o.p - pbeg), 2, ph + 1);
    if (in->ref_md5) {   // writeMd5@0x416b10: setID(8), 1-byte size 0x10, the 16 bytes
        uint8_t* d = o.take(1 + 1 + 16);
        if (!d) return -1;
        put_id(8, d);
        put_size(16, 1, d + 1);
        memcpy(d + 2, in->ref_md5, 16);
    }
    // ---- writeBlockLenArry: ID 7, size4, raw block records ----
    const uint32_t rec = in->paired ? 40u : 32u;
    uint8_t* bh = o.take(1 + 4);
    if (!bh) return -1;
    put_id(7, bh);
    put_size((uint64_t)rec * n, 4, bh + 1);
    uint64_t off = 16, in1 = 0, in2 = 0;
    for (uint32_t b = 0; b < n; b++) {
        uint8_t* r = o.take(rec);
        if (!r) return -1;
        memset(r, 0, rec);
        // outPutData@0x412040: size << 1 | SeqArcMemBuf+0x2 (long-read flag)
        put_le(((uint64_t)blk[b].size << 1 | (blk[b].long_reads ? 1u : 0u)) & 0xffffffffu, 4, r);
        if (in->paired) {   // getdata@0x412da0 / addBlockPEInfo@0x412f30
            put_le(blk[b].text1, 4, r + 4);
            put_le(blk[b].text2, 4, r + 8);
            put_le(off, 8, r + 0x10);
            put_le(in1, 8, r + 0x18);
            put_le(in2, 8, r + 0x20);
        } else {            // getdata@0x411e60 / addBlockSEInfo@0x411f10
            put_le((0u << 1) | (in->bare_plus ? 1u : 0u), 4, r + 4);   // input file index 0
            put_le(blk[b].text1, 4, r + 8);
            put_le(off, 8, r + 0x10);
            put_le(in1, 8, r + 0x18);
        }
        off += blk[b].size;
        in1 += blk[b].text1;
        in2 += blk[b].text2;
    }
    put_size((uint64_t)(o.p - top - 5), 4, top + 1);
    return o.p - out;
}

int64_t sa_arc_trailer(const sa_arc_info* in, const sa_arc_block* blk, uint32_t n, uint8_t* out, uint64_t cap)
{
    return sa_arc_trailer2(in, 7, blk, n, out, cap);
}

}  // extern "C"
