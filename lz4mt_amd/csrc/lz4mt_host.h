// lz4mt_host.h — host-side helpers of the product library: XXH32 (the
// serial stream checksum and the header check byte), little-endian I/O and
// the frame-header codec (reference src/lz4mt.cpp:69-161, 335-369, 541-590).
#pragma once

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/lz4mt.h"

namespace lz4mt {

constexpr uint32_t kMagic = 0x184D2204u;
constexpr uint32_t kSkippableMin = 0x184D2A50u;
constexpr uint32_t kSkippableMax = 0x184D2A5Fu;
constexpr uint32_t kRawBit = 0x80000000u;
constexpr int kMaxHeader = 4 + 2 + 8 + 4 + 1;

inline uint32_t get32(const void* p) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}
inline void put32(void* p, uint32_t v) {
    uint8_t* b = static_cast<uint8_t*>(p);
    b[0] = (uint8_t)v; b[1] = (uint8_t)(v >> 8); b[2] = (uint8_t)(v >> 16); b[3] = (uint8_t)(v >> 24);
}

// Streaming XXH32, seed 0 in every lz4mt use (reference src/lz4mt.cpp:23).
class HostXxh32 {
public:
    explicit HostXxh32(uint32_t seed = 0) { reset(seed); }
    void reset(uint32_t seed) {
        seed_ = seed; total_ = 0; fill_ = 0;
        v_[0] = seed + P1 + P2; v_[1] = seed + P2; v_[2] = seed; v_[3] = seed - P1;
    }
    void update(const void* in, size_t len) {
        const uint8_t* p = static_cast<const uint8_t*>(in);
        total_ += len;
        if (fill_) {
            const size_t take = (16 - fill_) < len ? (16 - fill_) : len;
            memcpy(buf_ + fill_, p, take);
            fill_ += (uint32_t)take; p += take; len -= take;
            if (fill_ < 16) return;
            stripe(buf_);
            fill_ = 0;
        }
        // bulk: the four lanes in locals (stores to v_ through `this` would
        // alias the byte pointer and pin them to memory every stripe)
        uint32_t a = v_[0], b = v_[1], c = v_[2], d = v_[3];
        for (; len >= 16; p += 16, len -= 16) {
            a = rotl(a + get32(p) * P2, 13) * P1;
            b = rotl(b + get32(p + 4) * P2, 13) * P1;
            c = rotl(c + get32(p + 8) * P2, 13) * P1;
            d = rotl(d + get32(p + 12) * P2, 13) * P1;
        }
        v_[0] = a; v_[1] = b; v_[2] = c; v_[3] = d;
        memcpy(buf_, p, len);
        fill_ = (uint32_t)len;
    }
    uint32_t digest() const {
        uint32_t h = total_ >= 16 ? rotl(v_[0], 1) + rotl(v_[1], 7) + rotl(v_[2], 12) + rotl(v_[3], 18)
                                  : seed_ + P5;
        h += (uint32_t)total_;
        const uint8_t* p = buf_;
        size_t n = fill_;
        for (; n >= 4; n -= 4, p += 4) h = rotl(h + get32(p) * P3, 17) * P4;
        for (; n > 0; --n, ++p) h = rotl(h + (*p) * P5, 11) * P1;
        h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
        return h;
    }
    static uint32_t oneshot(const void* p, size_t len, uint32_t seed = 0) {
        HostXxh32 x(seed);
        x.update(p, len);
        return x.digest();
    }

private:
    static constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                              P5 = 374761393u;
    static uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
    void stripe(const uint8_t* p) {
        for (int i = 0; i < 4; ++i) v_[i] = rotl(v_[i] + get32(p + 4 * i) * P2, 13) * P1;
    }
    uint32_t v_[4];
    uint32_t seed_;
    uint64_t total_;
    uint8_t buf_[16];
    uint32_t fill_;
};

inline int block_max_bytes(int id) { return 1 << (8 + 2 * id); }

// validateStreamDescriptor (reference src/lz4mt.cpp:139-161), same order.
inline Lz4MtResult validate_sd(const Lz4MtStreamDescriptor* sd) {
    if (sd->flg.versionNumber != 1) return LZ4MT_RESULT_INVALID_VERSION;
    if (sd->flg.presetDictionary != 0) return LZ4MT_RESULT_PRESET_DICTIONARY_IS_NOT_SUPPORTED_YET;
    if (sd->flg.reserved1 != 0) return LZ4MT_RESULT_INVALID_HEADER_RESERVED1;
    if (sd->bd.blockMaximumSize < 4 || sd->bd.blockMaximumSize > 7) return LZ4MT_RESULT_INVALID_BLOCK_MAXIMUM_SIZE;
    if (sd->bd.reserved3 != 0) return LZ4MT_RESULT_INVALID_HEADER_RESERVED3;
    if (sd->bd.reserved2 != 0) return LZ4MT_RESULT_INVALID_HEADER_RESERVED2;
    return LZ4MT_RESULT_OK;
}

inline uint8_t flg_byte(const Lz4MtFlg& f) {
    return (uint8_t)(((f.presetDictionary & 1) << 0) | ((f.reserved1 & 1) << 1) | ((f.streamChecksum & 1) << 2) |
                     ((f.streamSize & 1) << 3) | ((f.blockChecksum & 1) << 4) | ((f.blockIndependence & 1) << 5) |
                     ((f.versionNumber & 3) << 6));
}
inline uint8_t bd_byte(const Lz4MtBd& b) {
    return (uint8_t)(((b.reserved3 & 15) << 0) | ((b.blockMaximumSize & 7) << 4) | ((b.reserved2 & 1) << 7));
}
inline void parse_flg(uint8_t c, Lz4MtFlg* f) {
    f->presetDictionary = (char)(c & 1);
    f->reserved1 = (char)((c >> 1) & 1);
    f->streamChecksum = (char)((c >> 2) & 1);
    f->streamSize = (char)((c >> 3) & 1);
    f->blockChecksum = (char)((c >> 4) & 1);
    f->blockIndependence = (char)((c >> 5) & 1);
    f->versionNumber = (char)((c >> 6) & 3);
}
inline void parse_bd(uint8_t c, Lz4MtBd* b) {
    b->reserved3 = (char)(c & 15);
    b->blockMaximumSize = (char)((c >> 4) & 7);
    b->reserved2 = (char)((c >> 7) & 1);
}

// Writes the frame header (makeHeader, reference src/lz4mt.cpp:335-369).
// Returns the header length; `out` must hold kMaxHeader bytes.
inline int build_header(const Lz4MtStreamDescriptor* sd, uint8_t* out) {
    int o = 0;
    put32(out, kMagic);
    o = 4;
    out[o++] = flg_byte(sd->flg);
    out[o++] = bd_byte(sd->bd);
    if (sd->flg.streamSize) {
        put32(out + o, (uint32_t)sd->streamSize);
        put32(out + o + 4, (uint32_t)(sd->streamSize >> 32));
        o += 8;
    }
    if (sd->flg.presetDictionary) { put32(out + o, sd->dictId); o += 4; }
    out[o] = (uint8_t)((HostXxh32::oneshot(out + 4, (size_t)(o - 4)) >> 8) & 0xFF);
    return o + 1;
}

// Parses FLG/BD (+ optional fields + check byte) from `p` (the bytes after
// the magic, `avail` of them).  Returns OK and sets *hdrBodyLen to the
// bytes consumed after the magic, or the reference's error code
// (readHeader, src/lz4mt.cpp:541-590).
inline Lz4MtResult parse_header(const uint8_t* p, size_t avail, Lz4MtStreamDescriptor* sd, int* hdrBodyLen) {
    if (avail < 2) return LZ4MT_RESULT_INVALID_HEADER;
    parse_flg(p[0], &sd->flg);
    parse_bd(p[1], &sd->bd);
    const Lz4MtResult r = validate_sd(sd);
    if (r != LZ4MT_RESULT_OK) return r;
    const int nex = (sd->flg.streamSize ? 8 : 0) + (sd->flg.presetDictionary ? 4 : 0) + 1;
    if (avail < (size_t)(2 + nex)) return LZ4MT_RESULT_INVALID_HEADER;
    int o = 2;
    if (sd->flg.streamSize) {
        sd->streamSize = (uint64_t)get32(p + o) | ((uint64_t)get32(p + o + 4) << 32);
        o += 8;
    }
    if (sd->flg.presetDictionary) { sd->dictId = get32(p + o); o += 4; }
    const uint8_t hc = (uint8_t)((HostXxh32::oneshot(p, (size_t)o) >> 8) & 0xFF);
    if (hc != p[o]) return LZ4MT_RESULT_INVALID_HEADER_CHECKSUM;
    *hdrBodyLen = o + 1;
    return LZ4MT_RESULT_OK;
}

// Replays, block by block, the state that decides how the reference's
// block-dependent compressor (compressBlockDependency, src/lz4mt.cpp:460-538)
// calls LZ4 1.9.3's LZ4_compress_limitedOutput_continue: its input buffer of
// max(blockMax + 64 KiB, 1088 KiB) bytes, LZ4_slideInputBuffer when the next
// block would not fit (it returns the stream's dictionary pointer in 1.9.3),
// and the stream's dictionary bookkeeping in LZ4_compress_fast_continue
// (renormalisation, tiny-dictionary reset, overlap trimming, prefix vs
// external-dictionary mode, dictSmall).  For 1 and 4 MiB blocks the
// reference reads each block over its own dictionary (its frames then need
// not decode back); those sizes follow one contiguous buffer instead -- the
// same stream without that defect.
// next() returns the block's catch-up bounds and dictSmall limit in the
// coordinates of k_encode_linked (block at 65536, history below).
// refBuffer: replay the reference's input buffer for 1 and 4 MiB blocks too
// (LZ4MT_AMD_BD_REFERENCE=1).  There lz4 1.9.3's LZ4_slideInputBuffer hands
// back the dictionary's own address, so from the second block on each full
// block is read over its dictionary: its "history" is its own last 64 KiB
// (the table still indexes the previous block).  `shift` then says where a
// history byte lives: position p < 65536 (block coordinates) reads the
// block's byte p - 65536 + shift; 0 = the true history before the block.
// bad: a history that is partly the block and partly older bytes (no such
// case in the reference's loop; refused rather than guessed).
struct BdSim {
    uint64_t bm = 0, bufSize = 0;   // bufSize 0: one contiguous buffer
    uint64_t inStart = 0, dict = 0, dictSize = 0, cur = 0;
    bool dictNull = true, bad = false;
    explicit BdSim(int blockMaxId, bool refBuffer = false) {
        bm = (uint64_t)1 << (8 + 2 * blockMaxId);
        const uint64_t b = bm + 65536, m = (1024 + 64) * 1024;
        bufSize = (blockMaxId <= 5 || refBuffer) ? (b > m ? b : m) : 0;
    }
    void next(uint32_t n, uint32_t* lowIn, uint32_t* lowDict, uint32_t* candLow, uint32_t* shift = nullptr) {
        if (bufSize && inStart + bm > bufSize) inStart = dict;   // translate()
        uint64_t dictEnd = dict + dictSize;
        if (cur + n > 0x80000000ull) {                           // LZ4_renormDictT
            cur = 65536;
            if (dictSize > 65536) dictSize = 65536;
            dict = dictEnd - dictSize;
        }
        if ((uint32_t)(dictSize - 1) < 3u && (dictNull || dictEnd != inStart)) {   // invalidate tiny dictionaries
            dictSize = 0; dict = inStart; dictNull = false; dictEnd = inStart;
        }
        const uint64_t srcEnd = inStart + n;
        if (!dictNull && srcEnd > dict && srcEnd < dictEnd) {   // overlapping input / dictionary
            dictSize = dictEnd - srcEnd;
            if (dictSize > 65536) dictSize = 65536;
            if (dictSize < 4) dictSize = 0;
            dict = dictEnd - dictSize;
        }
        const bool prefix = !dictNull && dictEnd == inStart;
        const bool small = dictSize < 65536 && dictSize < cur;
        const uint32_t ds = (uint32_t)(dictSize < 65536 ? dictSize : 65536);
        *lowDict = 65536 - ds;
        *lowIn = prefix ? 65536 - ds : 65536;
        *candLow = small ? 65536 - ds : 0;
        if (shift) {   // where the ds history bytes [dictEnd - ds, dictEnd) of the buffer stand
            *shift = 0;
            const uint64_t h0 = dict + dictSize - ds, h1 = dict + dictSize;
            if (!prefix && ds && h0 >= inStart && h1 <= inStart + n) *shift = (uint32_t)(h1 - inStart);
            else if (!prefix && ds && h0 < inStart + n && h1 > inStart) bad = true;
        }
        cur += n;
        if (prefix) dictSize += n;
        else { dict = inStart; dictSize = n; dictNull = false; }
        inStart += n;
    }
};

// -BD at level >= 3 (the same loop over the HC stream, src/lz4mt.cpp:295-332):
// LZ4_slideInputBufferHC resets lz4 1.9.3's HC stream, and the next block
// starts a new segment at the front of the buffer; inside a segment every
// block continues the one before it (one prefix, every position inserted).
// next() returns the stream offset where the next block's segment starts.
struct HcBdSim {
    uint64_t bm = 0, bufSize = 0, inStart = 0, pos = 0, seg = 0;
    explicit HcBdSim(int blockMaxId) {
        bm = (uint64_t)1 << (8 + 2 * blockMaxId);
        const uint64_t b = bm + 65536, m = (1024 + 64) * 1024;
        bufSize = b > m ? b : m;
    }
    uint64_t next(uint32_t n) {
        if (inStart + bm > bufSize) { inStart = 0; seg = pos; }   // translate(): a fresh stream
        inStart += n;
        pos += n;
        return seg;
    }
};

// The segments of a batch of blocks for k_hc_prev_seg / k_encode_hc_bd:
// segAbs[b] = stream offset of block b's segment (HcBdSim), the batch
// starting at stream offset A with `hist` (<= 64 KiB) bytes of history
// before it, `total` input bytes.  Packs begin[nSeg], end[nSeg] (int64,
// relative to A; a begin before A - hist is clamped there: no match or chain
// link reaches more than 64 KiB back) and blockSeg[nb] (uint32) into `out`.
inline uint32_t hc_bd_pack(const uint64_t* segAbs, uint64_t nb, uint64_t A, uint64_t total, uint64_t hist,
                           std::vector<uint8_t>& out, uint64_t bm = 0, bool* perBlock = nullptr) {
    std::vector<int64_t> begin, end;
    std::vector<uint32_t> blockSeg(nb);
    for (uint64_t b = 0; b < nb; ++b) {
        if (b == 0 || segAbs[b] != segAbs[b - 1]) {
            const int64_t lo = (int64_t)segAbs[b] - (int64_t)A, floor = -(int64_t)hist;
            if (!begin.empty()) end.push_back(lo);
            begin.push_back(lo > floor ? lo : floor);
        }
        blockSeg[b] = (uint32_t)(begin.size() - 1);
    }
    end.push_back((int64_t)total);
    const uint32_t nSeg = (uint32_t)begin.size();
    if (perBlock) {   // segment k = block k: the blocks are independent level-9 parses (cap n - 1)
        bool pb = nSeg == nb;
        for (uint64_t k = 0; pb && k < nSeg; ++k) pb = begin[k] == (int64_t)(k * bm);
        *perBlock = pb;
    }
    out.resize(16 * (size_t)nSeg + 4 * nb);
    memcpy(out.data(), begin.data(), 8 * (size_t)nSeg);
    memcpy(out.data() + 8 * (size_t)nSeg, end.data(), 8 * (size_t)nSeg);
    memcpy(out.data() + 16 * (size_t)nSeg, blockSeg.data(), 4 * nb);
    return nSeg;
}

}  // namespace lz4mt
