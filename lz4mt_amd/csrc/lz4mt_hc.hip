// lz4mt_hc.hip — LZ4-HC (compression levels 3..12) for gfx950: the codec
// lz4mt selects for level >= 3, LZ4_compressHC2_limitedOutput(src, dst, n,
// cap = n, level) (reference src/main.cpp:778-785, src/lz4mt.cpp:391), i.e.
// lz4 1.9.3's LZ4_compress_HC -> LZ4HC_compress_hashChain.  Bit-exact with
// oracle/lz4hc_oracle.c (pinned against liblz4 1.9.3).
//
// Two kernels, one wavefront per block each:
//   k_hc_prev    the hash chain of the block: for every position p the
//                distance to the previous position with the same 4-byte hash
//                (u16; 0 = none within 64 KiB).  LZ4HC_Insert inserts every
//                position in order before each search, so the chain lz4hc
//                walks at a search is exactly this "previous same hash" list
//                (its chainTable delta, capped at 65535, and its hashTable
//                head).  The "last position per hash" table (32768 x u32)
//                sits in LDS; 64 positions per step, equal hashes inside a
//                step resolved by ballot.
//   k_encode_hc  the hashChain parse (InsertAndFindBestMatch, the Search2 /
//                Search3 lazy evaluation, pattern analysis at level 9) with
//                the parse state wave-uniform; the lanes run the data-parallel
//                parts: forward match count (64 x 4 bytes per round), the
//                backward count, byte-run lengths and the literal copies.
//                The chain walk is serial (one dependent delta load per
//                candidate, with the candidate's bytes in the same round).
#include "lz4mt_device.h"

#include <stdlib.h>

#include <stdio.h>

#include <algorithm>
#include <vector>

namespace lz4mt {

// Lanes of one wavefront hand data to each other through LDS.  LDS
// operations of a wave execute in order, so no wait is needed, but the
// COMPILER must neither move LDS accesses across this point nor forward a
// lane's own store to its later load (another lane may have overwritten the
// word): wave_barrier alone has no memory effect in LLVM, so the
// wavefront-scope fences (no instructions on gfx950) carry the ordering.
#define WAVE_SYNC()                                              \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
    } while (0)

typedef const __attribute__((address_space(1))) uint8_t g_cu8;
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef const __attribute__((address_space(1))) uint16_t g_cu16;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(3))) uint8_t l_u8;
typedef __attribute__((address_space(3))) uint32_t l_u32;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ uint32_t laneid() { return __lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint32_t ffs64(uint64_t m) { return m ? (uint32_t)__builtin_ctzll(m) : 64u; }

constexpr uint32_t kHashLog = 15;
constexpr uint32_t kHcDist = 65535;
constexpr int kOptimalML = 18;   // (ML_MASK - 1) + MINMATCH

__device__ __forceinline__ uint32_t rd32(g_cu8* p) {   // little-endian, any alignment (bytes inside the block)
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t rd16(g_cu8* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
__device__ __forceinline__ uint32_t hc_hash(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

}  // namespace

// ---------------------------------------------------------------------------
// k_hc_prev: delta[p] = p - (previous position with the same hash), 0 if
// none within 65535, for p in [0, n - 4] (positions lz4hc may insert)
// ---------------------------------------------------------------------------
constexpr uint32_t kPrevThreads = 256;   // 4 waves share one last-position table

// 16 bytes per thread of the 4 KiB chunk at c0 (0 past n): one dwordx4 load
// when the source is 16-byte aligned, bytes at the segment's end
__device__ __forceinline__ v4u hc_chunk_load(g_cu8* s, uint32_t n, uint32_t c0, bool al) {
    const uint32_t x = c0 + 16 * threadIdx.x;
    if (al && x + 16 <= n) return *(const __attribute__((address_space(1))) v4u*)(s + x);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t i = 0; i < 16; ++i)
        if (x + i < n) w[i >> 2] |= (uint32_t)s[x + i] << (8 * (i & 3));
    return (v4u){w[0], w[1], w[2], w[3]};
}

// One workgroup (4 waves) over the n bytes at s: dl[p] for p in [0, n - 4].
// Steps of 256 positions, wave w taking positions 64w .. 64w + 63 of the
// step: equal hashes inside a wave are resolved by ballot (the group's
// earlier member is the predecessor, its last member records its position);
// the waves then read / update the last-position table in wave order, so a
// position without a predecessor in its own wave sees the earlier waves'
// positions.  The source goes through an 8 KiB LDS ring, one 4 KiB chunk
// (16 steps) at a time, the next chunk's load in flight meanwhile.
__device__ void hc_prev_range(g_cu8* s, uint32_t n, g_u16* dl, l_u32* last, l_u8* dd, l_u32* ring) {
    const uint32_t t = threadIdx.x, L = laneid(), wv = t >> 6;
    for (uint32_t i = t; i < (1u << kHashLog); i += kPrevThreads) last[i] = 0;
    if (n < 4) return;
    const uint32_t np = n - 3;   // positions with 4 readable bytes
    const bool al = ((uintptr_t)s & 15) == 0;
    typedef __attribute__((address_space(3))) v4u l_v4u;
    ((l_v4u*)ring)[t] = hc_chunk_load(s, n, 0, al);
    v4u nxt = hc_chunk_load(s, n, 4096, al);
    l_u8* ddw = dd + 1024 * wv;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < np; c0 += 4096) {
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t base = c0 + 256 * k;
            if (base >= np) break;
            if (k == 15) {   // the last step reads 3 bytes of the next chunk
                ((l_v4u*)ring)[(((c0 + 4096) >> 4) + t) & 511] = nxt;
                __syncthreads();
            }
            const uint32_t p = base + t;
            const bool live = p < np;
            const uint32_t w = p >> 2;
            const uint32_t word = __builtin_amdgcn_alignbyte(ring[(w + 1) & 2047], ring[w & 2047], p & 3);
            const uint32_t h = live ? hc_hash(word) : 0u;
            if (live) ddw[h & 1023] = (uint8_t)L;
            WAVE_SYNC();
            const uint32_t sv = live ? ddw[h & 1023] : L;
            uint64_t pending = ballot(live && sv != L);
            int pred = -1;
            uint64_t gm = 1ull << L;
            while (pending) {
                const uint32_t leader = ffs64(pending);
                const uint32_t key = rdlane(h, (int)leader);
                const uint64_t m = ballot(live && h == key);
                if ((m >> L) & 1) {
                    gm = m;
                    const uint64_t below = m & ((1ull << L) - 1ull);
                    pred = below ? 63 - __clzll((long long)below) : -1;
                }
                pending &= ~m;
            }
            const bool groupLast = live && !(gm & ~((2ull << L) - 1ull));
            uint32_t q1 = pred >= 0 ? base + 64 * wv + (uint32_t)pred + 1 : 0u;   // position + 1 of the previous
            for (uint32_t u = 0; u < kPrevThreads / 64; ++u) {
                if (wv == u) {
                    if (live && pred < 0) q1 = last[h];
                    WAVE_SYNC();
                    if (groupLast) last[h] = p + 1;
                }
                __syncthreads();
            }
            if (live) dl[p] = (uint16_t)((q1 && p + 1 - q1 <= kHcDist) ? p + 1 - q1 : 0u);
        }
        nxt = hc_chunk_load(s, n, c0 + 8192, al);
    }
}

__global__ void __launch_bounds__(kPrevThreads) k_hc_prev(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                          uint32_t blockSize, uint16_t* __restrict__ delta) {
    __shared__ uint32_t last[1u << kHashLog];   // position + 1 of the latest occurrence (0 = none)
    __shared__ uint8_t dd[4 * 1024];            // duplicate-hash detection inside a wave's step
    __shared__ __attribute__((aligned(16))) uint32_t ring[2048];   // 8 KiB source ring
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    hc_prev_range((g_cu8*)src + off, n, (g_u16*)delta + off, (l_u32*)last, (l_u8*)dd, (l_u32*)ring);
}

// -BD at level >= 3: the chain over each stream segment (the bytes between
// two resets of the reference's HC stream), segment k = src[begin, end)
// (begin may lie up to 64 KiB before src: the previous batch's history)
__global__ void __launch_bounds__(kPrevThreads) k_hc_prev_seg(const uint8_t* __restrict__ src,
                                                              const int64_t* __restrict__ begin,
                                                              const int64_t* __restrict__ end,
                                                              uint16_t* __restrict__ delta0) {
    __shared__ uint32_t last[1u << kHashLog];
    __shared__ uint8_t dd[4 * 1024];
    __shared__ __attribute__((aligned(16))) uint32_t ring[2048];
    const uint32_t k = blockIdx.x;
    const int64_t b0 = begin[k];
    hc_prev_range((g_cu8*)src + b0, (uint32_t)(end[k] - b0), (g_u16*)delta0 + b0, (l_u32*)last, (l_u8*)dd,
                  (l_u32*)ring);
}

// ---------------------------------------------------------------------------
// k_encode_hc
// ---------------------------------------------------------------------------
namespace {

struct HcBlock {
    g_cu8* s;             // block source
    uint32_t n;
    g_cu16* dl;           // k_hc_prev output
    uint32_t maxAttempts;
    bool pattern;         // pattern analysis (level 9)

    // chain delta as lz4hc's chainTable holds it (capped 65535 = "none")
    __device__ __forceinline__ uint32_t chain(uint32_t m) const {
        const uint32_t d = dl[m];
        return d ? d : kHcDist;
    }
    // LZ4_count(a, b, limit): equal bytes of [a, limit) and [b, ...), 256 per round
    __device__ uint32_t count_fwd(uint32_t a, uint32_t b, uint32_t limit) const {
        const uint32_t L = laneid();
        uint32_t c = 0;
        for (;;) {
            const uint32_t x = a + c + 4 * L;
            uint32_t eq = 0;
            if (x < limit) {
                const uint32_t av = rd32(s + x), bv = rd32(s + b + c + 4 * L);
                const uint32_t diff = av ^ bv;
                eq = diff ? ((uint32_t)__builtin_ctz(diff) >> 3) : 4u;
                eq = min(eq, limit - x);
            }
            const uint64_t nf = ballot(eq < 4);
            if (nf) {
                const uint32_t f = ffs64(nf);
                return c + 4 * f + rdlane(eq, (int)f);
            }
            c += 256;
        }
    }
    // LZ4HC_countBack: <= 0, bounded by max(iMin - ip, mMin - match)
    __device__ int count_back(uint32_t ip, uint32_t match, uint32_t iMin, uint32_t mMin) const {
        const uint32_t L = laneid();
        const uint32_t lim = min(ip - iMin, match - mMin);   // steps allowed
        uint32_t k = 0;
        for (;;) {
            const uint32_t j = k + L + 1;
            const bool same = j <= lim && s[ip - j] == s[match - j];
            const uint64_t stop = ballot(!same);
            if (stop != 0) return -(int)(k + ffs64(stop));
            k += 64;
        }
    }
    // length of the run of byte v starting at p, up to end
    __device__ uint32_t run_fwd(uint32_t p, uint32_t end, uint32_t v) const {
        const uint32_t L = laneid();
        for (uint32_t c = 0;; c += 64) {
            const uint32_t x = p + c + L;
            const uint64_t stop = ballot(!(x < end && s[x] == v));
            if (stop) return c + ffs64(stop);
        }
    }
    // length of the run of byte v ending just before p, down to low
    __device__ uint32_t run_back(uint32_t p, uint32_t low, uint32_t v) const {
        const uint32_t L = laneid();
        for (uint32_t c = 0;; c += 64) {
            const uint32_t j = c + L + 1;
            const uint64_t stop = ballot(!(j <= p - low && s[p - j] == v));
            if (stop) return c + ffs64(stop);
        }
    }

    // LZ4HC_InsertAndGetWiderMatch (single segment); positions are block
    // offsets.  Returns longest; *mpos / *spos as lz4hc's matchpos /
    // startpos.  CS: chainSwap (the optimal parser's searches; lookBack 0).
    template <bool CS = false>
    __device__ int wider(uint32_t ip, uint32_t iLow, uint32_t iHigh, int longest, uint32_t* mpos,
                         uint32_t* spos) const {
        const uint32_t lowest = ip > kHcDist ? ip - kHcDist : 0u;
        const uint32_t lookBack = ip - iLow;
        int nbAttempts = (int)maxAttempts;
        const uint32_t pat = rd32(s + ip);
        int repeat = 0;   // 0 untested, 1 confirmed, 2 not
        uint32_t srcPatLen = 0;
        uint32_t mcp = 0;   // matchChainPos
        const uint32_t d0 = uni(dl[ip]);
        if (d0 == 0) return longest;   // no earlier position with this hash in the window
        uint32_t m = ip - d0;
        while (m >= lowest && nbAttempts > 0) {
            --nbAttempts;
            // the candidate's filter bytes and its chain link, one round
            const uint32_t f16 = uni(rd16(s + m - lookBack + (uint32_t)longest - 1));
            const uint32_t m32 = uni(rd32(s + m));
            const uint32_t dnext = uni(dl[m]);
            int matchLength = 0;
            if (uni(rd16(s + iLow + (uint32_t)longest - 1)) == f16 && m32 == pat) {
                const int back = lookBack ? count_back(ip, m, iLow, 0) : 0;
                int ml = 4 + (int)count_fwd(ip + 4, m + 4, iHigh);
                ml -= back;
                matchLength = ml;
                if (ml > longest) {
                    longest = ml;
                    *mpos = m + (uint32_t)back;
                    *spos = ip + (uint32_t)back;
                }
            }
            if (CS && matchLength == longest && m + (uint32_t)longest <= ip) {
                // a better chain: the position of the match whose chain link
                // reaches furthest back (lz4hc's accelerating scan), 64
                // links per load round
                uint32_t dtn = 1;
                const int end = longest - 4 + 1;
                int step = 1, accel = 1 << 4;
                int pos = 0, base = -64;
                uint32_t lk = 0;
                while (pos < end) {
                    if (pos >= base + 64) {   // links of [pos, pos + 64)
                        base = pos;
                        const uint32_t q = m + (uint32_t)pos + laneid();
                        lk = dl[q];
                        lk = lk ? lk : kHcDist;
                    }
                    const uint32_t cdist = rdlane(lk, pos - base);
                    step = accel++ >> 4;
                    if (cdist > dtn) {
                        dtn = cdist;
                        mcp = (uint32_t)pos;
                        accel = 1 << 4;
                    }
                    pos += step;
                }
                if (dtn > 1) {
                    if (dtn > m) break;   // below the block: under `lowest`
                    m -= dtn;
                    continue;
                }
            }
            const uint32_t distNext = dnext ? dnext : kHcDist;
            if (pattern && distNext == 1 && (!CS || mcp == 0)) {
                const uint32_t cand = m - 1;
                if (repeat == 0) {
                    if (((pat & 0xFFFF) == (pat >> 16)) & ((pat & 0xFF) == (pat >> 24))) {
                        repeat = 1;
                        srcPatLen = run_fwd(ip + 4, iHigh, pat & 255u) + 4;
                    } else {
                        repeat = 2;
                    }
                }
                if (repeat == 1 && cand >= lowest && uni(rd32(s + cand)) == pat) {   // good candidate
                    const uint32_t fwdLen = run_fwd(cand + 4, iHigh, pat & 255u) + 4;
                    uint32_t backLen = run_back(cand, 0, pat & 255u);
                    {
                        const uint32_t lo = cand - backLen;
                        backLen = cand - (lo > lowest ? lo : lowest);
                    }
                    const uint32_t segLen = backLen + fwdLen;
                    if (segLen >= srcPatLen && fwdLen <= srcPatLen) {
                        m = cand + fwdLen - srcPatLen;
                    } else {
                        m = cand - backLen;
                        if (lookBack == 0) {
                            const uint32_t maxML = segLen < srcPatLen ? segLen : srcPatLen;
                            if ((uint32_t)longest < maxML) {
                                if (ip - m > kHcDist) break;
                                longest = (int)maxML;
                                *mpos = m;
                                *spos = ip;
                            }
                            const uint32_t dn = chain(m);
                            if (dn > m + 65536u) break;   // lz4hc: distToNextPattern > matchIndex (index = offset + 64 KiB)
                            m -= dn;
                            if ((int32_t)m < 0) break;     // below the block: under `lowest`
                        }
                    }
                    continue;
                }
            }
            const uint32_t dfol = (CS && mcp) ? chain(m + mcp) : distNext;   // follow the current chain
            if (m < dfol) break;   // would go below the block: under `lowest`
            m -= dfol;
        }
        return longest;
    }
};

// LZ4HC_encodeSequence into d; returns false on overflow (limitedOutput)
__device__ bool hc_encode(g_cu8* s, g_u8* d, uint32_t& ip, uint32_t& op, uint32_t& anchor, int ml, uint32_t ref,
                          bool limit, uint32_t cap) {
    const uint32_t L = laneid();
    const uint32_t token = op;
    uint32_t o = op + 1;
    const uint32_t lit = ip - anchor;
    if (limit && (uint64_t)o + lit / 255 + lit + (2 + 1 + 5) > cap) return false;
    uint32_t tk;
    if (lit >= 15) {
        tk = 15u << 4;
        const uint32_t ext = (lit - 15) / 255 + 1, rem = (lit - 15) % 255;
        for (uint32_t c = 0; c < ext; c += 64)
            if (c + L < ext) d[o + c + L] = (uint8_t)(c + L + 1 < ext ? 255u : rem);
        o += ext;
    } else {
        tk = lit << 4;
    }
    for (uint32_t c = 0; c < lit; c += 64)
        if (c + L < lit) d[o + c + L] = s[anchor + c + L];
    o += lit;
    const uint32_t off = ip - ref;
    if (L == 0) { d[o] = (uint8_t)off; d[o + 1] = (uint8_t)(off >> 8); }
    o += 2;
    uint32_t len = (uint32_t)ml - 4;
    if (limit && (uint64_t)o + len / 255 + (1 + 5) > cap) return false;
    if (len >= 15) {
        tk += 15;
        len -= 15;
        // 255 pairs, then one 255 when >= 255 remains, then the remainder:
        // the same bytes as (len / 255) 255s and len % 255
        const uint32_t ext = len / 255 + 1, rem = len % 255;
        for (uint32_t c = 0; c < ext; c += 64)
            if (c + L < ext) d[o + c + L] = (uint8_t)(c + L + 1 < ext ? 255u : rem);
        o += ext;
    } else {
        tk += len;
    }
    if (L == 0) d[token] = (uint8_t)tk;
    WAVE_SYNC();
    op = o;
    ip += (uint32_t)ml;
    anchor = ip;
    return true;
}

// Loop-top hooks of a split parse (one block parsed by several waves, each
// from its own start, spliced where two of them meet; see k_hc_heads).  At
// the top of LZ4HC_compress_hashChain's main loop the whole parse state is
// (ip, anchor, op): every later match decision depends on ip alone (the
// searches take ip, never anchor, as their low limit) and anchor only sets
// the literal run of the next sequence.  Two parses at a loop top with the
// same ip and anchor == ip write the same bytes from there on.
enum : uint32_t { kHcRun = 0, kHcEnd = 1, kHcSync = 2, kHcFail = 3 };
struct HcState {
    uint32_t ip, anchor, op, status, cnt;   // cnt: loop tops recorded (MODE 1)
};
struct HcHooks {
    // MODE 1: record loop tops with anchor == ip (position, op) into hp / ho,
    // stop after R of them or at ip >= hlim (a loop top), state saved
    __attribute__((address_space(1))) uint32_t* hp;
    __attribute__((address_space(1))) uint32_t* ho;
    uint32_t R, hlim;
    // MODE 2: from xlo on, stop at the first loop top with anchor == ip whose
    // ip is in np[0 .. nR) (ascending); past np[nR - 1], fail
    const __attribute__((address_space(1))) uint32_t* np;
    uint32_t nR, xlo;
};

// LZ4HC_compress_hashChain from the loop-top state st; returns the state it
// stops in.  MODE 0: to the block end (last literals; status kHcEnd, or
// kHcFail when the output does not fit cap); 1 / 2: see HcHooks.
template <int MODE>
__device__ HcState hc_parse(const HcBlock& B, g_u8* d, uint32_t cap, bool limit, HcState st, const HcHooks& hk,
                           bool fresh = false) {
    const uint32_t L = laneid();
    const uint32_t n = B.n;
    g_cu8* s = B.s;
    uint32_t ip = st.ip, anchor = st.anchor, op = st.op;
    const uint32_t mflimit = n >= 12 ? n - 12 : 0, matchlimit = n >= 5 ? n - 5 : 0;
    int ml0, ml, ml2, ml3;
    uint32_t start0 = 0, ref0 = 0, ref = 0, start2 = 0, ref2 = 0, start3 = 0, ref3 = 0;
    uint32_t cnt = 0, k = 0, lastHead = 0;
    if (MODE == 2) lastHead = hk.nR ? hk.np[hk.nR - 1] : 0u;
    if (MODE == 0 && fresh && n - ip < 13) goto last_literals;   // inputSize < LZ4_minLength
    while (ip <= mflimit) {
        if (MODE == 1) {
            if (anchor == ip) {
                if (L == 0) { hk.hp[cnt] = ip; hk.ho[cnt] = op; }
                ++cnt;
            }
            if (cnt == hk.R || ip >= hk.hlim) return HcState{ip, anchor, op, kHcRun, cnt};
        }
        if (MODE == 2 && ip >= hk.xlo) {
            if (ip > lastHead) return HcState{ip, anchor, op, kHcFail, cnt};
            if (anchor == ip) {
                while (hk.np[k] < ip) ++k;
                if (hk.np[k] == ip) return HcState{ip, anchor, op, kHcSync};
            }
        }
        {
            uint32_t useless = ip;
            ml = B.wider(ip, ip, matchlimit, 3, &ref, &useless);
        }
        if (ml < 4) { ++ip; continue; }
        start0 = ip; ref0 = ref; ml0 = ml;
    search2:
        if (ip + (uint32_t)ml <= mflimit) ml2 = B.wider(ip + (uint32_t)ml - 2, ip, matchlimit, ml, &ref2, &start2);
        else ml2 = ml;
        if (ml2 == ml) {
            if (!hc_encode(s, d, ip, op, anchor, ml, ref, limit, cap)) return HcState{ip, anchor, op, kHcFail, cnt};
            continue;
        }
        if (start0 < ip && start2 < ip + (uint32_t)ml0) { ip = start0; ref = ref0; ml = ml0; }
        if (start2 - ip < 3) {
            ml = ml2; ip = start2; ref = ref2;
            goto search2;
        }
    search3:
        if (start2 - ip < (uint32_t)kOptimalML) {
            int nml = ml;
            if (nml > kOptimalML) nml = kOptimalML;
            if (ip + (uint32_t)nml > start2 + (uint32_t)ml2 - 4) nml = (int)(start2 - ip) + ml2 - 4;
            const int corr = nml - (int)(start2 - ip);
            if (corr > 0) { start2 += (uint32_t)corr; ref2 += (uint32_t)corr; ml2 -= corr; }
        }
        if (start2 + (uint32_t)ml2 <= mflimit) ml3 = B.wider(start2 + (uint32_t)ml2 - 3, start2, matchlimit, ml2, &ref3, &start3);
        else ml3 = ml2;
        if (ml3 == ml2) {
            if (start2 < ip + (uint32_t)ml) ml = (int)(start2 - ip);
            if (!hc_encode(s, d, ip, op, anchor, ml, ref, limit, cap)) return HcState{ip, anchor, op, kHcFail, cnt};
            ip = start2;
            if (!hc_encode(s, d, ip, op, anchor, ml2, ref2, limit, cap)) return HcState{ip, anchor, op, kHcFail, cnt};
            continue;
        }
        if (start3 < ip + (uint32_t)ml + 3) {
            if (start3 >= ip + (uint32_t)ml) {
                if (start2 < ip + (uint32_t)ml) {
                    const int corr = (int)(ip + (uint32_t)ml - start2);
                    start2 += (uint32_t)corr; ref2 += (uint32_t)corr; ml2 -= corr;
                    if (ml2 < 4) { start2 = start3; ref2 = ref3; ml2 = ml3; }
                }
                if (!hc_encode(s, d, ip, op, anchor, ml, ref, limit, cap)) return HcState{ip, anchor, op, kHcFail, cnt};
                ip = start3; ref = ref3; ml = ml3;
                start0 = start2; ref0 = ref2; ml0 = ml2;
                goto search2;
            }
            start2 = start3; ref2 = ref3; ml2 = ml3;
            goto search3;
        }
        if (start2 < ip + (uint32_t)ml) {
            if (start2 - ip < (uint32_t)kOptimalML) {
                if (ml > kOptimalML) ml = kOptimalML;
                if (ip + (uint32_t)ml > start2 + (uint32_t)ml2 - 4) ml = (int)(start2 - ip) + ml2 - 4;
                const int corr = ml - (int)(start2 - ip);
                if (corr > 0) { start2 += (uint32_t)corr; ref2 += (uint32_t)corr; ml2 -= corr; }
            } else {
                ml = (int)(start2 - ip);
            }
        }
        if (!hc_encode(s, d, ip, op, anchor, ml, ref, limit, cap)) return HcState{ip, anchor, op, kHcFail, cnt};
        ip = start2; ref = ref2; ml = ml2;
        start2 = start3; ref2 = ref3; ml2 = ml3;
        goto search3;
    }
    if (MODE == 1) return HcState{ip, anchor, op, kHcRun, cnt};   // past mflimit: MODE 0 writes the last literals
    if (MODE == 2) return HcState{ip, anchor, op, kHcFail, cnt};
last_literals : {
    const uint32_t run = n - anchor;
    const uint32_t llAdd = (run + 255 - 15) / 255;
    if (limit && (uint64_t)op + 1 + llAdd + run > cap) return HcState{ip, anchor, op, kHcFail, cnt};
    uint32_t o = op;
    if (run >= 15) {
        if (L == 0) d[o] = (uint8_t)(15u << 4);
        ++o;
        const uint32_t ext = (run - 15) / 255 + 1, rem = (run - 15) % 255;
        for (uint32_t c = 0; c < ext; c += 64)
            if (c + L < ext) d[o + c + L] = (uint8_t)(c + L + 1 < ext ? 255u : rem);
        o += ext;
    } else {
        if (L == 0) d[o] = (uint8_t)(run << 4);
        ++o;
    }
    for (uint32_t c = 0; c < run; c += 64)
        if (c + L < run) d[o + c + L] = s[anchor + c + L];
    op = o + run;
}
    return HcState{n, n, op, kHcEnd};
}


// LZ4HC_compress_hashChain over [start, B.n) of B.s (start > 0: the rest of
// a stream segment before it, -BD at level >= 3); 0 = does not fit cap
// (store raw)
__device__ int32_t encode_block_hc(const HcBlock& B, g_u8* d, uint32_t cap, uint32_t start = 0) {
    const uint32_t blen = B.n - start;
    const bool limit = (uint64_t)cap < (uint64_t)blen + blen / 255 + 16;
    const HcState r = hc_parse<0>(B, d, cap, limit, HcState{start, start, 0, 0, 0}, HcHooks{}, true);
    return r.status == kHcEnd ? (int32_t)r.op : 0;
}

// ---------------------------------------------------------------------------
// Levels 10..12 (and above, clamped to 12: the reference CLI's -A asks for
// 17, src/main.cpp:377): lz4 1.9.3's LZ4HC_compress_optimal, restated in
// oracle/lz4hc_oracle.c (hc_compress_optimal).  One wave per block; the
// parser state is wave-uniform, its price table (LZ4_OPT_NUM + 3 entries)
// is four arrays in a per-block scratch, and the lanes run the searches'
// counts, the price updates of a match (one lane per match length) and the
// byte writes.
// ---------------------------------------------------------------------------
constexpr int kOptNum = 4096;                 // LZ4_OPT_NUM
constexpr int kOptEntries = kOptNum + 3 + 1;  // + TRAILING_LITERALS (+ pad)
// opt[] of LZ4HC_compress_optimal, structure of arrays, in LDS (AS 3) or in
// a per-block global scratch (AS 1).  The wave reads back what its lanes
// wrote: uniform reads are relaxed atomic loads, so they stay vector loads
// (never the scalar cache, which does not see vector stores).
template <int AS>
struct HcOpt {
    typedef __attribute__((address_space(AS))) int32_t i32;
    typedef __attribute__((address_space(AS))) uint16_t u16;
    i32* price;
    i32* litlen;
    i32* mlen;
    u16* off;
    template <class P>
    static __device__ __forceinline__ int rd(P p) { return (int)uni((uint32_t)__atomic_load_n(p, __ATOMIC_RELAXED)); }
};
constexpr uint64_t kOptBlockBytes = (uint64_t)kOptEntries * 14 + 256;   // one block's scratch (AS 1)

__device__ __forceinline__ int hc_lit_price(int litlen) { return litlen + (litlen >= 15 ? 1 + (litlen - 15) / 255 : 0); }
__device__ __forceinline__ int hc_seq_price(int litlen, int mlen) {
    return 3 + hc_lit_price(litlen) + (mlen >= 19 ? 1 + (mlen - 19) / 255 : 0);
}

// LZ4HC_compress_optimal (favorCompressionRatio) from the loop-top state st;
// MODE 0: to the block end (kHcEnd, or kHcFail when the output does not fit
// cap); 1 / 2: the split parse's hooks (HcHooks), as in hc_parse.  Its loop
// top has the same property: with anchor == ip the literal run is empty, the
// chain is a function of the input and the price table is rebuilt from ip,
// so two parses there with the same ip write the same bytes from then on.
template <int MODE, int AS>
__device__ HcState hc_opt_parse(const HcBlock& B, g_u8* d, uint32_t cap, bool limit, HcState st, const HcHooks& hk,
                                const HcOpt<AS>& O, int suff, bool fullUpdate, bool fresh = false) {
    typedef HcOpt<AS> OT;
    const uint32_t L = laneid();
    const uint32_t n = B.n;
    g_cu8* s = B.s;
    uint32_t ip = st.ip, anchor = st.anchor, op = st.op;
    uint32_t cnt = 0, k = 0, lastHead = 0;
    if (MODE == 2) lastHead = hk.nR ? hk.np[hk.nR - 1] : 0u;
    if (suff >= kOptNum) suff = kOptNum - 1;
    // FindLongerMatch: a match longer than minLen at p (pattern analysis and chain swap on)
    auto longer = [&](uint32_t p, int minLen, int& len, int& off) {
        uint32_t mpos = 0, spos = p;
        const int ml = B.wider<true>(p, p, n - 5, minLen, &mpos, &spos);
        len = ml > minLen ? ml : 0;
        off = ml > minLen ? (int)(spos - mpos) : 0;
    };
    auto trailing = [&](int last) {   // literals after the last match position
        WAVE_SYNC();
        const int p0 = OT::rd(&O.price[last]);
        if (L >= 1 && L <= 3) {
            O.mlen[last + L] = 1; O.off[last + L] = 0; O.litlen[last + L] = (int)L;
            O.price[last + L] = p0 + hc_lit_price((int)L);
        }
        WAVE_SYNC();
    };
    if (!(fresh && n < 13)) {   // (a fresh block below 13 bytes has no match: straight to the last literals)
        const uint32_t mflimit = n >= 12 ? n - 12 : 0;
        while (ip <= mflimit) {
            if (MODE == 1) {
                if (anchor == ip) {
                    if (L == 0) { hk.hp[cnt] = ip; hk.ho[cnt] = op; }
                    ++cnt;
                }
                if (cnt == hk.R || ip >= hk.hlim) return HcState{ip, anchor, op, kHcRun, cnt};
            }
            if (MODE == 2 && ip >= hk.xlo) {
                if (ip > lastHead) return HcState{ip, anchor, op, kHcFail, cnt};
                if (anchor == ip) {
                    while (hk.np[k] < ip) ++k;
                    if (hk.np[k] == ip) return HcState{ip, anchor, op, kHcSync};
                }
            }
            const int llen = (int)(ip - anchor);
            int best_mlen, best_off, cur, last;
            int fmLen, fmOff;
            longer(ip, 3, fmLen, fmOff);
            if (fmLen == 0) { ++ip; continue; }
            if (fmLen > suff) {   // good enough: immediate encoding
                if (!hc_encode(s, d, ip, op, anchor, fmLen, ip - (uint32_t)fmOff, limit, cap))
                    return HcState{ip, anchor, op, kHcFail, cnt};
                continue;
            }
            WAVE_SYNC();
            if (L < 4) {   // literals at the first positions
                O.mlen[L] = 1; O.off[L] = 0; O.litlen[L] = llen + (int)L; O.price[L] = hc_lit_price(llen + (int)L);
            }
            for (int b0 = 4; b0 <= fmLen; b0 += 64) {   // the first match
                const int ml = b0 + (int)L;
                if (ml <= fmLen) {
                    O.mlen[ml] = ml; O.off[ml] = (uint16_t)fmOff; O.litlen[ml] = llen; O.price[ml] = hc_seq_price(llen, ml);
                }
            }
            last = fmLen;
            trailing(last);
            for (cur = 1; cur < last; cur++) {
                if (ip + (uint32_t)cur > mflimit) break;
                const int pc = OT::rd(&O.price[cur]);
                const int pc1 = OT::rd(&O.price[cur + 1]);
                if (fullUpdate) {
                    if (pc1 <= pc && OT::rd(&O.price[cur + 4]) < pc + 3) continue;
                } else {
                    if (pc1 <= pc) continue;
                }
                int nmLen, nmOff;
                longer(ip + (uint32_t)cur, fullUpdate ? 3 : last - cur, nmLen, nmOff);
                if (!nmLen) continue;
                if (nmLen > suff || nmLen + cur >= kOptNum) {   // immediate encoding
                    best_mlen = nmLen;
                    best_off = nmOff;
                    last = cur + 1;
                    goto encode;
                }
                {   // before the match: literals after the path to cur
                    const int bl = OT::rd(&O.litlen[cur]);
                    if (L >= 1 && L <= 3) {
                        const int price = pc - hc_lit_price(bl) + hc_lit_price(bl + (int)L);
                        const int pos = cur + (int)L;
                        if (price < O.price[pos]) {
                            O.mlen[pos] = 1; O.off[pos] = 0; O.litlen[pos] = bl + (int)L; O.price[pos] = price;
                        }
                    }
                    WAVE_SYNC();
                }
                {   // the match at cur, one lane per length
                    const int mlc = OT::rd(&O.mlen[cur]);
                    int ll, basePrice;
                    if (mlc == 1) {
                        ll = OT::rd(&O.litlen[cur]);
                        basePrice = cur > ll ? OT::rd(&O.price[cur - ll]) : 0;
                    } else {
                        ll = 0;
                        basePrice = pc;
                    }
                    const int lastPre = last;
                    bool lastTaken = false;
                    for (int b0 = 4; b0 <= nmLen; b0 += 64) {
                        const int ml = b0 + (int)L;
                        const int pos = cur + ml;
                        bool take = false;
                        if (ml <= nmLen) {
                            const int price = basePrice + hc_seq_price(ll, ml);
                            take = pos > lastPre + 3 || price <= O.price[pos];
                            if (take) {
                                O.mlen[pos] = ml; O.off[pos] = (uint16_t)nmOff; O.litlen[pos] = ll; O.price[pos] = price;
                            }
                        }
                        if (ballot(take && ml == nmLen)) lastTaken = true;
                    }
                    if (lastTaken && lastPre < cur + nmLen) last = cur + nmLen;
                    trailing(last);
                }
            }
            best_mlen = OT::rd(&O.mlen[last]);
            best_off = OT::rd(&O.off[last]);
            cur = last - best_mlen;
        encode:
            {   // reverse traversal: the shortest path's sequences
                int cp = cur, sml = best_mlen, soff = best_off;
                for (;;) {
                    const int nml = OT::rd(&O.mlen[cp]);
                    const int noff = OT::rd(&O.off[cp]);
                    WAVE_SYNC();
                    if (L == 0) { O.mlen[cp] = sml; O.off[cp] = (uint16_t)soff; }
                    WAVE_SYNC();
                    sml = nml;
                    soff = noff;
                    if (nml > cp) break;
                    cp -= nml;
                }
            }
            {
                int rPos = 0;
                while (rPos < last) {
                    const int ml = OT::rd(&O.mlen[rPos]);
                    const int off = OT::rd(&O.off[rPos]);
                    if (ml == 1) { ++ip; ++rPos; continue; }
                    rPos += ml;
                    if (!hc_encode(s, d, ip, op, anchor, ml, ip - (uint32_t)off, limit, cap))
                        return HcState{ip, anchor, op, kHcFail, cnt};
                }
            }
        }
    }
    if (MODE == 1) return HcState{ip, anchor, op, kHcRun, cnt};   // past mflimit: MODE 0 writes the last literals
    if (MODE == 2) return HcState{ip, anchor, op, kHcFail, cnt};
    {   // last literals
        const uint32_t run = n - anchor;
        const uint32_t llAdd = (run + 255 - 15) / 255;
        if (limit && (uint64_t)op + 1 + llAdd + run > cap) return HcState{ip, anchor, op, kHcFail, cnt};
        uint32_t o = op;
        if (run >= 15) {
            if (L == 0) d[o] = (uint8_t)(15u << 4);
            ++o;
            const uint32_t ext = (run - 15) / 255 + 1, rem = (run - 15) % 255;
            for (uint32_t c = 0; c < ext; c += 64)
                if (c + L < ext) d[o + c + L] = (uint8_t)(c + L + 1 < ext ? 255u : rem);
            o += ext;
        } else {
            if (L == 0) d[o] = (uint8_t)(run << 4);
            ++o;
        }
        for (uint32_t c = 0; c < run; c += 64)
            if (c + L < run) d[o + c + L] = s[anchor + c + L];
        return HcState{n, n, o + run, kHcEnd};
    }
}

// the optimal parse of a whole block; 0 = does not fit cap (store raw)
template <int AS>
__device__ int32_t encode_block_hc_opt(const HcBlock& B, g_u8* d, uint32_t cap, const HcOpt<AS>& O, int suff,
                                       bool fullUpdate) {
    const bool limit = (uint64_t)cap < (uint64_t)B.n + B.n / 255 + 16;
    const HcState r = hc_opt_parse<0>(B, d, cap, limit, HcState{0, 0, 0, 0, 0}, HcHooks{}, O, suff, fullUpdate, true);
    return r.status == kHcEnd ? (int32_t)r.op : 0;
}

// cap of a block: capOverride, or n (0xFFFFFFFF, lz4mt) or n - 1 (0xFFFFFFFE, -BD)
__device__ __forceinline__ uint32_t hc_cap(uint32_t n, uint32_t capOverride) {
    return capOverride == 0xFFFFFFFFu ? n : capOverride == 0xFFFFFFFEu ? n - 1 : capOverride;
}

}  // namespace

__global__ void __launch_bounds__(64) k_encode_hc(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                  uint32_t blockSize, uint8_t* __restrict__ slots,
                                                  uint64_t slotStride, uint32_t capOverride,
                                                  const uint16_t* __restrict__ delta, uint32_t maxAttempts,
                                                  int32_t* __restrict__ csize, const uint32_t* __restrict__ redo) {
    const uint32_t b = blockIdx.x;
    if (redo && !redo[b]) return;   // done by the split parse
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const uint32_t cap = hc_cap(n, capOverride);   // lz4mt: cap = n; -BD: n - 1
    HcBlock B{(g_cu8*)src + off, n, (g_cu16*)delta + off, maxAttempts, maxAttempts > 128};
    const int32_t r = encode_block_hc(B, (g_u8*)slots + (uint64_t)b * slotStride, cap);
    if (laneid() == 0) csize[b] = r;
}

// price table number t of a scratch of kOptBlockBytes-sized tables
__device__ __forceinline__ HcOpt<1> hc_opt_at(uint8_t* ws, uint64_t t) {
    typedef HcOpt<1> OT;
    uint8_t* w = ws + t * kOptBlockBytes;
    return OT{(OT::i32*)w, (OT::i32*)(w + 4 * kOptEntries), (OT::i32*)(w + 8 * kOptEntries),
              (OT::u16*)(w + 12 * kOptEntries)};
}

// LZ4-HC levels 10..12: one wave per block, the price table in a global
// scratch of kOptBlockBytes per block (L2-resident; in LDS it would hold a
// CU to two of these waves)
__global__ void __launch_bounds__(64) k_encode_hc_opt_g(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                        uint32_t blockSize, uint8_t* __restrict__ slots,
                                                        uint64_t slotStride, uint32_t capOverride,
                                                        const uint16_t* __restrict__ delta, uint32_t nbSearches,
                                                        int32_t sufficientLen, int32_t fullUpdate, uint8_t* optWs,
                                                        uint32_t tableStride, const uint32_t* __restrict__ redo,
                                                        int32_t* __restrict__ csize) {
    const uint32_t b = blockIdx.x;
    if (redo && !redo[b]) return;   // done by the split parse
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const uint32_t cap = hc_cap(n, capOverride);
    HcBlock B{(g_cu8*)src + off, n, (g_cu16*)delta + off, nbSearches, true};   // pattern analysis always on
    const HcOpt<1> O = hc_opt_at(optWs, (uint64_t)b * tableStride);
    const int32_t r = encode_block_hc_opt(B, (g_u8*)slots + (uint64_t)b * slotStride, cap, O, sufficientLen,
                                          fullUpdate != 0);
    if (laneid() == 0) csize[b] = r;
}

// ---------------------------------------------------------------------------
// Split parse of large blocks.  A 4 MiB block is one serial hashChain parse
// (k_encode_hc: 2048 waves for 8 GiB, latency-bound); here stream j of a
// block starts its own parse at M_j = j * sub (j = 0: the block start) and
// the streams are spliced where they meet:
//   k_hc_heads  stream j >= 1 parses from (M_j, M_j) until it has recorded
//               kHcHeads loop tops with anchor == ip (position, output
//               offset) or passed M_j + sub / 4; its state is kept.
//   k_hc_exit   stream j resumes (j = 0 starts at 0) and, past M_{j+1},
//               stops at its first loop top with anchor == ip at a position
//               stream j+1 recorded: from there both parses are the same
//               (hc_parse's note), so the block is stream 0 up to that
//               point, stream 1 from it, ...  The last stream runs to the
//               block end.
//   k_hc_join   per block: checks the chain of meeting points (each at or
//               after the previous one, where the stream is exact), sums
//               the pieces (raw iff the total exceeds cap: every
//               limitedOutput check of lz4hc implies it) and compacts them
//               in the slot; a block that did not meet is re-run whole by
//               k_encode_hc (flag).
// Stream j writes at slot + M_j, capped at its region [M_j, M_{j+1}).
// ---------------------------------------------------------------------------
constexpr uint32_t kHcHeads = 64;

struct HcSplitWs {
    uint32_t* hp;      // streams x kHcHeads
    uint32_t* ho;
    HcState* st1;      // after k_hc_heads
    HcState* st2;      // after k_hc_exit
    uint32_t* redo;    // per block: 1 = run k_encode_hc on it
};

__device__ __forceinline__ uint32_t hc_streams(uint32_t n, uint32_t sub) { return n >= 2 * sub ? n / sub : 1u; }


__global__ void __launch_bounds__(64) k_hc_heads(const uint8_t* __restrict__ src, uint64_t srcSize, uint32_t blockSize,
                                                 uint8_t* __restrict__ slots, uint64_t slotStride,
                                                 const uint16_t* __restrict__ delta, uint32_t maxAttempts,
                                                 uint32_t sub, uint32_t smax, HcSplitWs w) {
    const uint32_t id = blockIdx.x, b = id / smax, j = id % smax;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const uint32_t S = hc_streams(n, sub);
    if (j == 0 || j >= S) return;
    const uint32_t M = j * sub, end = j + 1 < S ? M + sub : n;
    HcBlock B{(g_cu8*)src + off, n, (g_cu16*)delta + off, maxAttempts, maxAttempts > 128};
    HcHooks hk{};
    hk.hp = (__attribute__((address_space(1))) uint32_t*)w.hp + (uint64_t)id * kHcHeads;
    hk.ho = (__attribute__((address_space(1))) uint32_t*)w.ho + (uint64_t)id * kHcHeads;
    hk.R = kHcHeads;
    hk.hlim = M + sub / 4;
    const HcState r = hc_parse<1>(B, (g_u8*)slots + (uint64_t)b * slotStride + M, end - M, true,
                                  HcState{M, M, 0, 0, 0}, hk);
    if (laneid() == 0) w.st1[id] = r;
}

__global__ void __launch_bounds__(64) k_hc_exit(const uint8_t* __restrict__ src, uint64_t srcSize, uint32_t blockSize,
                                                uint8_t* __restrict__ slots, uint64_t slotStride,
                                                const uint16_t* __restrict__ delta, uint32_t maxAttempts,
                                                uint32_t sub, uint32_t smax, HcSplitWs w) {
    const uint32_t id = blockIdx.x, b = id / smax, j = id % smax;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const uint32_t S = hc_streams(n, sub);
    if (S == 1 || j >= S) return;
    const uint32_t M = j * sub, end = j + 1 < S ? M + sub : n;
    HcState st = j ? w.st1[id] : HcState{0, 0, 0, kHcRun, 0};
    st.ip = uni(st.ip); st.anchor = uni(st.anchor); st.op = uni(st.op); st.status = uni(st.status);
    HcState r = st;
    if (st.status == kHcRun) {
        HcBlock B{(g_cu8*)src + off, n, (g_cu16*)delta + off, maxAttempts, maxAttempts > 128};
        g_u8* d = (g_u8*)slots + (uint64_t)b * slotStride + M;
        if (j + 1 < S) {
            const HcState nx = w.st1[id + 1];
            HcHooks hk{};
            hk.np = (const __attribute__((address_space(1))) uint32_t*)w.hp + (uint64_t)(id + 1) * kHcHeads;
            hk.nR = nx.status == kHcFail ? 0u : uni(nx.cnt);
            hk.xlo = M + sub;
            r = hc_parse<2>(B, d, end - M, true, st, hk);
        } else {
            r = hc_parse<0>(B, d, end - M, true, st, HcHooks{});
        }
    }
    if (laneid() == 0) w.st2[id] = r;
}

// The split parse of the optimal parser (levels >= 10): the same streams,
// meeting points and join as above, each stream with its own price table
__global__ void __launch_bounds__(64) k_hc_opt_heads(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                     uint32_t blockSize, uint8_t* __restrict__ slots,
                                                     uint64_t slotStride, const uint16_t* __restrict__ delta,
                                                     uint32_t nbSearches, int32_t suff, int32_t full, uint32_t sub,
                                                     uint32_t smax, HcSplitWs w, uint8_t* optT) {
    const uint32_t id = blockIdx.x, b = id / smax, j = id % smax;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const uint32_t S = hc_streams(n, sub);
    if (j == 0 || j >= S) return;
    const uint32_t M = j * sub, end = j + 1 < S ? M + sub : n;
    HcBlock B{(g_cu8*)src + off, n, (g_cu16*)delta + off, nbSearches, true};
    HcHooks hk{};
    hk.hp = (__attribute__((address_space(1))) uint32_t*)w.hp + (uint64_t)id * kHcHeads;
    hk.ho = (__attribute__((address_space(1))) uint32_t*)w.ho + (uint64_t)id * kHcHeads;
    hk.R = kHcHeads;
    hk.hlim = M + sub / 4;
    const HcState r = hc_opt_parse<1>(B, (g_u8*)slots + (uint64_t)b * slotStride + M, end - M, true,
                                      HcState{M, M, 0, 0, 0}, hk, hc_opt_at(optT, id), suff, full != 0);
    if (laneid() == 0) w.st1[id] = r;
}

__global__ void __launch_bounds__(64) k_hc_opt_exit(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                    uint32_t blockSize, uint8_t* __restrict__ slots,
                                                    uint64_t slotStride, const uint16_t* __restrict__ delta,
                                                    uint32_t nbSearches, int32_t suff, int32_t full, uint32_t sub,
                                                    uint32_t smax, HcSplitWs w, uint8_t* optT) {
    const uint32_t id = blockIdx.x, b = id / smax, j = id % smax;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const uint32_t S = hc_streams(n, sub);
    if (S == 1 || j >= S) return;
    const uint32_t M = j * sub, end = j + 1 < S ? M + sub : n;
    HcState st = j ? w.st1[id] : HcState{0, 0, 0, kHcRun, 0};
    st.ip = uni(st.ip); st.anchor = uni(st.anchor); st.op = uni(st.op); st.status = uni(st.status);
    HcState r = st;
    if (st.status == kHcRun) {
        HcBlock B{(g_cu8*)src + off, n, (g_cu16*)delta + off, nbSearches, true};
        g_u8* d = (g_u8*)slots + (uint64_t)b * slotStride + M;
        const HcOpt<1> O = hc_opt_at(optT, id);
        if (j + 1 < S) {
            const HcState nx = w.st1[id + 1];
            HcHooks hk{};
            hk.np = (const __attribute__((address_space(1))) uint32_t*)w.hp + (uint64_t)(id + 1) * kHcHeads;
            hk.nR = nx.status == kHcFail ? 0u : uni(nx.cnt);
            hk.xlo = M + sub;
            r = hc_opt_parse<2>(B, d, end - M, true, st, hk, O, suff, full != 0);
        } else {
            r = hc_opt_parse<0>(B, d, end - M, true, st, HcHooks{}, O, suff, full != 0);
        }
    }
    if (laneid() == 0) w.st2[id] = r;
}

// one workgroup (256 threads) per block
__global__ void __launch_bounds__(256) k_hc_join(uint64_t srcSize, uint32_t blockSize, uint8_t* __restrict__ slots,
                                                 uint64_t slotStride, uint32_t capOverride, uint32_t sub, uint32_t smax,
                                                 HcSplitWs w, int32_t* __restrict__ csize) {
    __shared__ uint32_t pieceSrc[64], pieceLen[64];
    __shared__ uint32_t verdict;   // 0 ok, 1 redo, 2 raw
    __shared__ uint32_t total;
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const uint32_t S = hc_streams(n, sub);
    if (S == 1) {   // not split: k_encode_hc parses it
        if (t == 0) w.redo[b] = 1;
        return;
    }
    if (t == 0) {
        uint32_t v = S <= 64 ? 0u : 1u, F = 0, prevE = 0;
        const uint64_t base = (uint64_t)b * smax;
        for (uint32_t j = 0; j < S && v == 0; ++j) {
            const HcState x = w.st2[base + j];
            uint32_t from = 0;
            if (j) {   // stream j's output offset at prevE, a loop top it recorded
                const HcState h = w.st1[base + j];
                const uint32_t* hp = w.hp + (base + j) * kHcHeads;
                const uint32_t* ho = w.ho + (base + j) * kHcHeads;
                uint32_t k = 0;
                while (k < h.cnt && hp[k] < prevE) ++k;
                if (h.status == kHcFail || k == h.cnt || hp[k] != prevE) { v = 1; break; }
                from = ho[k];
            }
            const bool last = j + 1 == S;
            if (last ? x.status != kHcEnd : (x.status != kHcSync || x.ip < prevE)) { v = 1; break; }
            pieceSrc[j] = j * sub + from;
            pieceLen[j] = x.op - from;
            F += x.op - from;
            prevE = x.ip;
        }
        if (v == 0 && F > hc_cap(n, capOverride)) v = 2;
        verdict = v;
        total = F;
        w.redo[b] = v == 1;
    }
    __syncthreads();
    if (verdict != 0) {
        if (verdict == 2 && t == 0) csize[b] = 0;
        return;
    }
    // compact the pieces in order (each destination at or before its source)
    uint8_t* d = slots + (uint64_t)b * slotStride;
    uint32_t dst = pieceLen[0];
    for (uint32_t j = 1; j < S; ++j) {
        const uint32_t ps = pieceSrc[j], len = pieceLen[j];
        if (ps != dst) {
            for (uint32_t c = 0; c < len; c += 256 * 16) {
                uint8_t v[16];
                const uint32_t x = c + 16 * t;
                const uint32_t m = x < len ? min(16u, len - x) : 0u;
                for (uint32_t q = 0; q < m; ++q) v[q] = d[ps + x + q];
                __syncthreads();
                for (uint32_t q = 0; q < m; ++q) d[dst + x + q] = v[q];
                __syncthreads();
            }
        }
        dst += len;
    }
    if (t == 0) csize[b] = (int32_t)total;
}

// -BD at level >= 3 (compressBlockDependency with the HC stream, reference
// src/lz4mt.cpp:295-332): LZ4_resetStreamStateHC leaves the stream at lz4hc's
// default level 9 whatever the context asks for, LZ4_slideInputBufferHC
// resets it, and every position is inserted into the chain (LZ4HC_Insert),
// so block b's parse depends only on the bytes of its segment before it:
// the hashChain parse of [o, o + len) over the segment, lowest match index
// = the segment start (or 64 KiB back), chain = k_hc_prev_seg.  No rounds.
__global__ void __launch_bounds__(64) k_encode_hc_bd(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                     uint32_t blockSize, uint8_t* __restrict__ slots,
                                                     const int64_t* __restrict__ begin,
                                                     const uint32_t* __restrict__ blockSeg,
                                                     const uint16_t* __restrict__ delta0,
                                                     int32_t* __restrict__ csize) {
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t len = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const int64_t S = begin[blockSeg[b]];
    const uint32_t o = (uint32_t)((int64_t)off - S);
    HcBlock B{(g_cu8*)src + S, o + len, (g_cu16*)delta0 + S, 256u, true};   // level 9
    const int32_t r = encode_block_hc(B, (g_u8*)slots + off, len - 1, o);   // cap = inSize - 1
    if (laneid() == 0) csize[b] = r;
}

hipError_t launch_encode_hc_bd(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                               uint8_t* slots, const int64_t* segBegin, const int64_t* segEnd, uint32_t nSeg,
                               const uint32_t* blockSeg, uint16_t* delta0, int32_t* csize, hipStream_t st) {
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hc_prev_seg, dim3(nSeg), dim3(kPrevThreads), 0, st, src, segBegin, segEnd, delta0);
    hipLaunchKernelGGL(k_encode_hc_bd, dim3(nBlocks), dim3(64), 0, st, src, srcSize, blockSize, slots, segBegin,
                       blockSeg, (const uint16_t*)delta0, csize);
    return hipGetLastError();
}

// level -> maxNbAttempts / nbSearches (lz4 1.9.3 clTable; < 1 = default 9,
// > 12 = LZ4HC_CLEVEL_MAX)
uint32_t hc_attempts(int level) {
    static const uint32_t kA[13] = {2, 2, 2, 4, 8, 16, 32, 64, 128, 256, 96, 512, 16384};
    if (level < 1) level = 9;
    return kA[level > 12 ? 12 : level];
}

// stream length of the split parse (LZ4MT_AMD_HC_SUB_KIB, default 256; 0 = off)
uint32_t hc_split_sub() {
    const char* e = getenv("LZ4MT_AMD_HC_SUB_KIB");
    const long k = e ? atol(e) : 256;
    return k > 0 ? (uint32_t)std::max<long>(k, 64) << 10 : 0u;
}

static uint32_t hc_smax(uint32_t blockSize) {
    const uint32_t sub = hc_split_sub();
    return sub && blockSize >= 2 * sub ? blockSize / sub : 0u;
}

uint64_t hc_split_bytes(uint64_t nBlocks, uint32_t blockSize) {
    const uint64_t sm = hc_smax(blockSize), streams = nBlocks * sm;
    if (!sm) return 0;
    return streams * (2 * kHcHeads * 4 + 2 * sizeof(HcState)) + (nBlocks + 1) * 4 + 256;
}

// HC scratch of a launch: the split parse's records (levels 3..9), or the
// optimal parser's price tables (levels >= 10)
static uint64_t hc_opt_tables_at(uint64_t nBlocks, uint32_t blockSize) {   // after the split records
    return (hc_split_bytes(nBlocks, blockSize) + 255) & ~uint64_t(255);
}
uint64_t hc_ws_bytes(uint64_t nBlocks, uint32_t blockSize, int level) {
    if (level < 10) return hc_split_bytes(nBlocks, blockSize);
    const uint64_t tables = std::max<uint64_t>(nBlocks, nBlocks * hc_smax(blockSize));   // one per stream (or block)
    return hc_opt_tables_at(nBlocks, blockSize) + tables * kOptBlockBytes + 256;
}

static HcSplitWs carve_split(uint8_t* p, uint64_t nBlocks, uint32_t blockSize) {
    const uint64_t streams = nBlocks * hc_smax(blockSize);
    HcSplitWs w;
    w.hp = reinterpret_cast<uint32_t*>(p);
    w.ho = w.hp + streams * kHcHeads;
    w.st1 = reinterpret_cast<HcState*>(w.ho + streams * kHcHeads);
    w.st2 = w.st1 + streams;
    w.redo = reinterpret_cast<uint32_t*>(w.st2 + streams);
    return w;
}

hipError_t launch_encode_hc(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                            uint8_t* slots, uint64_t slotStride, uint32_t capOverride, int level, uint16_t* delta,
                            int32_t* csize, hipStream_t st, uint8_t* splitWs) {
    const uint32_t att = hc_attempts(level);
    if (att == 0) return hipErrorInvalidValue;
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hc_prev, dim3(nBlocks), dim3(kPrevThreads), 0, st, src, srcSize, blockSize, delta);
    if (level >= 10) {   // the optimal parser: target length 64 / 128 / LZ4_OPT_NUM, full update at 12
        const int lv = level > 12 ? 12 : level;
        const int32_t tl = lv == 10 ? 64 : lv == 11 ? 128 : kOptNum, fu = lv == 12 ? 1 : 0;
        if (!splitWs) return hipErrorInvalidValue;   // hc_ws_bytes(nBlocks, blockSize, level) of price tables
        uint8_t* optT = splitWs + hc_opt_tables_at(nBlocks, blockSize);
        const uint32_t sm = hc_smax(blockSize), sub = hc_split_sub();
        if (sm && slotStride >= blockSize) {   // large blocks: split parse, whole-block re-run where it fails
            const HcSplitWs w = carve_split(splitWs, nBlocks, blockSize);
            const uint32_t grid = nBlocks * sm;
            hipLaunchKernelGGL(k_hc_opt_heads, dim3(grid), dim3(64), 0, st, src, srcSize, blockSize, slots,
                               slotStride, (const uint16_t*)delta, att, tl, fu, sub, sm, w, optT);
            hipLaunchKernelGGL(k_hc_opt_exit, dim3(grid), dim3(64), 0, st, src, srcSize, blockSize, slots,
                               slotStride, (const uint16_t*)delta, att, tl, fu, sub, sm, w, optT);
            hipLaunchKernelGGL(k_hc_join, dim3(nBlocks), dim3(256), 0, st, srcSize, blockSize, slots, slotStride,
                               capOverride, sub, sm, w, csize);
            hipLaunchKernelGGL(k_encode_hc_opt_g, dim3(nBlocks), dim3(64), 0, st, src, srcSize, blockSize, slots,
                               slotStride, capOverride, (const uint16_t*)delta, att, tl, fu, optT, sm,
                               (const uint32_t*)w.redo, csize);
            return hipGetLastError();
        }
        hipLaunchKernelGGL(k_encode_hc_opt_g, dim3(nBlocks), dim3(64), 0, st, src, srcSize, blockSize, slots,
                           slotStride, capOverride, (const uint16_t*)delta, att, tl, fu, optT, 1u,
                           (const uint32_t*)nullptr, csize);
        return hipGetLastError();
    }
    const uint32_t sm = hc_smax(blockSize), sub = hc_split_sub();
    if (splitWs && sm && slotStride >= blockSize) {   // large blocks: split parse, whole-block re-run where it fails
        const HcSplitWs w = carve_split(splitWs, nBlocks, blockSize);
        const uint32_t grid = nBlocks * sm;
        hipLaunchKernelGGL(k_hc_heads, dim3(grid), dim3(64), 0, st, src, srcSize, blockSize, slots, slotStride,
                           (const uint16_t*)delta, att, sub, sm, w);
        hipLaunchKernelGGL(k_hc_exit, dim3(grid), dim3(64), 0, st, src, srcSize, blockSize, slots, slotStride,
                           (const uint16_t*)delta, att, sub, sm, w);
        hipLaunchKernelGGL(k_hc_join, dim3(nBlocks), dim3(256), 0, st, srcSize, blockSize, slots, slotStride,
                           capOverride, sub, sm, w, csize);
        if (getenv("LZ4MT_AMD_HC_STATS")) {   // diagnostics: blocks the split parse left to k_encode_hc
            std::vector<uint32_t> r(nBlocks);
            if (hipMemcpyAsync(r.data(), w.redo, nBlocks * 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
                hipStreamSynchronize(st) == hipSuccess) {
                uint32_t c = 0;
                for (uint32_t x : r) c += x;
                fprintf(stderr, "[hc split] sub %u KiB, %u streams/block: %u of %u blocks re-run whole\n", sub >> 10,
                        sm, c, nBlocks);
            }
        }
        hipLaunchKernelGGL(k_encode_hc, dim3(nBlocks), dim3(64), 0, st, src, srcSize, blockSize, slots, slotStride,
                           capOverride, (const uint16_t*)delta, att, csize, (const uint32_t*)w.redo);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_encode_hc, dim3(nBlocks), dim3(64), 0, st, src, srcSize, blockSize, slots, slotStride,
                       capOverride, (const uint16_t*)delta, att, csize, (const uint32_t*)nullptr);
    return hipGetLastError();
}

}  // namespace lz4mt
