// lz4mt_kernels.hip — hand-written CDNA4 (gfx950) kernels for the lz4mt hot path.
//
//   k_encode        LZ4 1.9.3 greedy parse, one wavefront per frame block
//                   (replaces ctx.compress = LZ4_compress_limitedOutput,
//                   reference src/lz4mt.cpp:391, src/main.cpp:749-751)
//   k_decode        LZ4_decompress_safe 1.9.3 state machine, one wavefront
//                   per block (replaces ctx.decompress, src/lz4mt.cpp:645-646)
//   k_xxh32_*       XXH32 seed 0 of stored blocks / whole streams
//                   (replaces Lz4Mt::Xxh32, src/lz4mt_xxh32.cpp:14-58)
//   k_frame_*       exclusive scan + scatter of the block records into one
//                   contiguous frame (replaces the ordered write chain,
//                   src/lz4mt.cpp:407-428), and the device-side frame walk
//                   (src/lz4mt.cpp:685-727)
//   k_gen_synthetic the pinned synthetic input
//
// Wave-level design: every block is an independent serial
// parse, so a block is owned by ONE 64-lane wavefront; lanes work on the
// data-parallel parts (64 speculative match probes per step, 64-lane
// backward/forward match extension, lane-parallel literal/match copies),
// while the parse state lives in wave-uniform registers.  The hash table
// (16 KiB) and the decoder's history ring (16 KiB) sit in LDS.
#include "lz4mt_device.h"
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>

// LZ4MT_PART splits this file into two objects so each half gets its own
// scheduler flags (Makefile): 1 = everything but the decoder kernels,
// 2 = the decoder kernels only, 0 (default) = all.
#ifndef LZ4MT_PART
#define LZ4MT_PART 0
#endif

namespace lz4mt {

// LZ4MT_AMD_BD_COLD=1: -BD encode rounds start from all-stale tables (A/B of k_link_warm)
[[maybe_unused]] static bool link_cold() {
    const char* e = getenv("LZ4MT_AMD_BD_COLD");
    return e && e[0] == '1';
}

// LZ4MT_AMD_BD_STATS=1: print the -BD rounds' work (blocks redone per
// round, first unsettled block) to stderr -- synchronises the stream
static void link_stats(const char* what, const uint32_t* changed, const uint32_t* firstU, int rounds,
                       uint32_t nBlocks, hipStream_t st) {
    const char* e = getenv("LZ4MT_AMD_BD_STATS");
    if (!e || e[0] != '1') return;
    uint32_t c[kLinkRounds + 1], f[kLinkRounds + 1];
    if (hipMemcpyAsync(c, changed, sizeof(c), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(f, firstU, sizeof(f), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return;
    fprintf(stderr, "[lz4mt -BD %s] %u blocks, queued per round:", what, nBlocks);
    int last = 0;
    for (int r = 1; r <= rounds; ++r) if (c[r]) last = r;
    for (int r = 1; r <= last; ++r) fprintf(stderr, " %u", c[r]);
    fprintf(stderr, "%s\n", c[rounds] ? " (serial finish)" : "");
}

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
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

// Address-space-typed pointers.  Every global (1) and LDS (3) access goes
// through these so the compiler emits global_* / ds_* instructions: a
// generic pointer (e.g. an LDS array kept in a struct) becomes flat_*,
// which counts against both vmcnt and lgkmcnt and serialises the wave.
typedef const __attribute__((address_space(1))) uint8_t g_cu8;
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef const __attribute__((address_space(1))) uint32_t g_cu32;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) v4u g_cu4;
typedef __attribute__((address_space(1))) v4u g_u4;
typedef __attribute__((address_space(1))) v2u g_u2;
typedef __attribute__((address_space(3))) uint8_t l_u8;
typedef __attribute__((address_space(3))) uint16_t l_u16;
typedef __attribute__((address_space(3))) uint32_t l_u32;
typedef __attribute__((address_space(3))) v4u l_u4;
typedef __attribute__((address_space(3))) v2u l_u2;
__device__ __forceinline__ g_cu8* gptr(const uint8_t* p) { return (g_cu8*)p; }
__device__ __forceinline__ g_u8* gptr(uint8_t* p) { return (g_u8*)p; }

__device__ __forceinline__ uint32_t laneid() { return __lane_id(); }

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// mask of lanes <= L (L in [0,63]; at 63 the shift drops the bit: 0 - 1 = all)
__device__ __forceinline__ uint64_t mask_le(uint32_t L) { return (2ull << L) - 1ull; }

// Little-endian 32-bit read at an arbitrary byte address.  Only the aligned
// dwords that hold requested bytes are touched, so it never reads a dword
// that lies wholly past the last requested byte.
__device__ __forceinline__ uint32_t ld32u(g_cu8* p) {
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    g_cu32* q = (g_cu32*)(p - sh);
    const uint32_t lo = q[0];
    const uint32_t hi = sh ? q[1] : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// Diagnostic stamps (separate kernels, never in the product launch):
// accumulate s_memtime deltas per phase into uniform registers.
#define STAMP_T() (ST ? (uint64_t)__builtin_amdgcn_s_memtime() : 0ull)
#define STAMP_ADD(i, t0)                          \
    do {                                          \
        if (ST) {                                 \
            const uint64_t t1_ = STAMP_T();       \
            acc[i] += t1_ - (t0);                 \
            t0 = t1_;                             \
        }                                         \
    } while (0)

[[maybe_unused]] constexpr uint32_t kP1 = 2654435761u, kP2 = 2246822519u, kP3 = 3266489917u, kP4 = 668265263u, kP5 = 374761393u;

// ---------------------------------------------------------------------------
// Encoder
// ---------------------------------------------------------------------------
// Probe schedule of LZ4_compress_generic's search loop: probe k sits at
// s + F(k) with step(k) = max(1, (63 + k) >> 6)  (searchMatchNb >> 6).
__device__ __forceinline__ uint32_t probe_off(uint32_t k) {
    if (k == 0) return 0;
    const uint32_t q = (k - 1) >> 6, r = (k - 1) & 63;
    return 1 + 32 * q * (q + 1) + r * (q + 1);
}
__device__ __forceinline__ uint32_t probe_step(uint32_t k) { return k == 0 ? 1u : ((63 + k) >> 6); }

template <bool U16>
__device__ __forceinline__ uint32_t lz4_hash(uint32_t w0, uint32_t w1) {
    if (U16) return (w0 * 2654435761u) >> 19;                         // hash4, 13 bits
    const uint64_t v = ((uint64_t)w1 << 32) | w0;                     // hash5, 12 bits
    return (uint32_t)(((v << 24) * 889523592379ull) >> 52);
}

// u32-table entries (blocks >= 65547 B, at most 4 MiB = 2^22 positions) keep
// the position in the low 22 bits and a 10-bit tag of the 4 bytes AT that
// position in the high bits.  LZ4 accepts a candidate only if those 4 bytes
// equal the probe's, so a tag mismatch proves "no match" without touching
// memory; only tag-equal candidates outside the LDS ring cost a global load
// (then folded into the count round trip).  Exact: every accepted match is
// still confirmed by a full 4-byte compare.
constexpr uint32_t kPosBits = 22;
constexpr uint32_t kPosMask = (1u << kPosBits) - 1u;
__device__ __forceinline__ uint32_t cand_tag(uint32_t w0) { return (w0 * 0x85EBCA77u) >> kPosBits; }

// One window of up to 64 probes.  Lane roles: [INSERT][TEST] SEARCH...
//   INSERT: table insertion only (position 0 at block start, ip-2 after a match)
//   TEST:   LZ4's "test next position" probe right after a match
//   SEARCH: probe k0 + j of the skip-accelerated search loop
struct Win {
    uint32_t hasIns, hasTest, insPos, testPos, s, k0;
    __device__ __forceinline__ uint32_t pos(uint32_t L) const {
        const uint32_t ns = hasIns + hasTest;
        if (L < hasIns) return insPos;
        if (L < ns) return testPos;
        return s + probe_off(k0 + (L - ns));
    }
};

// Source view of one block: a 2 KiB LDS ring holding src[B, B + kRingE)
// (B a multiple of 512, advanced as the parse moves) in front of global
// memory.  Every read falls back to global for positions outside the ring,
// so the ring only changes speed, never results.  The next 512-byte chunk
// is prefetched into registers one advance ahead, so an advance normally
// finds its data already landed.
constexpr uint32_t kRingE = 2048;
constexpr uint32_t kRingMaskW = kRingE / 4 - 1;   // ring index mask in dwords
constexpr uint32_t kDedup = 1024;                 // duplicate-hash scratch entries
constexpr uint32_t kOutRing = 1024;               // LDS staging of the compressed output
constexpr uint32_t kOutFlush = 512;               // flush granule (64 lanes x 8 B)

struct SrcView {
    g_cu8* s;
    uint32_t n;
    l_u32* ring;      // kRingE bytes
    uint32_t B;
    uint32_t pfPos;   // position of the prefetched chunk in (pa, pb)
    uint32_t pa, pb;

    __device__ __forceinline__ void fetch(uint32_t c, uint32_t& a, uint32_t& b) const {
        const uint32_t pos = c + 8 * laneid();
        a = 0; b = 0;
        if (pos < n) a = *(g_cu32*)(s + pos);
        if (pos + 4 < n) b = *(g_cu32*)(s + pos + 4);
    }
    __device__ __forceinline__ void store(uint32_t c, uint32_t a, uint32_t b) {
        const uint32_t w = (c >> 2) + 2 * laneid();
        ring[w & kRingMaskW] = a;
        ring[(w + 1) & kRingMaskW] = b;
    }
    __device__ __forceinline__ void init(uint32_t b0 = 0) {   // b0: a multiple of 512
        B = b0;
        for (uint32_t c = b0; c < b0 + kRingE; c += 512) {
            uint32_t a, b;
            fetch(c, a, b);
            store(c, a, b);
        }
        pfPos = b0 + kRingE;
        fetch(pfPos, pa, pb);
        WAVE_SYNC();
    }
    // make the ring end at or beyond `hi` (uniform)
    __device__ __forceinline__ void cover(uint32_t hi) {
        if (hi <= B + kRingE) return;
        WAVE_SYNC();
        const uint32_t nb = (hi - kRingE + 511) & ~511u;
        if (nb == B + 512 && pfPos == B + kRingE) {   // common case: one chunk, already prefetched
            store(pfPos, pa, pb);
        } else {
            const uint32_t from = (nb >= B + kRingE) ? nb : B + kRingE;
            for (uint32_t c = from; c < nb + kRingE; c += 512) {
                uint32_t a, b;
                if (c == pfPos) { a = pa; b = pb; } else fetch(c, a, b);
                store(c, a, b);
            }
        }
        B = nb;
        pfPos = B + kRingE;
        fetch(pfPos, pa, pb);   // next advance's chunk: in flight, not waited on
        WAVE_SYNC();
    }
    __device__ __forceinline__ bool in_ring(uint32_t pos, uint32_t len) const {
        return pos >= B && pos + len <= B + kRingE;
    }
    __device__ __forceinline__ uint32_t rd4(uint32_t pos) const {   // bytes [pos, pos+4) little-endian
        if (in_ring(pos, 4)) {
            const uint32_t w = pos >> 2, sh = pos & 3;
            const uint32_t lo = ring[w & kRingMaskW];
            const uint32_t hi = sh ? ring[(w + 1) & kRingMaskW] : 0u;
            return __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
        return ld32u(s + pos);
    }
    __device__ __forceinline__ uint32_t rd1(uint32_t pos) const {
        if (in_ring(pos, 1)) return (ring[(pos >> 2) & kRingMaskW] >> (8 * (pos & 3))) & 255u;
        return s[pos];
    }
};

// Compressed output staged in a 1 KiB LDS ring; complete 512-byte chunks are
// flushed with 8-byte stores.  Global stores are rare, so the vmcnt waits of
// the candidate loads do not queue behind byte stores.
struct OutView {
    g_u8* d;          // block slot (8-byte aligned)
    l_u8* ring;       // kOutRing bytes
    uint32_t flushed;

    __device__ __forceinline__ void put(uint32_t pos, uint32_t v) { ring[pos & (kOutRing - 1)] = (uint8_t)v; }
    __device__ __forceinline__ void flush_to(uint32_t upto) {   // flush complete chunks below `upto`
        while (flushed + kOutFlush <= upto) {
            WAVE_SYNC();
            const uint32_t o = flushed + 8 * laneid();
            const v2u v = *(l_u2*)(ring + (o & (kOutRing - 1)));
            *(g_u2*)(d + o) = v;
            flushed += kOutFlush;
        }
    }
    __device__ __forceinline__ void finish(uint32_t op) {
        flush_to(op);
        WAVE_SYNC();
        for (uint32_t o = flushed + laneid(); o < op; o += 64) d[o] = ring[o & (kOutRing - 1)];
        flushed = op;
    }
};

// bytes of a 4-bit length field's extension: (v - 15) / 255 + 1 for v >= 15,
// else 0 -- one formula for both: (v + 240) / 255
__device__ __forceinline__ uint32_t ext_len(uint32_t v) { return (v + 240) / 255; }

// Stages literal bytes src[from + i] for i in [i0, i1) at out position
// base + i, 4 per lane, flushing complete chunks below `safe + i` between
// pieces (bytes below `safe` are final).
__device__ __forceinline__ void stage_lits(const SrcView& V, OutView& O, uint32_t from, uint32_t i0, uint32_t i1,
                                           uint32_t base, bool flush, uint32_t safe) {
    const uint32_t L = laneid();
    for (uint32_t piece = i0; piece < i1; piece += 256) {
        if (flush) O.flush_to(safe + piece);
        const uint32_t i = piece + 4 * L;
        if (i < i1) {
            uint32_t v;
            if (i + 4 <= i1) {
                v = V.rd4(from + i);
            } else {   // tail: never touch bytes past the run (the block may end the buffer)
                v = V.rd1(from + i);
                if (i + 1 < i1) v |= V.rd1(from + i + 1) << 8;
                if (i + 2 < i1) v |= V.rd1(from + i + 2) << 16;
            }
            O.put(base + i, v);
            if (i + 1 < i1) O.put(base + i + 1, v >> 8);
            if (i + 2 < i1) O.put(base + i + 2, v >> 16);
            if (i + 3 < i1) O.put(base + i + 3, v >> 24);
        }
        WAVE_SYNC();
    }
}

// `cnt` length bytes (255 ... 255 rem) at pos, flushing between 64-byte
// pieces; every byte below pos is final.
__device__ __forceinline__ void put_ext(OutView& O, uint32_t pos, uint32_t cnt, uint32_t rem) {
    for (uint32_t base = 0; base < cnt; base += 64) {
        O.flush_to(pos + base);
        const uint32_t x = base + laneid();
        if (x < cnt) O.put(pos + x, x + 1 < cnt ? 255u : rem);
        WAVE_SYNC();
    }
}

// token + literal-length bytes at op (everything below op is final)
__device__ __forceinline__ void put_head(OutView& O, uint32_t op, uint32_t lit, uint32_t mcNibble) {
    const uint32_t token = ((lit < 15 ? lit : 15) << 4) | mcNibble;
    O.flush_to(op);
    if (laneid() == 0) O.put(op, token);
    WAVE_SYNC();
    put_ext(O, op + 1, ext_len(lit), lit >= 15 ? (lit - 15) % 255 : 0);
}

// Block-dependent (-BD) parameters of encode_block<..., LINK = true>: the
// block is compressed as one step of LZ4 1.9.3's LZ4_compress_fast_continue
// (byU32 table carried over from the previous blocks, history before the
// block).  Positions are "s'-coordinates": s points 64 KiB before the block,
// so the block is [kLinkO0, kLinkO0 + len) and its history [0, kLinkO0).
//   lowIn / lowDict  catch-up lower bound (lz4's lowLimit) for candidates in
//                    the block / in the history: the source start in
//                    usingExtDict mode, the prefix start in withPrefix64k mode
//   candLow          dictSmall: candidates below it are out of the valid area
//   fresh            a new stream: the table starts at the block's position 0
constexpr uint32_t kLinkO0 = 65536;
//   shift            (LZ4MT_AMD_BD_REFERENCE) history position p reads the
//                    block's own byte p - kLinkO0 + shift (LinkPlan.shift)
struct LinkArgs {
    uint32_t lowIn, lowDict, candLow;
    bool fresh;
    uint32_t shift = 0;
};

template <bool U16, bool TAG, bool ST, bool LINK = false>
__device__ __forceinline__ int32_t encode_block(g_cu8* __restrict__ s, uint32_t n, g_u8* __restrict__ d, uint32_t cap,
                                l_u32* __restrict__ Traw, l_u8* __restrict__ S, l_u32* __restrict__ ringE,
                                l_u8* __restrict__ outRing, uint64_t* acc, LinkArgs lk = LinkArgs{0, 0, 0, true}) {
    const uint32_t L = laneid();
    uint64_t ts = STAMP_T();
    const uint32_t o0 = LINK ? kLinkO0 : 0u;   // position of the block's first byte
    const uint32_t blen = n - o0;
    const uint32_t bound = blen + blen / 255 + 16;
    const bool limited = cap < bound;
    if (blen == 0) {
        if (limited && cap == 0) return 0;
        if (L == 0) d[0] = 0;
        return 1;
    }
    l_u16* T16 = (l_u16*)Traw;
    if (!LINK || lk.fresh) {
        // a fresh entry is position 0 -- a real candidate in LZ4 1.9.3 --
        // so tagged tables start with the tag of the bytes at 0
        const uint32_t t0 = TAG ? (cand_tag(ld32u(s)) << kPosBits) : o0;
        l_u4* T4 = (l_u4*)Traw;
        for (uint32_t i = L; i < 1024; i += 64) T4[i] = (v4u){t0, t0, t0, t0};
    }
    SrcView V{s, n, ringE, 0, 0, 0, 0};
    V.init(o0);
    OutView O{d, outRing, 0};

    const uint32_t mflimitP1 = n - kMfLimit + 1;
    const uint32_t matchlimit = n - kLastLiterals;
    uint32_t anchor = o0, op = 0;

    if (blen < (uint32_t)kMinLength) goto last_literals;
    {
        Win W{1, 0, o0, 0, o0 + 1, 0};  // T[h(0)] = 0; search from ip = 1
        for (;;) {
            // ---------------- one probe window ----------------
            if (ST) acc[10] += 1;
            STAMP_ADD(9, ts);
            const uint32_t ns = W.hasIns + W.hasTest;
            const bool isIns = L < W.hasIns;
            const bool isTest = !isIns && L < ns;
            const bool isSearch = L >= ns;
            const uint32_t k = W.k0 + (L - ns);
            const uint32_t p = W.pos(L);
            const bool live = !isSearch || p <= mflimitP1;
            const bool term = isSearch && live && (p + probe_step(k) > mflimitP1);
            {
                const uint32_t plast = W.pos(63);
                V.cover((plast < mflimitP1 ? plast : mflimitP1) + 8);
            }
            uint32_t w0 = 0, w1 = 0;
            if (live) {
                w0 = V.rd4(p);
                if (!U16) w1 = V.rd4(p + 4);
            }
            const uint32_t h = live ? lz4_hash<U16>(w0, w1) : 0u;
            const uint32_t mytag = TAG ? cand_tag(w0) : 0u;
            STAMP_ADD(0, ts);
            // duplicate-hash detection inside the window (aliasing of the
            // scratch index only costs an extra group iteration)
            S[h & (kDedup - 1)] = (uint8_t)L;
            const uint32_t told = U16 ? (uint32_t)T16[h] : Traw[h];
            WAVE_SYNC();
            const uint32_t sv = S[h & (kDedup - 1)];
            uint64_t pending = ballot(live && sv != L);
            int pred = -1;
            uint64_t gmask = 1ull << L;
            while (pending) {  // one iteration per group of equal hashes
                const int leader = __ffsll((long long)pending) - 1;
                const uint32_t key = rdlane(h, leader);
                const uint64_t m = ballot(live && h == key);
                if ((m >> L) & 1) {
                    gmask = m;
                    const uint64_t below = m & ((1ull << L) - 1ull);
                    pred = below ? 63 - __clzll((long long)below) : -1;
                }
                pending &= ~m;
            }
            const uint32_t cand = pred >= 0 ? W.pos((uint32_t)pred) : (TAG ? (told & kPosMask) : told);
            STAMP_ADD(1, ts);
            // ok: verified match (4-byte compare); maybe: tag-equal table
            // candidate outside the ring, confirmed in the count round trip
            bool ok = false, maybe = false;
            if (live && !isIns && !term) {
                const bool distok = (U16 || (cand + kDistMax >= p)) && (!LINK || cand >= lk.candLow);
                if (distok) {
                    if (TAG && pred < 0 && !V.in_ring(cand, 4)) maybe = (told >> kPosBits) == mytag;
                    else ok = (V.rd4(cand) == w0);
                }
            }
            uint64_t sm = ballot(live && (term || ok || maybe));
            const uint64_t mm = ballot(maybe), tmk = ballot(term);
            STAMP_ADD(2, ts);
            // resolve the first stop; a tag-equal lane issues the count round
            // (with its 4-byte check) and drops out if the check fails
            int w;
            uint32_t ip = 0, cd = 0, maxb = 0, lim = 0, lit0 = 0;
            bool wasTest = false, early = false, beq = false;
            uint32_t eqb = 0;
            for (;;) {
                w = sm ? __ffsll((long long)sm) - 1 : 64;
                if (w == 64 || ((tmk >> w) & 1)) break;
                ip = rdlane(p, w);
                cd = rdlane(cand, w);
                wasTest = (ballot(isTest) >> w) & 1;
                // Catch-up and forward count in one round: with back = catch-up
                // length, LZ4_count from the caught-up position equals
                // back + count from ip+4 (the skipped bytes are known equal).
                {
                    const uint32_t lowL = !LINK ? 0u : (cd >= o0 ? lk.lowIn : lk.lowDict);
                    maxb = wasTest ? 0u : min(ip - anchor, cd > lowL ? cd - lowL : 0u);
                }
                lim = matchlimit - (ip + kMinMatch);
                V.cover(min(ip + kMinMatch + 256, n));
                // round-0 operands (the cd side is the global round trip)
                const bool needV = (mm >> w) & 1;
                uint32_t vx = 0;
                if (needV && L == 0) vx = ld32u(s + cd) ^ rdlane(w0, w);
                beq = false;
                if (L + 1 <= maxb) beq = V.rd1(ip - L - 1) == V.rd1(cd - L - 1);
                eqb = 0;
                if (4 * L < lim) {
                    const uint32_t x = V.rd4(ip + kMinMatch + 4 * L) ^ V.rd4(cd + kMinMatch + 4 * L);
                    eqb = x ? ((uint32_t)__builtin_ctz(x) >> 3) : 4u;
                    eqb = min(eqb, lim - 4 * L);
                }
                STAMP_ADD(3, ts);
                if (ST) acc[12] += (mm >> w) & 1;
                // while those loads fly: stage the literals assuming no catch-up
                lit0 = ip - anchor;
                early = lit0 <= 256 && op + 1 + ext_len(lit0) + lit0 + 64 <= O.flushed + kOutRing;
                if (early) stage_lits(V, O, anchor, 0, lit0, op + 1 + ext_len(lit0), false, 0);
                STAMP_ADD(4, ts);
                if (needV && (ballot(L == 0 && vx != 0) & 1)) {   // tag alias: not a match
                    if (ST) acc[11] += 1;
                    sm &= ~(1ull << w);
                    STAMP_ADD(5, ts);
                    continue;
                }
                if (ST) {   // round trip of the count loads (waited here)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                STAMP_ADD(5, ts);
                break;
            }
            const bool wTerm = (w < 64) && ((tmk >> w) & 1);
            const int wlim = (w == 64) ? 63 : (wTerm ? w - 1 : w);
            // table writes: last member of each hash group among lanes <= wlim
            if (wlim >= 0 && live && (int)L <= wlim) {
                const uint64_t later = gmask & ~mask_le(L) & mask_le((uint32_t)wlim);
                if (!later) {
                    if (U16) T16[h] = (uint16_t)p;
                    else Traw[h] = TAG ? (p | (mytag << kPosBits)) : p;
                }
            }
            WAVE_SYNC();
            STAMP_ADD(6, ts);
            if (w == 64) {  // no stop: continue the search
                W.k0 += 64 - ns;
                W.hasIns = 0; W.hasTest = 0;
                continue;
            }
            if (wTerm) goto last_literals;

            // ---------------- match found ----------------
            uint32_t back = 0, mc = 0;
            bool backDone = maxb == 0, cntDone = false;
            for (;;) {
                if (!backDone) {
                    const uint64_t fm = ballot(!beq);
                    if (fm) { back += (uint32_t)(__ffsll((long long)fm) - 1); backDone = true; }
                    else { back += 64; backDone = back >= maxb; }
                }
                if (!cntDone) {
                    const uint64_t nf = ballot(eqb < 4);
                    if (nf) {
                        const int f = __ffsll((long long)nf) - 1;
                        mc += 4 * (uint32_t)f + rdlane(eqb, f);
                        cntDone = true;
                    } else {
                        mc += 256;
                    }
                }
                if (backDone && cntDone) break;
                beq = false;
                eqb = 0;
                const uint32_t kk = back + L + 1;
                if (!backDone && kk <= maxb) beq = V.rd1(ip - kk) == V.rd1(cd - kk);
                const uint32_t rel = mc + 4 * L;
                if (!cntDone && rel < lim) {
                    const uint32_t x = V.rd4(ip + kMinMatch + rel) ^ V.rd4(cd + kMinMatch + rel);
                    eqb = x ? ((uint32_t)__builtin_ctz(x) >> 3) : 4u;
                    eqb = min(eqb, lim - rel);
                }
            }
            STAMP_ADD(7, ts);
            const uint32_t mcf = mc + back;          // LZ4_count from the caught-up start + 4
            const uint32_t lit = lit0 - back;
            const uint32_t litExt = ext_len(lit);
            const uint32_t mlExt = ext_len(mcf);
            if (limited) {
                if (!wasTest && op + 1 + lit + 8 + lit / 255 > cap) return 0;
                if (op + 1 + litExt + lit + 2 + 6 + (mcf + 240) / 255 > cap) return 0;
            }
            const uint32_t litPos = op + 1 + litExt;
            if (!early || litExt != ext_len(lit0)) {
                put_head(O, op, lit, mcf < 15 ? mcf : 15);
                WAVE_SYNC();
                stage_lits(V, O, anchor, 0, lit, litPos, true, litPos);
            } else {
                put_head(O, op, lit, mcf < 15 ? mcf : 15);
            }
            {   // offset + match-length bytes
                const uint32_t off = ip - cd, tpos = litPos + lit;
                O.flush_to(tpos);
                if (L < 2) O.put(tpos + L, L == 0 ? (off & 255) : (off >> 8));
                WAVE_SYNC();
                put_ext(O, tpos + 2, mlExt, mcf >= 15 ? (mcf - 15) % 255 : 0);
            }
            op = litPos + lit + 2 + mlExt;
            WAVE_SYNC();
            O.flush_to(op);
            STAMP_ADD(8, ts);
            const uint32_t ipe = ip + kMinMatch + mc;  // = caught-up start + mcf + 4
            anchor = ipe;
            if (ipe >= mflimitP1) goto last_literals;
            W = Win{1, 1, ipe - 2, ipe, ipe + 1, 0};
        }
    }
last_literals : {
    const uint32_t run = n - anchor;
    if (limited && op + run + 1 + (run + 240) / 255 > cap) return 0;
    put_head(O, op, run, 0);
    const uint32_t litPos = op + 1 + ext_len(run);
    WAVE_SYNC();
    stage_lits(V, O, anchor, 0, run, litPos, true, litPos);
    op = litPos + run;
    O.finish(op);
}
    return (int32_t)op;
}

// ---------------------------------------------------------------------------
// Lean encoder for the frame path: tagged u32 table, 65547 <= n <= 4 MiB.
// Same parse and bytes as encode_block (LZ4 1.9.3); the
// window is organised around ONE global round trip:
//   hash inputs   unaligned ds_read_b64 from a mirrored 2 KiB source ring
//                 (global loads when the window spans more than 1 KiB)
//   candidates    in-window predecessor: its bytes via ds_bpermute (exact);
//                 table entry: distance + 10-bit tag filter
//   round trip    verify word, both sides of the forward count, catch-up
//                 bytes and the literal bytes, all issued together
//   emit          coalesced byte stores straight into the block slot
// ---------------------------------------------------------------------------
typedef const __attribute__((address_space(1))) uint32_t __attribute__((aligned(1))) g_cu32u;
typedef const __attribute__((address_space(1))) uint64_t __attribute__((aligned(1))) g_cu64u;
typedef __attribute__((address_space(3))) uint64_t __attribute__((aligned(1))) l_u64u;
typedef __attribute__((address_space(3))) uint32_t __attribute__((aligned(1))) l_u32u;
typedef __attribute__((address_space(3))) uint16_t __attribute__((aligned(1))) l_u16u;
typedef __attribute__((address_space(3))) uint64_t l_u64;

constexpr uint32_t kSR = 2048;        // source ring bytes
// forward-count words the v5 round trip loads per side (the first 4 * this
// many bytes after the minimum match; longer matches take 256-byte rounds)
#ifndef LZ4MT_COUNT_LANES
#define LZ4MT_COUNT_LANES 32
#endif
constexpr uint32_t kCountLanes = LZ4MT_COUNT_LANES;
// catch-up bytes the round trip loads per side (the bytes just before ip
// and before the candidate); longer catch-ups take 64-byte rounds
#ifndef LZ4MT_CATCH_LANES
#define LZ4MT_CATCH_LANES 64
#endif
constexpr uint32_t kCatchLanes = LZ4MT_CATCH_LANES;
static_assert(kCatchLanes >= 1 && kCatchLanes <= 64, "catch-up lanes");
constexpr uint64_t kCatchMask = kCatchLanes >= 64 ? ~0ull : (1ull << kCatchLanes) - 1ull;
static_assert(kCountLanes >= 1 && kCountLanes <= 63, "count lanes");
constexpr uint32_t kSRMirror = 64;    // ring[kSR .. kSR+64) mirrors ring[0 .. 64)
// ds_mskor_rtn_b32 on two LDS dwords (one position half, one tag byte): each
// word becomes (word & ~mask) | data; returns the old words
__device__ __forceinline__ void mskor2_rtn(l_u32* w16, uint32_t m16, uint32_t d16, l_u32* w8, uint32_t m8,
                                           uint32_t d8, uint32_t& o16, uint32_t& o8) {
    asm volatile("ds_mskor_rtn_b32 %0, %2, %3, %4\n\t"
                 "ds_mskor_rtn_b32 %1, %5, %6, %7\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(o16), "=&v"(o8)
                 : "v"((uint32_t)(uintptr_t)w16), "v"(m16), "v"(d16), "v"((uint32_t)(uintptr_t)w8), "v"(m8), "v"(d8)
                 : "memory");
}

__device__ __forceinline__ uint32_t gld4u(g_cu8* p) { return *(g_cu32u*)p; }
__device__ __forceinline__ uint64_t gld8u(g_cu8* p) { return *(g_cu64u*)p; }

struct SrcRing {
    g_cu8* s;
    uint32_t n;
    l_u8* r;          // kSR + kSRMirror bytes
    uint32_t B;       // ring holds src[B, B + kSR), B a multiple of 512
    uint32_t pfPos;   // chunk prefetched into pf
    uint64_t pf;

    __device__ __forceinline__ uint64_t fetch(uint32_t c) const {
        const uint32_t pos = c + 8 * laneid();
        if (pos + 8 <= n) return gld8u(s + pos);
        uint64_t v = 0;
        for (uint32_t i = 0; i < 8; ++i)
            if (pos + i < n) v |= (uint64_t)s[pos + i] << (8 * i);
        return v;
    }
    __device__ __forceinline__ void store(uint32_t c, uint64_t v) {
        const uint32_t o = (c & (kSR - 1)) + 8 * laneid();
        *(l_u64*)(r + o) = v;
        if (o < kSRMirror) *(l_u64*)(r + kSR + o) = v;
    }
    __device__ __forceinline__ void init(uint32_t b0 = 0) {   // b0: a multiple of 512
        B = b0;
        for (uint32_t c = b0; c < b0 + kSR; c += 512) store(c, fetch(c));
        pfPos = b0 + kSR;
        pf = fetch(pfPos);
        WAVE_SYNC();
    }
    // make [lo, hi) readable (requires hi - lo <= 1024 and lo >= B)
    __device__ __forceinline__ void cover(uint32_t hi) {
        if (hi <= B + kSR) return;
        const uint32_t nb = (hi - kSR + 511) & ~511u;
        WAVE_SYNC();
        for (uint32_t c = (nb > B + kSR ? nb : B + kSR); c < nb + kSR; c += 512) store(c, c == pfPos ? pf : fetch(c));
        B = nb;
        pfPos = B + kSR;
        pf = fetch(pfPos);   // next advance's chunk, in flight
        WAVE_SYNC();
    }
    __device__ __forceinline__ uint64_t rd8(uint32_t pos) const { return *(l_u64u*)(r + (pos & (kSR - 1))); }
};

// ---------------------------------------------------------------------------
// Encoder v5: the frame path's encoder for 65547 <= n <= 4 MiB (same parse
// and bytes as encode_block, LZ4 1.9.3 SURVEY.md App. A),
// laid out for the fewest instructions per window:
//   * fixed lane roles: lane 0 INSERT, lane 1 TEST, lanes 2..63 SEARCH
//     probes k0 .. k0+61 (step 1 for the first 64 probes: p = sPos + L - 2)
//   * every LDS op is branch-free: lanes with nothing to do address their
//     own dummy slot (T[4096 + L]) instead of toggling EXEC
//   * the table is probed with the lane's FINAL entry as marker (position |
//     tag); a readback that differs flags a same-bucket collision, and the
//     exact predecessor resolution runs only when a collision reaches a lane
//     at or before the first stop (about 1 window in 20)
//   * ballots go straight to SGPRs (no v_cndmask + v_cmp per ballot)
//   * the previous sequence's bytes are stored during this window's round
//     trip, literal bytes taken from the LDS source ring
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t bal(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t sff1(uint64_t m) { return m ? (uint32_t)__builtin_ctzll(m) : 64u; }
// Table geometry per table type: lz4 1.9.3 uses byU32 (4096 entries,
// hash5) from 65 547 bytes up and byU16 (8192 entries, hash4) below.  An
// entry is position | tag << PB; the tag is 32 - PB more bits of the
// sequence's own hash.  T[kTE + L] is lane L's dummy slot.
// SPLIT (byU16 only): positions in a u16 array and 8-bit tags in a u8
// array (26 KiB of LDS in all: 6 waves per CU instead of 4); the marker
// readback compares positions only (distinct per live lane).
// P17: the byU32 table in 3 bytes per entry (u16 + u8 arrays, 12 KiB): a
// 17-bit position (mod 2^17) + a 7-bit tag, kept exact by a sweep every
// 32 KiB (sweep_p17) so that every live entry lies within 96 KiB of ip.
template <bool U16, bool SPLIT = false, bool LINK = false, bool P17 = false> struct V5Geo {
    static constexpr uint32_t kTE = U16 ? 8192u : 4096u;
    // LINK: positions in the block-dependent coordinates (64 KiB of history
    // before the block) need one more bit: 23-bit positions, 9-bit tags
    static constexpr uint32_t PB = P17 ? 17u : U16 ? 16u : (LINK ? kPosBits + 1 : kPosBits);
    static constexpr uint32_t PM = (1u << PB) - 1u;
    static constexpr bool SP = SPLIT || P17;                  // u16 + u8 storage
    static constexpr uint32_t TB = P17 ? 7u : SPLIT ? 8u : 32u - PB;   // tag bits
    // tag from the hash product (one multiply for hash and tag): the u32
    // table takes bits 42..51 of the hash5 product (bits 52..63 are the
    // hash); those bits depend on the word's first 28 bits only, so equal
    // words keep equal tags, and within one bucket equal low 28 bits force
    // equal words, so the filter is as sharp (profiles/r04htag_encoder_ab.txt).
    // The byU16 split table takes its hash4 product's bits 19 - TB .. 18 (B4
    // 218.0 -> 216.3 ms); not P17, whose 7 bits from the hash5 product filter
    // a little worse (132.0 -> 132.3 ms at B5; profiles/r04htsp_encoder_ab.txt)
    static constexpr bool HT = !SP || U16;
    static __device__ __forceinline__ uint32_t tag(uint32_t w0) {
        if constexpr (HT && U16) return ((w0 * 2654435761u) >> (19 - TB)) & ((1u << TB) - 1u);
        else if constexpr (HT) return (uint32_t)(((uint64_t)w0 << 24) * 889523592379ull >> (52 - TB)) & ((1u << TB) - 1u);
        else return (w0 * 0x85EBCA77u) >> (32 - TB);
    }
    l_u32* T;
    __device__ __forceinline__ l_u16* T16() const { return (l_u16*)T; }
    __device__ __forceinline__ l_u8* TG() const { return (l_u8*)T + 2 * (kTE + 64); }
    __device__ __forceinline__ uint32_t ld(uint32_t i) const {
        return SP ? ((uint32_t)T16()[i] | ((uint32_t)TG()[i] << 16)) : T[i];
    }
    __device__ __forceinline__ void st(uint32_t i, uint32_t e) const {
        if (SP) { T16()[i] = (uint16_t)e; TG()[i] = (uint8_t)(e >> 16); } else T[i] = e;
    }
    __device__ __forceinline__ uint32_t rb(uint32_t i) const { return SP ? (uint32_t)T16()[i] : T[i]; }
    // store e, return the entry it replaced (lane-ordered within a wave)
    __device__ __forceinline__ uint32_t xchg(uint32_t i, uint32_t e) const {
        if constexpr (SP) {
            const uint32_t s16 = (i & 1u) * 16u, s8 = (i & 3u) * 8u;
            uint32_t o16, o8;
            mskor2_rtn((l_u32*)T16() + (i >> 1), 0xFFFFu << s16, (e & 0xFFFFu) << s16, (l_u32*)TG() + (i >> 2),
                       0xFFu << s8, ((e >> 16) & 0xFFu) << s8, o16, o8);
            return ((o16 >> s16) & 0xFFFFu) | (((o8 >> s8) & 0xFFu) << 16);
        } else {
            return __hip_atomic_exchange(T + i, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
    }
    static constexpr uint32_t kRbMask = SP ? 0xFFFFu : 0xFFFFFFFFu;
    // P17: at T (a multiple of 32 KiB, every table write so far below T +
    // 32 KiB, every live entry at or above T - 96 KiB): entries more than
    // 64 KiB below T can never be a candidate again -- they become a marker
    // (T + 64 KiB mod 2^17) that reads as out of range until the next sweep
    // re-marks it.  Entries at or above T - 64 KiB (and those written ahead,
    // at or above T) keep their distance (< 2^17) exact.
    __device__ __forceinline__ void sweep(uint32_t Tp) const {
        const uint32_t L = laneid();
        const uint32_t mk = (Tp + 65536u) & PM;
        for (uint32_t i = L; i < kTE; i += 64) {
            const uint32_t d = (Tp - ld(i)) & PM;
            if (d > 65536u && d <= 98304u) st(i, mk);
        }
        WAVE_SYNC();
    }
    __device__ __forceinline__ void init(uint32_t e0) const {
        const uint32_t L = laneid();
        if (SP) {
            const uint32_t p2 = (e0 & 0xFFFFu) * 0x10001u, t4 = (e0 >> 16) * 0x01010101u;
            for (uint32_t i = L; i < kTE / 8; i += 64) ((l_u4*)T16())[i] = (v4u){p2, p2, p2, p2};
            for (uint32_t i = L; i < kTE / 16; i += 64) ((l_u4*)TG())[i] = (v4u){t4, t4, t4, t4};
        } else {
            for (uint32_t i = L; i < kTE / 4; i += 64) ((l_u4*)T)[i] = (v4u){e0, e0, e0, e0};
        }
    }
};

// one encoded sequence whose bytes are stored during the next round trip
// (few loop-carried fields; the layout is derived at store time).  The
// extension lengths come from the window, which computes them for its own
// output cursor anyway: the layout then needs no division by 255 (two
// quarter-rate v_mul_hi_u32 and two v_mad_u64_u32 fewer per sequence); with
// the do-while byte rounds below and the hash input read without an else
// branch, k_encode 151.1 -> 146.7 ms at 8 GiB B7 (136.3 vs 139.6 at B6;
// profiles/r06/r06k_trim_ab.txt)
struct PendSeq {
    uint32_t op, lit, mcf, off, anchor;
    uint32_t litExt, mlExt;   // ext_len(lit), ext_len(mcf)
};
template <bool R8> struct SeqLayout {
    uint32_t total, a1, a2, token, litRem, mlRem, off;
    __device__ __forceinline__ explicit SeqLayout(const PendSeq& e) {
        a1 = 1 + e.litExt;
        a2 = a1 + e.lit;
        total = a2 + 2 + e.mlExt;
        token = ((e.lit < 15 ? e.lit : 15) << 4) | (e.mcf < 15 ? e.mcf : 15);
        if (R8) {   // (lit - 15) % 255 mod 256, as it is stored (-255 = 1 mod 256): no multiply
            litRem = e.lit + 240 + e.litExt;
            mlRem = e.mcf + 240 + e.mlExt;
        } else {    // (lit - 15) % 255 when an extension exists
            litRem = e.lit + 240 - __umul24(255u, e.litExt);
            mlRem = e.mcf + 240 - __umul24(255u, e.mlExt);
        }
        off = e.off;
    }
};
// byte x of a sequence: token | literal-length ext | literals | offset | match-length ext
// (flat selects: a nested ?: here is turned into an EXEC-mask branch)
template <bool R8>
__device__ __forceinline__ uint32_t pend_byte(const SeqLayout<R8>& e, uint32_t x, uint32_t litByte) {
    const uint32_t vM = x + 1 < e.total ? 255u : e.mlRem;
    const uint32_t vL = x + 1 < e.a1 ? 255u : e.litRem;
    const uint32_t vO = x == e.a2 ? e.off & 255u : e.off >> 8;
    uint32_t v = x < e.a2 + 2 ? vO : vM;
    v = x < e.a2 ? litByte : v;
    v = x < e.a1 ? vL : v;
    asm volatile("" : "+v"(v));
    return x == 0 ? e.token : v;
}
// The literal byte is made opaque right after its load, so the select chain
// stays selects (no load sunk into a branch) and the store waits only on the
// counter of its own load: LDS (ring, the common case) never waits on the
// round-trip loads in flight.
template <bool R8>
__device__ __forceinline__ void store_pend(const PendSeq& p, const SrcRing& V, g_cu8* __restrict__ s,
                                           g_u8* __restrict__ d) {
    const uint32_t L = laneid();
    // the layout in VALU (uniform values in VGPRs): the scalar unit is the
    // CU's busiest port in the encoder window, the vector ALU is not
    PendSeq q = p;
    asm volatile("" : "+v"(q.lit), "+v"(q.mcf), "+v"(q.off), "+v"(q.litExt), "+v"(q.mlExt));
    const SeqLayout<R8> e(q);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readfirstlane((int)e.total);
    // a sequence is at least 5 bytes: the first round always runs (no
    // zero-trip test before the loop)
    if (p.anchor >= V.B && p.anchor + p.lit <= V.B + kSR) {
        uint32_t base = 0;
        do {
            const uint32_t x = min(base + L, e.total - 1);   // lanes past the end repeat the last byte
            uint32_t lv = V.r[(p.anchor + x - e.a1) & (kSR - 1)];
            asm volatile("" : "+v"(lv));
            // (plain stores: non-temporal ones saved 0.3 % of k_encode but
            // reach HBM uncombined, profiles/r03s_enc_nt_ab.txt; with no
            // stores at all the encoder is only 1.4 % faster)
            d[p.op + x] = (uint8_t)pend_byte(e, x, lv);
            base += 64;
        } while (base < total);
    } else {   // literals no longer (or not yet) in the ring: global bytes
        uint32_t base = 0;
        do {
            const uint32_t x = min(base + L, e.total - 1);
            uint32_t lv = s[(x >= e.a1 && x < e.a2) ? p.anchor + x - e.a1 : p.anchor];
            asm volatile("" : "+v"(lv));
            d[p.op + x] = (uint8_t)pend_byte(e, x, lv);
            base += 64;
        } while (base < total);
    }
}

// LINK: one step of LZ4_compress_fast_continue (block-dependent frames):
// positions in the coordinates of k_encode_linked (block at o0 = 65536, its
// 64 KiB history below), the table carried in T unless lk.fresh, candidates
// bounded by lk (see LinkArgs); n = o0 + block length.
// PUB (the block-sharded streamed gather, lz4mt_shard.hip): every time the
// output crosses a multiple of kPubBytes, the bytes written so far are
// published -- the wave drains its stores, writes its XCD's L2 back (agent
// release) and stores the byte count to *pub (relaxed, agent scope): a
// concurrent kernel that reads *pub and then (after its own agent acquire,
// e.g. a new launch) the slot's bytes below it sees them final
// (MI355X_MICROARCH.md, valid hand-off forms).
constexpr uint32_t kPubShift = 16;   // publish every 64 KiB of output
// pub[b] at the end of block b: the stored size | kPubDone, or kPubDone |
// kPubRaw when the block is stored raw (its source bytes are the payload)
[[maybe_unused]] constexpr uint32_t kPubDone = 0x80000000u, kPubRaw = 0x40000000u, kPubLen = 0x3FFFFFFFu;
__device__ __forceinline__ void publish_progress(uint32_t* pub, uint32_t v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (laneid() == 0) __hip_atomic_store(pub, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// XH (LINK only): the history below o0 is the block's own bytes at
// p - o0 + lk.shift (the reference's -BD buffer with 1 / 4 MiB blocks,
// LZ4MT_AMD_BD_REFERENCE): every candidate-side load goes through xld4 /
// xld1, and the carried entries' tags are recomputed from the bytes those
// positions now hold (lz4 compares the memory as it is, not as it was).
// XCHG (the product path): the table probe is ONE LDS exchange per lane
// (ds_wrxchg_rtn_b32; on the split u16 + u8 tables a masked OR with return,
// ds_mskor_rtn_b32, on the dword of the lane's position half and on the one of
// its tag byte).  A wave's same-address exchanges take effect in ascending
// lane order on gfx950 (tools/probe/lds_xchg_order.hip, lds_mskor_order.hip:
// 6.4 M lanes, every one), lanes are in position order, so each lane gets
// exactly the entry LZ4's sequential inserts leave for it -- its in-window
// predecessor's mark, or the table's -- with no readback and no predecessor
// resolution.  That order is not architected: encoder_path() checks it once
// per device (k_xchg_order) and runs the !XCHG instantiation -- read, write
// the marker, read back, resolve same-bucket predecessors exactly -- when the
// check fails (or LZ4MT_AMD_ENC_PROBE=readback forces it).
// DUP: no effect on the code; a separate instantiation for a kernel that
// must not share (and so outline) another kernel's one (k_encode_stream).
// (k_decode_walk, k_xxh32_walked; ctl words described at k_decode_walk)
// waits until records [0, need) are published or the walk ended; returns the
// published count (0 after 30 s, which the caller treats as the end).  The
// walker publishes ctl[0] = count (| kWalkEnded at the end) with agent-scope
// atomics behind a release fence; this polls it with relaxed agent loads and
// takes ONE agent acquire once it matches.  ctl is uncached device memory
// (DecodeBuffers::ensure_ctl): a poll is served by the reader's own XCD L2,
// and with cached memory that copy stayed stale until the 30 s bound.
constexpr uint32_t kWalkEnded = 0x80000000u;
__device__ __forceinline__ uint32_t walked_wait(uint32_t* ctl, uint32_t need) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        uint32_t v = 0;
        if (laneid() == 0) v = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
        if ((v & ~kWalkEnded) >= need || (v & kWalkEnded)) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every lane: the records as published
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return v & ~kWalkEnded;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull) {
#if LZ4MT_WALK_DIAG
            if (laneid() == 0) {
                __hip_atomic_fetch_add(ctl + 5, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(ctl + 6, need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(ctl + 7, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#endif
            return 0;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}
// the walker's publication: its records were stored write-through (sc1), so
// waiting for them is the whole release -- an agent release fence here
// (buffer_wbl2) also wrote back every output line the decoders had dirtied
// in the walker's XCD L2, once per publication: B7 decompress 152 GiB/s
__device__ __forceinline__ void walk_publish(uint32_t* ctl, uint32_t v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    (void)__hip_atomic_exchange(ctl, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// SIMD-mate priority (encode_block_v5, byU32 blocks >= 1 MiB).  The waves
// sharing a SIMD issue oldest first, so with one generation of 2048 blocks
// (8 GiB of 4 MiB blocks, 8 waves per CU) the younger wave of each pair is
// starved while both run: slot-0 blocks ended at 118.6 ms on average,
// slot-1 blocks at 137.9, and the kernel at 146.3 (per-block wall clocks of
// the product kernel, profiles/r06/r06t_tail.txt).  Each wave publishes
// its projected finish time (a 100 MHz wall clock, linear in its input
// progress) every 1/128 of its block and takes the SIMD's issue priority
// (s_setprio by rank) while it is projected to finish after its SIMD-mates,
// so pairs end together: k_encode 146.0 -> 139.8 ms at B7, 136.2 -> 132.5
// at B6; at B5 / B4 (many generations, 2-3 and 1-2 waves per SIMD) it cost
// 2-5 %, so it is not used there (profiles/r06/r06tu_simd_priority_ab.txt).
// Slots: [SIMD key: XCC, SE, SH, CU, SIMD] x 16 wave slots.  A finished wave
// clears its slot; a slot whose projected finish is already past (a previous
// launch) is not a live SIMD-mate, so no reset between launches is needed.
constexpr uint32_t kPrioSimds = 8 * 8 * 2 * 16 * 4;
__device__ uint32_t g_simdFinish[kPrioSimds * 16];
struct SimdPrio {
    uint32_t base, slot;   // this SIMD's 16 slots, this wave's slot
    uint64_t t0;
    __device__ __forceinline__ void start() {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
        const uint32_t key = ((((xcc & 7) * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 15)) * 4 +
                             ((hw >> 4) & 3);
        base = key * 16;
        slot = hw & 15;
        t0 = __builtin_amdgcn_s_memrealtime();
    }
    // done / total of this wave's bytes are parsed
    __device__ __forceinline__ void tick(uint32_t done, uint32_t total) const {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        const float frac = (float)done / (float)total;
        const uint32_t fin = (uint32_t)t0 + (uint32_t)((float)(uint32_t)(now - t0) / (frac > 1e-3f ? frac : 1e-3f));
        const uint32_t L = laneid();
        if (L == 0) __hip_atomic_store(g_simdFinish + base + slot, fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if LZ4MT_EXP_CUPRIO   // rank among the CU's waves (4 SIMDs x 16 slots), priority = rank / 2
        const uint32_t cb = base & ~63u;
        const uint32_t e = __hip_atomic_load(g_simdFinish + cb + L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool live = cb + L != base + slot && (int32_t)(e - (uint32_t)now) > 0;
        const uint32_t rank = (uint32_t)__builtin_popcountll(bal(live && (int32_t)(e - fin) < 0)) >> 1;
#else
        const uint32_t e = L < 16 ? __hip_atomic_load(g_simdFinish + base + L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : 0u;
        // live SIMD-mates projected to finish before this wave
        const bool live = L < 16 && L != slot && (int32_t)(e - (uint32_t)now) > 0;
        const uint32_t rank = (uint32_t)__builtin_popcountll(bal(live && (int32_t)(e - fin) < 0));
#endif
        if (rank >= 3) __builtin_amdgcn_s_setprio(3);
        else if (rank == 2) __builtin_amdgcn_s_setprio(2);
        else if (rank == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    }
    __device__ __forceinline__ void done() const {
        if (laneid() == 0) __hip_atomic_store(g_simdFinish + base + slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_setprio(0);
    }
};
template <bool ST, bool U16, bool SPLIT = false, bool LINK = false, bool P17 = false, bool PUB = false,
          bool XH = false, bool XCHG = true, bool DUP = false>
__device__ int32_t encode_block_v5(g_cu8* __restrict__ s, uint32_t n, g_u8* __restrict__ d, uint32_t cap,
                                   l_u32* __restrict__ T, l_u8* __restrict__ R, uint64_t* acc,
                                   LinkArgs lk = LinkArgs{0, 0, 0, true}, uint32_t* pub = nullptr) {
    using G = V5Geo<U16, SPLIT, LINK, P17>;
    const G tab{T};
    const uint32_t L = laneid();
    uint64_t ts = STAMP_T();
    const uint32_t o0 = LINK ? kLinkO0 : 0u;   // position of the block's first byte
    // candidate-side loads (a candidate may lie in the history)
    auto xld4 = [&](uint32_t pos) -> uint32_t {
        if constexpr (!XH) {
            return gld4u(s + pos);
        } else {
            if (pos >= o0) return gld4u(s + pos);
            if (pos + 4 <= o0) return gld4u(s + pos + lk.shift);
            uint32_t v = 0;   // straddles the history's end: the rest is the block's start
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t q = pos + j;
                v |= (uint32_t)s[q < o0 ? q + lk.shift : q] << (8 * j);
            }
            return v;
        }
    };
    auto xld1 = [&](uint32_t pos) -> uint32_t {
        if constexpr (!XH) return s[pos];
        else return s[pos < o0 ? pos + lk.shift : pos];
    };
    const uint32_t blen = n - o0;
    const uint32_t bound = blen + blen / 255 + 16;
    const bool limited = cap < bound;
    if (blen < (uint32_t)kMinLength) {   // too short to search: one literal run (1.9.3 _last_literals)
        if (limited && (LINK && blen == 0 ? cap == 0 : blen + 1 + (blen + 240) / 255 > cap)) return 0;
        if (L == 0) d[0] = (uint8_t)(blen << 4);
        for (uint32_t x = L; x < blen; x += 64) d[1 + x] = s[o0 + x];
        return (int32_t)(blen + 1);
    }
    if (!LINK || lk.fresh) {
        // a fresh entry is the block's position 0 -- a real candidate in LZ4 1.9.3
        tab.init(o0 | (G::tag(gld4u(s + o0)) << G::PB));
    }
    if constexpr (XH) {
        if (!lk.fresh && lk.shift) {   // history entries: the tag of the bytes they point at now
            for (uint32_t i = L; i < G::kTE; i += 64) {
                const uint32_t e = tab.ld(i), pos = e & G::PM;
                if (pos != 0 && pos < o0) tab.st(i, pos | (G::tag(xld4(pos)) << G::PB));
            }
            WAVE_SYNC();
        }
    }
    SrcRing V{s, n, R, 0, 0, 0};
    V.init(o0);
    // SIMD-mate priority: the byU32 encoder on blocks of 1 MiB and more
    // (LZ4MT_NO_SIMD_PRIO: off, for A/B builds)
#ifndef LZ4MT_NO_SIMD_PRIO
    constexpr bool kPrioT = !ST && !U16 && !SPLIT && !LINK && !P17 && !XH;
#else
    constexpr bool kPrioT = false;
#endif
    const bool prioOn = kPrioT && blen >= (1u << 20);
    SimdPrio prio{};
    uint32_t tickShift = 31;
    if (prioOn) {
        prio.start();
#ifndef LZ4MT_EXP_PRIO_SHIFT
#define LZ4MT_EXP_PRIO_SHIFT 7
#endif
        tickShift = (31 - __builtin_clz(blen)) - LZ4MT_EXP_PRIO_SHIFT;   // a check every 1/128 of the block
    }
    const uint32_t capL = limited ? cap : 0xFFFFFFFFu;   // one SGPR for the per-sequence margin test
    const uint32_t mflimitP1 = n - kMfLimit + 1;
    const uint32_t matchlimit = n - kLastLiterals;
    const uint32_t last4 = n - 4;
    const uint32_t dumIdx = G::kTE + L;
    uint32_t anchor = o0, op = 0;
    PendSeq pe{};
    bool havePe = false;
    bool done = false, fail = false;
    // (the layout is settled right after the count: deferring it into the
    // next round trip's shadow cost 3.2 ms, profiles/r04late_encoder_layout_ab.txt)
    auto store_pending = [&]() {
        // remainders mod 256 without a multiply: B4 -2.6 %, B5 -1.4 %; on the
        // byU32 encoder +0.5 % (profiles/r06/r06pq_quarter_rate_ab.txt)
#ifndef LZ4MT_EXP_R8ALL
        store_pend<U16 || P17>(pe, V, s, d);
#else
        store_pend<LZ4MT_EXP_R8ALL != 0>(pe, V, s, d);
#endif
        havePe = false;
    };
    // window: lane 0 INSERT insPos, lane 1 TEST testPos, lane L >= 2 SEARCH
    // probe k0 + L - 2 (at sBase + F(k) - F(k0), sBase = first search position)
    // window state: sBase, k0 (+ s0, j1 derived from it) and the mode
    // (0 continuation: search only; 1 after a match ending at sBase - 1:
    // INSERT sBase - 3, TEST sBase - 1; 2 first window: INSERT 0)
    uint32_t sBase = o0 + 1, k0 = 0, s0 = 1, j1 = 65, mode = 2;
    // 61 * s0 + max(0, 61 - j1): the last SEARCH probe's offset from sBase,
    // carried as loop state (61 after every match) rather than recomputed
    uint32_t spanHi = 61;
    uint32_t nextSweep = 32768;   // P17
    // ONE exit and no continue: the structurizer then needs no flow
    // variables and the loop-carried state stays in place across windows
    while (!done) {
      // windows without a stop (continuations) loop here, inside: the
      // match-path state (anchor, op, pe) is not touched by them
      uint32_t w, ip, cd, maxb, cw, iw, bi, bc;
      bool wTerm;
      do {
        if (ST) acc[10] += 1;
        if (P17) {
            while (sBase >= nextSweep) {   // (long matches cross several)
                tab.sweep(nextSweep);
                nextSweep += 32768;
            }
        }
        // ---- probe positions.  SEARCH lane L probes k = k0 + j (j = L - 2) at
        // sBase + j*s0 + max(0, j - j1): the step s0 = step(k0) rises by one at
        // most once inside a window (at j = j1; never in the k0 = 0 window)
        const uint32_t j = L - 2;
        const int32_t jx = (int32_t)j - (int32_t)j1;
        // j < 62 and the step s0 < 2^24: a full-rate 24-bit multiply (lanes 0
        // and 1 wrap j, but take the INSERT / TEST position below)
        uint32_t p = sBase + __umul24(j, s0) + (uint32_t)max(jx, 0);
        const uint32_t step = s0 + (jx >= 0 ? 1u : 0u);
        const uint32_t sHi = sBase + spanHi;
        const bool insOn = mode != 0;
        const uint32_t insPos = mode == 2 ? o0 : sBase - 3, testPos = sBase - 1;
        p = L == 0 ? insPos : (L == 1 ? testPos : p);
        // lane predicates as wave masks (SALU), turned back into per-lane
        // conditions with inverse_ballot (the mask is the select's condition):
        // no 0/1 materialisation chains.  Lane 0 / 1's bits come straight
        // from the mode (2: INSERT only, 1: both, 0: neither)
        const uint64_t roleM = (uint64_t)((0x130u >> (4 * mode)) & 3u);
        const uint64_t liveM = (bal(p <= mflimitP1) & ~3ull) | roleM;
        const uint64_t tmk = bal(p + step > mflimitP1) & liveM & ~3ull;
        const bool live = __builtin_amdgcn_inverse_ballot_w64(liveM);
        const bool term = __builtin_amdgcn_inverse_ballot_w64(tmk);
        const uint32_t lo = insOn ? insPos : sBase;
        const uint32_t hi = (sHi < mflimitP1 ? sHi : mflimitP1) + 8;
        uint64_t v8;
        // two if-regions and no else: the ring read is issued on both paths
        // (wasted, harmless, in the rare wide case), so the common path
        // carries no structurizer flow variable
        const bool wide = hi - lo > 1024;
        if constexpr (kPrioT) {   // the check rides on the ring's advance (every 512 B of input or more)
            if (!wide && hi > V.B + kSR) {
                const uint32_t oldB = V.B;
                V.cover(hi);
                if (prioOn && ((oldB ^ V.B) >> tickShift)) prio.tick(V.B - o0, blen);
            }
        } else {
            if (!wide) V.cover(hi);
        }
        v8 = V.rd8(p);
        if (wide) {   // wide window (long searches): hash inputs straight from global
            if (ST) acc[13] += 1;
            v8 = gld8u(s + (p < n - 8 ? p : n - 8));
            uint32_t a = (uint32_t)v8, b = (uint32_t)(v8 >> 32);
            asm volatile("" : "+v"(a), "+v"(b));   // land it here, not at the join
            v8 = ((uint64_t)b << 32) | a;
        }
        const uint32_t w0 = (uint32_t)v8;
        uint32_t h, tg;
        if constexpr (G::HT && U16) {   // one product: hash4 = bits 19..31, tag = the TB bits below
            const uint32_t P = w0 * 2654435761u;
            h = P >> 19;
            tg = (P >> (19 - G::TB)) & ((1u << G::TB) - 1u);
        } else if constexpr (G::HT) {   // one product: hash5 = bits 52..63, tag = the TB bits below
            const uint64_t P = (v8 << 24) * 889523592379ull;
            h = (uint32_t)(P >> 52);
            tg = (uint32_t)(P >> (52 - G::TB)) & ((1u << G::TB) - 1u);
        } else {
            h = lz4_hash<U16>(w0, (uint32_t)(v8 >> 32));
            tg = G::tag(w0);
        }
        const uint32_t mark = (P17 ? p & G::PM : p) | (tg << G::PB);   // the lane's final table entry
        // ---- table probe: read, write the marker, read back (LDS ops of a wave run in order)
        const uint32_t ti = live ? h : dumIdx;
        uint32_t told;
        uint64_t pend = 0;   // same-bucket collisions inside the window (XCHG: none to resolve)
        if constexpr (XCHG) {
            told = tab.xchg(ti, mark);
        } else {
            told = tab.ld(ti);
            tab.st(ti, mark);
            WAVE_SYNC();
            const uint32_t sv = tab.rb(ti);
            pend = bal(sv != (mark & G::kRbMask));
        }
        const uint32_t dq = (p - told) & G::PM;   // P17: the distance, exact below 2^17
        uint32_t cand = P17 ? p - dq : told & G::PM;
        const uint64_t cokM = bal((P17 ? dq <= kDistMax : cand + kDistMax >= p) && (!LINK || cand >= lk.candLow)) &
                              liveM & ~tmk & ~1ull;
        uint64_t mm = cokM & bal((told >> G::PB) == (mark >> G::PB));
        bool maybe = __builtin_amdgcn_inverse_ballot_w64(mm);
        uint64_t sm = mm | tmk;
        STAMP_ADD(0, ts);
        // ---- resolve the first stop.  Exact in-window predecessors are
        // resolved (once) whenever a collision reaches the current stop
        // candidate -- also after a tag alias moved the stop further out.
        // The round trip: verify word + forward count words, catch-up bytes;
        // the previous sequence's stores go out behind them.
        w = 64;
        bool dd = false, twDone = false, twRedo = false;
        uint64_t gmask, aliased = 0;   // gmask: read only after dd set it
        // table writes for stop w: lanes past the stop put the old entry
        // back; on a collision (or when redone after a tag alias moved the
        // stop) the lanes up to the stop re-insert (last member of each group)
        // pB: the position of lane wlim (the last lane whose insert stays)
        auto table_writes = [&](uint32_t ws, bool wsTerm, uint32_t pB) {
            // (an SGPR-pinned version of this, w - ((tmk >> w) & 1) under an
            // asm "+s" constraint, drops a v_readfirstlane but costs 1 ms:
            // profiles/r04tidy_encoder_ab.txt)
            const int wlim = (ws == 64) ? 63 : (wsTerm ? (int)ws - 1 : (int)ws);
            const bool le = (int)L <= wlim;
            if constexpr (XCHG) {
                // after an alias moved the stop: the lanes up to it insert again
                // (exchanges, so the last of each bucket wins)
                if (twRedo) (void)tab.xchg((live && le) ? h : dumIdx, mark);
                // lanes past the stop: the first of each bucket puts back the
                // entry it displaced (the last mark up to the stop, or the
                // table's entry); a later one displaced a lane past the stop.
                // Lanes are in position order and every entry a lane can
                // displace is an older table entry or an earlier lane's
                // mark, so "displaced by no lane past the stop" is "its
                // position is at most lane wlim's" (P17 keeps positions
                // mod 2^17: compare distances from p)
                const bool first = P17 ? dq >= p - pB : (told & G::PM) <= pB;
                tab.st((live && !le && first) ? h : dumIdx, told);
            } else {
                tab.st((live && !le) ? h : dumIdx, told);
                if (pend || twRedo) {
                    const uint64_t upto = wlim < 0 ? 0ull : mask_le((uint32_t)wlim);
                    const bool lastM = !dd || !(gmask & ~mask_le(L) & upto);
                    tab.st((live && le && lastM) ? h : dumIdx, mark);
                }
            }
            WAVE_SYNC();
        };
        // ip .. bc and wTerm are set on the path that reads them (a stop
        // inside the window): no per-window zeroing
        bool again = true;
        while (again) {
            w = sff1(sm);
            if (!dd && (pend & mask_le(w < 63 ? w : 63))) {
                if (ST) acc[12] += 1;
                dd = true;
                int pred = -1;
                gmask = 1ull << L;
                uint64_t todo = pend;
                while (todo) {   // one iteration per group of equal hashes
                    const uint32_t key = rdlane(h, (int)sff1(todo));
                    const uint64_t m = bal(live && h == key);
                    const bool inG = (m >> L) & 1;
                    const uint64_t below = m & ((1ull << L) - 1ull);
                    pred = inG ? (below ? 63 - __clzll((long long)below) : -1) : pred;
                    gmask = inG ? m : gmask;
                    todo &= ~m;
                }
                const int pi = (pred < 0 ? 0 : pred) * 4;
                const uint32_t pw = (uint32_t)__builtin_amdgcn_ds_bpermute(pi, (int)w0);   // predecessor's bytes
                const uint32_t pp = (uint32_t)__builtin_amdgcn_ds_bpermute(pi, (int)p);    // and position
                const bool ok = live && L != 0 && !term && pred >= 0 && pp + kDistMax >= p && pw == w0 &&
                                (!LINK || pp >= lk.candLow);
                maybe = maybe && pred < 0;
                cand = pred >= 0 ? pp : cand;
                mm = bal(maybe);
                sm = (bal(ok) | mm | tmk) & ~aliased;
            } else {
                wTerm = w < 64 && ((tmk >> w) & 1);
                again = false;
                if (w < 64 && !wTerm) {
                    ip = rdlane(p, (int)w);
                    cd = rdlane(cand, (int)w);
                    {   // catch-up bound: lz4's lowLimit for the candidate's side
                        const uint32_t lowL = !LINK ? 0u : (cd >= o0 ? lk.lowIn : lk.lowDict);
                        maxb = w == 1 ? 0u : min(ip - anchor, cd > lowL ? cd - lowL : 0u);
                    }
                    // lane 0: verify word; lanes 1 .. kCountLanes: count words; the
                    // rest repeat lane 0's address (no further lines touched)
                    const bool cOn = L <= kCountLanes;
                    const uint32_t ci = cOn ? cd + 4 * L : cd, ii = cOn ? ip + 4 * L : ip;
                    const bool bOn = L < maxb && L < kCatchLanes;
                    // every side from global memory: reading the near side(s)
                    // from the LDS ring when they lie in it was slower
                    // (profiles/r03j_encoder_ring_rt_ab.txt, r04s_encoder_ip_ring_ab.txt)
                    cw = xld4(ci < last4 ? ci : last4);
                    iw = gld4u(s + (ii < last4 ? ii : last4));
                    uint32_t bix = bOn ? ip - L - 1 : o0, bcx = bOn ? cd - L - 1 : o0;   // (o0: a byte of the block itself)
                    asm volatile("" : "+v"(bix), "+v"(bcx));   // 32-bit offsets, SGPR-base loads
                    bi = s[bix];
                    bc = xld1(bcx);
                    if (havePe) store_pending();
                    table_writes(w, false, ip);   // in the round trip's shadow; redone if w moves
                    twDone = true;
                    if (((mm >> w) & 1) && rdlane(cw, 0) != rdlane(w0, (int)w)) {   // tag alias: no match here
                        if (ST) acc[11] += 1;
                        // drain this try's loads here, so the loop head's load
                        // registers carry nothing pending into the common path
                        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
                        aliased |= 1ull << w;
                        sm &= ~(1ull << w);
                        again = true;
                        twDone = false;
                        twRedo = true;
                    }
                }
            }
        }
        if (havePe) store_pending();
        // no stop in the window (w == 64): every insert stays, nothing to put
        // back -- unless an alias moved the stop here after the lanes past the
        // old one were put back (twRedo: they insert again)
        if (!twDone && (!XCHG || w < 64 || twRedo)) table_writes(w, wTerm, rdlane(p, (int)(w < 64 ? w - 1 : 63)));
        STAMP_ADD(1, ts);
        STAMP_ADD(2, ts);
        if (w == 64) {   // no stop: the search goes on
            sBase += 62 * s0 + (62 > j1 ? 62 - j1 : 0u);
            k0 += 62;
            s0 = (63 + k0) >> 6;   // k0 >= 62: no max(1, .) needed
            j1 = (k0 < 65 ? 65u : ((k0 - 1) & ~63u) + 65) - k0;
            mode = 0;
            spanHi = 61 * s0 + (61 > j1 ? 61 - j1 : 0u);
        }
      } while (w == 64);
        if (wTerm) {
            done = true;
        } else {
            // ---- catch-up (backwards) and LZ4_count (forwards from ip + 4).
            // bi/bc are consumed on every path, so no load of this window is
            // left pending into the next window's round trip.
            asm volatile("" ::"v"(bi), "v"(bc));
            uint64_t fm = ~(bal(L < maxb) & bal(bi == bc)) & kCatchMask;
            uint32_t back = 0;
            if (kCatchLanes < 64 && fm == 0) {   // every loaded byte matched, the limit lies beyond them
                back = kCatchLanes;
                const uint32_t kb = back + L + 1;
                const bool on = kb <= maxb;
                fm = ~bal(on && s[on ? ip - kb : o0] == xld1(on ? cd - kb : o0));
            }
            while (fm == 0 && back + 64 < maxb) {   // catch-up longer than 64 bytes
                back += 64;
                const uint32_t kb = back + L + 1;
                const bool on = kb <= maxb;
                fm = ~bal(on && s[on ? ip - kb : o0] == xld1(on ? cd - kb : o0));
            }
            back = fm ? back + (uint32_t)__builtin_ctzll(fm) : maxb;
            const uint32_t lim = matchlimit - (ip + kMinMatch);
            uint32_t mc;
            {
                const uint32_t rel = 4 * L - 4;
                const uint32_t x = cw ^ iw;
                uint32_t e = min(x ? ((uint32_t)__builtin_ctz(x) >> 3) : 4u, lim - rel);
                e = rel < lim ? e : 0u;   // (lane 0's e is masked out below)
                const uint64_t nf = bal(e < 4) & (mask_le(kCountLanes) & ~1ull);
                if (nf) {
                    const uint32_t f = (uint32_t)__builtin_ctzll(nf);
                    mc = 4 * (f - 1) + rdlane(e, (int)f);
                } else {
                    mc = 4 * kCountLanes;
                    uint64_t nf2 = 0;
                    while (!nf2) {   // long match: 256 bytes per round
                        const uint32_t r2 = mc + 4 * L;
                        const uint32_t a2 = ip + kMinMatch + r2, c2 = cd + kMinMatch + r2;
                        const uint32_t x2 = gld4u(s + (a2 < last4 ? a2 : last4)) ^ xld4(c2 < last4 ? c2 : last4);
                        uint32_t e2 = min(x2 ? ((uint32_t)__builtin_ctz(x2) >> 3) : 4u, lim - r2);
                        e2 = r2 < lim ? e2 : 0u;
                        nf2 = bal(e2 < 4);
                        mc += nf2 ? 4 * (uint32_t)__builtin_ctzll(nf2) + rdlane(e2, (int)__builtin_ctzll(nf2))
                                  : 256u;
                    }
                }
            }
            STAMP_ADD(3, ts);
            // ---- sequence layout (stored during the next round trip)
            const uint32_t lit = ip - anchor - back, mcf = mc + back;
            pe.lit = lit;
            pe.mcf = mcf;
            pe.off = ip - cd;
            pe.anchor = anchor;
            {
                const uint32_t litExt = ext_len(lit), mlExt = ext_len(mcf);
                pe.litExt = litExt;
                pe.mlExt = mlExt;
                // 1.9.3's limitedOutput margins; both hold whenever
                // op + 2 (lit + mcf) + 16 <= cap, so the exact test runs rarely
                if (op + 2 * (lit + mcf) + 16 > capL) {
                    fail = (w != 1 && op + 1 + lit + 8 + lit / 255 > cap) ||
                           (op + 1 + litExt + lit + 2 + 6 + (mcf + 240) / 255 > cap);
                }
                pe.op = op;
                havePe = !fail;
                if constexpr (PUB) {   // every sequence before this one has been stored: [0, op) is final
                    if ((op ^ (op + 1 + litExt + lit + 2 + mlExt)) >> kPubShift) publish_progress(pub, op);
                }
                op += 1 + litExt + lit + 2 + mlExt;
            }
            const uint32_t ipe = ip + kMinMatch + mc;
            anchor = ipe;
            done = fail || ipe >= mflimitP1;
            mode = 1;
            sBase = ipe + 1;
            k0 = 0;
            s0 = 1;
            j1 = 65;
            spanHi = 61;
            STAMP_ADD(4, ts);
        }
    }
    if (prioOn) prio.done();
    if (fail) return 0;
    if (havePe) store_pending();
    // ---- last literals
    {
        const uint32_t run = n - anchor;
        if (limited && op + run + 1 + (run + 240) / 255 > cap) return 0;
        const uint32_t ext = ext_len(run), rem = run >= 15 ? (run - 15) % 255 : 0u;
        if (L == 0) d[op] = (uint8_t)((run < 15 ? run : 15) << 4);
        for (uint32_t x = L; x < ext; x += 64) d[op + 1 + x] = (uint8_t)(x + 1 < ext ? 255u : rem);
        op += 1 + ext;
        for (uint32_t x = L; x < run; x += 64) d[op + x] = s[anchor + x];
        op += run;
    }
    return (int32_t)op;
}

// 20 KiB per wave (8 waves per CU), one array so lanes can address dummy
// slots branch-free:
//   [0, 16 KiB)          hash table (4096 x u32, or 8192 x u16)
//   [16 KiB, 17 KiB)     dedup scratch (encode_block) / dummy slots (v5)
//   [17 KiB, 20 KiB)     encode_block: 2 KiB source ring + 1 KiB output ring;
//                        v5: 2 KiB + 64 B mirrored source ring
#define ENCODE_LDS                                                     \
    __shared__ __attribute__((aligned(16))) uint32_t ELDS[5120];       \
    uint32_t* const T = ELDS;                                          \
    uint8_t* const S = (uint8_t*)(ELDS + 4096);                        \
    uint32_t* const X = ELDS + 4352;
static_assert(kSR + kSRMirror <= 3072, "ring exceeds the shared scratch");
static_assert(kDedup == 1024, "scratch layout");

#if LZ4MT_PART != 2
#if LZ4MT_EXP_BLKTIME
constexpr uint32_t kExpBlkMax = 16384;
__device__ uint64_t g_expBlk[3 * kExpBlkMax];
#endif
// XC: the exchange probe (true, the product) or the read-back probe (false,
// the fallback when k_xchg_order fails); see encode_block_v5
template <bool XC>
__global__ void __launch_bounds__(64) k_encode(const uint8_t* __restrict__ src, uint64_t srcSize, uint32_t blockSize,
                                               uint8_t* __restrict__ slots, uint64_t slotStride,
                                               uint32_t capOverride, int32_t* __restrict__ csize) {
    ENCODE_LDS
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)((srcSize - off) < blockSize ? (srcSize - off) : blockSize);
    const uint32_t cap = (capOverride == 0xFFFFFFFFu) ? n : capOverride;   // lz4mt: cap = n
    g_cu8* s = gptr(src) + off;
    g_u8* d = gptr(slots) + (uint64_t)b * slotStride;
    l_u32* Tl = (l_u32*)T;
    l_u8* Sl = (l_u8*)S;
    l_u8* Xl = (l_u8*)X;
#if LZ4MT_EXP_BLKTIME
    const uint64_t t0 = wall_clock64();
#endif
    int32_t r;
    if (n < (uint32_t)kLimit64K)
        r = encode_block<true, false, false>(s, n, d, cap, Tl, Sl, (l_u32*)Xl, Xl + kRingE, nullptr);
    else if (n <= (1u << kPosBits))
        [[clang::always_inline]] r =
            encode_block_v5<false, false, false, false, false, false, false, XC>(s, n, d, cap, Tl, Xl, nullptr);
    else
        r = encode_block<false, false, false>(s, n, d, cap, Tl, Sl, (l_u32*)Xl, Xl + kRingE, nullptr);
    if (laneid() == 0) csize[b] = r;
#if LZ4MT_EXP_BLKTIME
    if (laneid() == 0 && b < kExpBlkMax) {   // experiment builds only: per-block start / end / placement
        g_expBlk[3 * b] = t0;
        g_expBlk[3 * b + 1] = wall_clock64();
        g_expBlk[3 * b + 2] = ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32) |
                              (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
#endif
}
#if LZ4MT_EXP_BLKTIME
// (tools/blocktimes.py reads it through lz4mtHipExpBlockTimes)
extern "C" int lz4mtHipExpBlockTimes(uint64_t* out, uint32_t nb) {
    if (nb > kExpBlkMax) nb = kExpBlkMax;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_expBlk), (size_t)nb * 24) == hipSuccess ? (int)nb : -1;
}
#endif

// k_encode with progress publishing (the block checksums' follower, the
// block-sharded streamed gather): the same parse and bytes; pub[b] = bytes
// of slot b already final, while the block encodes (the v5 path, 65 547 B ..
// 4 MiB blocks, every 64 KiB of output), then kPubDone | size (or kPubRaw).
template <bool XC>
__global__ void __launch_bounds__(64) k_encode_pub(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                   uint32_t blockSize, uint8_t* __restrict__ slots,
                                                   uint64_t slotStride, int32_t* __restrict__ csize,
                                                   uint32_t* __restrict__ pub) {
    ENCODE_LDS
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)((srcSize - off) < blockSize ? (srcSize - off) : blockSize);
    g_cu8* s = gptr(src) + off;
    g_u8* d = gptr(slots) + (uint64_t)b * slotStride;
    l_u32* Tl = (l_u32*)T;
    l_u8* Sl = (l_u8*)S;
    l_u8* Xl = (l_u8*)X;
    int32_t r;
    if (n < (uint32_t)kLimit64K)
        r = encode_block<true, false, false>(s, n, d, n, Tl, Sl, (l_u32*)Xl, Xl + kRingE, nullptr);
    else if (n <= (1u << kPosBits))
        r = encode_block_v5<false, false, false, false, false, true, false, XC>(s, n, d, n, Tl, Xl, nullptr,
                                                                                LinkArgs{0, 0, 0, true}, pub + b);
    else
        r = encode_block<false, false, false>(s, n, d, n, Tl, Sl, (l_u32*)Xl, Xl + kRingE, nullptr);
    if (laneid() == 0) csize[b] = r;
    publish_progress(pub + b, kPubDone | (r > 0 ? (uint32_t)r : kPubRaw));   // the block is final
}

// The exchange table probes rely on one wave's same-address LDS exchanges
// (ds_wrxchg_rtn_b32) and masked ORs (ds_mskor_rtn_b32) taking effect in
// ascending lane order.  k_xchg_order checks it on the device in use (one
// wave; three exchange address patterns, masked ORs on 16- and 8-bit
// fields): *ok = 1 when every lane got its lower same-address neighbour's
// value (or the initial one) and every word ends with its highest lane's.
__global__ void __launch_bounds__(64) k_xchg_order(uint32_t* ok) {
    __shared__ uint32_t W[64];
    const uint32_t L = laneid();
    bool good = true;
    for (uint32_t pat = 0; pat < 3; ++pat) {
        W[L] = 0xFFFF0000u | L;
        WAVE_SYNC();
        const uint32_t a = pat == 0 ? 0u : pat == 1 ? (L & 3u) : (L * 37u) % 7u;
        const uint32_t got = __hip_atomic_exchange((l_u32*)W + a, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        WAVE_SYNC();
        uint32_t want = 0xFFFF0000u | a, last = 64;
        for (uint32_t j = 0; j < 64; ++j) {   // (uniform loop: every lane walks the pattern)
            const uint32_t aj = pat == 0 ? 0u : pat == 1 ? (j & 3u) : (j * 37u) % 7u;
            if (aj == a && j < L) want = j;
            if (aj == L) last = j;
        }
        good = good && got == want && (last == 64 || W[L] == last);
        WAVE_SYNC();
    }
    // the split tables' masked ORs (16-bit and 8-bit fields of shared dwords)
    for (uint32_t fb = 16; fb >= 8; fb -= 8) {
        const uint32_t nf = 32u / fb, fm = (1u << fb) - 1u;
        W[L] = 0xA5A5A5A5u ^ L;
        WAVE_SYNC();
        const uint32_t sel = (L * 5u) % (4u * nf), a = sel / nf, sh = (sel % nf) * fb;
        uint32_t o16, o8;   // (the second op hits a word no lane reads back)
        mskor2_rtn((l_u32*)W + a, fm << sh, ((L + 1u) & fm) << sh, (l_u32*)W + 63, 0u, 0u, o16, o8);
        WAVE_SYNC();
        uint32_t want = ((0xA5A5A5A5u ^ a) >> sh) & fm, fin = 0xA5A5A5A5u ^ L;
        for (uint32_t j = 0; j < 64; ++j) {
            const uint32_t sj = (j * 5u) % (4u * nf), shj = (sj % nf) * fb;
            if (sj == sel && j < L) want = (j + 1u) & fm;
            if (sj / nf == L) fin = (fin & ~(fm << shj)) | (((j + 1u) & fm) << shj);
        }
        good = good && ((o16 >> sh) & fm) == want && (L >= 4 || W[L] == fin);
        WAVE_SYNC();
    }
    const bool all = __builtin_amdgcn_ballot_w64(!good) == 0;
    if (L == 0) *ok = all ? 1u : 0u;
}

// Which table probe the frame encoders run on the current device (*xc):
//   true   the exchange probe: k_xchg_order passed on this device (run once);
//   false  the read-back probe (no ordering assumed): the check failed (one
//          stderr line), LZ4MT_AMD_ENC_PROBE=readback forces it, or `st` is
//          being captured into a graph before any uncaptured call checked
//          this device (the check synchronises; the read-back probe is exact
//          on any device, so the captured graph is right either way).
// Returns a HIP error only when the check itself could not run.
static std::atomic<int> g_xchg_state[64];   // per device: 0 unchecked, 1 passed, -1 failed
static bool probe_forced_readback() {
    const char* e = getenv("LZ4MT_AMD_ENC_PROBE");
    return e && !strcmp(e, "readback");
}
static hipError_t xchg_check(int dev) {   // runs k_xchg_order once on `dev` (the current device)
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    if (g_xchg_state[dev].load()) return hipSuccess;
    hipStream_t ps = nullptr;
    uint32_t* d = nullptr;
    uint32_t h = 0;
    hipError_t e = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&d, 4);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_xchg_order, dim3(1), dim3(64), 0, ps, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, ps);
    if (e == hipSuccess) e = hipStreamSynchronize(ps);
    if (d) (void)hipFree(d);
    if (ps) (void)hipStreamDestroy(ps);
    if (e != hipSuccess) return e;
    g_xchg_state[dev].store(h == 1 ? 1 : -1, std::memory_order_release);
    if (h != 1)
        fprintf(stderr, "lz4mt_amd: device %d does not apply a wave's same-address LDS exchanges in lane order; "
                        "the block encoders use the read-back table probe there\n", dev);
    return hipSuccess;
}
hipError_t encoder_path(hipStream_t st, bool* xc) {
    *xc = false;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (probe_forced_readback()) return hipSuccess;
    int v = g_xchg_state[dev].load(std::memory_order_acquire);
    if (v == 0) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (st && hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return hipSuccess;
        if (const hipError_t e = xchg_check(dev); e != hipSuccess) return e;
        v = g_xchg_state[dev].load(std::memory_order_acquire);
    }
    *xc = v > 0;
    return hipSuccess;
}
// the diagnostic kernels exist only with the exchange probe
hipError_t encoder_ready(hipStream_t st) {
    bool xc = false;
    if (const hipError_t e = encoder_path(st, &xc); e != hipSuccess) return e;
    return xc ? hipSuccess : hipErrorNotSupported;
}

extern "C" int lz4mtHipCheckEncoderOrder(void) {
    int n = 0, dev = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return -1;
    if (g_xchg_state[dev].load() == 0 && xchg_check(dev) != hipSuccess) return -1;
    return g_xchg_state[dev].load() > 0 ? 1 : 0;
}

extern "C" int lz4mtHipEncoderProbe(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -1;
    bool xc = false;
    if (encoder_path(nullptr, &xc) != hipSuccess) return -1;
    return xc ? 1 : 0;
}

hipError_t launch_encode_pub(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                             uint8_t* slots, int32_t* csize, uint32_t* pub, hipStream_t st) {
    bool xc = true;
    if (const hipError_t r = encoder_path(st, &xc); r != hipSuccess) return r;
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(xc ? k_encode_pub<true> : k_encode_pub<false>, dim3(nBlocks), dim3(64), 0, st, src, srcSize,
                       blockSize, slots, (uint64_t)blockSize, csize, pub);
    return hipGetLastError();
}

// The v5 encoder with the 3-byte table (V5Geo P17): 14.25 KiB of LDS, 11
// waves per CU instead of 8.  Blocks of 65 547 B .. 4 MiB; others are left
// to k_encode (csize untouched here).
template <bool XC>
__global__ void __launch_bounds__(64) k_encode_p17(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                   uint32_t blockSize, uint8_t* __restrict__ slots,
                                                   uint64_t slotStride, uint32_t capOverride,
                                                   int32_t* __restrict__ csize) {
    __shared__ __attribute__((aligned(16))) uint32_t PLDS[(2 * (4096 + 64) + (4096 + 64) + kSR + kSRMirror) / 4];
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)((srcSize - off) < blockSize ? (srcSize - off) : blockSize);
    if (n < (uint32_t)kLimit64K || n > (1u << kPosBits)) return;
    const uint32_t cap = (capOverride == 0xFFFFFFFFu) ? n : capOverride;   // lz4mt: cap = n
    l_u8* Xl = (l_u8*)PLDS + 3 * (4096 + 64);
    int32_t r;
    [[clang::always_inline]] r = encode_block_v5<false, false, false, false, true, false, false, XC>(
        gptr(src) + off, n, gptr(slots) + (uint64_t)b * slotStride, cap, (l_u32*)PLDS, Xl, nullptr);
    if (laneid() == 0) csize[b] = r;
}

// diagnostic twin of k_encode: per-block phase cycle counts in stats[b*16 .. +16]
__global__ void __launch_bounds__(64) k_encode_stats(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                     uint32_t blockSize, uint8_t* __restrict__ slots,
                                                     uint64_t slotStride, int32_t* __restrict__ csize,
                                                     uint64_t* __restrict__ stats) {
    ENCODE_LDS
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)((srcSize - off) < blockSize ? (srcSize - off) : blockSize);
    uint64_t acc[16] = {0};
    int32_t r;
    g_cu8* s = gptr(src) + off;
    g_u8* d = gptr(slots) + b * slotStride;
    l_u8* Xl = (l_u8*)X;
    if (n < (uint32_t)kLimit64K)
        r = encode_block<true, false, true>(s, n, d, n, (l_u32*)T, (l_u8*)S, (l_u32*)Xl, Xl + kRingE, acc);
    else if (n <= (1u << kPosBits))
        r = encode_block_v5<true, false>(s, n, d, n, (l_u32*)T, Xl, acc);
    else
        r = encode_block<false, false, true>(s, n, d, n, (l_u32*)T, (l_u8*)S, (l_u32*)Xl, Xl + kRingE, acc);
    if (laneid() == 0) {
        csize[b] = r;
        for (int i = 0; i < 16; ++i) stats[b * 16 + i] = acc[i];
    }
}

// Frames of blocks below 65 547 bytes (-B4: 64 KiB): every block uses the
// byU16 table, so the kernel carries the 8192-entry table (34.3 KiB of LDS,
// 4 waves per CU) instead of k_encode's 20 KiB.
// The table is split (u16 positions + u8 tags, 26.3 KiB, 6 waves per CU).
constexpr uint32_t kE16TabWords = (8192 + 64) * 3 / 4;
constexpr uint32_t kE16Words = kE16TabWords + (kSR + kSRMirror) / 4;
template <bool XC>
__global__ void __launch_bounds__(64) k_encode16(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                 uint32_t blockSize, uint8_t* __restrict__ slots,
                                                 uint64_t slotStride, uint32_t capOverride,
                                                 int32_t* __restrict__ csize) {
    __shared__ uint32_t E16[kE16Words];
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)((srcSize - off) < blockSize ? (srcSize - off) : blockSize);
    const uint32_t cap = (capOverride == 0xFFFFFFFFu) ? n : capOverride;   // lz4mt: cap = n
    const int32_t r = encode_block_v5<false, true, true, false, false, false, false, XC>(
        gptr(src) + off, n, gptr(slots) + (uint64_t)b * slotStride, cap, (l_u32*)E16, (l_u8*)(E16 + kE16TabWords),
        nullptr);
    if (laneid() == 0) csize[b] = r;
}

// A block-dependent table entry (position | tag, V5Geo<false, false, true>)
// in the next block's coordinates: position x -> x - n; positions at or
// below n (older than the next block's 64 KiB window) -> 0, stale like an
// empty entry.
constexpr uint32_t kLinkPM = (1u << (kPosBits + 1)) - 1u;
__device__ __forceinline__ uint32_t link_rebase(uint32_t e, uint32_t n) {
    const uint32_t pos = e & kLinkPM;
    return pos > n ? (e & ~kLinkPM) | (pos - n) : 0u;
}

// Block-dependent frames (-BD, reference compressBlockDependency,
// src/lz4mt.cpp:460-538): ONE wave encodes the blocks in order, as lz4's
// LZ4_compress_limitedOutput_continue does (cap = inSize - 1): the byU32
// table stays in LDS from block to block (rebased to the next block's
// coordinates, entries older than 64 KiB dropped) and each block sees the 64
// KiB of input before it (src[-65536, 0) must be readable from block 1 on:
// the previous batch's tail when called per batch).  `table` (16 KiB) passes
// the table between calls: read unless `fresh`, written at the end.  The
// per-block lz4 mode (prefix / external dictionary, dictionary size) comes
// from the host's replay of the reference's buffer handling (LinkPlan).
template <bool XH, bool XC>
__global__ void __launch_bounds__(64) k_encode_linked(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                      uint32_t blockSize, uint32_t nBlocks,
                                                      uint8_t* __restrict__ slots, const LinkPlan* __restrict__ plan,
                                                      uint32_t* __restrict__ table, int fresh,
                                                      int32_t* __restrict__ csize, const uint32_t* __restrict__ gate,
                                                      const uint32_t* __restrict__ startp,
                                                      const uint32_t* __restrict__ entry) {
    if (gate && *gate == 0) return;   // the parallel rounds settled: nothing to redo
    ENCODE_LDS
    l_u32* Tl = (l_u32*)T;
    (void)S;
    l_u8* Xl = (l_u8*)X;
    const uint32_t L = laneid();
    // after parallel rounds: resume at the first unsettled block, whose
    // entry table is exact (its predecessors are)
    const uint32_t b0 = startp ? *startp : 0u;
    if (b0 >= nBlocks) return;
    if (b0 > 0 || !fresh) {
        const uint32_t* in = b0 > 0 ? entry + (uint64_t)b0 * 4096 : table;
        for (uint32_t i = L; i < 4096; i += 64) Tl[i] = in[i];
        WAVE_SYNC();
    }
    for (uint32_t b = b0; b < nBlocks; ++b) {
        const uint64_t off = (uint64_t)b * blockSize;
        const uint32_t n = (uint32_t)((srcSize - off) < blockSize ? (srcSize - off) : blockSize);
        const LinkPlan pl = plan[b];
        const LinkArgs lk{pl.lowIn, pl.lowDict, pl.candLow, fresh && b == 0, pl.shift};
        const int32_t r = encode_block_v5<false, false, false, true, false, false, XH, XC>(
            gptr(src) + off - kLinkO0, kLinkO0 + n, gptr(slots) + off, n - 1, Tl, Xl, nullptr, lk);
        if (L == 0) csize[b] = r;
        WAVE_SYNC();
        // the next block's coordinates: x -> x - n; older than the window -> 0
        for (uint32_t i = L; i < 4096; i += 64) {
            const uint32_t e = Tl[i];
            Tl[i] = link_rebase(e, n);
        }
        WAVE_SYNC();
    }
    for (uint32_t i = L; i < 4096; i += 64) table[i] = Tl[i];
}

hipError_t launch_encode_linked(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                                uint8_t* slots, const LinkPlan* plan, uint32_t* table, bool fresh, bool xh,
                                int32_t* csize, hipStream_t st) {
    bool xc = true;
    if (const hipError_t r = encoder_path(st, &xc); r != hipSuccess) return r;
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(xh ? (xc ? k_encode_linked<true, true> : k_encode_linked<true, false>)
                          : (xc ? k_encode_linked<false, true> : k_encode_linked<false, false>),
                       dim3(1), dim3(64), 0, st, src, srcSize,
                       blockSize, nBlocks, slots, plan, table, fresh ? 1 : 0, csize, (const uint32_t*)nullptr,
                       (const uint32_t*)nullptr, (const uint32_t*)nullptr);
    return hipGetLastError();
}

// Block-dependent encode in parallel: the only state one block hands the
// next is the lz4 table (its entries within 64 KiB of the next block; the
// history bytes are input).  Round 0 encodes every block at once, block b
// from a guessed entry table (all stale; block 0 from the call's first
// table, exact), and writes its exit table rebased to block b+1 (stale
// entries -> 0, which behave exactly like any other stale entry).  After
// round r, k_link_settle compares exit[b-1] with entry[b] for every block
// whose predecessor was re-encoded in round r; a differing entry is
// replaced and its block queued for round r+1 (flag[b] = r+1).  Once no
// entry changes, every block started from its predecessor's true exit
// table: by induction from block 0 the output is exactly the serial
// stream's.  A parse forgets a wrong start within a few KiB, so chains of
// wrong tables die out geometrically and rounds after the first re-encode
// few blocks.  If kLinkRounds rounds do not settle, the serial kernel
// finishes from the first unsettled block (its entry is exact).
//   ctl words: changed[kLinkRounds + 1] | first[kLinkRounds + 1] |
//              flag[nBlocks] | enc[nBlocks]
template <bool XH, bool XC>
__global__ void __launch_bounds__(64) k_encode_linked_round(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                            uint32_t blockSize, uint8_t* __restrict__ slots,
                                                            const LinkPlan* __restrict__ plan,
                                                            const uint32_t* __restrict__ first, int fresh,
                                                            const uint32_t* __restrict__ entry,
                                                            uint32_t* __restrict__ exitT, int32_t* __restrict__ csize,
                                                            const uint32_t* __restrict__ gate,
                                                            const uint32_t* __restrict__ flag,
                                                            uint32_t* __restrict__ enc, uint32_t round) {
    const uint32_t b = blockIdx.x;
    if (*gate == 0 || flag[b] != round) return;   // settled / this block's entry did not change
    ENCODE_LDS
    (void)S;
    l_u32* Tl = (l_u32*)T;
    const uint32_t L = laneid();
    const uint32_t* in = b == 0 ? first : entry + (uint64_t)b * 4096;
    const bool fr = b == 0 && fresh;
    if (!fr) {
        for (uint32_t i = L; i < 4096; i += 64) Tl[i] = in[i];
        WAVE_SYNC();
    }
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)((srcSize - off) < blockSize ? (srcSize - off) : blockSize);
    const LinkPlan pl = plan[b];
    const LinkArgs lk{pl.lowIn, pl.lowDict, pl.candLow, fr, pl.shift};
    const int32_t r = encode_block_v5<false, false, false, true, false, false, XH, XC>(
        gptr(src) + off - kLinkO0, kLinkO0 + n, gptr(slots) + off, n - 1, Tl, (l_u8*)X, nullptr, lk);
    if (L == 0) {
        csize[b] = r;
        enc[b] = round;
    }
    WAVE_SYNC();
    uint32_t* o = exitT + (uint64_t)b * 4096;
    for (uint32_t i = L; i < 4096; i += 64) {
        const uint32_t e = Tl[i];
        o[i] = link_rebase(e, n);
    }
}

__global__ void __launch_bounds__(256) k_link_settle(const uint32_t* __restrict__ exitT, uint32_t* __restrict__ entry,
                                                     uint32_t nBlocks, const uint32_t* __restrict__ gate,
                                                     const uint32_t* __restrict__ enc, uint32_t* __restrict__ flag,
                                                     uint32_t* __restrict__ changedNext,
                                                     uint32_t* __restrict__ firstNext, uint32_t round) {
    const uint32_t b = blockIdx.x + 1;   // entry[b] <- exit[b-1]
    if (b >= nBlocks || *gate == 0 || enc[b - 1] != round) return;   // exit[b-1] unchanged
    const uint32_t* x = exitT + (uint64_t)(b - 1) * 4096;
    uint32_t* e = entry + (uint64_t)b * 4096;
    __shared__ uint32_t diff;
    if (threadIdx.x == 0) diff = 0;
    __syncthreads();
    uint32_t d = 0;
    for (uint32_t i = threadIdx.x; i < 4096; i += 256) {
        const uint32_t v = x[i];
        d |= (e[i] != v) ? 1u : 0u;
        e[i] = v;
    }
    if (d) atomicOr(&diff, 1u);
    __syncthreads();
    if (threadIdx.x == 0 && diff) {
        flag[b] = round + 1;
        atomicAdd(changedNext, 1u);
        atomicMin(firstNext, b);
    }
}

// Chained rounds (blocks of 256 KiB and less): one table guess per block
// needs ~1-1.5 MiB of parse to be forgotten, i.e. 16-24 rounds of 64 KiB
// blocks.  Instead a wave encodes a chain of G consecutive blocks serially
// (exactly as k_encode_linked does), so only chain heads start from a guess;
// a wrong head entry is forgotten inside the chain, whose last exit table is
// then (almost always) right, and the next round re-runs only the chains
// whose head entry changed.  Blocks inside a chain are exact given the head,
// so only chain heads are compared (k_link_settle_chain) and can be the
// serial kernel's first unsettled block.
template <bool XC>
__global__ void __launch_bounds__(64) k_encode_linked_chain(const uint8_t* __restrict__ src, uint64_t srcSize,
                                                            uint32_t blockSize, uint32_t nBlocks, uint32_t G,
                                                            uint8_t* __restrict__ slots,
                                                            const LinkPlan* __restrict__ plan,
                                                            const uint32_t* __restrict__ first, int fresh,
                                                            const uint32_t* __restrict__ entry,
                                                            uint32_t* __restrict__ exitT, int32_t* __restrict__ csize,
                                                            const uint32_t* __restrict__ gate,
                                                            const uint32_t* __restrict__ flag,
                                                            uint32_t* __restrict__ enc, uint32_t round) {
    const uint32_t h = blockIdx.x * G;
    if (h >= nBlocks || *gate == 0 || flag[h] != round) return;   // settled / head entry unchanged
    ENCODE_LDS
    (void)S;
    l_u32* Tl = (l_u32*)T;
    const uint32_t L = laneid();
    const bool fr = h == 0 && fresh;
    if (!fr) {
        const uint32_t* in = h == 0 ? first : entry + (uint64_t)h * 4096;
        for (uint32_t i = L; i < 4096; i += 64) Tl[i] = in[i];
        WAVE_SYNC();
    }
    const uint32_t e = min(h + G, nBlocks);
    for (uint32_t b = h; b < e; ++b) {
        const uint64_t off = (uint64_t)b * blockSize;
        const uint32_t n = (uint32_t)((srcSize - off) < blockSize ? (srcSize - off) : blockSize);
        const LinkPlan pl = plan[b];
        const LinkArgs lk{pl.lowIn, pl.lowDict, pl.candLow, fr && b == 0};
        const int32_t r = encode_block_v5<false, false, false, true, false, false, false, XC>(
            gptr(src) + off - kLinkO0, kLinkO0 + n, gptr(slots) + off, n - 1, Tl, (l_u8*)X, nullptr, lk);
        if (L == 0) csize[b] = r;
        WAVE_SYNC();
        for (uint32_t i = L; i < 4096; i += 64) Tl[i] = link_rebase(Tl[i], n);
        WAVE_SYNC();
    }
    uint32_t* o = exitT + (uint64_t)(e - 1) * 4096;
    for (uint32_t i = L; i < 4096; i += 64) o[i] = Tl[i];
    if (L == 0) enc[e - 1] = round;
}

__global__ void __launch_bounds__(256) k_link_settle_chain(const uint32_t* __restrict__ exitT,
                                                           uint32_t* __restrict__ entry, uint32_t nBlocks, uint32_t G,
                                                           const uint32_t* __restrict__ gate,
                                                           const uint32_t* __restrict__ enc, uint32_t* __restrict__ flag,
                                                           uint32_t* __restrict__ changedNext,
                                                           uint32_t* __restrict__ firstNext, uint32_t round) {
    const uint32_t b = (blockIdx.x + 1) * G;   // chain head: entry[b] <- exit[b-1]
    if (b >= nBlocks || *gate == 0 || enc[b - 1] != round) return;
    const uint32_t* x = exitT + (uint64_t)(b - 1) * 4096;
    uint32_t* e = entry + (uint64_t)b * 4096;
    __shared__ uint32_t diff;
    if (threadIdx.x == 0) diff = 0;
    __syncthreads();
    uint32_t d = 0;
    for (uint32_t i = threadIdx.x; i < 4096; i += 256) {
        const uint32_t v = x[i];
        d |= (e[i] != v) ? 1u : 0u;
        e[i] = v;
    }
    if (d) atomicOr(&diff, 1u);
    __syncthreads();
    if (threadIdx.x == 0 && diff) {
        flag[b] = round + 1;
        atomicAdd(changedNext, 1u);
        atomicMin(firstNext, b);
    }
}

__global__ void k_link_final(const uint32_t* __restrict__ exitT, uint32_t nBlocks, const uint32_t* __restrict__ gate,
                             uint32_t* __restrict__ table) {
    if (*gate != 0) return;   // not settled: the serial kernel writes the table
    const uint32_t* x = exitT + (uint64_t)(nBlocks - 1) * 4096;
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) table[i] = x[i];
}

__global__ void k_link_init(uint32_t* __restrict__ ctl, uint32_t nBlocks) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t R = kLinkRounds + 1;
    if (i < R) ctl[i] = i == 0 ? 1u : 0u;                  // changed: round 0 open
    else if (i < 2 * R) ctl[i] = 0xFFFFFFFFu;             // first unsettled block
    else if (i < 2 * R + nBlocks) ctl[i] = 0u;            // flag: every block in round 0
}

// The first guess of block b's entry table for 4 MiB blocks:
// lz4's table after block b-1 holds only positions of b-1's last 64 KiB
// (older ones are stale), and two greedy parses of the same bytes from
// different tables end up making the same choices once their tables agree
// on the window (see link_warm_bytes for how long that takes).  So the table after
// parsing b-1's last W bytes from an empty table is, almost always, exactly
// the table the stream has, and round 0 then rarely needs a second round.
// The warm parse writes its (discarded) output into block b's own slot,
// which round 0 overwrites.  A wrong guess costs a round, never a byte.
template <bool XC>
__global__ void __launch_bounds__(64) k_link_warm(const uint8_t* __restrict__ src, uint32_t blockSize, uint32_t W,
                                                  uint8_t* __restrict__ slots, uint32_t* __restrict__ entry) {
    ENCODE_LDS
    (void)S;
    l_u32* Tl = (l_u32*)T;
    const uint32_t L = laneid();
    const uint32_t b = blockIdx.x + 1;
    const uint64_t off = (uint64_t)b * blockSize;   // block b's start; the warm bytes end there
    const LinkArgs lk{kLinkO0, kLinkO0, kLinkO0, true};   // no history: a fresh stream over the W bytes
    (void)encode_block_v5<false, false, false, true, false, false, false, XC>(
        gptr(src) + off - W - kLinkO0, kLinkO0 + W, gptr(slots) + off, W + W / 255 + 16, Tl, (l_u8*)X, nullptr, lk);
    WAVE_SYNC();
    uint32_t* o = entry + (uint64_t)b * 4096;
    for (uint32_t i = L; i < 4096; i += 64) {
        const uint32_t e = Tl[i];
        o[i] = link_rebase(e, W);
    }
}

// bytes of the warm parse for a block size (0 = no warm start):
// LZ4MT_AMD_BD_WARM_KIB overrides (A/B)
static uint32_t link_warm_bytes(uint32_t blockSize) {
    const char* e = getenv("LZ4MT_AMD_BD_WARM_KIB");
    // measured on App. F (LZ4MT_AMD_BD_STATS=1; profiles/r02_bd_warm_sweep*): two
    // parses agree only after ~0.5-1.5 MiB -- 4 MiB blocks with W = 256 / 512
    // / 1024 KiB leave 212 / 47 / 0 of 255 entries wrong at 1 GiB, W = 1024 /
    // 1536 KiB leave 15 / 0 of 2047 at 8 GiB (19.6 / 29.0 GiB/s compress);
    // 1 MiB blocks cannot hold a long enough warm-up (512 KiB: 147 of 1023
    // wrong), so they start cold
    uint32_t w = blockSize >= (4u << 20) ? (1536u << 10) : 0u;
    if (e) w = (uint32_t)atoi(e) << 10;
    if (w + kLinkO0 > blockSize) w = 0;   // the warm bytes and their 64 KiB lie in the previous block
    return w;
}

// blocks per chain of the chained rounds: ~1.5 MiB of parse (0 = one block
// per wave, the plain rounds); LZ4MT_AMD_BD_CHAIN overrides (A/B)
static uint32_t link_chain(uint32_t blockSize) {
    const char* e = getenv("LZ4MT_AMD_BD_CHAIN");
    if (e) return (uint32_t)std::max(0, atoi(e));
    return blockSize <= (256u << 10) ? (1536u << 10) / blockSize : 0u;
}

uint64_t link_round_bytes(uint64_t nBlocks) {
    return nBlocks * 4096 * 4 * 2 + (2 * (uint64_t)(kLinkRounds + 1) + 2 * nBlocks) * 4;
}

// The whole block-dependent encode of one call, asynchronously: up to
// kLinkRounds parallel rounds, each skipped on the device once one settled,
// then the serial kernel from the first unsettled block, which runs only if
// none settled (exact either way).  scratch: link_round_bytes(nBlocks).
hipError_t launch_encode_linked_par(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                                    uint8_t* slots, const LinkPlan* plan, uint32_t* table, bool fresh, bool xh,
                                    uint32_t* scratch, int32_t* csize, int rounds, hipStream_t st) {
    bool xc = true;
    if (const hipError_t r = encoder_path(st, &xc); r != hipSuccess) return r;
    if (nBlocks == 0) return hipSuccess;
    if (rounds < 1 || rounds > kLinkRounds) rounds = kLinkRounds;
    uint32_t* entry = scratch;
    uint32_t* exitT = entry + (uint64_t)nBlocks * 4096;
    uint32_t* ctl = exitT + (uint64_t)nBlocks * 4096;
    uint32_t* changed = ctl;
    uint32_t* firstU = ctl + kLinkRounds + 1;
    uint32_t* flag = firstU + kLinkRounds + 1;
    uint32_t* enc = flag + nBlocks;
    // first guess: blocks 1.. start from the warm table (blocks of 256 KiB and
    // up, k_link_warm) or an all-stale one
    if (hipMemsetAsync(entry, 0, (uint64_t)nBlocks * 4096 * 4, st) != hipSuccess) return hipErrorUnknown;
    const uint32_t warm = link_cold() ? 0u : link_warm_bytes(blockSize);
    if (nBlocks > 1 && warm)
        hipLaunchKernelGGL(xc ? k_link_warm<true> : k_link_warm<false>, dim3(nBlocks - 1), dim3(64), 0, st, src, blockSize, warm, slots, entry);
    const uint32_t nInit = 2 * (kLinkRounds + 1) + nBlocks;
    hipLaunchKernelGGL(k_link_init, dim3((nInit + 255) / 256), dim3(256), 0, st, ctl, nBlocks);
    // chains only below 1 MiB; the reference's own-history blocks (xh) are 1 / 4 MiB
    const uint32_t G = xh ? 0u : link_chain(blockSize);
    for (int r = 0; r < rounds && G > 1; ++r) {   // chained rounds
        const uint32_t nc = (nBlocks + G - 1) / G;
        hipLaunchKernelGGL(xc ? k_encode_linked_chain<true> : k_encode_linked_chain<false>, dim3(nc), dim3(64), 0, st, src, srcSize, blockSize, nBlocks, G, slots,
                           plan, (const uint32_t*)table, fresh ? 1 : 0, (const uint32_t*)entry, exitT, csize,
                           (const uint32_t*)(changed + r), (const uint32_t*)flag, enc, (uint32_t)r);
        if (nc > 1)
            hipLaunchKernelGGL(k_link_settle_chain, dim3(nc - 1), dim3(256), 0, st, (const uint32_t*)exitT, entry,
                               nBlocks, G, (const uint32_t*)(changed + r), (const uint32_t*)enc, flag, changed + r + 1,
                               firstU + r + 1, (uint32_t)r);
    }
    for (int r = 0; r < rounds && G <= 1; ++r) {
        hipLaunchKernelGGL(xh ? (xc ? k_encode_linked_round<true, true> : k_encode_linked_round<true, false>)
                              : (xc ? k_encode_linked_round<false, true> : k_encode_linked_round<false, false>),
                           dim3(nBlocks), dim3(64), 0,
                           st, src, srcSize, blockSize, slots, plan, (const uint32_t*)table, fresh ? 1 : 0,
                           (const uint32_t*)entry, exitT, csize, (const uint32_t*)(changed + r), (const uint32_t*)flag,
                           enc, (uint32_t)r);
        if (nBlocks > 1)
            hipLaunchKernelGGL(k_link_settle, dim3(nBlocks - 1), dim3(256), 0, st, (const uint32_t*)exitT, entry,
                               nBlocks, (const uint32_t*)(changed + r), (const uint32_t*)enc, flag, changed + r + 1,
                               firstU + r + 1, (uint32_t)r);
    }
    // a single block settles in round 0 (changed[1] stays 0)
    hipLaunchKernelGGL(xh ? (xc ? k_encode_linked<true, true> : k_encode_linked<true, false>)
                          : (xc ? k_encode_linked<false, true> : k_encode_linked<false, false>),
                       dim3(1), dim3(64), 0, st, src, srcSize, blockSize, nBlocks, slots, plan, table, fresh ? 1 : 0, csize,
                       (const uint32_t*)(changed + rounds), (const uint32_t*)(firstU + rounds),
                       (const uint32_t*)entry);
    hipLaunchKernelGGL(k_link_final, dim3(1), dim3(256), 0, st, (const uint32_t*)exitT, nBlocks,
                       (const uint32_t*)(changed + rounds), table);
    link_stats("encode", changed, firstU, rounds, nBlocks, st);
    return hipGetLastError();
}

// k_encode_p17 (the 3-byte table, 11 waves per CU) for 256 KiB blocks: with
// the exchange probe on both tables (XCHG, XCHG_SP) it is 134.7 ms per 8 GiB
// there against k_encode's 141.4; at 1 / 4 MiB blocks k_encode wins (150.2 /
// 161.5 vs 154.6 / 175.9: the 7-bit tags' extra round trips, and 4 MiB blocks
// fill only 8 waves per CU anyway; profiles/r04xsp_encoder_split_xchg_ab.txt).
// LZ4MT_AMD_ENC=p17 / base forces one (A/B)
static bool enc_p17(uint32_t blockSize) {
    const char* e = getenv("LZ4MT_AMD_ENC");
    if (e && !strcmp(e, "p17")) return true;
    if (e && !strcmp(e, "base")) return false;
    return blockSize <= (256u << 10);
}

// The parse work of a split parse (timing only): stream b of S
// bytes is parsed from `ov` bytes before its start -- the overlap its join
// with stream b-1 needs -- into slot b (stride S + ov); k_encode's table
// (P17 = 0) or the 3-byte one (P17 = 1).  No join: this is the part of the
// split parse's cost that the joins would only add to.
template <bool P17>
__global__ void __launch_bounds__(64) k_encode_overlap(const uint8_t* __restrict__ src, uint64_t srcSize, uint32_t S,
                                                       uint32_t ov, uint8_t* __restrict__ slots,
                                                       int32_t* __restrict__ csize) {
    constexpr uint32_t kWords = P17 ? (2 * (4096 + 64) + (4096 + 64) + kSR + kSRMirror) / 4 : 5120;
    __shared__ __attribute__((aligned(16))) uint32_t OLDS[kWords];
    const uint32_t b = blockIdx.x;
    const uint64_t lo = (uint64_t)b * S > ov ? (uint64_t)b * S - ov : 0u;
    const uint64_t hi = min<uint64_t>((uint64_t)(b + 1) * S, srcSize);
    const uint32_t n = (uint32_t)(hi - lo);
    if (n < (uint32_t)kLimit64K || n > (1u << kPosBits)) {   // not a v5 block: no size
        if (laneid() == 0) csize[b] = -1;
        return;
    }
    l_u8* ring = P17 ? (l_u8*)OLDS + 3 * (4096 + 64) : (l_u8*)(OLDS + 4352);
    // inlined here, so k_encode / k_encode_p17 stay the only call sites of
    // their instantiations (a second call site outlines the encoder into a
    // called function in the product kernels too)
    int32_t r;
    [[clang::always_inline]] r = encode_block_v5<false, false, false, false, P17>(gptr(src) + lo, n,
                                                                             gptr(slots) + (uint64_t)b * (S + ov),
                                                                             n, (l_u32*)OLDS, ring, nullptr);
    if (laneid() == 0) csize[b] = r;
}

hipError_t launch_encode_overlap(const uint8_t* src, uint64_t srcSize, uint32_t S, uint32_t ov, bool p17,
                                 uint8_t* slots, int32_t* csize, hipStream_t st) {
    if (const hipError_t r = encoder_ready(st); r != hipSuccess) return r;
    const uint32_t nb = (uint32_t)((srcSize + S - 1) / S);
    if (nb == 0) return hipSuccess;
    if (p17) hipLaunchKernelGGL(k_encode_overlap<true>, dim3(nb), dim3(64), 0, st, src, srcSize, S, ov, slots, csize);
    else hipLaunchKernelGGL(k_encode_overlap<false>, dim3(nb), dim3(64), 0, st, src, srcSize, S, ov, slots, csize);
    return hipGetLastError();
}

// LZ4MT_AMD_ENC_LDS_PAD=<bytes>: dynamic LDS added to the frame encoder's
// launch, i.e. fewer resident waves per CU (occupancy sweeps, timing only;
// profiles/r04a_occupancy_sweep.txt)
static uint32_t enc_lds_pad() {
    const char* e = getenv("LZ4MT_AMD_ENC_LDS_PAD");
    return e ? (uint32_t)atoi(e) : 0u;
}

hipError_t launch_encode(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks, uint8_t* slots,
                         uint64_t slotStride, uint32_t capOverride, int32_t* csize, hipStream_t st) {
    bool xc = true;
    if (const hipError_t r = encoder_path(st, &xc); r != hipSuccess) return r;
    if (nBlocks == 0) return hipSuccess;
    const uint32_t pad = enc_lds_pad();
    const auto kEnc = xc ? k_encode<true> : k_encode<false>;
    if (blockSize < (uint32_t)kLimit64K)
        hipLaunchKernelGGL(xc ? k_encode16<true> : k_encode16<false>, dim3(nBlocks), dim3(64), pad, st, src, srcSize, blockSize, slots, slotStride,
                           capOverride, csize);
    else if (enc_p17(blockSize) && blockSize <= (1u << kPosBits)) {   // 3-byte table; a short last block on k_encode
        hipLaunchKernelGGL(xc ? k_encode_p17<true> : k_encode_p17<false>, dim3(nBlocks), dim3(64), pad, st, src, srcSize, blockSize, slots, slotStride,
                           capOverride, csize);
        const uint64_t lastOff = (uint64_t)(nBlocks - 1) * blockSize;
        if (srcSize - lastOff < (uint64_t)kLimit64K)
            hipLaunchKernelGGL(kEnc, dim3(1), dim3(64), 0, st, src + lastOff, srcSize - lastOff, blockSize,
                               slots + (nBlocks - 1) * slotStride, slotStride, capOverride, csize + (nBlocks - 1));
    } else
        hipLaunchKernelGGL(kEnc, dim3(nBlocks), dim3(64), pad, st, src, srcSize, blockSize, slots, slotStride,
                           capOverride, csize);
    return hipGetLastError();
}
#endif


// ---------------------------------------------------------------------------
// Wave-wide inclusive prefix sum and max (DPP row shifts + 3 cross-row adds)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    const uint32_t r0 = rdlane(v, 15), r1 = rdlane(v, 31), r2 = rdlane(v, 47);
    const uint32_t row = laneid() >> 4;
    return v + (row >= 1 ? r0 : 0u) + (row >= 2 ? r1 : 0u) + (row >= 3 ? r2 : 0u);
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
    return max(max(rdlane(v, 15), rdlane(v, 31)), max(rdlane(v, 47), rdlane(v, 63)));
}

// ---------------------------------------------------------------------------
// Decoder
// ---------------------------------------------------------------------------
#ifndef LZ4MT_DEC_RING
#define LZ4MT_DEC_RING 16384
#endif
constexpr int32_t kRing = LZ4MT_DEC_RING;   // LDS history ring (bytes; A/B: -DLZ4MT_DEC_RING=8192 / 32768)
static_assert((kRing & (kRing - 1)) == 0 && kRing >= 4096, "history ring: a power of two");
constexpr int32_t kInWin = 2048;   // LDS input window (bytes)
constexpr int32_t kFlush = 1024;   // ring -> HBM flush granule (64 lanes x 16 B)
// next-sequence table of a batch: u16 per candidate token position (512),
// plus PAST (element 512) and DEAD (element 513); values are BYTE offsets
// into the table, so a hop is one dependent ds_read_u16
constexpr int32_t kNxOff = kInWin + 128;      // inside the win[] allocation
constexpr uint32_t kNxPast = 1024, kNxDead = 1026;
// far matches of a batch whose bytes load together (LZ4MT_FAR_TAB, A/B):
// App. F batches hold ~31 sequences, ~8 of them far (offset > the ring);
// the rest are loaded one at a time
#ifndef LZ4MT_FAR_TAB
#define LZ4MT_FAR_TAB 8
#endif
constexpr int kFarTab = LZ4MT_FAR_TAB;
// A batch's far-match parameters are read straight from their lanes (s_ff1
// over the far mask + v_readlane) instead of a rank-ordered LDS table read
// back by broadcast, so no far load waits on an LDS round trip (k_decode
// 31.36 -> 31.03 ms at 8 GiB B7, profiles/r04c_decoder_ab.txt); the ordered
// matches (5d) likewise (31.03 -> 30.90 ms, r04f_decoder_ordlanes_ab.txt).
// Rejected (records kept): deferring a batch's far-byte writes to the next
// batch (34.1 ms: vmcnt retires in issue order and the loop-carried far
// registers double the VGPRs, r04g_decoder_far_defer_ab.txt); a two-hop
// table beside the next table (33.9 ms, r04c_decoder_ab.txt).
static_assert(kFarTab >= 1 && kFarTab <= 24, "far table");
// (the window allocation keeps the 16 B x kFarTab the far table had: the
// decoder's LDS layout, and so its timing, is unchanged by its removal)
constexpr int32_t kFpOff = kInWin + 128 + 1040;
[[maybe_unused]] constexpr int32_t kWinAlloc = kFpOff + 16 * kFarTab;
static_assert(kRing + kWinAlloc <= 20480 || kRing != 16384, "decoder LDS: 8 waves per CU need <= 20 KiB each");

template <bool ST>
struct Dec {
    uint64_t* acc;
    uint64_t ts;
    g_cu8* src;           // compressed block
    int64_t len;
    g_u8* dst;            // block's output slot (16-B aligned)
    int64_t physcap;      // bytes of the slot that exist
    l_u8* ring;
    l_u8* win;
    int64_t wlo;          // block-relative position of win[0]
    int64_t labase;       // block position of the register lookahead's byte 0
    uint32_t la;          // lookahead: lane L holds bytes [labase + 4L, labase + 4L + 4)
    int64_t flushed;      // [0, flushed) stored to dst
    int64_t completed;    // [0, completed) known complete in memory
    int32_t lowP;         // lowest position a match may read: 0, or -65536 with a 64 KiB prefix before dst
    __device__ __forceinline__ void refill(int64_t i) {
        const uintptr_t base = (reinterpret_cast<uintptr_t>(src) + (uintptr_t)i) & ~uintptr_t(15);
        wlo = (int64_t)(base - reinterpret_cast<uintptr_t>(src));
        const uintptr_t end = reinterpret_cast<uintptr_t>(src) + (uintptr_t)len;
        const uint32_t L = laneid();
        WAVE_SYNC();
#pragma unroll
        for (int h = 0; h < kInWin / 1024; ++h) {
            const uintptr_t a = base + (uintptr_t)(h * 1024 + 16 * L);
            g_cu32* q = (g_cu32*)(src + (a - reinterpret_cast<uintptr_t>(src)));
            v4u v = {0, 0, 0, 0};   // dword-granular: never past the block's last dword
            if (a + 12 < end) v = *(g_cu4*)q;
            else {
                if (a < end) v.x = q[0];
                if (a + 4 < end) v.y = q[1];
                if (a + 8 < end) v.z = q[2];
            }
            *(l_u4*)(win + h * 1024 + 16 * L) = v;
        }
        WAVE_SYNC();
    }
    // 256-byte register lookahead of the token stream: the serial parser
    // extracts bytes with v_readlane (no LDS round trip per byte)
    __device__ __forceinline__ void refill_la(int64_t i) {
        if (i < wlo || i + 256 > wlo + kInWin) refill(i);
        labase = wlo + ((i - wlo) & ~int64_t(3));
        la = *(l_u32*)(win + (labase - wlo) + 4 * laneid());
    }
    __device__ __forceinline__ uint32_t in8(int64_t i) {
        if (i < 0 || i >= len) return 0;
        int64_t k = i - labase;
        if (k < 0 || k >= 256) {
            refill_la(i);
            k = i - labase;
        }
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)la, (int)(k >> 2));
        return (w >> ((uint32_t)(k & 3) * 8)) & 255u;
    }
    // flush every complete kFlush chunk below `upto`
    __device__ __forceinline__ void flush_to(int64_t upto) {
        const uint32_t L = laneid();
        while (flushed + kFlush <= upto) {
            const v4u v = *(l_u4*)(ring + ((flushed & (kRing - 1)) + 16 * L));
            const int64_t o = flushed + 16 * L;
            if (o + 16 <= physcap) *(g_u4*)(dst + o) = v;
            flushed += kFlush;
        }
    }
    __device__ __forceinline__ void flush_tail(int64_t op) {
        flush_to(op);
        const uint32_t L = laneid();
        for (int64_t o = flushed + L; o < op; o += 64)
            if (o < physcap) dst[o] = ring[o & (kRing - 1)];
        flushed = op;
    }
    __device__ __forceinline__ void copy_lit(int64_t ip, int64_t op, int64_t n) {
        STAMP_ADD(0, ts);
        const uint32_t L = laneid();
        const bool inWin = ip >= wlo && ip + n <= wlo + kInWin;
        for (int64_t c = 0; c < n; c += 64) {
            flush_to(op + c);
            const int64_t i = ip + c + L;
            if (c + L < n) {
                const uint32_t v = inWin ? win[i - wlo] : src[i];
                ring[(op + c + L) & (kRing - 1)] = (uint8_t)v;
            }
            WAVE_SYNC();
        }
        STAMP_ADD(1, ts);
    }
    __device__ __forceinline__ void copy_match(int64_t op, uint32_t offset, int64_t n) {
        STAMP_ADD(0, ts);
        if (ST) { acc[6] += 1; acc[7] += (int64_t)offset > kRing ? 1 : 0; }
        const uint32_t L = laneid();
        // out[x] = out[op - offset + ((x - op) mod offset)]; offset 0 => zeros (LZ4 1.9.3)
        const uint32_t magic = (offset > 0 && offset < 64) ? (65536u + offset - 1) / offset : 0u;
        for (int64_t c = 0; c < n; c += 64) {
            const int64_t o = op + c;
            flush_to(o);
            if ((int64_t)offset > kRing && completed < o - kRing) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                completed = flushed;
            }
            if (c + L < n) {
                uint32_t v = 0;
                if (offset) {
                    int64_t sp;
                    if (offset >= 64) sp = o + L - offset;
                    else {
                        const uint32_t kq = (L * magic) >> 16;   // L / offset for L < 64
                        sp = o + L - (int64_t)(kq + 1) * offset;
                    }
                    v = (sp >= o - kRing && sp >= 0) ? ring[sp & (kRing - 1)] : dst[sp];
                }
                ring[(o + L) & (kRing - 1)] = (uint8_t)v;
            }
            WAVE_SYNC();
        }
        STAMP_ADD((int64_t)offset > kRing ? 3 : 2, ts);
    }
    // literal [ipl, ipl+lit) -> [opl, opl+lit), then a match of mlen bytes at
    // opl+lit with `off`.  When the whole sequence fits one wave step and the
    // match source lies wholly before the sequence, it is ONE LDS read (lanes
    // pick the input window or the history ring) and ONE LDS write.
    __device__ __forceinline__ void copy_seq(int64_t ipl, int64_t opl, int64_t lit, uint32_t off, int64_t mlen) {
        const int64_t tot = lit + mlen;
        if (tot <= 64 && (int64_t)off >= tot && (int64_t)off <= kRing - 128 && ipl >= wlo &&
            ipl + lit <= wlo + kInWin && opl + lit >= (int64_t)off) {
            STAMP_ADD(0, ts);
            if (ST) acc[6] += 1;
            flush_to(opl);
            const int64_t x = laneid();
            uint32_t v = 0;
            if (x < lit) v = win[ipl + x - wlo];
            else if (x < tot) v = ring[(opl + x - off) & (kRing - 1)];
            if (x < tot) ring[(opl + x) & (kRing - 1)] = (uint8_t)v;
            WAVE_SYNC();
            STAMP_ADD(2, ts);
            return;
        }
        if (lit) copy_lit(ipl, opl, lit);
        copy_match(opl + lit, off, mlen);
    }
    // ---------------------------------------------------------------------
    // Batch fast path.  Called at the top of the 1.9.3 fast loop.  Consumes
    // the longest run of sequences (<= 64) that the fast loop would process
    // on its normal path -- no error, no detour to safe_literal_copy /
    // safe_match_copy, one-byte length extensions, offset != 0 -- so the
    // serial state machine resumes at the same loop top with identical
    // state.  Returns the number of sequences consumed (0: run serially).
    // Positions are 32-bit block-relative here (blocks are < 2^31 bytes).
    //   1. next-token delta for 512 candidate positions (8 per lane, one
    //      LDS round trip; the match-length byte is checked in step 3)
    //   2. serial hop over the packed deltas (v_readlane), one lane per sequence
    //   3. lane-parallel field decode, DPP prefix sum of output lengths
    //   4. lane-parallel check of the fast-loop conditions, cut at the first miss
    //   5. copies: far-match loads issued first (HBM, lane per byte); literal
    //      runs and short matches whose source lies before the batch, 8
    //      sequences per group (all reads, then all writes); far bytes into
    //      the ring; then, in order, matches sourcing the batch's own output
    //      and matches longer than one group slot (128 B)
    // ---------------------------------------------------------------------
    __device__ __forceinline__ int decode_batch(int64_t& ip64, int64_t& op64, int64_t iend64, int64_t oend64) {
        // every sequence is validated against 1.9.3's fast-loop conditions
        // below; this guard only keeps the batch machinery inside the block
        if (ip64 + 17 > iend64 || op64 + 64 > oend64) {
            return 0;
        }
        STAMP_ADD(0, ts);
        if (ip64 < wlo || ip64 + 1024 > wlo + kInWin) refill(ip64);
        STAMP_ADD(10, ts);
        const uint32_t L = laneid();
        const int32_t ip = (int32_t)ip64, op = (int32_t)op64, iend = (int32_t)iend64, oend = (int32_t)oend64;
        const uint32_t w0 = (uint32_t)(ip64 - wlo);
        // 1. candidate deltas for positions 8L .. 8L+7 (bytes 8L .. 8L+8)
        uint32_t pk0 = 0, pk1 = 0;
        {
            const uint64_t q = *(l_u64u*)(win + w0 + 8 * L);
            const uint32_t q8 = win[w0 + 8 * L + 8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const uint32_t t = (uint32_t)(q >> (8 * e)) & 255u;
                const uint32_t b1 = e < 7 ? (uint32_t)(q >> (8 * e + 8)) & 255u : q8;
                const bool l15 = (t >> 4) == 15;
                const uint32_t lit = (t >> 4) + (l15 ? b1 : 0u);
                const uint32_t d = 3 + (l15 ? 1u : 0u) + lit + ((t & 15) == 15 ? 1u : 0u);
                const bool cx = (l15 && b1 == 255) || d > 255;   // deltas are bytes
                if (e < 4) pk0 |= (cx ? 0u : d) << (8 * e);
                else pk1 |= (cx ? 0u : d) << (8 * (e - 4));
            }
        }
        STAMP_ADD(11, ts);
        // 2. hop.  next(i) = i + delta(i) goes into an LDS table (8 entries
        // per lane, one ds_write_b128); the chain from position 0 is then
        // one dependent ds_read_u16 per sequence, with every lane running it
        // redundantly (uniform broadcast reads) and lane m recording x_m and
        // x_(m+1).  A zero delta (complex token) leads to DEAD, a start past
        // the 512 candidates to PAST (whose sequence still counts).
        uint32_t startRel, cnt;
        {
            l_u8* const nxb = win + kNxOff;
            uint32_t nv[4];
#pragma unroll
            for (int e2 = 0; e2 < 4; ++e2) {
                uint32_t pr = 0;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int e = 2 * e2 + h;
                    const uint32_t d = ((e < 4 ? pk0 : pk1) >> (8 * (e & 3))) & 255u;
                    const uint32_t pos = 8 * L + (uint32_t)e;
                    const uint32_t nx = d == 0 ? kNxDead : (pos + d < 512 ? 2 * (pos + d) : kNxPast);
                    pr |= nx << (16 * h);
                }
                nv[e2] = pr;
            }
            *(l_u4*)(nxb + 16 * L) = (v4u){nv[0], nv[1], nv[2], nv[3]};
            WAVE_SYNC();
            uint32_t x = 0, startA = 0, nextA = kNxDead;
            for (uint32_t m0 = 0; m0 < 64; m0 += 8) {
#pragma unroll
                for (uint32_t e = 0; e < 8; ++e) {
                    x = *(l_u16*)(nxb + x);
                    nextA = L == m0 + e ? x : nextA;
                    startA = L == m0 + e + 1 ? x : startA;
                }
                if ((uint32_t)__builtin_amdgcn_readfirstlane((int)x) == kNxDead) break;
            }
            cnt = (uint32_t)__popcll(bal(nextA != kNxDead));
            startRel = startA >> 1;
        }
        STAMP_ADD(12, ts);
        if (cnt == 0) return 0;
        if (ST) acc[4] += 1;
        // 3. fields (lane j = sequence j), branch-free
        const bool act = L < cnt;
        const uint32_t sw = w0 + (act ? startRel : 0u);
        const uint32_t tb = *(l_u16u*)(win + sw);   // token, first literal-length byte
        const uint32_t tok = tb & 255u, b1 = tb >> 8;
        const bool l15 = (tok >> 4) == 15, m15 = (tok & 15) == 15;
        const uint32_t e1 = l15 ? 1u : 0u;
        const uint32_t lit = (tok >> 4) + (l15 ? b1 : 0u);
        const uint32_t ow = sw + 1 + e1 + lit;
        const uint32_t ob = *(l_u32u*)(win + ow);   // offset lo, hi, match-length byte
        const uint32_t off = ob & 0xFFFFu;
        const uint32_t b2 = (ob >> 16) & 255u;
        const uint32_t e2 = m15 ? 1u : 0u;
        const uint32_t mlen = (tok & 15) + kMinMatch + (m15 ? b2 : 0u);
        const uint32_t olen = act ? lit + mlen : 0u;
        const uint32_t incl = wave_scan_incl(olen);
        const int32_t oj = op + (int32_t)(incl - olen);      // sequence output start
        const int32_t ipT = ip + (int32_t)startRel + 1;      // just after the token
        const int32_t lp = ipT + (int32_t)e1;                // literal start
        const int32_t om = oj + (int32_t)lit;                // match output start
        const int32_t src = om - (int32_t)off;
        const int32_t ringLo = max(op + 4096 - kRing, 0);   // prefix bytes (< 0) are never in the ring
        // 4. fast-loop conditions (lz4 1.9.3, see decode_block)
        bool ok = act && off != 0 && !(m15 && b2 == 255) && incl <= 4096;
        ok = ok && (l15 ? (ipT < iend - 15 && ipT + 1 < iend - 15 && oj + (int32_t)lit <= oend - 32 &&
                           lp + (int32_t)lit <= iend - 32)
                        : ipT <= iend - 17);
        ok = ok && om - (int32_t)off >= lowP;
        // a prefix source running into the block reads bytes not yet flushed
        // from the ring: the serial path copies those byte by byte
        ok = ok && !(src < 0 && src + (int32_t)mlen > 0);
        ok = ok && (!m15 || lp + (int32_t)lit + 3 < iend - kLastLiterals + 1);
        ok = ok && om + (int32_t)mlen < oend - 64;
        ok = ok && !(src < ringLo && mlen > 128);   // far loads carry at most 128 bytes
        const uint64_t bad = ballot(act && !ok);
        const uint32_t nb = bad ? (uint32_t)(__ffsll((long long)bad) - 1) : cnt;
        STAMP_ADD(13, ts);
        if (nb == 0) return 0;
        const bool in = L < nb;
        if (ST) { acc[6] += nb; acc[8] += nb; }
        flush_to(op64);
        STAMP_ADD(14, ts);
        // 5. classes: far (source older than the ring keeps), ordered (source
        // reaches into this batch's output, or longer than a group slot),
        // else copied in groups
        const bool far = in && src < ringLo;
        const bool longLit = in && lit > 64;
        const bool ord = in && !far && (longLit || src + (int32_t)mlen > op || lit + mlen > 128);
        const uint64_t farM = ballot(far), ordM = ballot(ord);
        // 5a. far loads (up to 8 sequences, lane per byte), in flight during 5b.
        // Each far sequence's parameters come from its lane (v_readlane).
        uint32_t fv[kFarTab], fv2[kFarTab];
        const uint32_t fr = __builtin_amdgcn_mbcnt_hi((uint32_t)(farM >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)farM, 0u));
        const uint32_t nf8 = min((uint32_t)__popcll(farM), (uint32_t)kFarTab);
        uint32_t flane[kFarTab];   // lane of the g-th far sequence (uniform)
        if (farM) {
            if (completed < (int64_t)ringLo) {   // their bytes were stored to dst: make sure the stores landed
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                completed = flushed;
            }
            if (ST) acc[7] += __popcll(farM);
            uint64_t fm = farM;
#pragma unroll
            for (int g = 0; g < kFarTab; ++g) {
                fv[g] = 0; fv2[g] = 0; flane[g] = 0;
                if ((uint32_t)g < nf8) {
                    const uint32_t lg = (uint32_t)__builtin_ctzll(fm);
                    fm &= fm - 1;
                    flane[g] = lg;
                    const int64_t fs = (int32_t)rdlane((uint32_t)src, (int)lg);   // a prefix source is negative
                    const uint32_t fz = rdlane(mlen, (int)lg);
                    fv[g] = dst[fs + min(L, fz - 1)];   // bytes past the match repeat its last one (never written)
                    if (fz > 64) fv2[g] = dst[fs + min(L + 64, fz - 1)];
                }
            }
        }
        STAMP_ADD(15, ts);
        // 5b. literal runs of every sequence + grouped matches, 8 per group
        const uint32_t tot = longLit ? 0u : lit + ((in && !far && !ord) ? mlen : 0u);
        const uint32_t pA = lit | (tot << 8) | ((uint32_t)(lp - (int32_t)wlo) << 16);     // lw < 2048
        const uint32_t pB = (uint32_t)(oj - op) | ((((uint32_t)src - lit) & (kRing - 1)) << 16);   // ojrel < 4096
        l_u8* const winp = win;
        l_u8* const ringp = ring;
        l_u8* const dummy = win + kInWin;   // 128 scratch bytes: target of masked-off lane writes
        const uint64_t bigM = ballot(tot > 64);
        // Fast path: each sequence's copy parameters are precomputed by its
        // lane as LDS byte addresses (literal source, match source, target)
        // and broadcast to the wave with one ds_read_b128 (the hop table is
        // dead by now) -- no v_readlane / SALU unpacking per sequence.  It
        // needs every copied range to stay clear of the ring's end (true for
        // ~15 batches in 16); otherwise the masked per-sequence path below.
        const uint32_t jt0 = in ? tot : 0u;
        const uint32_t r2i = ((uint32_t)src - lit) & (kRing - 1), wi = (uint32_t)oj & (kRing - 1);
        const bool wrapJ = jt0 && (wi + jt0 > (uint32_t)kRing || r2i + jt0 > (uint32_t)kRing);
        if (!ballot(wrapJ)) {
            const uint32_t ringA = (uint32_t)(uintptr_t)ringp, winA = (uint32_t)(uintptr_t)winp;
            l_u4* const prm = (l_u4*)(win + kNxOff);
            prm[L] = (v4u){winA + (uint32_t)(lp - (int32_t)wlo), ringA + r2i, ringA + wi, (lit & 255u) | (jt0 << 8)};
            WAVE_SYNC();
            const uint32_t dumA = (uint32_t)(uintptr_t)dummy;
            for (uint32_t j0 = 0; j0 < nb; j0 += 8) {
                uint32_t v[8], wa[8];
                const bool big = ((bigM >> j0) & 0xFFull) != 0;
#pragma unroll
                for (int g = 0; g < 8; ++g) {
                    const v4u q = prm[j0 + g];
                    const uint32_t jl = q.w & 255u, jt = q.w >> 8;
                    v[g] = *(l_u8*)(uintptr_t)((L < jl ? q.x : q.y) + L);
                    wa[g] = (L < jt ? q.z : dumA) + L;
                }
#pragma unroll
                for (int g = 0; g < 8; ++g) *(l_u8*)(uintptr_t)wa[g] = (uint8_t)v[g];
                if (big) {   // second 64-byte half of sequences longer than 64 bytes
#pragma unroll
                    for (int g = 0; g < 8; ++g) {
                        const v4u q = prm[j0 + g];
                        const uint32_t jl = q.w & 255u, jt = q.w >> 8, x = L + 64;
                        v[g] = *(l_u8*)(uintptr_t)((x < jl ? q.x : q.y) + x);
                        wa[g] = x < jt ? q.z + x : dumA + 64 + L;
                    }
#pragma unroll
                    for (int g = 0; g < 8; ++g) *(l_u8*)(uintptr_t)wa[g] = (uint8_t)v[g];
                }
            }
        } else {
            const uint64_t bigM = ballot(tot > 64);
            for (uint32_t j0 = 0; j0 < nb; j0 += 8) {
                uint32_t v[8];
                l_u8* wp[8];
                const bool big = ((bigM >> j0) & 0xFFull) != 0;
    #pragma unroll
                for (int g = 0; g < 8; ++g) {
                    const uint32_t j = min(j0 + g, 63u);
                    const uint32_t A = rdlane(pA, (int)j), Bv = rdlane(pB, (int)j);
                    const uint32_t jl = A & 255u, jt = (j0 + g < nb) ? (A >> 8) & 255u : 0u, jlw = A >> 16;
                    const uint32_t jo = (uint32_t)op + (Bv & 0xFFFFu), js = Bv >> 16;
                    l_u8* ra = L < jl ? winp + jlw + L : ringp + ((js + L) & (kRing - 1));
                    v[g] = *ra;
                    wp[g] = L < jt ? ringp + ((jo + L) & (kRing - 1)) : dummy + L;
                }
    #pragma unroll
                for (int g = 0; g < 8; ++g) *wp[g] = (uint8_t)v[g];
                if (big) {   // second 64-byte half of sequences longer than 64 bytes
    #pragma unroll
                    for (int g = 0; g < 8; ++g) {
                        const uint32_t j = min(j0 + g, 63u);
                        const uint32_t A = rdlane(pA, (int)j), Bv = rdlane(pB, (int)j);
                        const uint32_t jl = A & 255u, jt = (j0 + g < nb) ? (A >> 8) & 255u : 0u, jlw = A >> 16;
                        const uint32_t jo = (uint32_t)op + (Bv & 0xFFFFu), js = Bv >> 16;
                        const uint32_t x = L + 64;
                        l_u8* ra = x < jl ? winp + jlw + x : ringp + ((js + x) & (kRing - 1));
                        v[g] = *ra;
                        wp[g] = x < jt ? ringp + ((jo + x) & (kRing - 1)) : dummy + 64 + L;
                    }
    #pragma unroll
                    for (int g = 0; g < 8; ++g) *wp[g] = (uint8_t)v[g];
                }
            }
        }
        STAMP_ADD(1, ts);
        // 5b'. literal runs longer than 64 bytes (whole wave, 64 per step)
        uint64_t llLeft = ballot(longLit);
        while (llLeft) {
            const int j = __ffsll((long long)llLeft) - 1;
            llLeft &= llLeft - 1;
            const uint32_t A = rdlane(pA, j), jo = (uint32_t)op + (rdlane(pB, j) & 0xFFFFu);
            const uint32_t jl = A & 255u, jlw = A >> 16;
            for (uint32_t base = 0; base < jl; base += 64) {
                const uint32_t x = base + L;
                if (x < jl) ring[(jo + x) & (kRing - 1)] = win[jlw + x];
            }
        }
        // 5c. far bytes into the ring at the match outputs
        if (farM) {
#pragma unroll
            for (int g = 0; g < kFarTab; ++g) {
                if ((uint32_t)g < nf8) {
                    const uint32_t qy = rdlane((uint32_t)om, (int)flane[g]) & (kRing - 1);
                    const uint32_t qz = rdlane(mlen, (int)flane[g]);
                    *(L < qz ? ringp + ((qy + L) & (kRing - 1)) : dummy + L) = (uint8_t)fv[g];
                    if (qz > 64)
                        *(L + 64 < qz ? ringp + ((qy + 64 + L) & (kRing - 1)) : dummy + 64 + L) = (uint8_t)fv2[g];
                }
            }
            uint64_t farLeft = ballot(far && fr >= (uint32_t)kFarTab);
            while (farLeft) {   // more than kFarTab far matches: one at a time
                const int j = __ffsll((long long)farLeft) - 1;
                const uint32_t js = (uint32_t)rdlane((uint32_t)src, j), jm = rdlane(mlen, j);
                const uint32_t jo = (uint32_t)rdlane((uint32_t)om, j);
                const int64_t jsS = (int32_t)js;
                const uint32_t a0 = L < jm ? (uint32_t)dst[jsS + L] : 0u;
                const uint32_t a1 = L + 64 < jm ? (uint32_t)dst[jsS + 64 + L] : 0u;
                if (L < jm) ring[(jo + L) & (kRing - 1)] = (uint8_t)a0;
                if (L + 64 < jm) ring[(jo + 64 + L) & (kRing - 1)] = (uint8_t)a1;
                farLeft &= farLeft - 1;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            completed = flushed;
        }
        WAVE_SYNC();
        STAMP_ADD(3, ts);
        // 5d. ordered matches (k mod off when the source overlaps the match),
        // in sequence order; the ordered lanes publish their parameters by
        // rank into the (now free) copy table, read back by broadcast
        const uint32_t nOrd = (uint32_t)__popcll(ordM);
        if (nOrd) {
            const uint32_t magicL = (off > 0 && off < 64) ? (65536u + off - 1) / off : 0u;
            uint64_t oLeft = ordM;
            for (uint32_t g = 0; g < nOrd; ++g) {
                const int lg = (int)__builtin_ctzll(oLeft);
                oLeft &= oLeft - 1;
                const uint32_t jom = rdlane((uint32_t)om, lg) & (kRing - 1), joff = rdlane(off, lg);
                const uint32_t jm = rdlane(mlen, lg), magic = rdlane(magicL, lg);
                const uint32_t jmS = jm;
                for (uint32_t base = 0; base < jmS; base += 64) {
                    const uint32_t k = base + L;
                    const uint32_t kk = (joff >= 64 || k < joff) ? k : k - ((k * magic) >> 16) * joff;
                    const uint8_t v = ring[(jom - joff + kk) & (kRing - 1)];
                    *(k < jm ? ringp + ((jom + k) & (kRing - 1)) : dummy + L) = v;
                    WAVE_SYNC();
                }
            }
        }
        STAMP_ADD(2, ts);
        // advance past the last consumed sequence
        const int last = (int)nb - 1;
        ip64 = ip64 + (int64_t)rdlane(startRel, last) + 1 + rdlane(e1, last) + rdlane(lit, last) + 2 + rdlane(e2, last);
        op64 = op64 + (int64_t)rdlane(incl, last);
        return (int)nb;
    }
    // read_variable_length(); returns 0 ok, -1 initial error, -2 loop error
    __device__ __forceinline__ int rvl(int64_t& ip, int64_t lencheck, bool loopCheck, bool initialCheck,
                                       int64_t& length) {
        length = 0;
        if (initialCheck && ip >= lencheck) return -1;
        uint32_t sv;
        do {
            sv = in8(ip);
            ip++;
            length += sv;
            if (loopCheck && ip >= lencheck) return -2;
        } while (sv == 255);
        return 0;
    }
};

// LZ4_decompress_safe (lz4 1.9.3, LZ4_FAST_DEC_LOOP=1): same accept/reject
// decisions and return values as the oracle restatement (oracle/lz4_oracle.c).
template <bool ST>
__device__ int32_t decode_block(Dec<ST>& D, int64_t cap) {
    const int64_t iend = D.len, oend = cap;
    const int64_t shortiend = iend - 16, shortoend = oend - 32;
    int64_t ip = 0, op = 0, cpy = 0, match = 0, length = 0, ext = 0;
    int64_t plIp = 0, plOp = 0, plLen = 0;   // literal run deferred to its sequence's match copy
    uint32_t token = 0, offset = 0;
    int e;

    if (cap == 0) return (D.len == 1 && D.in8(0) == 0) ? 0 : -1;
    if (D.len == 0) return -1;
    *(l_u32*)(D.win + kNxOff + kNxPast) = kNxDead | (kNxDead << 16);   // next(PAST) = next(DEAD) = DEAD

#define PHYS_CHECK(end_) \
    if ((end_) > D.physcap) return kDecodeOutputTooSmall;

    // SIMD-mate priority as in the encoder (SimdPrio), on output progress,
    // blocks of 1 MiB and more (a finished wave's last projection is its
    // finish time, past at once, so no clearing is needed)
#ifndef LZ4MT_NO_DEC_PRIO
    const bool prioOn = !ST && cap >= (1 << 20);
#else
    const bool prioOn = false;
#endif
    SimdPrio prio{};
    uint32_t tickShift = 31, opTick = 0;
    if (prioOn) {
        prio.start();
        tickShift = (31 - __builtin_clz((uint32_t)cap)) - 7;   // a check every 1/128 of the block
    }
    if (oend - op < 64) goto safe_decode;
    for (;;) {
        if (D.decode_batch(ip, op, iend, oend)) {
            if (prioOn && ((opTick ^ (uint32_t)op) >> tickShift)) {
                opTick = (uint32_t)op;
                prio.tick(opTick, (uint32_t)cap);
            }
            continue;
        }
        if (ST) D.acc[9] += 1;
        token = D.in8(ip++);
        length = token >> 4;
        if (length == 15) {
            e = D.rvl(ip, iend - 15, true, true, ext);
            length += ext;
            if (e == -1) goto output_error;
            cpy = op + length;
            if (cpy > oend - 32 || ip + length > iend - 32) goto safe_literal_copy;
        } else {
            cpy = op + length;
            if (ip > iend - 17) goto safe_literal_copy;
        }
        PHYS_CHECK(cpy);
        plIp = ip; plOp = op; plLen = length;
        ip += length;
        op = cpy;
        offset = D.in8(ip) | (D.in8(ip + 1) << 8);
        ip += 2;
        match = op - (int64_t)offset;
        length = token & 15;
        if (length == 15) {
            if (match < D.lowP) goto output_error;
            e = D.rvl(ip, iend - kLastLiterals + 1, true, false, ext);
            length += ext;
            if (e != 0) goto output_error;
            length += kMinMatch;
            if (op + length >= oend - 64) goto safe_match_copy;
        } else {
            length += kMinMatch;
            if (op + length >= oend - 64) goto safe_match_copy;
            if (match >= D.lowP && offset >= 8) {
                PHYS_CHECK(op + length);
                D.copy_seq(plIp, plOp, plLen, offset, length);
                op += length;
                continue;
            }
        }
        if (match < D.lowP) goto output_error;
        cpy = op + length;
        PHYS_CHECK(cpy);
        D.copy_seq(plIp, plOp, plLen, offset, length);
        op = cpy;
    }

safe_decode:
    for (;;) {
        token = D.in8(ip++);
        length = token >> 4;
        if (length != 15 && ip < shortiend && op <= shortoend) {
            PHYS_CHECK(op + length);
            plIp = ip; plOp = op; plLen = length;
            op += length;
            ip += length;
            length = token & 15;
            offset = D.in8(ip) | (D.in8(ip + 1) << 8);
            ip += 2;
            match = op - (int64_t)offset;
            if (length != 15 && offset >= 8 && match >= D.lowP) {
                PHYS_CHECK(op + length + kMinMatch);
                D.copy_seq(plIp, plOp, plLen, offset, length + kMinMatch);
                op += length + kMinMatch;
                continue;
            }
            goto copy_match;
        }
        if (length == 15) {
            e = D.rvl(ip, iend - 15, true, true, ext);
            length += ext;
            if (e == -1) goto output_error;
        }
        cpy = op + length;
    safe_literal_copy:
        if (cpy > oend - kMfLimit || ip + length > iend - (2 + 1 + kLastLiterals)) {
            if (ip + length != iend || cpy > oend) goto output_error;
            PHYS_CHECK(cpy);
            D.copy_lit(ip, op, length);
            ip += length;
            op += length;
            break;
        }
        PHYS_CHECK(cpy);
        plIp = ip; plOp = op; plLen = length;
        ip += length;
        op = cpy;
        offset = D.in8(ip) | (D.in8(ip + 1) << 8);
        ip += 2;
        match = op - (int64_t)offset;
        length = token & 15;
    copy_match:
        if (length == 15) {
            e = D.rvl(ip, iend - kLastLiterals + 1, true, false, ext);
            length += ext;
            if (e != 0) goto output_error;
        }
        length += kMinMatch;
    safe_match_copy:
        if (match < D.lowP) goto output_error;
        cpy = op + length;
        if (cpy > oend - kLastLiterals) goto output_error;
        PHYS_CHECK(cpy);
        D.copy_seq(plIp, plOp, plLen, offset, length);
        op = cpy;
    }
#undef PHYS_CHECK
    D.flush_tail(op);
    return (int32_t)op;

output_error:
    return (int32_t)(-ip) - 1;
}

// raw (incompressible) block: src at any alignment -> dst 16-B aligned
__device__ void copy_raw(g_cu8* src, g_u8* dst, int64_t n) {
    const uint32_t L = laneid();
    const int64_t nd = n >> 2;   // whole destination dwords
    g_u32* d32 = (g_u32*)dst;
    for (int64_t base = 0; base < nd; base += 64 * 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t j = base + u * 64 + L;
            if (j < nd) d32[j] = ld32u(src + 4 * j);
        }
    }
    for (int64_t i = nd * 4 + L; i < n; i += 64) dst[i] = src[i];
}

#if LZ4MT_PART != 1
#if LZ4MT_EXP_BLKTIME
constexpr uint32_t kExpDecMax = 16384;
__device__ uint64_t g_expDec[3 * kExpDecMax];
#endif
// one block of an independent-block frame into its output slot (k_decode,
// k_decode_walk): the reference's decompressBlockIndependent body
__device__ __forceinline__ int32_t decode_one(const uint8_t* __restrict__ frame, const BlockRec& r, uint32_t b,
                                              uint32_t blockMax, uint8_t* __restrict__ out, uint64_t outCap,
                                              l_u8* ring, l_u8* win) {
    const uint64_t slot = (uint64_t)b * blockMax;
    const int64_t physcap = outCap > slot ? (int64_t)min<uint64_t>(blockMax, outCap - slot) : 0;
    const int64_t len = r.bits & 0x7FFFFFFFu;
    int32_t res;
    if (r.bits & 0x80000000u) {
        if (len > physcap) res = kDecodeOutputTooSmall;
        else { copy_raw(gptr(frame) + r.offset, gptr(out) + slot, len); res = (int32_t)len; }
    } else {
        Dec<false> D;
        D.acc = nullptr;
        D.ts = 0;
        D.src = gptr(frame) + r.offset;
        D.len = len;
        D.dst = gptr(out) + slot;
        D.physcap = physcap;
        D.ring = ring;
        D.win = win;
        D.wlo = INT64_MIN / 4;
        D.labase = INT64_MIN / 4;
        D.la = 0;
        D.flushed = 0;
        D.completed = 0;
        D.lowP = 0;
#if LZ4MT_EXP_BLKTIME
        const uint64_t t0 = wall_clock64();
#endif
        res = decode_block(D, (int64_t)blockMax);
#if LZ4MT_EXP_BLKTIME
        if (laneid() == 0 && b < kExpDecMax) {
            g_expDec[3 * b] = t0;
            g_expDec[3 * b + 1] = wall_clock64();
            g_expDec[3 * b + 2] = ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32) |
                                  (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        }
#endif
    }
    return res;
}

__global__ void __launch_bounds__(64) k_decode(const uint8_t* __restrict__ frame, const BlockRec* __restrict__ recs,
                                               uint32_t blockMax, uint8_t* __restrict__ out, uint64_t outCap,
                                               int32_t* __restrict__ dsize) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWinAlloc];   /* + dummy write area + hop table */
    const uint32_t b = blockIdx.x;
    const int32_t res = decode_one(frame, recs[b], b, blockMax, out, outCap, (l_u8*)ring, (l_u8*)win);
    if (laneid() == 0) dsize[b] = res;
}

// The serial frame walk fused with the decode (wherever the walk is serial,
// §4.6): workgroup 0's lane 0 follows the size words as k_frame_walk does,
// publishing the records found so far every kWalkPub blocks (agent-scope
// release of ctl[0]); every other wave takes block numbers from ctl[2] and
// decodes each one as soon as its record is published.  k_xxh32_walked hashes the blocks on a side stream the same
// way.  Waves wait only on the walker, a resident wave of this grid
// (workgroup 0 is dispatched first), so every wait ends; a 30 s bound keeps
// even a broken invariant from spinning for ever.
// ctl: [0] records published (| kWalkEnded once the walk ended), [2] next
// block to decode, [3] next block group to hash (k_xxh32_walked).
constexpr uint32_t kWalkPub = 8;
__global__ void __launch_bounds__(64) k_decode_walk(const uint8_t* __restrict__ frame, uint64_t frameSize,
                                                    uint64_t bodyPos, uint32_t blockMax, int blockChecksum,
                                                    uint32_t maxBlocks, BlockRec* __restrict__ recs,
                                                    WalkInfo* __restrict__ info, uint32_t* __restrict__ ctl,
                                                    uint8_t* __restrict__ out, uint64_t outCap,
                                                    int32_t* __restrict__ dsize) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWinAlloc];
    const uint32_t L = laneid();
    if (blockIdx.x == 0) __builtin_amdgcn_s_setprio(3);   // the walk gates every decoder: it issues first
    if (blockIdx.x == 0 && L == 0) {
        auto rd32 = [&](uint64_t p) -> uint32_t {
            return (uint32_t)frame[p] | ((uint32_t)frame[p + 1] << 8) | ((uint32_t)frame[p + 2] << 16) |
                   ((uint32_t)frame[p + 3] << 24);
        };
        uint64_t pos = bodyPos;
        uint32_t nb = 0;
        int32_t result = 0;
        for (;;) {   // result codes: src/lz4mt.cpp:685-727 (as k_frame_walk)
            if (pos + 4 > frameSize) { result = 12; break; }
            const uint32_t bits = rd32(pos);
            pos += 4;
            if (bits == 0) break;
            const uint32_t sz = bits & 0x7FFFFFFFu;
            if (sz > blockMax) { result = 20; break; }
            if (pos + sz > frameSize) { result = 13; pos = frameSize; break; }
            BlockRec r{pos, bits, 0};
            pos += sz;
            if (blockChecksum) {
                if (pos + 4 > frameSize) { result = 14; break; }
                r.checksum = rd32(pos);
                pos += 4;
            }
            if (nb >= maxBlocks) { result = 1; break; }
            // write-through (sc1) stores: see walk_publish
            __hip_atomic_store(&recs[nb].offset, r.offset, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(reinterpret_cast<uint64_t*>(&recs[nb].bits),
                               (uint64_t)r.bits | ((uint64_t)r.checksum << 32), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            ++nb;
            if (nb % kWalkPub == 0) walk_publish(ctl, nb);
        }
        const WalkInfo wi{pos, nb, result};
        *info = wi;
        walk_publish(ctl, nb | kWalkEnded);
    }
    // the walker's wave does not decode: after its lane-0 loop, a wave that
    // went on into the decode loop waited out the 30 s bound there (its first
    // poll never matched), so the walk has a wave of its own
    if (blockIdx.x == 0) return;
    for (;;) {
        uint32_t b = 0;
        if (L == 0) b = __hip_atomic_fetch_add(ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
        if (b >= walked_wait(ctl, b + 1)) return;
        const int32_t res = decode_one(frame, recs[b], b, blockMax, out, outCap, (l_u8*)ring, (l_u8*)win);
        // every lane stores the (uniform) result: a lane-0-only store here,
        // at the end of the loop body, was compiled as a divergent loop exit
        // that left lane 0 looping alone, and the wave then waited out the
        // 30 s bound with its other lanes parked
        dsize[b] = res;
        // decode_block's SIMD-mate priority is per block: a wave going back
        // to wait for the walk must not keep it
        __builtin_amdgcn_s_setprio(0);
    }
}

hipError_t launch_decode_walk(const uint8_t* frame, uint64_t frameSize, uint64_t bodyPos, uint32_t blockMax,
                              int blockChecksum, uint32_t maxBlocks, BlockRec* recs, WalkInfo* info, uint32_t* ctl,
                              uint8_t* out, uint64_t outCap, int32_t* dsize, uint32_t waves, hipStream_t st) {
    if (!waves || !maxBlocks) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_decode_walk, dim3(waves), dim3(64), 0, st, frame, frameSize, bodyPos, blockMax, blockChecksum,
                       maxBlocks, recs, info, ctl, out, outCap, dsize);
    return hipGetLastError();
}
#if LZ4MT_EXP_BLKTIME
extern "C" int lz4mtHipExpDecBlockTimes(uint64_t* out, uint32_t nb) {
    if (nb > kExpDecMax) nb = kExpDecMax;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_expDec), (size_t)nb * 24) == hipSuccess ? (int)nb : -1;
}
#endif

__global__ void __launch_bounds__(64) k_decode_stats(const uint8_t* __restrict__ frame,
                                                     const BlockRec* __restrict__ recs, uint32_t blockMax,
                                                     uint8_t* __restrict__ out, uint64_t outCap,
                                                     int32_t* __restrict__ dsize, uint64_t* __restrict__ stats) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWinAlloc];   /* + dummy write area + hop table */
    const uint32_t b = blockIdx.x;
    const BlockRec r = recs[b];
    const uint64_t slot = (uint64_t)b * blockMax;
    uint64_t acc[16] = {0};
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    Dec<true> D;
    D.acc = acc;
    D.ts = t0;
    D.src = gptr(frame) + r.offset;
    D.len = r.bits & 0x7FFFFFFFu;
    D.dst = gptr(out) + slot;
    D.physcap = (int64_t)min<uint64_t>(blockMax, outCap - slot);
    D.ring = (l_u8*)ring;
    D.win = (l_u8*)win;
    D.wlo = INT64_MIN / 4;
    D.labase = INT64_MIN / 4;
    D.la = 0;
    D.flushed = 0;
    D.completed = 0;
    D.lowP = 0;
    const int32_t res = decode_block(D, (int64_t)blockMax);
    acc[5] = __builtin_amdgcn_s_memtime() - t0;
    if (laneid() == 0) {
        dsize[b] = res;
        for (int i = 0; i < 16; ++i) stats[b * 16 + i] = acc[i];
    }
}

// byte copy by one wave; 16-byte pieces when both ends share the alignment
__device__ void wave_copy(g_u8* __restrict__ dst, g_cu8* __restrict__ src, int64_t n) {
    const uint32_t L = laneid();
    int64_t i = 0;
    if (((reinterpret_cast<uintptr_t>(dst) ^ reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
        const int64_t head = min<int64_t>(n, (int64_t)((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15));
        if ((int64_t)L < head) dst[L] = src[L];
        i = head;
        for (; i + 1024 <= n; i += 1024) *(g_u4*)(dst + i + 16 * L) = *(g_cu4*)(src + i + 16 * L);
    }
    for (; i < n; i += 64)
        if (i + L < n) dst[i + L] = src[i + L];
}

// Block-dependent frames (-BD, reference decompressBlockDependency,
// src/lz4mt.cpp:737-845): ONE wave decodes the blocks in order.  Each block
// is checked against its checksum BEFORE it is decoded (the reference's
// order there), then decoded by LZ4_decompress_safe_withPrefix64k rules
// into `slot` = [64 KiB history | blockMax], the history being the last 64
// KiB of (hist ++ this call's output so far); the bytes are then appended
// to out.  `hist` (64 KiB, device) is the history before the call (zeros
// for a new frame: the reference's zero-filled MemPool buffer) and receives
// the history after it.  status[0] = blocks completed, status[1] = the
// Lz4MtResult of the block that stopped the call (0 = none).
__global__ void __launch_bounds__(64) k_decode_linked(const uint8_t* __restrict__ frame,
                                                      const BlockRec* __restrict__ recs, uint32_t nBlocks,
                                                      uint32_t blockMax, uint8_t* __restrict__ out, uint64_t outCap,
                                                      uint8_t* __restrict__ slot, uint8_t* __restrict__ hist,
                                                      const uint32_t* __restrict__ digest, int bck,
                                                      int32_t* __restrict__ dsize, int32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWinAlloc];
    const uint32_t L = laneid();
    g_u8* const sl = gptr(slot);
    g_u8* const o = gptr(out);
    int64_t opos = 0;
    uint32_t b = 0;
    int32_t code = 0;
    // history [0, 65536) of the slot: the 64 KiB before output position opos
    auto load_hist = [&](int64_t at) {
        for (int64_t i = 16 * L; i < 65536; i += 1024) {
            const int64_t x = at - 65536 + i;
            v4u v;
            if (x >= 0) {
                g_cu8* p = (g_cu8*)o + x;
                v = (v4u){ld32u(p), ld32u(p + 4), ld32u(p + 8), ld32u(p + 12)};
            } else {   // (partly) before this call's output: bytes of hist
                uint8_t t[16];
                for (int k = 0; k < 16; ++k) t[k] = x + k < 0 ? gptr(hist)[65536 + x + k] : o[x + k];
                v = (v4u){(uint32_t)t[0] | t[1] << 8 | t[2] << 16 | (uint32_t)t[3] << 24,
                          (uint32_t)t[4] | t[5] << 8 | t[6] << 16 | (uint32_t)t[7] << 24,
                          (uint32_t)t[8] | t[9] << 8 | t[10] << 16 | (uint32_t)t[11] << 24,
                          (uint32_t)t[12] | t[13] << 8 | t[14] << 16 | (uint32_t)t[15] << 24};
            }
            *(g_u4*)(sl + i) = v;
        }
        // the slot is reused block after block: wait for these stores and
        // drop the vector L1's lines of it (the previous block's decode read
        // them), or this block's far reads could see the old bytes
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        WAVE_SYNC();
    };
    for (; b < nBlocks; ++b) {
        const BlockRec r = recs[b];
        const int64_t len = r.bits & 0x7FFFFFFFu;
        if (bck && digest[b] != r.checksum) { code = 16; break; }   // BLOCK_CHECKSUM_MISMATCH, nothing written
        load_hist(opos);
        int32_t res;
        if (r.bits & 0x80000000u) {
            copy_raw(gptr(frame) + r.offset, sl + 65536, len);
            res = (int32_t)len;
        } else {
            Dec<false> D;
            D.acc = nullptr;
            D.ts = 0;
            D.src = gptr(frame) + r.offset;
            D.len = len;
            D.dst = sl + 65536;
            D.physcap = blockMax;
            D.ring = (l_u8*)ring;
            D.win = (l_u8*)win;
            D.wlo = INT64_MIN / 4;
            D.labase = INT64_MIN / 4;
            D.la = 0;
            D.flushed = 0;
            D.completed = 0;
            D.lowP = -65536;
            res = decode_block(D, (int64_t)blockMax);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        WAVE_SYNC();
        if (L == 0) dsize[b] = res;
        if (res < 0) { code = 18; break; }                               // DECOMPRESS_FAIL
        if ((uint64_t)opos + (uint64_t)res > outCap) { code = 1; break; }   // ERROR: output too small
        wave_copy(o + opos, sl + 65536, res);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the next history read sees these bytes
        WAVE_SYNC();
        opos += res;
    }
    load_hist(opos);   // the history after this call -> hist
    for (int64_t i = 16 * L; i < 65536; i += 1024) *(g_u4*)(gptr(hist) + i) = *(g_cu4*)(sl + i);
    if (L == 0) { status[0] = (int32_t)b; status[1] = code; }
}

hipError_t launch_decode_linked(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t blockMax,
                                uint8_t* out, uint64_t outCap, uint8_t* slot, uint8_t* hist, const uint32_t* digest,
                                int blockChecksum, int32_t* dsize, int32_t* status, hipStream_t st) {
    hipLaunchKernelGGL(k_decode_linked, dim3(1), dim3(64), 0, st, frame, recs, nBlocks, blockMax, out, outCap, slot,
                       hist, digest, blockChecksum, dsize, status);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Block-dependent decode in parallel rounds.  Block b's output depends on
// the 64 KiB decoded before it; its SIZE and its errors do not (LZ4
// withPrefix64k rules: offsets, lengths and bounds come from the token
// stream alone).  So:
//   round 0   every block decodes at once into its slot [64 KiB history |
//             blockMax] (slot 0's history = the call's exact history, the
//             others a guess); k_dlink_plan turns the sizes, checksums and
//             outCap into output offsets and the first stopping block
//             (nOk, code: the serial order of checks);
//   gather    k_dlink_gather rebuilds every block's history from the
//             current outputs (the 64 KiB before start[b] in hist0 ++
//             outputs) and compares it with the one the block was decoded
//             against; a block whose history changed is queued for the next
//             round (flag[b] = r + 1);
//   rounds    only queued blocks decode again.
// A gather that changes nothing means every block decoded against the
// history its predecessors really produce: by induction from block 0 (exact
// history) the outputs are the serial decoder's.  Matches reach back at
// most 64 KiB, so wrong bytes die out within a few rounds on real data; if
// kLinkRounds do not settle, one wave finishes serially from the first
// unsettled block (k_dlink_serial).  k_dlink_compact then writes the
// outputs back to back and k_dlink_hist_out the history after the call.
//   ctl words: changed[R + 1] | first[R + 1] | flag[nBlocks] | nOk, code, pad, pad
//   then start[nBlocks] (u64, 8-byte aligned)
constexpr int64_t kDHist = 65536;
__host__ __device__ __forceinline__ uint64_t dlink_stride(uint32_t blockMax) {
    return (uint64_t)kDHist + (((uint64_t)blockMax + 15) & ~15ull);
}

__device__ __forceinline__ int32_t dlink_decode(const uint8_t* frame, const BlockRec& r, uint32_t blockMax,
                                                g_u8* out, l_u8* ring, l_u8* win) {
    const int64_t len = r.bits & 0x7FFFFFFFu;
    if (r.bits & 0x80000000u) {
        if (len > (int64_t)blockMax) return kDecodeOutputTooSmall;
        copy_raw(gptr(frame) + r.offset, out, len);
        return (int32_t)len;
    }
    Dec<false> D;
    D.acc = nullptr;
    D.ts = 0;
    D.src = gptr(frame) + r.offset;
    D.len = len;
    D.dst = out;
    D.physcap = blockMax;
    D.ring = ring;
    D.win = win;
    D.wlo = INT64_MIN / 4;
    D.labase = INT64_MIN / 4;
    D.la = 0;
    D.flushed = 0;
    D.completed = 0;
    D.lowP = -65536;
    return decode_block(D, (int64_t)blockMax);
}

__global__ void __launch_bounds__(64) k_dlink_round(const uint8_t* __restrict__ frame,
                                                    const BlockRec* __restrict__ recs, uint32_t blockMax,
                                                    uint8_t* __restrict__ slots, int32_t* __restrict__ dsize,
                                                    const uint32_t* __restrict__ gate,
                                                    const uint32_t* __restrict__ flag, const uint32_t* __restrict__ nOk,
                                                    uint32_t round) {
    const uint32_t b = blockIdx.x;
    if (*gate == 0 || flag[b] != round || (round > 0 && b >= *nOk)) return;
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWinAlloc];
    const BlockRec r = recs[b];
    const int32_t res = dlink_decode(frame, r, blockMax, gptr(slots) + b * dlink_stride(blockMax) + kDHist,
                                     (l_u8*)ring, (l_u8*)win);
    if (round == 0 && laneid() == 0) dsize[b] = res;
}

// The serial order of the per-block checks (k_decode_linked): checksum,
// decode, output room.  One workgroup; start[] = exclusive scan of the
// sizes up to the first stopping block.
__global__ void __launch_bounds__(1024) k_dlink_plan(const BlockRec* __restrict__ recs,
                                                     const uint32_t* __restrict__ digest, int bck,
                                                     const int32_t* __restrict__ dsize, uint32_t nBlocks,
                                                     uint64_t outCap, uint64_t* __restrict__ start,
                                                     uint32_t* __restrict__ misc, int32_t* __restrict__ status) {
    __shared__ uint64_t sc[1024];
    __shared__ uint32_t stopAt;
    const uint32_t t = threadIdx.x;
    uint64_t carry = 0;
    uint32_t nOk = nBlocks;
    int32_t code = 0;
    for (uint32_t c = 0; c < nBlocks; c += 1024) {
        const uint32_t b = c + t;
        int32_t bad = 0;
        uint64_t v = 0;
        if (b < nBlocks) {
            const BlockRec r = recs[b];
            const int32_t d = dsize[b];
            if (bck && digest[b] != r.checksum) bad = 16;
            else if (d < 0) bad = 18;
            else v = (uint64_t)d;
        }
        sc[t] = v;
        if (t == 0) stopAt = 0xFFFFFFFFu;
        __syncthreads();
        for (uint32_t k = 1; k < 1024; k <<= 1) {   // inclusive scan
            const uint64_t x = t >= k ? sc[t - k] : 0;
            __syncthreads();
            sc[t] += x;
            __syncthreads();
        }
        const uint64_t st = carry + sc[t] - v;
        if (b < nBlocks && !bad && st + v > outCap) bad = 1;
        if (bad) atomicMin(&stopAt, b);
        __syncthreads();
        const uint32_t stop = stopAt;
        if (b < nBlocks && b < stop) start[b] = st;
        if (stop != 0xFFFFFFFFu) {
            nOk = stop;
            if (b == stop) misc[1] = (uint32_t)bad;   // the stopping block's code
            break;
        }
        carry += sc[1023];
        __syncthreads();
    }
    __syncthreads();
    if (t == 0) {
        misc[0] = nOk;
        if (nOk == nBlocks) misc[1] = 0;
    }
    __syncthreads();
    if (t == 0) {
        status[0] = (int32_t)nOk;
        status[1] = (int32_t)misc[1];
    }
    (void)code;
}

// history byte g (< start of the call: hist0) of the stream hist0 ++ outputs
__device__ __forceinline__ uint8_t dlink_byte(int64_t g, uint32_t k, const uint64_t* start, const int32_t* dsize,
                                              g_cu8* slots, uint64_t stride, g_cu8* hist0) {
    (void)dsize;
    return g < 0 ? hist0[kDHist + g] : slots[k * stride + kDHist + (uint64_t)(g - (int64_t)start[k])];
}

// Rebuilds block b's history (the kDHist bytes before start[b]) with
// nThreads threads, comparing with (and overwriting) the slot's; returns
// this thread's "differs".  Fast path: the whole history inside block b-1's
// output at a 4-byte aligned offset.
__device__ bool dlink_gather(uint32_t b, uint32_t t, uint32_t nThreads, const uint64_t* start, const int32_t* dsize,
                             g_u8* slots, uint64_t stride, g_cu8* hist0) {
    const int64_t hi = b ? (int64_t)start[b] : 0, lo = hi - kDHist;
    g_u8* h = slots + b * stride;
    bool diff = false;
    if (b > 0 && (int64_t)start[b - 1] <= lo && (((uint64_t)(lo - (int64_t)start[b - 1])) & 3) == 0) {
        g_cu8* src = slots + (b - 1) * stride + kDHist + (uint64_t)(lo - (int64_t)start[b - 1]);
        for (uint32_t i = 4 * t; i < kDHist; i += 4 * nThreads) {
            const uint32_t v = *(g_cu32*)(src + i);
            g_u32* d = (g_u32*)(h + i);
            if (*d != v) { *d = v; diff = true; }
        }
        return diff;
    }
    // general: walk back over the blocks that hold [lo, hi)
    int64_t top = hi;
    for (int64_t k = (int64_t)b - 1; top > lo; --k) {
        const int64_t s0 = k >= 0 ? (int64_t)start[k] : INT64_MIN / 4;
        const int64_t from = s0 > lo ? s0 : lo;
        for (int64_t g = from + t; g < top; g += nThreads) {
            const uint8_t v = k >= 0 ? slots[(uint64_t)k * stride + kDHist + (uint64_t)(g - s0)]
                                     : hist0[kDHist + g];
            g_u8* d = h + (g - lo);
            if (*d != v) { *d = v; diff = true; }
        }
        top = from;
        if (k < 0) break;
    }
    return diff;
}

__global__ void __launch_bounds__(256) k_dlink_gather(uint8_t* __restrict__ slots, uint64_t stride,
                                                      const uint64_t* __restrict__ start,
                                                      const int32_t* __restrict__ dsize, const uint8_t* __restrict__ hist0,
                                                      const uint32_t* __restrict__ misc,
                                                      const uint32_t* __restrict__ gate, uint32_t* __restrict__ flag,
                                                      uint32_t* __restrict__ changedNext,
                                                      uint32_t* __restrict__ firstNext, uint32_t round) {
    const uint32_t b = blockIdx.x + 1;   // block 0's history is the call's: exact from the start
    if (*gate == 0 || b >= misc[0]) return;
    __shared__ uint32_t any;
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    if (dlink_gather(b, threadIdx.x, 256, start, dsize, gptr(slots), stride, gptr(hist0))) atomicOr(&any, 1u);
    __syncthreads();
    if (threadIdx.x == 0 && any) {
        flag[b] = round + 1;
        atomicAdd(changedNext, 1u);
        atomicMin(firstNext, b);
    }
}

// the rounds did not settle: one wave, in order, from the first unsettled block
__global__ void __launch_bounds__(64) k_dlink_serial(const uint8_t* __restrict__ frame,
                                                     const BlockRec* __restrict__ recs, uint32_t blockMax,
                                                     uint8_t* __restrict__ slots, const uint64_t* __restrict__ start,
                                                     const int32_t* __restrict__ dsize,
                                                     const uint8_t* __restrict__ hist0,
                                                     const uint32_t* __restrict__ misc,
                                                     const uint32_t* __restrict__ gate,
                                                     const uint32_t* __restrict__ firstp) {
    if (*gate == 0) return;
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWinAlloc];
    const uint64_t stride = dlink_stride(blockMax);
    const uint32_t nOk = misc[0];
    for (uint32_t b = *firstp; b < nOk; ++b) {
        dlink_gather(b, laneid(), 64, start, dsize, gptr(slots), stride, gptr(hist0));
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the decode's far reads see the new history
        WAVE_SYNC();
        dlink_decode(frame, recs[b], blockMax, gptr(slots) + b * stride + kDHist, (l_u8*)ring, (l_u8*)win);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the next gather sees these bytes
        WAVE_SYNC();
    }
}

__global__ void __launch_bounds__(256) k_dlink_compact(const uint8_t* __restrict__ slots, uint64_t stride,
                                                       const uint64_t* __restrict__ start,
                                                       const int32_t* __restrict__ dsize,
                                                       const uint32_t* __restrict__ misc, uint8_t* __restrict__ out) {
    const uint32_t b = blockIdx.x;
    if (b >= misc[0]) return;
    g_cu8* src = gptr(slots) + b * stride + kDHist;
    g_u8* dst = gptr(out) + start[b];
    const int64_t n = dsize[b];
    const uint32_t t = threadIdx.x;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        const int64_t n16 = n & ~int64_t(15);
        for (int64_t i = 16 * (int64_t)t; i < n16; i += 16 * 256) *(g_u4*)(dst + i) = *(g_cu4*)(src + i);
        for (int64_t i = n16 + t; i < n; i += 256) dst[i] = src[i];
    } else {
        for (int64_t i = t; i < n; i += 256) dst[i] = src[i];
    }
}

// the history after the call: the last 64 KiB of hist0 ++ out[0, end)
// (hist0 read from slot 0's copy: histOut may be the caller's hist0)
__global__ void __launch_bounds__(1024) k_dlink_hist_out(const uint8_t* __restrict__ out,
                                                         const uint8_t* __restrict__ slot0,
                                                         const uint64_t* __restrict__ start,
                                                         const int32_t* __restrict__ dsize,
                                                         const uint32_t* __restrict__ misc,
                                                         uint8_t* __restrict__ histOut) {
    const uint32_t nOk = misc[0];
    const int64_t end = nOk ? (int64_t)(start[nOk - 1] + (uint64_t)dsize[nOk - 1]) : 0;
    for (int64_t i = threadIdx.x; i < kDHist; i += 1024) {
        const int64_t g = end - kDHist + i;
        histOut[i] = g < 0 ? slot0[kDHist + g] : out[g];
    }
}

__global__ void k_dlink_init(uint32_t* __restrict__ ctl, uint32_t nBlocks) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t R = kLinkRounds + 1;
    if (i < R) ctl[i] = i == 0 ? 1u : 0u;
    else if (i < 2 * R) ctl[i] = 0xFFFFFFFFu;
    else if (i < 2 * R + nBlocks + 4) ctl[i] = 0u;
}

uint64_t dlink_scratch_bytes(uint64_t nBlocks, uint32_t blockMax) {
    const uint64_t ctl = ((2 * (uint64_t)(kLinkRounds + 1) + nBlocks + 4) * 4 + 15) & ~15ull;
    return nBlocks * dlink_stride(blockMax) + ctl + nBlocks * 8;
}

hipError_t launch_decode_linked_par(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t blockMax,
                                    uint8_t* out, uint64_t outCap, uint8_t* hist, const uint32_t* digest,
                                    int blockChecksum, int32_t* dsize, int32_t* status, uint8_t* scratch, int rounds,
                                    hipStream_t st) {
    if (rounds < 1 || rounds > kLinkRounds) rounds = kLinkRounds;
    if (nBlocks == 0) {   // nothing decoded: status {0, 0}, the history unchanged
        return hipMemsetAsync(status, 0, 8, st);
    }
    const uint64_t stride = dlink_stride(blockMax);
    uint8_t* slots = scratch;
    uint32_t* ctl = reinterpret_cast<uint32_t*>(scratch + nBlocks * stride);
    const uint32_t R = kLinkRounds + 1;
    uint32_t* changed = ctl;
    uint32_t* firstU = ctl + R;
    uint32_t* flag = firstU + R;
    uint32_t* misc = flag + nBlocks;
    uint64_t* start = reinterpret_cast<uint64_t*>(
        scratch + nBlocks * stride + (((2 * (uint64_t)R + nBlocks + 4) * 4 + 15) & ~15ull));
    // slot 0's history: the call's (exact); the others start from a guess
    if (hipMemcpyAsync(slots, hist, kDHist, hipMemcpyDeviceToDevice, st) != hipSuccess) return hipErrorUnknown;
    const uint32_t nInit = 2 * R + nBlocks + 4;
    hipLaunchKernelGGL(k_dlink_init, dim3((nInit + 255) / 256), dim3(256), 0, st, ctl, nBlocks);
    hipLaunchKernelGGL(k_dlink_round, dim3(nBlocks), dim3(64), 0, st, frame, recs, blockMax, slots, dsize,
                       (const uint32_t*)changed, (const uint32_t*)flag, (const uint32_t*)misc, 0u);
    hipLaunchKernelGGL(k_dlink_plan, dim3(1), dim3(1024), 0, st, recs, digest, blockChecksum, (const int32_t*)dsize,
                       nBlocks, outCap, start, misc, status);
    for (int r = 0; r < rounds; ++r) {
        if (r > 0)
            hipLaunchKernelGGL(k_dlink_round, dim3(nBlocks), dim3(64), 0, st, frame, recs, blockMax, slots, dsize,
                               (const uint32_t*)(changed + r), (const uint32_t*)flag, (const uint32_t*)misc,
                               (uint32_t)r);
        if (nBlocks > 1)
            hipLaunchKernelGGL(k_dlink_gather, dim3(nBlocks - 1), dim3(256), 0, st, slots, stride,
                               (const uint64_t*)start, (const int32_t*)dsize, (const uint8_t*)slots,
                               (const uint32_t*)misc, (const uint32_t*)(changed + r), flag, changed + r + 1,
                               firstU + r + 1, (uint32_t)r);
    }
    hipLaunchKernelGGL(k_dlink_serial, dim3(1), dim3(64), 0, st, frame, recs, blockMax, slots, (const uint64_t*)start,
                       (const int32_t*)dsize, (const uint8_t*)slots, (const uint32_t*)misc,
                       (const uint32_t*)(changed + rounds), (const uint32_t*)(firstU + rounds));
    hipLaunchKernelGGL(k_dlink_compact, dim3(nBlocks), dim3(256), 0, st, (const uint8_t*)slots, stride,
                       (const uint64_t*)start, (const int32_t*)dsize, (const uint32_t*)misc, out);
    hipLaunchKernelGGL(k_dlink_hist_out, dim3(1), dim3(1024), 0, st, (const uint8_t*)out, (const uint8_t*)slots,
                       (const uint64_t*)start, (const int32_t*)dsize, (const uint32_t*)misc, hist);
    link_stats("decode", changed, firstU, rounds, nBlocks, st);
    return hipGetLastError();
}

hipError_t launch_decode_stats(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t blockMax,
                               uint8_t* out, uint64_t outCap, int32_t* dsize, uint64_t* stats, hipStream_t st) {
    hipLaunchKernelGGL(k_decode_stats, dim3(nBlocks), dim3(64), 0, st, frame, recs, blockMax, out, outCap, dsize,
                       stats);
    return hipGetLastError();
}
#endif


#if LZ4MT_PART != 2
hipError_t launch_encode_stats(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                               uint8_t* slots, int32_t* csize, uint64_t* stats, hipStream_t st) {
    if (const hipError_t r = encoder_ready(st); r != hipSuccess) return r;
    hipLaunchKernelGGL(k_encode_stats, dim3(nBlocks), dim3(64), 0, st, src, srcSize, blockSize, slots,
                       (uint64_t)blockSize, csize, stats);
    return hipGetLastError();
}
#endif


#if LZ4MT_PART != 1
hipError_t launch_decode(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t blockMax, uint8_t* out,
                         uint64_t outCap, int32_t* dsize, hipStream_t st) {
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode, dim3(nBlocks), dim3(64), 0, st, frame, recs, blockMax, out, outCap, dsize);
    return hipGetLastError();
}
#endif


#if LZ4MT_PART != 2
// ---------------------------------------------------------------------------
// XXH32: 4 lanes per block (one per accumulator), 16 blocks per wavefront
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xround(uint32_t acc, uint32_t w) { return rotl32(acc + w * kP2, 13) * kP1; }
// a round on a word premultiplied by P2 (LLVM fuses the multiply with the
// next round's add into one v_mad_u64_u32: the chain is alignbit + mad;
// an unfused v_mul_lo_u32 + v_add_u32 was slower, profiles/r03n_xxh32_ab.txt)
__device__ __forceinline__ uint32_t xround_pm(uint32_t acc, uint32_t wp) { return rotl32(acc + wp, 13) * kP1; }

// One wavefront hashes one byte range: the range streams through LDS in
// 1 KiB chunks (64 lanes x 16 B, loaded one chunk ahead), lanes 0..3 run
// the four accumulator chains (v1..v4 of XXH32) over each chunk.
__device__ __forceinline__ v4u load16u(g_cu8* p) {   // 16 bytes at any alignment
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    g_cu32* q = (g_cu32*)(p - sh);
    const uint32_t a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
    const uint32_t a4 = sh ? q[4] : 0u;
    v4u v;
    v.x = __builtin_amdgcn_alignbyte(a1, a0, sh);
    v.y = __builtin_amdgcn_alignbyte(a2, a1, sh);
    v.z = __builtin_amdgcn_alignbyte(a3, a2, sh);
    v.w = __builtin_amdgcn_alignbyte(a4, a3, sh);
    return v;
}

__device__ uint32_t xxh32_wave(g_cu8* p, uint64_t len, l_u32* __restrict__ buf /* 512 dwords */) {
    const uint32_t L = laneid();
    uint32_t v = (L == 0) ? kP1 + kP2 : (L == 1) ? kP2 : (L == 2) ? 0u : (uint32_t)(0u - kP1);
    const uint64_t ns = len >> 4;            // whole 16-byte stripes
    const uint64_t nch = (ns + 63) >> 6;     // 1 KiB chunks
    v4u r = {0, 0, 0, 0};
    if (nch && (uint64_t)L < ns) r = load16u(p + 16 * L);
    uint32_t cur = 0;
    for (uint64_t ch = 0; ch < nch; ++ch) {
        // words stored premultiplied by P2 (64 lanes at once): the chain
        // below keeps only rotl + mul per round
        ((l_u4*)(buf + cur * 256))[L] = (v4u){r.x * kP2, r.y * kP2, r.z * kP2, r.w * kP2};
        const uint64_t nxt = (ch + 1) * 64 + L;
        if (ch + 1 < nch && nxt < ns) r = load16u(p + 16 * nxt);
        WAVE_SYNC();
        if (L < 4) {
            const uint32_t m = (uint32_t)min<uint64_t>(64, ns - ch * 64);
            const l_u32* cb = buf + cur * 256 + L;
            uint32_t i = 0;
            // a whole 1 KiB chunk: all 64 LDS reads in flight before its rounds
            // (k_xxh32_stored 4.05 -> 3.78 ms at 8 GiB, profiles/r03n_xxh32_ab.txt;
            // full-rate 24-bit multiplies for the round: 5.83 ms, r05ad_xxh32_m24_ab.txt)
            if (m == 64) {
                uint32_t w[64];
#pragma unroll
                for (int u = 0; u < 64; ++u) w[u] = cb[4 * u];
#pragma unroll
                for (int u = 0; u < 64; ++u) v = xround_pm(v, w[u]);
                i = 64;
            }
            for (; i + 8 <= m; i += 8) {
                uint32_t w[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) w[u] = cb[4 * (i + u)];
#pragma unroll
                for (int u = 0; u < 8; ++u) v = xround_pm(v, w[u]);
            }
            for (; i < m; ++i) v = xround_pm(v, cb[4 * i]);
        }
        WAVE_SYNC();
        cur ^= 1;
    }
    const uint32_t v1 = rdlane(v, 0), v2 = rdlane(v, 1), v3 = rdlane(v, 2), v4 = rdlane(v, 3);
    uint32_t h = len >= 16 ? rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18) : kP5;
    h += (uint32_t)len;
    uint64_t o = ns << 4;
    for (; o + 4 <= len; o += 4) h = rotl32(h + ld32u(p + o) * kP3, 17) * kP4;
    for (; o < len; ++o) h = rotl32(h + p[o] * kP5, 11) * kP1;
    h ^= h >> 15; h *= kP2; h ^= h >> 13; h *= kP3; h ^= h >> 16;
    return h;
}

// Block checksums: 16 blocks per wavefront, one quad of lanes per block,
// lane c of the quad runs accumulator v(c+1).  No LDS at all, so these waves
// can run beside the decode (whose eight 20 KiB waves fill a CU's LDS)
// without taking a decode slot.  Lane c reads the aligned dword 4s+c of
// stripe s (one coalesced 16 B per quad and stripe); the unaligned word is
// alignbyte(next, this) where `next` is the quad neighbour's dword (DPP
// quad rotate) or, for lane 3, lane 0's dword of the next stripe.  Only
// dwords holding requested bytes are read.  Loads run one batch ahead of
// the rounds.
constexpr int kXqBatch = 32;

__device__ __forceinline__ uint32_t quad_rot1(uint32_t x) {   // lane c <- lane (c+1)&3 of its quad
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x39, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t quad_get(uint32_t x, uint32_t c) {   // lane c of the caller's quad
    return (uint32_t)__shfl((int)x, (int)((laneid() & ~3u) | c), 64);
}

// dword index clamped to the last one holding a requested byte (no
// divergent loads; a clamped value is never used)
__device__ __forceinline__ void xq_load(uint32_t (&w)[kXqBatch], g_cu32* q, uint32_t s0, uint32_t c, uint32_t last) {
#pragma unroll
    for (int u = 0; u < kXqBatch; ++u) w[u] = q[min(4u * (s0 + u) + c, last)];
}

__device__ __forceinline__ uint32_t xq_rounds(uint32_t v, const uint32_t (&w)[kXqBatch], uint32_t nxt, uint32_t s0,
                                              uint32_t ns, uint32_t sh, bool lane3) {
#pragma unroll
    for (int u = 0; u < kXqBatch; ++u) {
        const uint32_t lo = w[u];
        const uint32_t r0 = quad_rot1(lo);
        const uint32_t r1 = quad_rot1(u + 1 < kXqBatch ? w[u + 1] : nxt);
        const uint32_t word = __builtin_amdgcn_alignbyte(lane3 ? r1 : r0, lo, sh);
        v = (s0 + u < ns) ? xround(v, word) : v;
    }
    return v;
}

// XXH32 (seed 0) of [p, p+len) for the quad's block; every lane of the quad
// returns the digest.  All 64 lanes must call it (DPP reads neighbours).
// Kept a called function (three call sites): inlined, the decode it runs
// beside is 0.3 ms slower (30.9 -> 31.2 ms at 8 GiB;
// profiles/r04m_xxh32_quad_inline_ab.txt)
__device__ __noinline__ uint32_t xxh32_quad(g_cu8* p, uint32_t len, g_cu8* safe /* any readable byte */) {
    const uint32_t c = laneid() & 3u;
    const uint32_t ns = len >> 4;
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    // dword i holds requested bytes iff i < 4ns + (sh != 0); with no stripe
    // the (unused) loads all read the dword holding `safe`
    g_cu8* base = ns ? p : safe;
    g_cu32* q = (g_cu32*)(base - (reinterpret_cast<uintptr_t>(base) & 3));
    const uint32_t last = ns ? 4u * ns - (sh ? 0u : 1u) : 0u;
    uint32_t nsMax = 0;
#pragma unroll
    for (int g = 0; g < 16; ++g) nsMax = max(nsMax, rdlane(ns, 4 * g));
    uint32_t v = (c == 0) ? kP1 + kP2 : (c == 1) ? kP2 : (c == 2) ? 0u : (uint32_t)(0u - kP1);
    const bool lane3 = (c == 3);
    uint32_t wa[kXqBatch], wb[kXqBatch];
    xq_load(wa, q, 0, c, last);
    for (uint32_t s0 = 0; s0 < nsMax; s0 += 2 * kXqBatch) {
        xq_load(wb, q, s0 + kXqBatch, c, last);
        v = xq_rounds(v, wa, wb[0], s0, ns, sh, lane3);
        if (s0 + kXqBatch >= nsMax) break;
        xq_load(wa, q, s0 + 2 * kXqBatch, c, last);
        v = xq_rounds(v, wb, wa[0], s0 + kXqBatch, ns, sh, lane3);
    }
    const uint32_t v1 = quad_get(v, 0), v2 = quad_get(v, 1), v3 = quad_get(v, 2), v4 = quad_get(v, 3);
    uint32_t h = len >= 16 ? rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18) : kP5;
    h += len;
    uint32_t o = ns << 4;
    for (; o + 4 <= len; o += 4) h = rotl32(h + ld32u(p + o) * kP3, 17) * kP4;
    for (; o < len; ++o) h = rotl32(h + p[o] * kP5, 11) * kP1;
    h ^= h >> 15; h *= kP2; h ^= h >> 13; h *= kP3; h ^= h >> 16;
    return h;
}

// stored bytes of compress-side block b: the slot if it compressed, else the
// source.  A wave per block (xxh32_wave): on the compress side the checksums
// run beside the short scan + assembly, where the wave-per-block kernel
// finishes sooner than the 16-blocks-per-wave one (measured 40.9 vs 41.5
// GiB/s compress at 8 GiB).
__global__ void __launch_bounds__(64) k_xxh32_stored(const uint8_t* __restrict__ src, const uint8_t* __restrict__ slots,
                                                     uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                                                     const int32_t* __restrict__ csize, uint32_t* __restrict__ digest) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[512];
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const int32_t cs = csize[b];
    const uint32_t h = xxh32_wave(cs > 0 ? gptr(slots) + off : gptr(src) + off, cs > 0 ? (uint64_t)cs : n, (l_u32*)buf);
    if (laneid() == 0) digest[b] = h;
}

// ---------------------------------------------------------------------------
// Streamed compress: lz4mtCompress over the callbacks (MODE_DEVICE, or a
// relinked PARALLEL caller), independent 1 / 4 MiB blocks, levels 0..2
// (reference compress(), src/lz4mt.cpp:372-457, and the
// FILE* reads of src/lz4mt_io_cstdio.cpp:112-118).  Batches of blocks staged
// to HBM and encoded by one launch each leave a whole block latency plus the
// last batch's copy after the final read(); here ONE persistent grid encodes
// every block as soon as the host has read it:
//   * the host reads block b into in[b % Rin] (coherent pinned memory: GPU
//     reads of it are never served from a GPU cache), then publishes its
//     length and b + 1 in that slot's control words;
//   * a wave takes the next block number (a device counter), waits for it
//     (system-scope polls with s_sleep), copies it into its own HBM buffer,
//     marks the staging slot free, encodes it (the frame encoder's code, its
//     own instantiation), hashes the stored bytes (block XXH32), waits until
//     out[b % Rout] is free, pushes the stored bytes there (coherent pinned)
//     and publishes size word, checksum and b + 1;
//   * a host writer thread calls write() record by record in block order as
//     they appear.
// Every wait gives up after `ticks` (LZ4MT_AMD_STREAM_TIMEOUT_S, 60 s by
// default) without progress of the other side -- its heartbeat word, or the
// host's liveness word, which a host thread bumps while a read() / write()
// callback is running (a slow pipe is not a hang) -- so the grid always
// drains; the host sets the block count once read() returns 0 and every wave
// still waiting leaves.
// Control words (u32, coherent pinned host memory):
//   g[0] blocks in the stream (0xFFFFFFFF until known)  g[1] abort (host)
//   g[2] blocks read (heartbeat)  g[3] records written (heartbeat)
//   g[4] error (GPU: a wait timed out)  g[5] host liveness (inside a callback)
//   g[7] park (host: a read() or a write() stalled -- waves waiting for an
//        unpublished block leave, waves waiting for an output slot leave
//        their block in their HBM buffers with a descriptor in pend[]; the
//        host relaunches the grid at its next block once the stall ends, and
//        each wave first finishes the block it parked with)
//   in[r]  {seq = b + 1, length, pulled = b + 1}   (4 words per slot)
//   out[r] {seq = b + 1, size word, XXH32, written = b + 1}
// A waiting wave sleeps in proportion to how far the awaited heartbeat is
// from its target (~35 us per block still to come, at most ~1.8 ms), so 2048
// waves waiting for blocks far ahead of the reader cost the PCIe link only a
// few hundred thousand small reads per second.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// n bytes, both sides 16-byte aligned: dwordx4 per lane, 8 in flight
__device__ __forceinline__ void wave_copy16(g_u8* d, g_cu8* s, uint32_t n) {
    const uint32_t L = laneid(), n16 = n >> 4;
    for (uint32_t i = L; i < n16; i += 64 * 8) {
        v4u v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (i + 64 * k < n16) v[k] = ((g_cu4*)s)[i + 64 * k];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (i + 64 * k < n16) ((g_u4*)d)[i + 64 * k] = v[k];
    }
    for (uint32_t i = (n16 << 4) + L; i < n; i += 64) d[i] = s[i];
}
// Waits until *w == want.  hb: the heartbeat (2 = blocks read, 3 = records
// written) that reaches `target` when *w is about to change.  kWaitOk, or
// kWaitStop on abort, on a timeout (`ticks` of s_memrealtime, 100 MHz,
// without a change of the heartbeat or of the host's liveness word g[5]; g[4]
// set), or -- endAt >= 0 -- once the stream is known to hold no block endAt
// (*ended); kWaitPark when the host parked the grid (g[7]): an input wait
// (hb 2) re-reads *w after seeing the park word, so a block published before
// the park is always taken (the host publishes nothing while parked).
constexpr int kWaitStop = 0, kWaitOk = 1, kWaitPark = 2;
__device__ __forceinline__ int stream_wait(const uint32_t* w, uint32_t want, uint32_t* g, uint32_t hb,
                                           uint32_t target, int64_t endAt, bool* ended, uint64_t ticks) {
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t beat = ld_sys(g + hb), alive = ld_sys(g + 5);
    for (;;) {
        if (ld_sys(w) == want) return kWaitOk;
        const uint32_t total = ld_sys(g), abort = ld_sys(g + 1), now = ld_sys(g + hb), live = ld_sys(g + 5);
        if (endAt >= 0 && (uint64_t)endAt >= total) { *ended = true; return kWaitStop; }
        if (abort) return kWaitStop;
        if (ld_sys(g + 7)) {   // parked
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            return hb == 2 && ld_sys(w) == want ? kWaitOk : kWaitPark;
        }
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        if (now != beat || live != alive) { beat = now; alive = live; t0 = t; }
        else if (t - t0 > ticks) {
            if (laneid() == 0) st_sys(g + 4, 1u);
            return kWaitStop;
        }
        const uint32_t dist = target > now ? min(target - now, 64u) : 0u;
        for (uint32_t k = 0; k < 8 * dist + 2; ++k) __builtin_amdgcn_s_sleep(127);
    }
}

// A wave's block parked on its output slot: {b + 1, word, sum} (lane 0's
// vector store; read back by the wave's relaunch, a kernel boundary later)
__device__ __forceinline__ void pend_store(uint32_t* pend, uint32_t b, uint32_t word, uint32_t sum) {
    if (laneid() == 0) {
        v4u v;
        v.x = b + 1;
        v.y = word;
        v.z = sum;
        v.w = 0;
        *(g_u4*)(gptr((uint8_t*)(pend + 4 * blockIdx.x))) = v;
    }
}

// B16: 64 KiB blocks (every block < 65 547 B): k_encode16's byU16 split
// table and LDS layout (26.3 KiB, 6 waves per CU); else k_encode's (1 MiB /
// 4 MiB, and 256 KiB blocks on the same v5 table: p17's sweeps would need
// their own instantiation for a path bound by the host's read())
template <bool XC, bool B16>
__global__ void __launch_bounds__(64) k_encode_stream(const uint8_t* __restrict__ hin, uint8_t* __restrict__ hout,
                                                      uint32_t* inCtl, uint32_t* outCtl, uint32_t* g,
                                                      uint32_t* __restrict__ next, uint32_t* pend,
                                                      uint8_t* __restrict__ dIn, uint8_t* __restrict__ dSlot,
                                                      uint32_t bm, uint32_t Rin, uint32_t Rout, int bck,
                                                      uint64_t ticks) {
    constexpr uint32_t kWords = B16 ? kE16Words : 5120;
    __shared__ __attribute__((aligned(16))) uint32_t ELDS[kWords];
    uint32_t* const T = ELDS;
    uint8_t* const S = (uint8_t*)(ELDS + 4096);
    uint32_t* const X = ELDS + 4352;
    const uint32_t L = laneid();
    g_u8* din = gptr(dIn) + (uint64_t)blockIdx.x * (bm + 64);
    g_u8* dsl = gptr(dSlot) + (uint64_t)blockIdx.x * (bm + 64);
    // a relaunch after a park: first the block this wave parked with
    uint32_t resumeB = pend[4 * blockIdx.x];
    for (;;) {
        uint32_t b, word, sum;
        bool ended = false;
        if (resumeB) {
            b = resumeB - 1;
            word = pend[4 * blockIdx.x + 1];
            sum = pend[4 * blockIdx.x + 2];
            resumeB = 0;
            pend_store(pend, 0xFFFFFFFFu, 0u, 0u);   // (seq 0: consumed)
        } else {
            b = 0;
            if (L == 0) b = atomicAdd(next, 1u);
            b = rdlane(b, 0);
            const uint32_t ri = b % Rin;
            if (stream_wait(inCtl + 4 * ri, b + 1, g, 2, b + 1, (int64_t)b, &ended, ticks) != kWaitOk) return;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            const uint32_t n = min(ld_sys(inCtl + 4 * ri + 1), bm);   // (the host never publishes more)
            wave_copy16(din, gptr(hin) + (uint64_t)ri * bm, n);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (L == 0) st_sys(inCtl + 4 * ri + 2, b + 1);   // the staging slot may be refilled
            int32_t r;
            if constexpr (B16)
                [[clang::always_inline]] r = encode_block_v5<false, true, true, false, false, false, false, XC, true>(
                    din, n, dsl, n, (l_u32*)ELDS, (l_u8*)(ELDS + kE16TabWords), nullptr);
            else if (n < (uint32_t)kLimit64K)
                r = encode_block<true, false, false>(din, n, dsl, n, (l_u32*)T, (l_u8*)S, (l_u32*)X,
                                                     (l_u8*)X + kRingE, nullptr);
            else
                [[clang::always_inline]] r = encode_block_v5<false, false, false, false, false, false, false, XC,
                                                             true>(din, n, dsl, n, (l_u32*)T, (l_u8*)X, nullptr);
            WAVE_SYNC();
            word = r > 0 ? (uint32_t)r : (n | 0x80000000u);
            sum = bck ? xxh32_wave(r > 0 ? dsl : din, r > 0 ? (uint32_t)r : n, (l_u32*)T) : 0u;
        }
        const uint32_t ro = b % Rout;
        // the record's slot in host memory: free once the writer wrote block b - Rout
        if (b >= Rout) {
            const int wr = stream_wait(outCtl + 4 * ro + 3, b - Rout + 1, g, 3, b - Rout + 1, -1, &ended, ticks);
            if (wr != kWaitOk) {
                if (wr == kWaitPark) pend_store(pend, b, word, sum);   // the block stays in din / dsl
                return;
            }
        }
        g_cu8* stored = (word & 0x80000000u) ? din : dsl;
        wave_copy16(gptr(hout) + (uint64_t)ro * bm, stored, word & 0x7FFFFFFFu);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (L == 0) {
            st_sys(outCtl + 4 * ro + 1, word);
            st_sys(outCtl + 4 * ro + 2, sum);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (L == 0) st_sys(outCtl + 4 * ro, b + 1);
    }
}

hipError_t launch_encode_stream(const uint8_t* hin, uint8_t* hout, uint32_t* inCtl, uint32_t* outCtl, uint32_t* g,
                                uint32_t* next, uint32_t* pend, uint8_t* dIn, uint8_t* dSlot, uint32_t bm,
                                uint32_t Rin, uint32_t Rout, uint32_t waves, int bck, uint64_t ticks,
                                hipStream_t st) {
    bool xc = true;
    if (const hipError_t r = encoder_path(st, &xc); r != hipSuccess) return r;
    if (bm < (64u << 10) || bm > (1u << kPosBits) || !waves || !Rin || !Rout || !pend) return hipErrorInvalidValue;
    const bool b16 = bm < (uint32_t)kLimit64K;
    const auto k = b16 ? (xc ? k_encode_stream<true, true> : k_encode_stream<false, true>)
                       : (xc ? k_encode_stream<true, false> : k_encode_stream<false, false>);
    hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, st, hin, hout, inCtl, outCtl, g, next, pend, dIn, dSlot, bm, Rin,
                       Rout, bck, ticks);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Streamed decompress: the mirror of the streamed compress above for
// lz4mtDecompress over the callbacks (independent 1 / 4 MiB blocks;
// reference decompress(), src/lz4mt.cpp:593-734).  The host reads each
// record (size word, stored bytes, block checksum) into in[b % Rin]; a wave
// takes block b, copies the stored bytes to HBM, frees the slot, hashes them
// (block XXH32) when the frame carries block checksums, decodes them with
// the frame decoder's code (LZ4_decompress_safe, cap = blockMax) or takes a
// raw block as is, waits for out[b % Rout] and pushes the decoded bytes
// there; a host writer thread writes them in block order.
//   in[r]  {seq = b + 1, size word, XXH32 from the frame, pulled = b + 1}
//   out[r] {seq = b + 1, decoded bytes or the decoder's negative result,
//           status (16 checksum mismatch, 18 decode failure, | 0x100 raw),
//           written = b + 1}
// Control words and waits as in k_encode_stream (g[2] heartbeat = records read).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_decode_stream(const uint8_t* __restrict__ hin, uint8_t* __restrict__ hout,
                                                      uint32_t* inCtl, uint32_t* outCtl, uint32_t* g,
                                                      uint32_t* __restrict__ next, uint32_t* pend,
                                                      uint8_t* __restrict__ dIn, uint8_t* __restrict__ dSlot,
                                                      uint32_t bm, uint32_t Rin, uint32_t Rout, int bck,
                                                      uint64_t ticks) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
    __shared__ __attribute__((aligned(16))) uint8_t win[kWinAlloc];   /* + dummy write area + hop table */
    const uint32_t L = laneid();
    g_u8* din = gptr(dIn) + (uint64_t)blockIdx.x * (bm + 64);
    g_u8* dsl = gptr(dSlot) + (uint64_t)blockIdx.x * (bm + 64);
    // a relaunch after a park: first the block this wave parked with
    uint32_t resumeB = pend[4 * blockIdx.x];
    for (;;) {
        uint32_t b, status;
        int32_t res;
        bool ended = false;
        if (resumeB) {
            b = resumeB - 1;
            res = (int32_t)pend[4 * blockIdx.x + 1];
            status = pend[4 * blockIdx.x + 2];
            resumeB = 0;
            pend_store(pend, 0xFFFFFFFFu, 0u, 0u);   // (seq 0: consumed)
        } else {
            b = 0;
            if (L == 0) b = atomicAdd(next, 1u);
            b = rdlane(b, 0);
            const uint32_t ri = b % Rin;
            if (stream_wait(inCtl + 4 * ri, b + 1, g, 2, b + 1, (int64_t)b, &ended, ticks) != kWaitOk) return;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            const uint32_t bits = ld_sys(inCtl + 4 * ri + 1), ck = ld_sys(inCtl + 4 * ri + 2);
            const uint32_t n = min(bits & 0x7FFFFFFFu, bm);   // (the host refuses n > bm)
            const bool raw = (bits & 0x80000000u) != 0;
            wave_copy16(din, gptr(hin) + (uint64_t)ri * bm, n);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (L == 0) st_sys(inCtl + 4 * ri + 3, b + 1);   // the staging slot may be refilled
            status = raw ? 0x100u : 0u;
            if (bck && xxh32_wave(din, n, (l_u32*)ring) != ck) status |= 16u;
            WAVE_SYNC();
            res = (int32_t)n;
            if (!raw) {
                Dec<false> D;
                D.acc = nullptr;
                D.ts = 0;
                D.src = din;
                D.len = n;
                D.dst = dsl;
                D.physcap = bm;
                D.ring = (l_u8*)ring;
                D.win = (l_u8*)win;
                D.wlo = INT64_MIN / 4;
                D.labase = INT64_MIN / 4;
                D.la = 0;
                D.flushed = 0;
                D.completed = 0;
                D.lowP = 0;
                res = decode_block(D, (int64_t)bm);   // cap = blockMax (src/lz4mt.cpp:645)
                if (res < 0) status = 18u;   // a decode failure wins over the checksum (src/lz4mt.cpp:619-681)
            }
        }
        const uint32_t ro = b % Rout;
        if (b >= Rout) {
            const int wr = stream_wait(outCtl + 4 * ro + 3, b - Rout + 1, g, 3, b - Rout + 1, -1, &ended, ticks);
            if (wr != kWaitOk) {
                if (wr == kWaitPark) pend_store(pend, b, (uint32_t)res, status);   // the block stays in din / dsl
                return;
            }
        }
        g_cu8* outp = (status & 0x100u) ? din : dsl;
        if (res > 0) wave_copy16(gptr(hout) + (uint64_t)ro * bm, outp, (uint32_t)res);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (L == 0) {
            st_sys(outCtl + 4 * ro + 1, (uint32_t)res);
            st_sys(outCtl + 4 * ro + 2, status);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (L == 0) st_sys(outCtl + 4 * ro, b + 1);
    }
}

hipError_t launch_decode_stream(const uint8_t* hin, uint8_t* hout, uint32_t* inCtl, uint32_t* outCtl, uint32_t* g,
                                uint32_t* next, uint32_t* pend, uint8_t* dIn, uint8_t* dSlot, uint32_t bm,
                                uint32_t Rin, uint32_t Rout, uint32_t waves, int bck, uint64_t ticks,
                                hipStream_t st) {
    if (bm < 64 || (bm & 15) || !waves || !Rin || !Rout || !pend) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_decode_stream, dim3(waves), dim3(64), 0, st, hin, hout, inCtl, outCtl, g, next, pend, dIn,
                       dSlot, bm, Rin, Rout, bck, ticks);
    return hipGetLastError();
}

__global__ void __launch_bounds__(64) k_xxh32_frame_blocks(const uint8_t* __restrict__ frame,
                                                           const BlockRec* __restrict__ recs, uint32_t nBlocks,
                                                           uint32_t* __restrict__ digest) {
    const uint32_t b = blockIdx.x * 16u + (laneid() >> 2);
    const bool ok = b < nBlocks;
    const BlockRec r = recs[ok ? b : 0u];
    const uint32_t h = xxh32_quad(gptr(frame) + r.offset, ok ? (r.bits & 0x7FFFFFFFu) : 0u, gptr(frame));
    if (ok && (laneid() & 3u) == 0) digest[b] = h;
}

// k_xxh32_frame_blocks beside k_decode_walk: 16 blocks per wave (lane
// quads), groups taken from ctl[3], each group hashed once the walk has
// published it (or ended short of it)
__global__ void __launch_bounds__(64) k_xxh32_walked(const uint8_t* __restrict__ frame,
                                                     const BlockRec* __restrict__ recs, uint32_t* __restrict__ ctl,
                                                     uint32_t* __restrict__ digest) {
    const uint32_t L = laneid();
    for (;;) {
        uint32_t g = 0;
        if (L == 0) g = __hip_atomic_fetch_add(ctl + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t first = 16u * (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
        const uint32_t w = walked_wait(ctl, first + 16);
        if (first >= w) return;
        const uint32_t b = first + (L >> 2);
        const bool ok = b < w;
        const BlockRec r = recs[ok ? b : first];
        const uint32_t h = xxh32_quad(gptr(frame) + r.offset, ok ? (r.bits & 0x7FFFFFFFu) : 0u, gptr(frame));
        if (ok && (L & 3u) == 0) digest[b] = h;
    }
}

hipError_t launch_xxh32_walked(const uint8_t* frame, const BlockRec* recs, uint32_t* ctl, uint32_t* digest,
                               uint32_t waves, hipStream_t st) {
    if (!waves) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_xxh32_walked, dim3(waves), dim3(64), 0, st, frame, recs, ctl, digest);
    return hipGetLastError();
}

// XXH32 of consecutive `chunk`-byte pieces of one range (the last one
// short), 16 pieces per wave, a lane quad per piece: the parallel "checksum
// of checksums" the large-config tests and the multi-GPU check compare.
__global__ void __launch_bounds__(64) k_xxh32_chunks(const uint8_t* __restrict__ p, uint64_t len, uint32_t chunk,
                                                     uint32_t nChunks, uint32_t* __restrict__ digest) {
    const uint32_t b = blockIdx.x * 16u + (laneid() >> 2);
    const bool ok = b < nChunks;
    const uint64_t off = ok ? (uint64_t)b * chunk : 0;
    const uint32_t n = ok ? (uint32_t)min<uint64_t>(chunk, len - off) : 0u;
    const uint32_t h = xxh32_quad(gptr(p) + off, n, gptr(p));
    if (ok && (laneid() & 3u) == 0) digest[b] = h;
}

hipError_t launch_xxh32_chunks(const uint8_t* p, uint64_t len, uint32_t chunk, uint32_t* digest, hipStream_t st) {
    if (len == 0 || chunk == 0) return hipSuccess;
    const uint64_t nc = (len + chunk - 1) / chunk;
    if (nc > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_xxh32_chunks, dim3((uint32_t)((nc + 15) / 16)), dim3(64), 0, st, p, len, chunk, (uint32_t)nc,
                       digest);
    return hipGetLastError();
}

// whole-stream XXH32 (lz4mt's serial content checksum): ONE wave, by design
__global__ void __launch_bounds__(64) k_xxh32_stream(const uint8_t* __restrict__ p, uint64_t len,
                                                     uint32_t* __restrict__ digest) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[512];
    const uint32_t h = xxh32_wave(gptr(p), len, (l_u32*)buf);
    if (laneid() == 0) *digest = h;
}

// Block checksums WHILE the encoder runs (k_encode_pub publishes pub[b]):
// a quad of lanes per block (lane c keeps XXH32 accumulator v_c), 16 blocks
// per wave, no LDS (every CU's LDS belongs to the encoder meanwhile).  A
// wave polls pub[] and hashes what became final -- whole 128-B lines only
// while a block is still encoding, so no line is ever cached half-written
// -- behind an agent-scope acquire; once a block is done it hashes the rest
// (or, for a block stored raw, its source bytes) and writes the digest and
// xdone[b] = 1.  Every wave leaves once its blocks are done, or after ~2 s
// without progress (k_xxh32_fixup then computes what is missing), so the
// grid always drains.  Replaces the k_xxh32_stored pass after the encode
// (~4.3 ms at 8 GiB) by the last blocks' tails.
constexpr int kFollowBatch = 8;   // stripes per lane loaded ahead

__global__ void __launch_bounds__(64) k_xxh32_follow(const uint8_t* __restrict__ src, const uint8_t* __restrict__ slots,
                                                     uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                                                     uint32_t* pub, uint32_t* __restrict__ digest,
                                                     uint32_t* __restrict__ xdone) {
    const uint32_t L = laneid(), c = L & 3u;
    const uint32_t b = blockIdx.x * 16u + (L >> 2);
    const bool ok = b < nBlocks;
    const uint64_t off = (uint64_t)(ok ? b : 0u) * blockSize;
    const uint32_t n = ok ? (uint32_t)min<uint64_t>(blockSize, srcSize - off) : 0u;
    const uint32_t vInit = (c == 0) ? kP1 + kP2 : (c == 1) ? kP2 : (c == 2) ? 0u : (uint32_t)(0u - kP1);
    uint32_t v = vInit;
    uint32_t hs = 0;              // stripes of the block hashed so far
    bool raw = false, fin = !ok;  // raw: hashing the source bytes (block stored raw)
    uint64_t tLast = __builtin_amdgcn_s_memrealtime();   // 100 MHz
    while (__builtin_amdgcn_ballot_w64(!fin)) {
        uint32_t pv = 0;
        if (!fin) pv = __hip_atomic_load(pub + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool done = !fin && (pv & kPubDone);
        if (done && (pv & kPubRaw) && !raw) {   // restart on the source bytes
            raw = true;
            v = vInit;
            hs = 0;
        }
        const uint32_t len = fin ? 0u : done ? (raw ? n : (pv & kPubLen)) : 0u;
        const uint32_t target = fin ? hs : done ? (len >> 4) : ((pv & kPubLen) & ~127u) >> 4;
        const uint32_t todo = target > hs ? target - hs : 0u;
        uint32_t most = todo;
        for (uint32_t d = 4; d < 64; d <<= 1) most = max(most, (uint32_t)__shfl_xor((int)most, (int)d, 64));
        most = (uint32_t)__builtin_amdgcn_readfirstlane((int)max(most, (uint32_t)__shfl_xor((int)most, 1, 64)));
        if (most == 0 && !__builtin_amdgcn_ballot_w64(done)) {   // nothing new: wait a little
            if (__builtin_amdgcn_s_memrealtime() - tLast > 200000000ull) break;   // ~2 s: leave it to the fixup
            __builtin_amdgcn_s_sleep(127);
            continue;
        }
        tLast = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the bytes behind the counts just read
        g_cu32* q = (g_cu32*)((raw ? gptr(src) : gptr(slots)) + off);
        const uint32_t lastW = target ? 4u * target - 1u : 0u;   // loads never pass the final lines
        for (uint32_t i = 0; i < most; i += kFollowBatch) {
            uint32_t w[kFollowBatch];
#pragma unroll
            for (int u = 0; u < kFollowBatch; ++u) w[u] = q[min(4u * (hs + i + u) + c, lastW)];
#pragma unroll
            for (int u = 0; u < kFollowBatch; ++u) v = (i + u < todo) ? xround(v, w[u]) : v;
        }
        hs += todo;
        // finish the blocks that are done: lane 0 of the quad folds the
        // accumulators, the length and the tail (len & 15 bytes)
        const uint32_t v1 = quad_get(v, 0), v2 = quad_get(v, 1), v3 = quad_get(v, 2), v4 = quad_get(v, 3);
        if (done) {
            if (c == 0) {
                g_cu8* p = (raw ? gptr(src) : gptr(slots)) + off;
                uint32_t h = len >= 16 ? rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18) : kP5;
                h += len;
                uint32_t o = len & ~15u;
                for (; o + 4 <= len; o += 4) h = rotl32(h + ld32u(p + o) * kP3, 17) * kP4;
                for (; o < len; ++o) h = rotl32(h + p[o] * kP5, 11) * kP1;
                h ^= h >> 15; h *= kP2; h ^= h >> 13; h *= kP3; h ^= h >> 16;
                digest[b] = h;
                xdone[b] = 1u;
            }
            fin = true;
        }
    }
}

// the blocks k_xxh32_follow did not finish (normally none): their digests
// from the stored bytes, after the encode
__global__ void __launch_bounds__(64) k_xxh32_fixup(const uint8_t* __restrict__ src, const uint8_t* __restrict__ slots,
                                                    uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                                                    const int32_t* __restrict__ csize, uint32_t* __restrict__ digest,
                                                    const uint32_t* __restrict__ xdone) {
    const uint32_t b = blockIdx.x * 16u + (laneid() >> 2);
    const bool ok = b < nBlocks;
    const bool need = ok && xdone[b] == 0u;
    if (!__builtin_amdgcn_ballot_w64(need)) return;
    const uint64_t off = (uint64_t)(ok ? b : 0u) * blockSize;
    const uint32_t n = ok ? (uint32_t)min<uint64_t>(blockSize, srcSize - off) : 0u;
    const int32_t cs = ok ? csize[b] : 0;
    g_cu8* p = cs > 0 ? gptr(slots) + off : gptr(src) + off;
    const uint32_t h = xxh32_quad(p, need ? (cs > 0 ? (uint32_t)cs : n) : 0u, gptr(src));
    if (need && (laneid() & 3u) == 0) digest[b] = h;
}

hipError_t launch_xxh32_follow(const uint8_t* src, const uint8_t* slots, uint64_t srcSize, uint32_t blockSize,
                               uint32_t nBlocks, uint32_t* pub, uint32_t* digest, uint32_t* xdone, hipStream_t st) {
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_xxh32_follow, dim3((nBlocks + 15) / 16), dim3(64), 0, st, src, slots, srcSize, blockSize,
                       nBlocks, pub, digest, xdone);
    return hipGetLastError();
}

hipError_t launch_xxh32_fixup(const uint8_t* src, const uint8_t* slots, uint64_t srcSize, uint32_t blockSize,
                              uint32_t nBlocks, const int32_t* csize, uint32_t* digest, const uint32_t* xdone,
                              hipStream_t st) {
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_xxh32_fixup, dim3((nBlocks + 15) / 16), dim3(64), 0, st, src, slots, srcSize, blockSize,
                       nBlocks, csize, digest, xdone);
    return hipGetLastError();
}

hipError_t launch_xxh32_stored(const uint8_t* src, const uint8_t* slots, uint64_t srcSize, uint32_t blockSize,
                               uint32_t nBlocks, const int32_t* csize, uint32_t* digest, hipStream_t st) {
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_xxh32_stored, dim3(nBlocks), dim3(64), 0, st, src, slots, srcSize, blockSize, nBlocks, csize,
                       digest);
    return hipGetLastError();
}

hipError_t launch_xxh32_frame_blocks(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t* digest,
                                     hipStream_t st) {
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_xxh32_frame_blocks, dim3((nBlocks + 15) / 16), dim3(64), 0, st, frame, recs, nBlocks,
                       digest);
    return hipGetLastError();
}

hipError_t launch_xxh32_stream(const uint8_t* p, uint64_t len, uint32_t* digest, hipStream_t st) {
    hipLaunchKernelGGL(k_xxh32_stream, dim3(1), dim3(64), 0, st, p, len, digest);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Frame assembly: record sizes -> exclusive scan -> scatter
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_frame_scan(const int32_t* __restrict__ csize, uint64_t srcSize,
                                                     uint32_t blockSize, uint32_t nBlocks, int blockChecksum,
                                                     uint64_t* __restrict__ recOff) {
    __shared__ uint64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nBlocks + 1023) / 1024;
    const uint32_t lo = min(nBlocks, t * per), hi = min(nBlocks, lo + per);
    auto recsz = [&](uint32_t b) -> uint64_t {
        const uint64_t off = (uint64_t)b * blockSize;
        const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
        const int32_t cs = csize[b];
        return 4ull + (cs > 0 ? (uint64_t)cs : n) + (blockChecksum ? 4ull : 0ull);
    };
    uint64_t sum = 0;
    for (uint32_t b = lo; b < hi; ++b) sum += recsz(b);
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;  // exclusive base
    for (uint32_t b = lo; b < hi; ++b) { recOff[b] = run; run += recsz(b); }
    if (t == 1023) recOff[nBlocks] = part[1023];
}

// chunks per thread in flight in the assembly's middle loop (A/B)
#ifndef LZ4MT_ASM_UNROLL
#define LZ4MT_ASM_UNROLL 1
#endif

__global__ void __launch_bounds__(256) k_frame_assemble(const uint8_t* __restrict__ src, const uint8_t* __restrict__ slots,
                                                        uint64_t srcSize, uint32_t blockSize,
                                                        const int32_t* __restrict__ csize,
                                                        const uint32_t* __restrict__ bsum,
                                                        const uint64_t* __restrict__ recOff, int blockChecksum,
                                                        uint8_t* __restrict__ frame, uint32_t hdrLen) {
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const int32_t cs = csize[b];
    g_cu8* sp = cs > 0 ? gptr(slots) + off : gptr(src) + off;   // 16-B aligned
    const uint64_t L = cs > 0 ? (uint64_t)cs : n;
    const uint32_t bits = cs > 0 ? (uint32_t)cs : (n | 0x80000000u);
    g_u8* rec = gptr(frame) + hdrLen + recOff[b];
    g_u8* D = rec + 4;
    if (t < 4) rec[t] = (uint8_t)(bits >> (8 * t));
    // blockChecksum 2: the words are written later by k_frame_sums
    if (blockChecksum == 1 && t >= 4 && t < 8) D[L + (t - 4)] = (uint8_t)(bsum[b] >> (8 * (t - 4)));
    const uintptr_t Da = reinterpret_cast<uintptr_t>(D);
    const uintptr_t A0 = (Da + 15) & ~uintptr_t(15);
    const uintptr_t E = Da + L, E0 = E & ~uintptr_t(15);
    if (A0 >= E0) {  // short payload: bytes only
        for (uint64_t i = t; i < L; i += 256) D[i] = sp[i];
        return;
    }
    const uint64_t head = A0 - Da, tailStart = E0 - Da;
    for (uint64_t i = t; i < head; i += 256) D[i] = sp[i];
    for (uint64_t i = tailStart + t; i < L; i += 256) D[i] = sp[i];
    // middle: 16-B aligned destination chunks gathered from the source
    const uint64_t nchunks = (E0 - A0) >> 4;
#pragma unroll LZ4MT_ASM_UNROLL
    for (uint64_t j = t; j < nchunks; j += 256) {
        const uint64_t so = head + 16 * j;                 // source byte offset of this chunk
        g_cu32* q = (g_cu32*)(sp + (so & ~3ull));
        const uint32_t s3 = (uint32_t)(so & 3);
        const uint32_t a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
        const uint32_t a4 = s3 ? q[4] : 0u;
        v4u v;
        v.x = __builtin_amdgcn_alignbyte(a1, a0, s3);
        v.y = __builtin_amdgcn_alignbyte(a2, a1, s3);
        v.z = __builtin_amdgcn_alignbyte(a3, a2, s3);
        v.w = __builtin_amdgcn_alignbyte(a4, a3, s3);
        *(g_u4*)(D + (A0 - Da) + 16 * j) = v;
    }
}

struct HdrBytes { uint8_t b[20]; };

__global__ void k_frame_finalize(uint8_t* __restrict__ frame, HdrBytes hdr, uint32_t hdrLen,
                                 const uint64_t* __restrict__ recOff, uint32_t nBlocks,
                                 const uint32_t* __restrict__ streamSum, uint64_t* __restrict__ frameSize) {
    const uint32_t t = threadIdx.x;
    if (t < hdrLen) frame[t] = hdr.b[t];
    const uint64_t eos = hdrLen + recOff[nBlocks];
    if (t < 4) frame[eos + t] = 0;
    uint64_t total = eos + 4;
    if (streamSum) {
        if (t < 4) frame[eos + 4 + t] = (uint8_t)(*streamSum >> (8 * t));
        total += 4;
    }
    if (t == 0) *frameSize = total;
}

hipError_t launch_frame_scan(const int32_t* csize, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                             int blockChecksum, uint64_t* recOff, hipStream_t st) {
    hipLaunchKernelGGL(k_frame_scan, dim3(1), dim3(1024), 0, st, csize, srcSize, blockSize, nBlocks, blockChecksum,
                       recOff);
    return hipGetLastError();
}

hipError_t launch_frame_assemble(const uint8_t* src, const uint8_t* slots, uint64_t srcSize, uint32_t blockSize,
                                 uint32_t nBlocks, const int32_t* csize, const uint32_t* bsum, const uint64_t* recOff,
                                 int blockChecksum, uint8_t* frame, uint32_t hdrLen, hipStream_t st) {
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_frame_assemble, dim3(nBlocks), dim3(256), 0, st, src, slots, srcSize, blockSize, csize, bsum,
                       recOff, blockChecksum, frame, hdrLen);
    return hipGetLastError();
}

// block checksum words of an assembled frame (when the checksums were
// computed beside the assembly, on another stream)
__global__ void __launch_bounds__(256) k_frame_sums(const int32_t* __restrict__ csize, uint64_t srcSize,
                                                    uint32_t blockSize, uint32_t nBlocks,
                                                    const uint32_t* __restrict__ bsum,
                                                    const uint64_t* __restrict__ recOff, uint8_t* __restrict__ frame,
                                                    uint32_t hdrLen) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nBlocks) return;
    const uint64_t off = (uint64_t)b * blockSize;
    const uint32_t n = (uint32_t)min<uint64_t>(blockSize, srcSize - off);
    const int32_t cs = csize[b];
    g_u8* w = gptr(frame) + hdrLen + recOff[b] + 4 + (cs > 0 ? (uint64_t)cs : n);
    const uint32_t v = bsum[b];
    w[0] = (uint8_t)v; w[1] = (uint8_t)(v >> 8); w[2] = (uint8_t)(v >> 16); w[3] = (uint8_t)(v >> 24);
}

hipError_t launch_frame_sums(const int32_t* csize, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                             const uint32_t* bsum, const uint64_t* recOff, uint8_t* frame, uint32_t hdrLen,
                             hipStream_t st) {
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_frame_sums, dim3((nBlocks + 255) / 256), dim3(256), 0, st, csize, srcSize, blockSize, nBlocks,
                       bsum, recOff, frame, hdrLen);
    return hipGetLastError();
}

hipError_t launch_frame_finalize(uint8_t* frame, const uint8_t* hdr, uint32_t hdrLen, const uint64_t* recOff,
                                 uint32_t nBlocks, const uint32_t* streamSum, uint64_t* frameSize, hipStream_t st) {
    HdrBytes h{};
    for (uint32_t i = 0; i < hdrLen && i < 20; ++i) h.b[i] = hdr[i];
    hipLaunchKernelGGL(k_frame_finalize, dim3(1), dim3(64), 0, st, frame, h, hdrLen, recOff, nBlocks, streamSum,
                       frameSize);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Frame walk (decompress side): follows the block size words serially.
// Result codes follow src/lz4mt.cpp:685-727.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rd32b(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__global__ void k_frame_walk(const uint8_t* __restrict__ frame, uint64_t frameSize, uint64_t pos, uint32_t blockMax,
                             int blockChecksum, uint32_t maxBlocks, BlockRec* __restrict__ recs,
                             WalkInfo* __restrict__ info) {
    if (threadIdx.x != 0) return;
    uint32_t nb = 0;
    int32_t result = 0;
    for (;;) {
        if (pos + 4 > frameSize) { result = 12; break; }             // CANNOT_READ_BLOCK_SIZE
        const uint32_t bits = rd32b(frame + pos);
        pos += 4;
        if (bits == 0) break;                                        // EOS
        const uint32_t sz = bits & 0x7FFFFFFFu;
        if (sz > blockMax) { result = 20; break; }                   // INVALID_BLOCK_SIZE
        if (pos + sz > frameSize) { result = 13; pos = frameSize; break; }  // CANNOT_READ_BLOCK_DATA
        BlockRec r{pos, bits, 0};
        pos += sz;
        if (blockChecksum) {
            if (pos + 4 > frameSize) { result = 14; break; }         // CANNOT_READ_BLOCK_CHECKSUM
            r.checksum = rd32b(frame + pos);
            pos += 4;
        }
        if (nb >= maxBlocks) { result = 1; break; }
        recs[nb++] = r;
    }
    info->endPos = pos;
    info->nBlocks = nb;
    info->result = result;
}

hipError_t launch_frame_walk(const uint8_t* frame, uint64_t frameSize, uint64_t bodyPos, uint32_t blockMax,
                             int blockChecksum, uint32_t maxBlocks, BlockRec* recs, WalkInfo* info, hipStream_t st) {
    hipLaunchKernelGGL(k_frame_walk, dim3(1), dim3(64), 0, st, frame, frameSize, bodyPos, blockMax, blockChecksum,
                       maxBlocks, recs, info);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Parallel frame walk.  The serial walk costs one dependent HBM load per
// block (~0.5 us: 70 ms for the 131 072 blocks of an 8 GiB -B4 stream).  This
// one finds the same chain without a serial pass:
//   1. every byte offset whose u32 could start a record (EOS, or a size word
//      <= blockMax whose record fits in the frame) is a candidate node; two
//      passes over 64 KiB chunks (count, scan, emit) list them in offset order;
//   2. each node points at the node its record ends on (or DEAD);
//   3. pointer doubling from the body start lists the path P[0..cap]:
//      P[s + k] = J_r[P[k]] for k < s = 2^r, with J_{r+1} = J_r o J_r;
//   4. the path gives the block records.  A path that ends on DEAD (a
//      malformed frame) reports result -1 and the host reruns the serial walk
//      for the reference's exact error code (src/lz4mt.cpp:685-727).
// EOS nodes point at themselves; node M (the candidate count) is DEAD.
// ---------------------------------------------------------------------------
// candidate mask of the 16 offsets o .. o+15 (bit j = offset o + j)
__device__ __forceinline__ uint32_t walk_group(g_cu8* f, uint64_t o, uint64_t frameSize, uint64_t pos0,
                                               uint32_t blockMax, uint32_t bck) {
    if (o + 4 > frameSize || o + 16 <= pos0) return 0;
    uint32_t wd[5];
    if (o + 20 <= frameSize) {
        for (int k = 0; k < 5; ++k) wd[k] = gld4u(f + o + 4 * k);
    } else {
        for (int k = 0; k < 5; ++k) {
            uint32_t v = 0;
            for (int b = 0; b < 4; ++b) {
                const uint64_t q = o + 4 * k + b;
                v |= (q < frameSize ? (uint32_t)f[q] : 0u) << (8 * b);
            }
            wd[k] = v;
        }
    }
    // a size word's top byte is 0x00 or 0x80: exact per-byte flags of that
    // (bit 7 of each byte), then bit j <=> byte o + j + 3 qualifies
    uint32_t fl = 0;
    for (int k = 0; k < 5; ++k) {
        const uint32_t t = wd[k] & 0x7F7F7F7Fu;
        const uint32_t z = ~((t + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
        fl |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * k);
    }
    uint32_t pre = (fl >> 3) & 0xFFFFu, m = 0;
    for (; pre; pre &= pre - 1) {
        const uint32_t j = (uint32_t)__builtin_ctz(pre);
        uint32_t w = wd[j >> 2];
        w = (j & 3) ? __builtin_amdgcn_alignbyte(wd[(j >> 2) + 1], w, j & 3) : w;
        const uint64_t p = o + j;
        const uint32_t sz = w & 0x7FFFFFFFu;
        const bool ok = p >= pos0 && p + 4 <= frameSize && (w == 0 || (sz <= blockMax && p + 4 + sz + bck <= frameSize));
        m |= ok ? 1u << j : 0u;
    }
    return m;
}

constexpr uint32_t kWalkIters = (1u << kWalkChunkLog) / 4096;   // 16-byte groups per thread per chunk

__global__ void __launch_bounds__(256) k_walk_count(const uint8_t* __restrict__ frame, uint64_t frameSize,
                                                    uint64_t pos0, uint32_t blockMax, int blockChecksum,
                                                    uint32_t* __restrict__ count) {
    __shared__ uint32_t part[4];
    const uint64_t c0 = (uint64_t)blockIdx.x << kWalkChunkLog;
    uint32_t n = 0;
    for (uint32_t it = 0; it < kWalkIters; ++it)
        n += __builtin_popcount(walk_group(gptr(frame), c0 + it * 4096 + threadIdx.x * 16, frameSize, pos0, blockMax,
                                           blockChecksum ? 4u : 0u));
    n = wave_scan_incl(n);
    if (laneid() == 63) part[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) count[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// exclusive scan of count[] -> base[] (u64); M = base[nChunks]
__global__ void __launch_bounds__(1024) k_walk_scan(const uint32_t* __restrict__ count, uint32_t nChunks,
                                                    uint64_t* __restrict__ base) {
    __shared__ uint64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nChunks + 1023) / 1024;
    const uint32_t lo = min(nChunks, t * per), hi = min(nChunks, lo + per);
    uint64_t sum = 0;
    for (uint32_t c = lo; c < hi; ++c) sum += count[c];
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;
    for (uint32_t c = lo; c < hi; ++c) { base[c] = run; run += count[c]; }
    if (t == 1023) base[nChunks] = part[1023];
}

// candidate offsets in frame order: pos[base[c] ..]
__global__ void __launch_bounds__(256) k_walk_emit(const uint8_t* __restrict__ frame, uint64_t frameSize,
                                                   uint64_t pos0, uint32_t blockMax, int blockChecksum,
                                                   const uint64_t* __restrict__ base, uint64_t* __restrict__ pos) {
    __shared__ uint32_t part[4];
    const uint64_t c0 = (uint64_t)blockIdx.x << kWalkChunkLog;
    uint64_t run = base[blockIdx.x];
    if (base[blockIdx.x + 1] == run) return;
    const uint32_t wv = threadIdx.x >> 6;
    for (uint32_t it = 0; it < kWalkIters; ++it) {
        const uint64_t o = c0 + it * 4096 + threadIdx.x * 16;
        uint32_t m = walk_group(gptr(frame), o, frameSize, pos0, blockMax, blockChecksum ? 4u : 0u);
        const uint32_t c = (uint32_t)__builtin_popcount(m);
        const uint32_t incl = wave_scan_incl(c);
        __syncthreads();   // part[] of the previous group has been read
        if (laneid() == 63) part[wv] = incl;
        __syncthreads();
        uint32_t before = incl - c;
        for (uint32_t q = 0; q < wv; ++q) before += part[q];
        for (uint64_t k = run + before; m; m &= m - 1, ++k) pos[k] = o + (uint32_t)__builtin_ctz(m);
        run += part[0] + part[1] + part[2] + part[3];
    }
}

__device__ __forceinline__ uint32_t walk_find(const uint64_t* __restrict__ base, const uint64_t* __restrict__ pos,
                                              uint64_t p, uint32_t dead) {
    const uint64_t c = p >> kWalkChunkLog;
    uint64_t lo = base[c], hi = base[c + 1];
    while (lo < hi) {   // first entry >= p
        const uint64_t mid = (lo + hi) >> 1;
        if (pos[mid] < p) lo = mid + 1; else hi = mid;
    }
    return (lo < base[c + 1] && pos[lo] == p) ? (uint32_t)lo : dead;
}

// J[i] = the node record i ends on (DEAD = M when that offset is no
// candidate); EOS nodes point at themselves.  Also P[0] and J[M] = M.
__global__ void __launch_bounds__(256) k_walk_next(const uint8_t* __restrict__ frame, uint64_t frameSize,
                                                   uint64_t pos0, int blockChecksum, uint32_t M,
                                                   const uint64_t* __restrict__ base,
                                                   const uint64_t* __restrict__ pos, uint32_t* __restrict__ J,
                                                   uint32_t* __restrict__ P) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) P[0] = walk_find(base, pos, pos0, M);
    if (i >= M) { if (i == M) J[M] = M; return; }
    const uint64_t p = pos[i];
    const uint32_t w = gld4u(gptr(frame) + p);
    if (w == 0) { J[i] = i; return; }
    const uint64_t np = p + 4 + (w & 0x7FFFFFFFu) + (blockChecksum ? 4u : 0u);
    J[i] = np + 4 <= frameSize ? walk_find(base, pos, np, M) : M;
}

__global__ void __launch_bounds__(256) k_walk_path(const uint32_t* __restrict__ J, uint32_t* __restrict__ P,
                                                   uint32_t span, uint32_t cap) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < span && span + k <= cap) P[span + k] = J[P[k]];
}

__global__ void __launch_bounds__(256) k_walk_jump(const uint32_t* __restrict__ Jin, uint32_t* __restrict__ Jout,
                                                   uint32_t M) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= M) Jout[i] = Jin[Jin[i]];
}

// P[0..cap] -> block records and the walk summary (one writer: the first
// path entry that is not a record, or entry cap when all are records)
__global__ void __launch_bounds__(256) k_walk_records(const uint8_t* __restrict__ frame, int blockChecksum,
                                                      uint32_t M, const uint64_t* __restrict__ pos,
                                                      const uint32_t* __restrict__ P, uint32_t cap,
                                                      BlockRec* __restrict__ recs, WalkInfo* __restrict__ info) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k > cap) return;
    g_cu8* f = gptr(frame);
    // 0 record, 1 EOS, 2 DEAD
    auto state = [&](uint32_t node, uint64_t* pp, uint32_t* pw) -> int {
        if (node == M) return 2;
        const uint64_t q = pos[node];
        const uint32_t w = gld4u(f + q);
        *pp = q; *pw = w;
        return w == 0 ? 1 : 0;
    };
    uint64_t p = 0, pp = 0;
    uint32_t w = 0, pw = 0;
    const int s = state(P[k], &p, &w);
    const int sPrev = k == 0 ? 0 : state(P[k - 1], &pp, &pw);
    if (s == 0) {
        if (k == cap) { info->endPos = p; info->nBlocks = cap; info->result = 1; return; }
        const uint32_t sz = w & 0x7FFFFFFFu;
        recs[k] = BlockRec{p + 4, w, blockChecksum ? gld4u(f + p + 4 + sz) : 0u};
    } else if (sPrev == 0) {
        info->endPos = s == 1 ? p + 4 : 0;
        info->nBlocks = k;
        info->result = s == 1 ? 0 : -1;
    }
}

uint64_t frame_walk_par_chunks(uint64_t frameSize) { return (frameSize + (1u << kWalkChunkLog) - 1) >> kWalkChunkLog; }

hipError_t launch_frame_walk_count(const uint8_t* frame, uint64_t frameSize, uint64_t bodyPos, uint32_t blockMax,
                                   int blockChecksum, const WalkScratch& ws, hipStream_t st) {
    const uint64_t nc = frame_walk_par_chunks(frameSize);
    hipLaunchKernelGGL(k_walk_count, dim3((uint32_t)nc), dim3(256), 0, st, frame, frameSize, bodyPos, blockMax,
                       blockChecksum, ws.count);
    hipLaunchKernelGGL(k_walk_scan, dim3(1), dim3(1024), 0, st, ws.count, (uint32_t)nc, ws.base);
    return hipGetLastError();
}

hipError_t launch_frame_walk_path(const uint8_t* frame, uint64_t frameSize, uint64_t bodyPos, uint32_t blockMax,
                                  int blockChecksum, uint32_t maxBlocks, uint32_t M, const WalkScratch& ws,
                                  BlockRec* recs, WalkInfo* info, hipStream_t st) {
    const uint64_t nc = frame_walk_par_chunks(frameSize);
    hipLaunchKernelGGL(k_walk_emit, dim3((uint32_t)nc), dim3(256), 0, st, frame, frameSize, bodyPos, blockMax,
                       blockChecksum, ws.base, ws.pos);
    hipLaunchKernelGGL(k_walk_next, dim3((M + 256) / 256), dim3(256), 0, st, frame, frameSize, bodyPos,
                       blockChecksum, M, ws.base, ws.pos, ws.Ja, ws.P);
    uint32_t* J = ws.Ja;
    uint32_t* Jn = ws.Jb;
    for (uint64_t span = 1; span <= maxBlocks; span <<= 1) {
        const uint32_t todo = (uint32_t)std::min<uint64_t>(span, maxBlocks + 1 - span);
        hipLaunchKernelGGL(k_walk_path, dim3((todo + 255) / 256), dim3(256), 0, st, J, ws.P, (uint32_t)span,
                           maxBlocks);
        if (span * 2 <= maxBlocks) {
            hipLaunchKernelGGL(k_walk_jump, dim3((M + 256) / 256), dim3(256), 0, st, J, Jn, M);
            std::swap(J, Jn);
        }
    }
    hipLaunchKernelGGL(k_walk_records, dim3((maxBlocks + 256) / 256), dim3(256), 0, st, frame, blockChecksum, M,
                       ws.pos, ws.P, maxBlocks, recs, info);
    return hipGetLastError();
}

// Per-block decode status in the reference's precedence: decode failure
// (src/lz4mt.cpp:647-650) before block checksum mismatch (675-681).
__global__ void k_block_verify(const BlockRec* __restrict__ recs, uint32_t nBlocks, const uint32_t* __restrict__ digest,
                               const int32_t* __restrict__ dsize, uint32_t blockMax, int blockChecksum,
                               int32_t* __restrict__ status) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nBlocks) return;
    int32_t st = 0;
    if (dsize[b] < 0) st = (dsize[b] == kDecodeOutputTooSmall) ? 1 : 18;   // ERROR / DECOMPRESS_FAIL
    else if (blockChecksum && digest[b] != recs[b].checksum) st = 16;      // BLOCK_CHECKSUM_MISMATCH
    status[b] = st;
}

// k_block_verify after k_decode_walk: the block count from the walk's info
__global__ void k_block_verify_walked(const BlockRec* __restrict__ recs, const WalkInfo* __restrict__ info,
                                      const uint32_t* __restrict__ digest, const int32_t* __restrict__ dsize,
                                      int blockChecksum, int32_t* __restrict__ status) {
    const uint32_t nb = info->nBlocks;
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gridDim.x * blockDim.x) {
        int32_t st = 0;
        if (dsize[b] < 0) st = (dsize[b] == kDecodeOutputTooSmall) ? 1 : 18;
        else if (blockChecksum && digest[b] != recs[b].checksum) st = 16;
        status[b] = st;
    }
}

hipError_t launch_block_verify_walked(const BlockRec* recs, const WalkInfo* info, const uint32_t* digest,
                                      const int32_t* dsize, int blockChecksum, int32_t* status, uint32_t maxBlocks,
                                      hipStream_t st) {
    const uint32_t need = (maxBlocks + 255) / 256 + 1, wg = need < 1024u ? need : 1024u;
    hipLaunchKernelGGL(k_block_verify_walked, dim3(wg), dim3(256), 0, st, recs, info, digest, dsize, blockChecksum,
                       status);
    return hipGetLastError();
}

hipError_t launch_block_verify(const BlockRec* recs, uint32_t nBlocks, const uint32_t* digest, const int32_t* dsize,
                               uint32_t blockMax, int blockChecksum, int32_t* status, hipStream_t st) {
    if (nBlocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_block_verify, dim3((nBlocks + 255) / 256), dim3(256), 0, st, recs, nBlocks, digest, dsize,
                       blockMax, blockChecksum, status);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Synthetic input: one workgroup per 64 KiB segment,
// generated serially by lane 0 in LDS (back-copies read LDS), then stored
// with coalesced 16-B writes.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t sm_next(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(64) k_gen_synthetic(uint8_t* __restrict__ dst, uint64_t n, uint64_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[65536 + 128];
    const uint64_t seg = blockIdx.x;
    if (threadIdx.x == 0) {
        uint64_t s = seed + seg * 0x9E3779B97F4A7C15ull;
        uint32_t len = 0;
        while (len < 65536) {
            const uint64_t r = sm_next(s);
            if (len >= 64 && (r & 255) < 76) {
                const uint32_t Lm = 4 + (uint32_t)((r >> 8) & 63);
                const uint32_t lim = len < 65535 ? len : 65535;
                const uint32_t off = 1 + (uint32_t)((r >> 16) % lim);
                for (uint32_t k = 0; k < Lm; ++k, ++len) buf[len] = buf[len - off];
            } else {
                const uint32_t cnt = (uint32_t)((r >> 8) & 15) + 1;
                for (uint32_t k = 0; k < cnt; ++k) buf[len++] = (uint8_t)(97 + (sm_next(s) >> 40) % 26);
            }
        }
    }
    __syncthreads();
    const uint64_t base = seg * 65536;
    const uint64_t take = (n - base) < 65536 ? (n - base) : 65536;
    if (take == 65536 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        for (uint32_t i = threadIdx.x; i < 4096; i += 64)
            reinterpret_cast<uint4*>(dst + base)[i] = reinterpret_cast<const uint4*>(buf)[i];
    } else {
        for (uint64_t i = threadIdx.x; i < take; i += 64) dst[base + i] = buf[i];
    }
}

hipError_t launch_gen_synthetic(uint8_t* dst, uint64_t n, uint64_t seed, hipStream_t st) {
    const uint64_t segs = (n + 65535) / 65536;
    if (segs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_synthetic, dim3((uint32_t)segs), dim3(64), 0, st, dst, n, seed);
    return hipGetLastError();
}

#endif  // LZ4MT_PART != 2

}  // namespace lz4mt
