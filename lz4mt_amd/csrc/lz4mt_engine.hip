// lz4mt_engine.hip — host side of the device engine: the lz4mt_hip.h C ABI.
//
// Compress path (device-resident frame, one lz4mt frame per call):
//   k_encode (wave per block, slots of blockMax) -> k_xxh32_stored (if FLG.4)
//   -> k_frame_scan (record offsets) -> k_frame_assemble (scatter into the
//   frame) -> [k_xxh32_stream if FLG.2] -> k_frame_finalize (header, EOS,
//   content checksum).  Replaces lz4mt's compress() scheduler and ordered
//   write chain (reference src/lz4mt.cpp:372-457, 898-935).
// Decompress path: host parses the header (one small D2H copy), k_frame_walk
//   builds the block table, k_decode (wave per block) -> k_xxh32_frame_blocks
//   + k_block_verify -> [k_xxh32_stream].  Replaces decompress() and
//   lz4mtDecompress (src/lz4mt.cpp:593-734, 938-1011).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/lz4mt_hip.h"
#include "lz4mt_device.h"
#include <chrono>
#include "lz4mt_host.h"

using namespace lz4mt;

// LZ4MT_AMD_FOLLOW=1: block checksums hashed beside the encode
// (k_xxh32_follow).  Off by default: measured, the encoder runs ~6 ms longer
// beside it at 8 GiB (185.9 vs 179.0 ms; the compress call 188.4 vs 184.3),
// more than the 4.3 ms of k_xxh32_stored it hides
// (profiles/r03e_follow_ab.txt).
bool follow_enabled() {
    static const bool on = [] {
        const char* e = getenv("LZ4MT_AMD_FOLLOW");
        return e && e[0] == '1';
    }();
    return on;
}


namespace {

#define HIPCHK(x)                                   \
    do {                                            \
        if ((x) != hipSuccess) return LZ4MT_RESULT_ERROR; \
    } while (0)

inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

bool have_device() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return false;
    return n > 0;
}

// ---- optional per-stage timing (thread-local hipEvents) -------------------
struct Timing {
    bool enabled = false;
    bool valid = false;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    void mark(int i, hipStream_t st) {
        if (!enabled) return;
        if (!ev[i]) hipEventCreate(&ev[i]);
        hipEventRecord(ev[i], st);
        if (i == 4) valid = true;
    }
};
thread_local Timing g_timing;

// ---- workspace layout for one compressed frame ----------------------------
struct CompressWs {
    uint8_t* slots;
    uint16_t* delta;   // LZ4-HC hash chain (level >= 3 only)
    uint8_t* hcSplit;  // LZ4-HC split-parse records (level >= 3, large blocks)
    int32_t* csize;
    uint32_t* bsum;
    uint64_t* recOff;
    uint32_t* ssum;
    uint64_t* fsize;
    uint32_t* pub;     // k_encode_pub's per-block progress (the checksum follower reads it)
    uint32_t* xdone;   // k_xxh32_follow's finished flags
    // block-dependent frames of the asynchronous calls (bd != 0): the host
    // plan copied in, the carried lz4 table, the parallel rounds' scratch
    // (bd == 1), or the HC stream's packed segments (bd == 2)
    uint8_t* bdPlan;
    uint32_t* bdTable;
    uint32_t* bdRounds;
    uint64_t bytes;
};

// bd: 0 independent blocks, 1 block-dependent fast LZ4, 2 block-dependent HC
CompressWs carve_compress(uint8_t* base, uint64_t nb, uint64_t bm, int level = 0, int bd = 0) {
    CompressWs w{};
    uint64_t o = 0;
    auto take = [&](uint64_t n) { uint8_t* p = base ? base + o : nullptr; o = align_up(o + n, 256); return p; };
    w.slots = take(nb * bm + 64);
    // (-BD: 64 Ki entries more, for a segment that starts in the history before src)
    w.delta = level >= 3 ? reinterpret_cast<uint16_t*>(take((nb * bm + 65536) * 2 + 64)) : nullptr;
    const uint64_t hs = level >= 3 ? hc_ws_bytes(nb, (uint32_t)bm, level) : 0;
    w.hcSplit = hs ? take(hs) : nullptr;
    w.csize = reinterpret_cast<int32_t*>(take((nb + 1) * 4));
    w.bsum = reinterpret_cast<uint32_t*>(take((nb + 1) * 4));
    w.recOff = reinterpret_cast<uint64_t*>(take((nb + 1) * 8));
    w.ssum = reinterpret_cast<uint32_t*>(take(16));
    w.fsize = reinterpret_cast<uint64_t*>(take(16));
    w.pub = reinterpret_cast<uint32_t*>(take(nb * 4 + 4));
    w.xdone = reinterpret_cast<uint32_t*>(take(nb * 4 + 4));
    const uint64_t nbp = nb > 0 ? nb : 1;
    if (bd == 1) {
        w.bdPlan = take(nbp * sizeof(LinkPlan));
        w.bdTable = reinterpret_cast<uint32_t*>(take(4096 * 4));
        w.bdRounds = reinterpret_cast<uint32_t*>(take(link_round_bytes(nbp)));
    } else if (bd == 2) {
        w.bdPlan = take(20 * nbp + 64);   // hc_bd_pack: 16 B per segment (<= nb) + 4 B per block
    }
    w.bytes = o;
    return w;
}

// ---- scratch for the block operators --------------------------------------
// A process-wide pool, not one per thread: the reference's scheduler runs
// each block on a fresh std::async thread (src/lz4mt.cpp:448,722), so a
// thread_local cache would leak a stream and two buffers per block.  Each
// call borrows a scratch object and returns it; the pool holds at most as
// many as ever ran concurrently.
struct BlockScratch {
    hipStream_t st = nullptr;
    uint8_t* dIn = nullptr;
    uint8_t* dOut = nullptr;
    uint64_t capIn = 0, capOut = 0;
    int32_t* dRes = nullptr;
    BlockRec* dRec = nullptr;
    uint16_t* dDelta = nullptr;   // LZ4-HC hash chain
    uint64_t capDelta = 0;
    uint8_t* dSplit = nullptr;    // LZ4-HC split-parse records
    uint64_t capSplit = 0;
    bool ensure_split(uint64_t bytes) {
        if (dSplit && bytes <= capSplit) return true;
        hipFree(dSplit);
        capSplit = std::max<uint64_t>(bytes, 64 << 10);
        if (hipMalloc(&dSplit, capSplit) != hipSuccess) { dSplit = nullptr; capSplit = 0; return false; }
        return true;
    }
    int dev = -1;
    bool ensure_delta(uint64_t n) {
        if (dDelta && n <= capDelta) return true;
        hipFree(dDelta);
        capDelta = std::max<uint64_t>(align_up(n + 64, 1 << 20), 1 << 20);
        if (hipMalloc(&dDelta, capDelta * 2) != hipSuccess) { dDelta = nullptr; capDelta = 0; return false; }
        return true;
    }
    void release() {
        if (st) hipStreamSynchronize(st);
        hipFree(dIn); hipFree(dOut); hipFree(dRes); hipFree(dRec); hipFree(dDelta); hipFree(dSplit);
        if (st) hipStreamDestroy(st);
        *this = BlockScratch();
    }
    bool init() {
        int d = -1;
        if (hipGetDevice(&d) != hipSuccess) return false;
        if (st && d == dev) return true;
        release();
        dev = d;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { st = nullptr; return false; }
        if (hipMalloc(&dRes, 256) != hipSuccess) { dRes = nullptr; return false; }
        if (hipMalloc(&dRec, 256) != hipSuccess) { dRec = nullptr; return false; }
        return true;
    }
    bool ensure(uint64_t in, uint64_t out) {
        if (in + 64 > capIn) {
            if (dIn) hipFree(dIn);
            capIn = std::max<uint64_t>(align_up(in + 64, 1 << 20), 1 << 20);
            if (hipMalloc(&dIn, capIn) != hipSuccess) { dIn = nullptr; capIn = 0; return false; }
        }
        if (out + 64 > capOut) {
            if (dOut) hipFree(dOut);
            capOut = std::max<uint64_t>(align_up(out + 64, 1 << 20), 1 << 20);
            if (hipMalloc(&dOut, capOut) != hipSuccess) { dOut = nullptr; capOut = 0; return false; }
        }
        return true;
    }
};

class ScratchPool {
public:
    BlockScratch* get() {
        {
            std::lock_guard<std::mutex> g(mu_);
            if (!free_.empty()) {
                BlockScratch* b = free_.back();
                free_.pop_back();
                return b;
            }
        }
        return new BlockScratch();
    }
    void put(BlockScratch* b) {
        std::lock_guard<std::mutex> g(mu_);
        free_.push_back(b);
    }
    void clear() {
        std::vector<BlockScratch*> v;
        {
            std::lock_guard<std::mutex> g(mu_);
            v.swap(free_);
        }
        for (BlockScratch* b : v) { b->release(); delete b; }
    }
    size_t idle() {
        std::lock_guard<std::mutex> g(mu_);
        return free_.size();
    }

private:
    std::mutex mu_;
    std::vector<BlockScratch*> free_;
};
// never destroyed: its buffers must not be freed after the HIP runtime's own
// teardown at exit
ScratchPool& scratch_pool() {
    static ScratchPool* p = new ScratchPool();
    return *p;
}
struct ScratchLease {
    BlockScratch* b;
    ScratchLease() : b(scratch_pool().get()) {}
    ~ScratchLease() { scratch_pool().put(b); }
    BlockScratch* operator->() { return b; }
};

// device buffer freed on every return path
struct DevBuf {
    uint8_t* p = nullptr;
    uint64_t cap = 0;
    int dev = -1;
    ~DevBuf() { hipFree(p); }
    bool ensure(uint64_t n) {
        int d = -1;
        if (hipGetDevice(&d) != hipSuccess) return false;
        if (p && n <= cap && d == dev) return true;
        hipFree(p);
        p = nullptr;
        cap = 0;
        dev = d;
        if (hipMalloc(reinterpret_cast<void**>(&p), n + 64) != hipSuccess) { p = nullptr; return false; }
        cap = n;
        return true;
    }
};

// A few bytes of device memory per thread and device (frame-size / digest
// results): no hipMalloc/hipFree per call (hipFree waits for the whole
// device).  One buffer per device ordinal, made on first use, so a thread
// that alternates devices reuses them instead of leaking one per switch.
uint8_t* small_dev() {
    constexpr int kMaxDev = 64;
    thread_local uint8_t* p[kMaxDev] = {};
    int d = -1;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDev) return nullptr;
    if (!p[d] && hipMalloc(reinterpret_cast<void**>(&p[d]), 256) != hipSuccess) {
        p[d] = nullptr;
        return nullptr;
    }
    return p[d];
}

// The content checksum (FLG.2) is ONE serial XXH32 chain:
// a GPU runs it on one wavefront at ~0.8 GB/s, a host core at several
// times that.  The synchronous frame calls therefore hash on the host:
// the bytes stream device -> pinned host memory in 64 MiB chunks on a copy
// stream (double-buffered: chunk i+1 in flight while chunk i is hashed),
// beside whatever the GPU does meanwhile (the encode reads the same input).
class HostHasher {
public:
    static constexpr uint64_t kChunk = 64ull << 20;
    ~HostHasher() { release(); }
    // XXH32 of d[0, len) once `ready` (recorded on the producing stream) has completed
    bool hash(const uint8_t* d, uint64_t len, hipEvent_t ready, uint32_t* out) {
        if (!ensure()) return false;
        HostXxh32 x(0);
        if (ready && hipStreamWaitEvent(cp_, ready, 0) != hipSuccess) return false;
        const uint64_t nc = (len + kChunk - 1) / kChunk;
        auto issue = [&](uint64_t i) {
            const uint64_t o = i * kChunk, k = std::min(kChunk, len - o);
            return hipMemcpyAsync(pin_[i & 1], d + o, k, hipMemcpyDeviceToHost, cp_) == hipSuccess &&
                   hipEventRecord(ev_[i & 1], cp_) == hipSuccess;
        };
        const char* st = getenv("LZ4MT_AMD_HASH_STATS");   // 1: wait / hash split to stderr
        const bool stats = st && st[0] == '1';
        double tWait = 0, tHash = 0;
        auto now = [] { return std::chrono::steady_clock::now(); };
        const auto t0 = now();
        if (nc && !issue(0)) return false;
        for (uint64_t i = 0; i < nc; ++i) {
            if (i + 1 < nc && !issue(i + 1)) return false;   // its buffer held chunk i-1, hashed already
            const auto a = now();
            if (hipEventSynchronize(ev_[i & 1]) != hipSuccess) return false;
            const auto b = now();
            const uint64_t o = i * kChunk;
            x.update(pin_[i & 1], std::min(kChunk, len - o));
            if (stats) {
                tWait += std::chrono::duration<double>(b - a).count();
                tHash += std::chrono::duration<double>(now() - b).count();
            }
        }
        *out = x.digest();
        if (stats)
            fprintf(stderr, "[lz4mt host hash] %.3f GB in %.1f ms: waiting for copies %.1f ms, hashing %.1f ms\n",
                    len / 1e9, std::chrono::duration<double>(now() - t0).count() * 1e3, tWait * 1e3, tHash * 1e3);
        return true;
    }
    hipStream_t stream() const { return cp_; }
    uint32_t* word() const { return word_; }   // pinned: a digest to copy to the device

private:
    bool ensure() {
        int d = -1;
        if (hipGetDevice(&d) != hipSuccess) return false;
        if (cp_ && d == dev_) return true;
        release();
        dev_ = d;
        if (hipStreamCreateWithFlags(&cp_, hipStreamNonBlocking) != hipSuccess) { cp_ = nullptr; return false; }
        for (int i = 0; i < 2; ++i)
            if (hipHostMalloc(reinterpret_cast<void**>(&pin_[i]), kChunk, 0) != hipSuccess ||
                hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming) != hipSuccess) {
                release();
                return false;
            }
        if (hipHostMalloc(reinterpret_cast<void**>(&word_), 64, 0) != hipSuccess) { release(); return false; }
        return true;
    }
    void release() {
        if (cp_) { hipStreamSynchronize(cp_); hipStreamDestroy(cp_); }
        for (int i = 0; i < 2; ++i) {
            if (pin_[i]) hipHostFree(pin_[i]);
            if (ev_[i]) hipEventDestroy(ev_[i]);
            pin_[i] = nullptr; ev_[i] = nullptr;
        }
        if (word_) hipHostFree(word_);
        word_ = nullptr; cp_ = nullptr; dev_ = -1;
    }
    hipStream_t cp_ = nullptr;
    uint8_t* pin_[2] = {nullptr, nullptr};
    hipEvent_t ev_[2] = {nullptr, nullptr};
    uint32_t* word_ = nullptr;
    int dev_ = -1;
};
thread_local HostHasher g_hasher;

}  // namespace

// ===========================================================================
// internal C++ API shared with the host frame engine (lz4mt_frame.cpp)
// ===========================================================================
namespace lz4mt {


// Compresses nb blocks (block b = src[b*bm, ...), last block short) into a
// frame BODY (records only) at `body`; total body size written to
// d_bodySize.  Used by the frame call and by the batched DEVICE mode.
// With an AuxStream the block checksums run on it, beside the scan and the
// assembly (both only read the encoded slots); the checksum words are
// written once both are done.
Lz4MtResult device_compress_body(const uint8_t* src, uint64_t n, uint32_t bm, int blockChecksum, uint8_t* ws,
                                 uint8_t* body, uint32_t hdrLen, hipStream_t st, uint64_t** d_recOffOut,
                                 const AuxStream* aux, const LinkState* link, int level) {
    const uint64_t nb = (n + bm - 1) / bm;
    CompressWs w = carve_compress(ws, nb, bm, level);
    // Independent 1 / 4 MiB blocks with block checksums and a side stream:
    // the encoder publishes its progress and k_xxh32_follow hashes the
    // stored bytes beside it (no LDS, so it runs while the encoder holds all
    // of it).  Never on one stream (a graph capture): the follower waits for
    // the encode, which would then queue behind it.
    const bool follow = !link && level < 3 && blockChecksum && aux && aux->st && aux->evMid && follow_enabled() &&
                        bm >= (1u << 20) && bm <= (4u << 20);
    if (follow) {
        HIPCHK(hipMemsetAsync(w.pub, 0, nb * 4 + 4, st));
        HIPCHK(hipMemsetAsync(w.xdone, 0, nb * 4 + 4, st));
        HIPCHK(hipEventRecord(aux->evIn, st));
    }
    g_timing.mark(0, st);
    if (link && level >= 3 && link->hcPerBlock) {   // -BD LZ4-HC, one segment per block: level 9, cap n - 1
        HIPCHK(launch_encode_hc(src, n, bm, (uint32_t)nb, w.slots, bm, 0xFFFFFFFEu, 9, w.delta, w.csize, st, w.hcSplit));
    } else if (link && level >= 3) {   // block-dependent LZ4-HC: the stream's segments, a wave per block
        const uint8_t* g = link->hcSegs;
        const uint32_t ns = link->nSeg;
        HIPCHK(launch_encode_hc_bd(src, n, bm, (uint32_t)nb, w.slots, reinterpret_cast<const int64_t*>(g),
                                   reinterpret_cast<const int64_t*>(g + 8 * (size_t)ns), ns,
                                   reinterpret_cast<const uint32_t*>(g + 16 * (size_t)ns), w.delta + 65536, w.csize,
                                   st));
    } else if (link && link->rounds && !bd_serial())   // block-dependent: parallel rounds (exact; serial fallback)
        HIPCHK(launch_encode_linked_par(src, n, bm, (uint32_t)nb, w.slots, link->plan, link->table, link->fresh,
                                        link->xh, link->rounds, w.csize, env_rounds(), st));
    else if (link)             // block-dependent frame: one wave, blocks in order (k_encode_linked)
        HIPCHK(launch_encode_linked(src, n, bm, (uint32_t)nb, w.slots, link->plan, link->table, link->fresh,
                                    link->xh, w.csize, st));
    else if (level >= 3)   // LZ4-HC, a wave per block (lz4mt_hc.hip)
        HIPCHK(launch_encode_hc(src, n, bm, (uint32_t)nb, w.slots, bm, 0xFFFFFFFFu, level, w.delta, w.csize, st,
                                w.hcSplit));
    else if (follow) {   // block checksums hashed beside the encode (k_xxh32_follow), as the output appears
        HIPCHK(launch_encode_pub(src, n, bm, (uint32_t)nb, w.slots, w.csize, w.pub, st));
        // launched AFTER the encoder: were the two streams ever mapped onto
        // one hardware queue, the follower would merely run after it
        HIPCHK(hipStreamWaitEvent(aux->st, aux->evIn, 0));
        HIPCHK(launch_xxh32_follow(src, w.slots, n, bm, (uint32_t)nb, w.pub, w.bsum, w.xdone, aux->st));
    }
    else
        HIPCHK(launch_encode(src, n, bm, (uint32_t)nb, w.slots, bm, 0xFFFFFFFFu, w.csize, st));
    g_timing.mark(1, st);
    const bool side = blockChecksum && aux && aux->st;
    if (follow) {   // the follower ends once every block is done; the fix-up waits for the encode
        HIPCHK(hipEventRecord(aux->evMid, st));
        HIPCHK(hipStreamWaitEvent(aux->st, aux->evMid, 0));
        HIPCHK(launch_xxh32_fixup(src, w.slots, n, bm, (uint32_t)nb, w.csize, w.bsum, w.xdone, aux->st));
        HIPCHK(hipEventRecord(aux->evOut, aux->st));
    } else if (side) {
        HIPCHK(hipEventRecord(aux->evIn, st));
        HIPCHK(hipStreamWaitEvent(aux->st, aux->evIn, 0));
        HIPCHK(launch_xxh32_stored(src, w.slots, n, bm, (uint32_t)nb, w.csize, w.bsum, aux->st));
        HIPCHK(hipEventRecord(aux->evOut, aux->st));
    } else if (blockChecksum) {
        HIPCHK(launch_xxh32_stored(src, w.slots, n, bm, (uint32_t)nb, w.csize, w.bsum, st));
    }
    g_timing.mark(2, st);
    HIPCHK(launch_frame_scan(w.csize, n, bm, (uint32_t)nb, blockChecksum, w.recOff, st));
    HIPCHK(launch_frame_assemble(src, w.slots, n, bm, (uint32_t)nb, w.csize, w.bsum, w.recOff,
                                 side ? 2 : blockChecksum, body, hdrLen, st));
    if (side) {
        HIPCHK(hipStreamWaitEvent(st, aux->evOut, 0));
        HIPCHK(launch_frame_sums(w.csize, n, bm, (uint32_t)nb, w.bsum, w.recOff, body, hdrLen, st));
    }
    if (d_recOffOut) *d_recOffOut = w.recOff;
    return LZ4MT_RESULT_OK;
}

bool AuxStream::ensure() {
    int d = -1;
    if (hipGetDevice(&d) != hipSuccess) return false;
    if (st && d == dev) return true;
    release();
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { st = nullptr; return false; }
    if (hipEventCreateWithFlags(&evIn, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&evMid, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&evOut, hipEventDisableTiming) != hipSuccess) {
        release();
        return false;
    }
    dev = d;
    return true;
}

void AuxStream::release() {
    if (st) { hipStreamSynchronize(st); hipStreamDestroy(st); }
    if (evIn) hipEventDestroy(evIn);
    if (evMid) hipEventDestroy(evMid);
    if (evOut) hipEventDestroy(evOut);
    st = nullptr; evIn = nullptr; evMid = nullptr; evOut = nullptr; dev = -1;
}

uint64_t compress_ws_bytes(uint64_t n, uint32_t bm, int level, int bd) {
    return carve_compress(nullptr, (n + bm - 1) / bm, bm, level, bd).bytes;
}

// the workspace kind of a descriptor + level (carve_compress's bd)
static int ws_bd_kind(const Lz4MtStreamDescriptor* sd, int level) {
    return (sd && !sd->flg.blockIndependence) ? (level >= 3 ? 2 : 1) : 0;
}

}  // namespace lz4mt

// ===========================================================================
// 1. block operators
// ===========================================================================
extern "C" int lz4mtHipCompressBound(int isize) {
    return ((unsigned)isize > 0x7E000000u) ? 0 : isize + isize / 255 + 16;
}

extern "C" int lz4mtHipCompressBlock(const char* src, char* dst, int isize, int maxOutputSize, int compressionLevel) {
    // levels >= 3: LZ4-HC (LZ4_compressHC2_limitedOutput): 3..9 hashChain,
    // 10..12 (and above, clamped to 12) the optimal parser
    const bool hc = compressionLevel >= 3;
    if (isize < 0 || (unsigned)isize > 0x7E000000u) return 0;
    if (maxOutputSize < 0) maxOutputSize = 0;
    if (!have_device()) return -1;
    ScratchLease g_blk;
    if (!g_blk->init()) return -1;
    const int bound = lz4mtHipCompressBound(isize);
    uint64_t outMax = (uint64_t)std::min(maxOutputSize, bound) + 16;
    // LZ4-HC on a large block: the split parse (one wave per 256 KiB stream)
    // writes each stream at its offset in an output of at least isize bytes
    const uint64_t splitBytes = hc ? hc_ws_bytes(1, (uint32_t)std::max(isize, 1), compressionLevel) : 0;
    if (splitBytes) outMax = std::max<uint64_t>(outMax, (uint64_t)isize + 16);
    if (!g_blk->ensure((uint64_t)isize, outMax)) return -1;
    if (hc && !g_blk->ensure_delta((uint64_t)isize)) return -1;
    if (splitBytes && !g_blk->ensure_split(splitBytes)) return -1;
    if (isize && hipMemcpyAsync(g_blk->dIn, src, (size_t)isize, hipMemcpyHostToDevice, g_blk->st) != hipSuccess) return -1;
    const hipError_t le = hc ? launch_encode_hc(g_blk->dIn, (uint64_t)isize, (uint32_t)std::max(isize, 1), 1, g_blk->dOut,
                                                splitBytes ? (uint64_t)isize : 0, (uint32_t)maxOutputSize,
                                                compressionLevel, g_blk->dDelta, g_blk->dRes, g_blk->st,
                                                splitBytes ? g_blk->dSplit : nullptr)
                             : launch_encode(g_blk->dIn, (uint64_t)isize, (uint32_t)std::max(isize, 1), 1, g_blk->dOut,
                                             0, (uint32_t)maxOutputSize, g_blk->dRes, g_blk->st);
    if (le != hipSuccess) return -1;
    int32_t r = 0;
    if (hipMemcpyAsync(&r, g_blk->dRes, 4, hipMemcpyDeviceToHost, g_blk->st) != hipSuccess) return -1;
    if (hipStreamSynchronize(g_blk->st) != hipSuccess) return -1;
    if (r > 0) {
        if (hipMemcpyAsync(dst, g_blk->dOut, (size_t)r, hipMemcpyDeviceToHost, g_blk->st) != hipSuccess) return -1;
        if (hipStreamSynchronize(g_blk->st) != hipSuccess) return -1;
    }
    return r;
}

extern "C" int lz4mtHipDecompressBlock(const char* src, char* dst, int isize, int maxOutputSize) {
    if (isize < 0 || maxOutputSize < 0) return -1;
    if (!have_device()) return -1;
    ScratchLease g_blk;
    if (!g_blk->init()) return -1;
    if (!g_blk->ensure((uint64_t)isize, (uint64_t)maxOutputSize)) return -1;
    if (isize && hipMemcpyAsync(g_blk->dIn, src, (size_t)isize, hipMemcpyHostToDevice, g_blk->st) != hipSuccess) return -1;
    BlockRec rec{0, (uint32_t)isize, 0};
    if (hipMemcpyAsync(g_blk->dRec, &rec, sizeof(rec), hipMemcpyHostToDevice, g_blk->st) != hipSuccess) return -1;
    if (launch_decode(g_blk->dIn, g_blk->dRec, 1, (uint32_t)maxOutputSize, g_blk->dOut, (uint64_t)maxOutputSize,
                      g_blk->dRes, g_blk->st) != hipSuccess)
        return -1;
    int32_t r = 0;
    if (hipMemcpyAsync(&r, g_blk->dRes, 4, hipMemcpyDeviceToHost, g_blk->st) != hipSuccess) return -1;
    if (hipStreamSynchronize(g_blk->st) != hipSuccess) return -1;
    if (r > 0) {
        if (hipMemcpyAsync(dst, g_blk->dOut, (size_t)r, hipMemcpyDeviceToHost, g_blk->st) != hipSuccess) return -1;
        if (hipStreamSynchronize(g_blk->st) != hipSuccess) return -1;
    }
    return r == kDecodeOutputTooSmall ? -1 : r;
}

// ===========================================================================
// 2. device-resident frame engine
// ===========================================================================
extern "C" uint64_t lz4mtHipFrameBound(uint64_t srcSize, const Lz4MtStreamDescriptor* sd) {
    const int id = sd ? sd->bd.blockMaximumSize : 7;
    const uint64_t bm = (id >= 4 && id <= 7) ? (uint64_t)block_max_bytes(id) : (4u << 20);
    const uint64_t nb = (srcSize + bm - 1) / bm;
    return (uint64_t)kMaxHeader + srcSize + nb * 8 + 8;
}

extern "C" uint64_t lz4mtHipCompressWorkspaceSizeEx(uint64_t srcSize, const Lz4MtStreamDescriptor* sd, int level) {
    const int id = sd ? sd->bd.blockMaximumSize : 7;
    const uint32_t bm = (id >= 4 && id <= 7) ? (uint32_t)block_max_bytes(id) : (4u << 20);
    return compress_ws_bytes(srcSize, bm, level < 3 ? 0 : level, ws_bd_kind(sd, level));
}

extern "C" uint64_t lz4mtHipCompressWorkspaceSize(uint64_t srcSize, const Lz4MtStreamDescriptor* sd) {
    return lz4mtHipCompressWorkspaceSizeEx(srcSize, sd, 0);
}

static Lz4MtResult compress_frame_impl(const void* d_src, uint64_t srcSize, void* d_frame, uint64_t frameCap,
                                       uint64_t* d_frameSize, const Lz4MtStreamDescriptor* sd, int level, void* d_ws,
                                       uint64_t wsSize, hipStream_t st, void** ownedWs, bool hostHash) {
    if (!sd || !d_frame || (!d_src && srcSize)) return LZ4MT_RESULT_BAD_ARG;
    const Lz4MtResult v = validate_sd(sd);
    if (v != LZ4MT_RESULT_OK) return v;
    if (!have_device()) return LZ4MT_RESULT_ERROR;
    if (frameCap < lz4mtHipFrameBound(srcSize, sd)) return LZ4MT_RESULT_BAD_ARG;
    // LZ4-HC on independent blocks: levels 3..9 the hashChain parser, 10..12
    // (and above, clamped) the optimal parser.  Block-dependent frames at any
    // level >= 3 are the reference's HC stream, which runs at level 9 (HcBdSim).
    if (level < 3) level = 0;
    const uint32_t bm = (uint32_t)block_max_bytes(sd->bd.blockMaximumSize);
    const int bdk = ws_bd_kind(sd, level);
    const uint64_t need = compress_ws_bytes(srcSize, bm, level, bdk);
    uint8_t* ws = static_cast<uint8_t*>(d_ws);
    if (!ws || wsSize < need) {
        if (hipMalloc(reinterpret_cast<void**>(&ws), need) != hipSuccess) return LZ4MT_RESULT_ERROR;
        *ownedWs = ws;
    }
    uint8_t hdr[kMaxHeader];
    const int hdrLen = build_header(sd, hdr);
    uint64_t* recOff = nullptr;
    // side streams (block checksums; the content checksum), except while
    // `st` is being captured into a graph (no stream creation inside a capture)
    thread_local AuxStream aux, auxStream;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    const bool capturing = hipStreamIsCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone;
    CompressWs w = carve_compress(ws, (srcSize + bm - 1) / bm, bm, level, bdk);
    // The content checksum (FLG.2) is one serial XXH32 chain over the input
    // (SURVEY.md §0.5).  It reads only d_src, so it starts at t = 0 on its
    // own stream, beside the encode, and the finalize waits for it.
    const bool sck = sd->flg.streamChecksum != 0;
    // the synchronous call hashes on the host (HostHasher), beside the
    // encode; the asynchronous one stays on the device (one wavefront)
    thread_local hipEvent_t srcReady = nullptr, sumDone = nullptr;
    const bool sckHost = sck && hostHash && !capturing &&
                         (srcReady || hipEventCreateWithFlags(&srcReady, hipEventDisableTiming) == hipSuccess) &&
                         (sumDone || hipEventCreateWithFlags(&sumDone, hipEventDisableTiming) == hipSuccess);
    if (sckHost) HIPCHK(hipEventRecord(srcReady, st));
    const bool sckSide = sck && !sckHost && !capturing && auxStream.ensure();
    if (sckSide) {
        HIPCHK(hipEventRecord(auxStream.evIn, st));
        HIPCHK(hipStreamWaitEvent(auxStream.st, auxStream.evIn, 0));
        HIPCHK(launch_xxh32_stream(static_cast<const uint8_t*>(d_src), srcSize, w.ssum, auxStream.st));
        HIPCHK(hipEventRecord(auxStream.evOut, auxStream.st));
    }
    // block-dependent frames: the per-block lz4 stream plan (BdSim), the
    // carried table and the rounds' scratch live in this call's workspace,
    // so asynchronous calls on other streams never share them (the host
    // plan is staged by the copy before hipMemcpyAsync returns: pageable
    // memory)
    LinkState ls{};
    const LinkState* lsp = nullptr;
    if (bdk == 2) {
        const uint64_t nb = (srcSize + bm - 1) / bm;
        std::vector<uint64_t> segAbs(nb, 0);
        std::vector<uint8_t> packed;
        HcBdSim sim(sd->bd.blockMaximumSize);
        for (uint64_t b = 0; b < nb; ++b) segAbs[b] = sim.next((uint32_t)std::min<uint64_t>(bm, srcSize - b * bm));
        ls.nSeg = hc_bd_pack(segAbs.data(), nb, 0, srcSize, 0, packed, bm, &ls.hcPerBlock);
        if (!packed.empty())
            HIPCHK(hipMemcpyAsync(w.bdPlan, packed.data(), packed.size(), hipMemcpyHostToDevice, st));
        ls.hcSegs = w.bdPlan;
        lsp = &ls;
    } else if (bdk == 1) {
        const uint64_t nb = (srcSize + bm - 1) / bm;
        std::vector<LinkPlan> hplan(std::max<uint64_t>(nb, 1), LinkPlan{});
        const bool refBytes = bd_reference_bytes();
        BdSim sim(sd->bd.blockMaximumSize, refBytes);
        bool xh = false;
        for (uint64_t b = 0; b < nb; ++b) {
            sim.next((uint32_t)std::min<uint64_t>(bm, srcSize - b * bm), &hplan[b].lowIn, &hplan[b].lowDict,
                     &hplan[b].candLow, refBytes ? &hplan[b].shift : nullptr);
            xh = xh || hplan[b].shift != 0;
        }
        if (sim.bad) return LZ4MT_RESULT_ERROR;
        HIPCHK(hipMemcpyAsync(w.bdPlan, hplan.data(), hplan.size() * sizeof(LinkPlan), hipMemcpyHostToDevice, st));
        ls = LinkState{reinterpret_cast<LinkPlan*>(w.bdPlan), w.bdTable, true, w.bdRounds};
        ls.xh = xh;
        lsp = &ls;
    }
    const Lz4MtResult r = device_compress_body(static_cast<const uint8_t*>(d_src), srcSize, bm, sd->flg.blockChecksum,
                                               ws, static_cast<uint8_t*>(d_frame), (uint32_t)hdrLen, st, &recOff,
                                               !capturing && aux.ensure() ? &aux : nullptr, lsp, level);
    if (r != LZ4MT_RESULT_OK) {
        if (sckSide) hipStreamWaitEvent(st, auxStream.evOut, 0);   // scratch outlives the side kernel
        return r;
    }
    if (sckHost) {   // the kernels above run while the host hashes
        uint32_t h = 0;
        if (!g_hasher.hash(static_cast<const uint8_t*>(d_src), srcSize, srcReady, &h)) return LZ4MT_RESULT_ERROR;
        *g_hasher.word() = h;
        HIPCHK(hipMemcpyAsync(w.ssum, g_hasher.word(), 4, hipMemcpyHostToDevice, g_hasher.stream()));
        HIPCHK(hipEventRecord(sumDone, g_hasher.stream()));
        HIPCHK(hipStreamWaitEvent(st, sumDone, 0));
    } else if (sckSide) {
        HIPCHK(hipStreamWaitEvent(st, auxStream.evOut, 0));
    } else if (sck) {
        HIPCHK(launch_xxh32_stream(static_cast<const uint8_t*>(d_src), srcSize, w.ssum, st));
    }
    g_timing.mark(3, st);
    HIPCHK(launch_frame_finalize(static_cast<uint8_t*>(d_frame), hdr, (uint32_t)hdrLen, recOff,
                                 (uint32_t)((srcSize + bm - 1) / bm), sd->flg.streamChecksum ? w.ssum : nullptr,
                                 d_frameSize ? d_frameSize : w.fsize, st));
    g_timing.mark(4, st);
    return LZ4MT_RESULT_OK;
}

extern "C" Lz4MtResult lz4mtHipCompressFrameAsyncEx(const void* d_src, uint64_t srcSize, void* d_frame,
                                                    uint64_t frameCap, uint64_t* d_frameSize,
                                                    const Lz4MtStreamDescriptor* sd, int level, void* d_workspace,
                                                    uint64_t workspaceSize, void* stream) {
    void* owned = nullptr;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const Lz4MtResult r = compress_frame_impl(d_src, srcSize, d_frame, frameCap, d_frameSize, sd, level, d_workspace,
                                              workspaceSize, st, &owned, false);
    if (owned) {  // library-owned scratch: must outlive the kernels
        hipStreamSynchronize(st);
        hipFree(owned);
    }
    return r;
}

extern "C" Lz4MtResult lz4mtHipCompressFrameAsync(const void* d_src, uint64_t srcSize, void* d_frame, uint64_t frameCap,
                                                  uint64_t* d_frameSize, const Lz4MtStreamDescriptor* sd,
                                                  void* d_workspace, uint64_t workspaceSize, void* stream) {
    void* owned = nullptr;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const Lz4MtResult r =
        compress_frame_impl(d_src, srcSize, d_frame, frameCap, d_frameSize, sd, 0, d_workspace, workspaceSize, st, &owned,
                            false);
    if (owned) {  // library-owned scratch: must outlive the kernels
        hipStreamSynchronize(st);
        hipFree(owned);
    }
    return r;
}

extern "C" Lz4MtResult lz4mtHipCompressFrameEx(const void* d_src, uint64_t srcSize, void* d_frame, uint64_t frameCap,
                                               uint64_t* frameSize, const Lz4MtStreamDescriptor* sd, int level,
                                               void* d_workspace, uint64_t workspaceSize, void* stream) {
    void* owned = nullptr;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    uint64_t* dfs = reinterpret_cast<uint64_t*>(small_dev());
    if (!dfs) return LZ4MT_RESULT_ERROR;
    Lz4MtResult r =
        compress_frame_impl(d_src, srcSize, d_frame, frameCap, dfs, sd, level, d_workspace, workspaceSize, st, &owned,
                            true);
    if (r == LZ4MT_RESULT_OK) {
        uint64_t fs = 0;
        if (hipMemcpyAsync(&fs, dfs, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            r = LZ4MT_RESULT_ERROR;
        if (frameSize) *frameSize = fs;
    } else {
        hipStreamSynchronize(st);
    }
    if (owned) hipFree(owned);
    return r;
}

extern "C" Lz4MtResult lz4mtHipCompressFrame(const void* d_src, uint64_t srcSize, void* d_frame, uint64_t frameCap,
                                             uint64_t* frameSize, const Lz4MtStreamDescriptor* sd, void* d_workspace,
                                             uint64_t workspaceSize, void* stream) {
    return lz4mtHipCompressFrameEx(d_src, srcSize, d_frame, frameCap, frameSize, sd, 0, d_workspace, workspaceSize,
                                   stream);
}

// ---------------------------------------------------------------------------
// decompress
// ---------------------------------------------------------------------------
namespace {

struct DecodeBuffers {
    BlockRec* recs = nullptr;
    uint32_t* digest = nullptr;
    int32_t* dsize = nullptr;
    int32_t* status = nullptr;
    WalkInfo* info = nullptr;
    uint32_t* ssum = nullptr;
    uint32_t* ctl = nullptr;   // k_decode_walk's published / ended / next words
    uint64_t cap = 0;
    ~DecodeBuffers() {
        release();
        if (ctl) hipFree(ctl);
    }
    // k_decode_walk's control words live in UNCACHED device memory: the
    // waves poll them from every XCD, and an sc1 load is served by the
    // reader's own L2, which is not coherent with the other XCDs' -- with
    // cached memory a poller read a stale copy of the walk's progress until
    // its 30 s bound (per-XCD L2s, MI355X_MICROARCH.md).  Some runtimes grant
    // the kind only in 2 MiB units.  False: the fused walk is not used.
    bool ensure_ctl() {
        if (ctl) return true;
        for (size_t sz : {size_t(32), size_t(2) << 20}) {
            void* p = nullptr;
            if (hipExtMallocWithFlags(&p, sz, hipDeviceMallocUncached) == hipSuccess && p) {
                ctl = static_cast<uint32_t*>(p);
                return true;
            }
            (void)hipGetLastError();
        }
        return false;
    }
    WalkScratch ws{};
    uint64_t wsChunks = 0, wsCap = 0, wsNodes = 0;
    void release() {
        hipFree(recs); hipFree(digest); hipFree(dsize); hipFree(status); hipFree(info); hipFree(ssum);
        recs = nullptr; digest = nullptr; dsize = nullptr; status = nullptr; info = nullptr; ssum = nullptr;
        cap = 0;
        release_walk();
    }
    void release_walk() {
        hipFree(ws.count); hipFree(ws.base); hipFree(ws.P);
        release_nodes();
        ws = WalkScratch{};
        wsChunks = 0; wsCap = 0;
    }
    void release_nodes() {
        hipFree(ws.pos); hipFree(ws.Ja); hipFree(ws.Jb);
        ws.pos = nullptr; ws.Ja = nullptr; ws.Jb = nullptr;
        wsNodes = 0;
    }
    bool ensure_walk(uint64_t chunks, uint64_t nb) {
        if (ws.P && chunks <= wsChunks && nb <= wsCap) return true;
        release_walk();
        wsChunks = chunks; wsCap = nb;
        return hipMalloc(reinterpret_cast<void**>(&ws.count), chunks * 4) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&ws.base), (chunks + 1) * 8) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&ws.P), (nb + 1) * 4) == hipSuccess;
    }
    bool ensure_nodes(uint64_t m) {
        if (ws.pos && m <= wsNodes) return true;
        release_nodes();
        wsNodes = std::max<uint64_t>(m, 1024);
        return hipMalloc(reinterpret_cast<void**>(&ws.pos), wsNodes * 8) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&ws.Ja), (wsNodes + 1) * 4) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&ws.Jb), (wsNodes + 1) * 4) == hipSuccess;
    }
    bool ensure(uint64_t nb) {
        if (info && nb <= cap) return true;
        release();
        cap = std::max<uint64_t>(nb, 64);
        return hipMalloc(reinterpret_cast<void**>(&recs), cap * sizeof(BlockRec)) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&digest), cap * 4) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&dsize), cap * 4) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&status), cap * 4) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&info), sizeof(WalkInfo)) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&ssum), 16) == hipSuccess;
    }
};

// Per-thread cache of the decode scratch (records, digests, walk scratch):
// no hipMalloc / hipFree per call -- hipFree waits for the whole device,
// which would also wait for unrelated work such as an RCCL transfer running
// beside the decode.  Re-made when the thread's current device changes.
DecodeBuffers& decode_cache() {
    thread_local DecodeBuffers B;
    thread_local int dev = -1;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) d = -1;
    if (d != dev) {
        B.release();
        dev = d;
    }
    return B;
}

// Walks one frame body; retries with a larger block table if needed.
Lz4MtResult walk_frame(const uint8_t* frame, uint64_t frameSize, uint64_t bodyPos, uint32_t bm, int bck,
                       DecodeBuffers& B, WalkInfo& wi, hipStream_t st) {
    uint64_t guess = std::min<uint64_t>((frameSize - bodyPos) / 4 + 1, (frameSize - bodyPos) / 1024 + 4096);
    // The serial walk pays one dependent load per block; the parallel one a
    // pass over the body.  Parallel wins once blocks are small (<= 1 MiB)
    // and many.
    // LZ4MT_AMD_WALK=serial|parallel forces one (tests run both on small frames).
    const char* fe = getenv("LZ4MT_AMD_WALK");
    const int force = !fe ? 0 : (strcmp(fe, "serial") == 0 ? 1 : (strcmp(fe, "parallel") == 0 ? 2 : 0));
    const bool autoPar = bm <= (1u << 20) && frameSize - bodyPos >= (64ull << 20);
    const bool par = frameSize < (1ull << 40) && frameSize >= bodyPos + 8 && (force == 2 || (force == 0 && autoPar));
    for (int attempt = 0; attempt < 2; ++attempt) {
        if (!B.ensure(guess)) return LZ4MT_RESULT_ERROR;
        wi.result = -1;
        if (par) {
            const uint64_t nc = frame_walk_par_chunks(frameSize);
            if (!B.ensure_walk(nc, B.cap)) return LZ4MT_RESULT_ERROR;
            HIPCHK(launch_frame_walk_count(frame, frameSize, bodyPos, bm, bck, B.ws, st));
            uint64_t M = 0;
            HIPCHK(hipMemcpyAsync(&M, B.ws.base + nc, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            // more candidates than 1 per 8 bytes: not worth it (and node ids are u32)
            if (M > 0 && M <= (frameSize - bodyPos) / 8 + 1024 && M < (1ull << 31)) {
                if (!B.ensure_nodes(M)) return LZ4MT_RESULT_ERROR;
                HIPCHK(launch_frame_walk_path(frame, frameSize, bodyPos, bm, bck, (uint32_t)B.cap, (uint32_t)M, B.ws,
                                              B.recs, B.info, st));
                HIPCHK(hipMemcpyAsync(&wi, B.info, sizeof(wi), hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
            }
        }
        if (wi.result == -1) {   // serial walk (also: malformed frames, for the exact error code)
            HIPCHK(launch_frame_walk(frame, frameSize, bodyPos, bm, bck, (uint32_t)B.cap, B.recs, B.info, st));
            HIPCHK(hipMemcpyAsync(&wi, B.info, sizeof(wi), hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
        }
        if (!(wi.result == 1 && wi.nBlocks == B.cap)) return LZ4MT_RESULT_OK;
        guess = (frameSize - bodyPos) / 4 + 1;
    }
    return LZ4MT_RESULT_OK;
}

// LZ4MT_AMD_WALK: fused (the serial walk inside the decode kernel), serial
// (the separate serial walk kernel), parallel (the candidate walk, the
// default for blocks <= 1 MiB over 64 MiB)
// Fused by default only where the walk is serial and the frame surely spans
// more than one decode generation (8 resident decoders per CU; body /
// (bm + 8) is a lower bound on its block count): the walk then
// overlaps the earlier generations (32 GiB B7: 270.6 -> 273.2 GiB/s), while
// with one generation the last block's record arrives only at the walk's end
// (8 GiB B7: 262.4 -> 258.3; profiles/r06/r06ae_fused_walk_ab.txt).
bool fused_walk(uint32_t bm, uint64_t body) {
    const char* fe = getenv("LZ4MT_AMD_WALK");
    if (fe && strcmp(fe, "fused") == 0) return true;
    if (fe && (strcmp(fe, "serial") == 0 || strcmp(fe, "parallel") == 0)) return false;
    static const uint64_t kDecoders = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return (uint64_t)cus * 8;
    }();
    const bool serialWalk = !(bm <= (1u << 20) && body >= (64ull << 20));
    return serialWalk && body / ((uint64_t)bm + 8) > kDecoders;
}

// The fused walk + decode of an independent-block frame body into target
// (k_decode_walk), with the block checksums (k_xxh32_walked, on the aux
// stream) and the verify launched behind it: nothing waits on the host
// until the walk's info is read back at the end.  Returns false, with
// nothing to undo, when the record table overflowed (the caller then walks
// separately with a larger one); otherwise wi is the walk's result and
// dsize / status hold the blocks [0, wi.nBlocks).
bool decode_walk_fused(const uint8_t* f, uint64_t frameSize, uint64_t bodyPos, uint32_t bm, int bck, uint8_t* target,
                       uint64_t targetCap, DecodeBuffers& B, AuxStream& aux, WalkInfo& wi, Lz4MtResult& result,
                       hipStream_t st) {
    static const uint32_t kCus = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return (uint32_t)cus;
    }();
    const uint64_t guess = std::min<uint64_t>((frameSize - bodyPos) / 4 + 1, (frameSize - bodyPos) / 1024 + 4096);
    result = LZ4MT_RESULT_OK;
    if (!B.ensure(guess)) { result = LZ4MT_RESULT_ERROR; return true; }
    const uint32_t cap = (uint32_t)std::min<uint64_t>(B.cap, 0xFFFFFFFFu);
    const bool side = bck && aux.ensure();
    bool ok = hipMemsetAsync(B.ctl, 0, 32, st) == hipSuccess;
    if (ok && side) ok = hipEventRecord(aux.evIn, st) == hipSuccess && hipStreamWaitEvent(aux.st, aux.evIn, 0) == hipSuccess;
    static const bool trace = getenv("LZ4MT_AMD_WALK_TRACE") != nullptr;
    static hipEvent_t ev[6] = {};
    if (trace && !ev[0])
        for (auto& e : ev) hipEventCreate(&e);
    if (trace) hipEventRecord(ev[0], st);
    // k_decode's LDS allows 8 resident waves per CU: the walker + 8 decoders per
    // CU (the last one resident once the walk ends); with one decoder fewer, one
    // wave decoded two blocks of a one-generation frame back to back
    ok = ok && launch_decode_walk(f, frameSize, bodyPos, bm, bck, cap, B.recs, B.info, B.ctl, target, targetCap, B.dsize,
                                  std::min<uint32_t>(kCus * 8, cap) + 1, st) == hipSuccess;
    if (trace) hipEventRecord(ev[1], st);
    if (ok && bck) {   // 16 blocks per wave, as k_xxh32_frame_blocks; at most 2 waves per CU
        const uint32_t xw = std::min<uint32_t>(kCus * 2, (cap + 15) / 16);
        if (trace) hipEventRecord(ev[2], side ? aux.st : st);
        ok = launch_xxh32_walked(f, B.recs, B.ctl, B.digest, xw, side ? aux.st : st) == hipSuccess;
        if (trace) hipEventRecord(ev[3], side ? aux.st : st);
        if (ok && side) ok = hipEventRecord(aux.evOut, aux.st) == hipSuccess && hipStreamWaitEvent(st, aux.evOut, 0) == hipSuccess;
    }
    ok = ok && launch_block_verify_walked(B.recs, B.info, B.digest, B.dsize, bck, B.status, cap, st) == hipSuccess &&
         hipMemcpyAsync(&wi, B.info, sizeof(wi), hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
    if (trace) {
        float a = -1, b = -1, c = -1;
        hipEventSynchronize(ev[1]);
        hipEventElapsedTime(&a, ev[0], ev[1]);
        if (bck) {
            hipEventSynchronize(ev[3]);
            hipEventElapsedTime(&b, ev[2], ev[3]);
            hipEventElapsedTime(&c, ev[0], ev[2]);
        }
        fprintf(stderr, "fused walk: k_decode_walk %.3f ms, k_xxh32_walked %.3f ms (starting %.3f ms after the decode "
                "kernel's start)\n", a, b, c);
    }
    if (!ok) { result = LZ4MT_RESULT_ERROR; return true; }
#if LZ4MT_WALK_DIAG
    {
        uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        hipMemcpy(c, B.ctl, 32, hipMemcpyDeviceToHost);
        fprintf(stderr, "fused walk diag: ctl %08x next %u groups %u; timeouts %u (last: need %u saw %08x)\n", c[0],
                c[2], c[3], c[5], c[6], c[7]);
    }
#endif
    if (wi.result == 1 && wi.nBlocks == cap) return false;   // record table full: walk separately, larger
    return true;
}

}  // namespace

extern "C" Lz4MtResult lz4mtHipFrameInfo(const void* d_frame, uint64_t frameSize, Lz4MtStreamDescriptor* sd,
                                         uint64_t* decodedBound, uint64_t* nBlocks, void* stream) {
    if (!d_frame || !sd) return LZ4MT_RESULT_BAD_ARG;
    if (!have_device()) return LZ4MT_RESULT_ERROR;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const uint8_t* f = static_cast<const uint8_t*>(d_frame);
    uint64_t pos = 0;
    for (;;) {  // skip skippable frames
        uint8_t h[kMaxHeader + 8] = {0};
        const uint64_t avail = std::min<uint64_t>(sizeof(h), frameSize - pos);
        HIPCHK(hipMemcpyAsync(h, f + pos, avail, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (avail < 4) return LZ4MT_RESULT_INVALID_HEADER;
        const uint32_t magic = get32(h);
        if (magic >= kSkippableMin && magic <= kSkippableMax) {
            if (avail < 8) return LZ4MT_RESULT_INVALID_HEADER_SKIPPABLE_SIZE_UNREADABLE;
            pos += 8 + (uint64_t)get32(h + 4);
            if (pos >= frameSize) return LZ4MT_RESULT_INVALID_MAGIC_NUMBER;
            continue;
        }
        if (magic != kMagic) return LZ4MT_RESULT_INVALID_MAGIC_NUMBER;
        int hb = 0;
        const Lz4MtResult r = parse_header(h + 4, avail - 4, sd, &hb);
        if (r != LZ4MT_RESULT_OK) return r;
        const uint32_t bm = (uint32_t)block_max_bytes(sd->bd.blockMaximumSize);
        DecodeBuffers B;
        WalkInfo wi{};
        const Lz4MtResult wr = walk_frame(f, frameSize, pos + 4 + hb, bm, sd->flg.blockChecksum, B, wi, st);
        if (wr != LZ4MT_RESULT_OK) return wr;
        if (decodedBound) *decodedBound = (uint64_t)wi.nBlocks * bm;
        if (nBlocks) *nBlocks = wi.nBlocks;
        return wi.result ? (Lz4MtResult)wi.result : LZ4MT_RESULT_OK;
    }
}

// Header of the frame (or skippable frame) at `pos`: kind 0 = lz4mt frame
// (sd, hdrLen filled), 1 = skippable (skip = bytes to jump), 2 = end
// (fewer than 4 bytes, or non-magic data after a frame), or an error code.
namespace {
struct HeadInfo {
    int kind = 0;
    int hdrLen = 0;
    uint64_t skip = 0;
    Lz4MtResult err = LZ4MT_RESULT_OK;
};
HeadInfo read_head(const uint8_t* f, uint64_t frameSize, uint64_t pos, bool seen, Lz4MtStreamDescriptor* sd,
                   hipStream_t st) {
    HeadInfo hi;
    uint8_t h[kMaxHeader + 8] = {0};
    const uint64_t avail = std::min<uint64_t>(sizeof(h), frameSize - pos);
    if (hipMemcpyAsync(h, f + pos, avail, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
        hi.err = LZ4MT_RESULT_ERROR;
        return hi;
    }
    if (avail < 4) { hi.kind = 2; return hi; }
    const uint32_t magic = get32(h);
    if (magic != kMagic) {
        if (magic >= kSkippableMin && magic <= kSkippableMax) {
            if (avail < 8) { hi.err = LZ4MT_RESULT_INVALID_HEADER_SKIPPABLE_SIZE_UNREADABLE; return hi; }
            hi.kind = 1;
            hi.skip = 8 + (uint64_t)get32(h + 4);
            return hi;
        }
        if (!seen) hi.err = LZ4MT_RESULT_INVALID_MAGIC_NUMBER;
        hi.kind = 2;
        return hi;
    }
    int hb = 0;
    hi.err = parse_header(h + 4, avail - 4, sd, &hb);
    hi.hdrLen = 4 + hb;
    return hi;
}
}  // namespace

extern "C" Lz4MtResult lz4mtHipStreamBound(const void* d_frame, uint64_t frameSize, uint64_t* decodedBound,
                                           void* stream) {
    if (!d_frame || !decodedBound) return LZ4MT_RESULT_BAD_ARG;
    if (!have_device()) return LZ4MT_RESULT_ERROR;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const uint8_t* f = static_cast<const uint8_t*>(d_frame);
    DecodeBuffers& B = decode_cache();
    uint64_t pos = 0, bound = 0;
    bool seen = false;
    *decodedBound = 0;
    while (pos < frameSize) {
        Lz4MtStreamDescriptor sd = lz4mtInitStreamDescriptor();
        const HeadInfo hi = read_head(f, frameSize, pos, seen, &sd, st);
        if (hi.err != LZ4MT_RESULT_OK) return hi.err;
        if (hi.kind == 2) break;
        if (hi.kind == 1) { pos = std::min<uint64_t>(frameSize, pos + hi.skip); continue; }
        seen = true;
        const uint32_t bm = (uint32_t)block_max_bytes(sd.bd.blockMaximumSize);
        WalkInfo wi{};
        const Lz4MtResult wr = walk_frame(f, frameSize, pos + hi.hdrLen, bm, sd.flg.blockChecksum, B, wi, st);
        if (wr != LZ4MT_RESULT_OK) return wr;
        bound += (uint64_t)wi.nBlocks * bm;
        if (wi.result != 0) break;   // a damaged frame: the decoder stops inside it
        pos = wi.endPos + (sd.flg.streamChecksum ? 4 : 0);
    }
    *decodedBound = bound;
    return LZ4MT_RESULT_OK;
}

extern "C" Lz4MtResult lz4mtHipFrameRecords(const void* d_frame, uint64_t frameSize, uint64_t* recordStart,
                                            uint64_t cap, uint64_t* nBlocks, int* hdrLen,
                                            Lz4MtStreamDescriptor* sd, void* stream) {
    if (!d_frame || !nBlocks || !sd) return LZ4MT_RESULT_BAD_ARG;
    if (!have_device()) return LZ4MT_RESULT_ERROR;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const uint8_t* f = static_cast<const uint8_t*>(d_frame);
    const HeadInfo hi = read_head(f, frameSize, 0, false, sd, st);
    if (hi.err != LZ4MT_RESULT_OK) return hi.err;
    if (hi.kind != 0) return LZ4MT_RESULT_INVALID_MAGIC_NUMBER;
    const uint32_t bm = (uint32_t)block_max_bytes(sd->bd.blockMaximumSize);
    DecodeBuffers& B = decode_cache();
    WalkInfo wi{};
    const Lz4MtResult wr = walk_frame(f, frameSize, (uint64_t)hi.hdrLen, bm, sd->flg.blockChecksum, B, wi, st);
    if (wr != LZ4MT_RESULT_OK) return wr;
    if (wi.result != 0) return (Lz4MtResult)wi.result;
    *nBlocks = wi.nBlocks;
    if (hdrLen) *hdrLen = hi.hdrLen;
    if (recordStart && cap >= (uint64_t)wi.nBlocks + 1) {
        std::vector<BlockRec> r(wi.nBlocks);
        if (wi.nBlocks) {
            HIPCHK(hipMemcpyAsync(r.data(), B.recs, wi.nBlocks * sizeof(BlockRec), hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
        }
        for (uint64_t i = 0; i < wi.nBlocks; ++i) recordStart[i] = r[i].offset - 4;   // the size word
        recordStart[wi.nBlocks] = wi.endPos - 4;                                      // the EOS word
    } else if (recordStart) {
        return LZ4MT_RESULT_BAD_ARG;
    }
    return LZ4MT_RESULT_OK;
}

extern "C" Lz4MtResult lz4mtHipDecompressFrame(const void* d_frame, uint64_t frameSize, void* d_out, uint64_t outCap,
                                               uint64_t* outSize, Lz4MtStreamDescriptor* sd, void* stream) {
    if (!d_frame || !sd || (!d_out && outCap)) return LZ4MT_RESULT_BAD_ARG;
    if (!have_device()) return LZ4MT_RESULT_ERROR;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const uint8_t* f = static_cast<const uint8_t*>(d_frame);
    uint8_t* out = static_cast<uint8_t*>(d_out);
    uint64_t pos = 0, opos = 0;
    bool seen = false;
    Lz4MtResult result = LZ4MT_RESULT_OK;
    DecodeBuffers& B = decode_cache();
    thread_local AuxStream aux;   // block checksums beside the decode
    DevBuf tmp;   // staging when a frame's output is unaligned or needs compaction (freed on every return)
    if (outSize) *outSize = 0;
    while (pos < frameSize) {
        uint8_t h[kMaxHeader + 8] = {0};
        const uint64_t avail = std::min<uint64_t>(sizeof(h), frameSize - pos);
        HIPCHK(hipMemcpyAsync(h, f + pos, avail, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (avail < 4) break;  // 1-3 trailing bytes: end of stream (reference: OK at EOF)
        const uint32_t magic = get32(h);
        if (magic != kMagic) {
            if (magic >= kSkippableMin && magic <= kSkippableMax) {
                if (avail < 8) { result = LZ4MT_RESULT_INVALID_HEADER_SKIPPABLE_SIZE_UNREADABLE; break; }
                pos = std::min<uint64_t>(frameSize, pos + 8 + (uint64_t)get32(h + 4));
                continue;
            }
            // non-magic data: error before any frame, end of stream after one
            // (the reference spins forever here, src/lz4mt.cpp:971-979)
            if (!seen) result = LZ4MT_RESULT_INVALID_MAGIC_NUMBER;
            break;
        }
        seen = true;
        int hb = 0;
        result = parse_header(h + 4, avail - 4, sd, &hb);
        if (result != LZ4MT_RESULT_OK) break;
        const uint32_t bm = (uint32_t)block_max_bytes(sd->bd.blockMaximumSize);
        const int bck = sd->flg.blockChecksum, sck = sd->flg.streamChecksum;
        WalkInfo wi{};
        g_timing.mark(0, st);
        const uint64_t bodyPos = pos + 4 + hb;
        uint64_t produced = 0;
        if (!sd->flg.blockIndependence) {
            result = walk_frame(f, frameSize, bodyPos, bm, bck, B, wi, st);
            if (result != LZ4MT_RESULT_OK) break;
            const uint64_t nb = wi.nBlocks;
            // block-dependent frame (decompressBlockDependency, src/lz4mt.cpp:
            // 737-845): one wave decodes the blocks in order, each against the
            // 64 KiB before it (zeros before the frame's first byte)
            // (parallel rounds, k_dlink_*; LZ4MT_AMD_BD_SERIAL=1: the one-wave kernel)
            thread_local DevBuf slotBuf, histBuf;
            const bool serial = bd_serial();
            const uint64_t scratch = serial ? 65536 + (uint64_t)bm + 64 : dlink_scratch_bytes(nb, bm);
            if (!slotBuf.ensure(scratch) || !histBuf.ensure(65536)) { result = LZ4MT_RESULT_ERROR; break; }
            HIPCHK(hipMemsetAsync(histBuf.p, 0, 65536, st));
            if (bck && nb) HIPCHK(launch_xxh32_frame_blocks(f, B.recs, (uint32_t)nb, B.digest, st));
            const uint64_t room = outCap > opos ? outCap - opos : 0;
            g_timing.mark(1, st);
            if (serial)
                HIPCHK(launch_decode_linked(f, B.recs, (uint32_t)nb, bm, out + opos, room, slotBuf.p, histBuf.p,
                                            B.digest, bck, B.dsize, B.status, st));
            else
                HIPCHK(launch_decode_linked_par(f, B.recs, (uint32_t)nb, bm, out + opos, room, histBuf.p, B.digest,
                                                bck, B.dsize, B.status, slotBuf.p, env_rounds(), st));
            g_timing.mark(2, st);
            g_timing.mark(3, st);
            int32_t stat[2] = {0, 0};
            std::vector<int32_t> ds(nb);
            HIPCHK(hipMemcpyAsync(stat, B.status, 8, hipMemcpyDeviceToHost, st));
            if (nb) HIPCHK(hipMemcpyAsync(ds.data(), B.dsize, nb * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            for (int32_t i = 0; i < stat[0] && (uint64_t)i < nb; ++i) produced += (uint64_t)ds[i];
            if (stat[1] == 16) result = LZ4MT_RESULT_BLOCK_CHECKSUM_MISMATCH;   // checked before writing
            else if (stat[1] == 18) result = LZ4MT_RESULT_DECOMPRESS_FAIL;
            else if (stat[1] != 0) result = LZ4MT_RESULT_ERROR;
            else if (wi.result != 0) result = (Lz4MtResult)wi.result;
        } else {
        // decode target: in place when 16-B aligned, else a staging buffer
        const bool aligned = ((reinterpret_cast<uintptr_t>(out) + opos) & 15) == 0;
        const uint64_t room = outCap > opos ? outCap - opos : 0;
        uint8_t* target = out + opos;
        uint64_t targetCap = room;
        // The block checksums run on a side stream beside the decode: the
        // checksum kernel uses no LDS (16 blocks per wave), so its waves do
        // not take a slot from the decode's eight 20 KiB waves per CU.
        bool side = false, fused = false;
        if (aligned && fused_walk(bm, frameSize - bodyPos) && B.ensure_ctl()) {   // walk inside the decode (k_decode_walk)
            g_timing.mark(1, st);
            fused = decode_walk_fused(f, frameSize, bodyPos, bm, bck, target, targetCap, B, aux, wi, result, st);
            if (fused && result != LZ4MT_RESULT_OK) break;
            if (fused) {
                g_timing.mark(2, st);
                g_timing.mark(3, st);
            }
        }
        if (!fused) {
            result = walk_frame(f, frameSize, bodyPos, bm, bck, B, wi, st);
            if (result != LZ4MT_RESULT_OK) break;
        }
        const uint64_t nb = wi.nBlocks;
        if (!fused) {
            if (!aligned) {
                if (!tmp.ensure(nb * bm)) { result = LZ4MT_RESULT_ERROR; break; }
                target = tmp.p;
                targetCap = std::min<uint64_t>(room, nb * bm);
            }
            side = bck && nb && aux.ensure();
            if (side) {
                HIPCHK(hipEventRecord(aux.evIn, st));
                HIPCHK(hipStreamWaitEvent(aux.st, aux.evIn, 0));
                HIPCHK(launch_xxh32_frame_blocks(f, B.recs, (uint32_t)nb, B.digest, aux.st));
                HIPCHK(hipEventRecord(aux.evOut, aux.st));
            }
            g_timing.mark(1, st);
            HIPCHK(launch_decode(f, B.recs, (uint32_t)nb, bm, target, targetCap, B.dsize, st));
            g_timing.mark(2, st);
            if (side) HIPCHK(hipStreamWaitEvent(st, aux.evOut, 0));
            else if (bck) HIPCHK(launch_xxh32_frame_blocks(f, B.recs, (uint32_t)nb, B.digest, st));
        }
        if (!fused) {
            HIPCHK(launch_block_verify(B.recs, (uint32_t)nb, B.digest, B.dsize, bm, bck, B.status, st));
            g_timing.mark(3, st);
        }
        std::vector<int32_t> ds(nb), stv(nb);
        if (nb) {
            HIPCHK(hipMemcpyAsync(ds.data(), B.dsize, nb * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(stv.data(), B.status, nb * 4, hipMemcpyDeviceToHost, st));
        }
        HIPCHK(hipStreamSynchronize(st));
        // first failing block wins, then the walk's own error (block order)
        uint64_t good = nb;
        for (uint64_t i = 0; i < nb; ++i)
            if (stv[i] != 0) { good = i; result = (Lz4MtResult)stv[i]; break; }
        if (good == nb && wi.result != 0) result = (Lz4MtResult)wi.result;
        // gather decoded bytes of blocks [0, good) contiguously at out + opos
        bool contiguous = aligned;
        for (uint64_t i = 0; i < good; ++i) {
            if (i + 1 < good && (uint64_t)ds[i] != bm) contiguous = false;
            produced += (uint64_t)ds[i];
        }
        if (produced > room) { result = LZ4MT_RESULT_ERROR; break; }
        if (!contiguous) {
            // compaction: copy slots through staging in block order
            uint8_t* srcBase = target;
            if (aligned) {  // slots live in the output itself: stage them first
                if (!tmp.ensure(good * (uint64_t)bm)) { result = LZ4MT_RESULT_ERROR; break; }
                HIPCHK(hipMemcpyAsync(tmp.p, target, std::min<uint64_t>(good * (uint64_t)bm, targetCap), hipMemcpyDeviceToDevice, st));
                srcBase = tmp.p;
            }
            uint64_t w = 0;
            for (uint64_t i = 0; i < good; ++i) {
                if (ds[i] > 0)
                    HIPCHK(hipMemcpyAsync(out + opos + w, srcBase + i * bm, (size_t)ds[i], hipMemcpyDeviceToDevice, st));
                w += (uint64_t)ds[i];
            }
        }
        }   // independent blocks
        if (result != LZ4MT_RESULT_OK) { opos += produced; break; }
        uint64_t next = wi.endPos;
        if (sck) {
            if (next + 4 > frameSize) { opos += produced; result = LZ4MT_RESULT_CANNOT_READ_STREAM_CHECKSUM; break; }
            uint8_t want[4];
            HIPCHK(hipMemcpyAsync(want, f + next, 4, hipMemcpyDeviceToHost, st));
            // the serial content checksum on the host (HostHasher)
            thread_local hipEvent_t outReady = nullptr;
            if (!outReady) HIPCHK(hipEventCreateWithFlags(&outReady, hipEventDisableTiming));
            HIPCHK(hipEventRecord(outReady, st));
            uint32_t got = 0;
            if (!g_hasher.hash(out + opos, produced, outReady, &got)) { result = LZ4MT_RESULT_ERROR; break; }
            HIPCHK(hipStreamSynchronize(st));
            next += 4;
            if (got != get32(want)) { opos += produced; result = LZ4MT_RESULT_STREAM_CHECKSUM_MISMATCH; break; }
        }
        g_timing.mark(4, st);
        opos += produced;
        pos = next;
    }
    hipStreamSynchronize(st);
    if (outSize) *outSize = opos;
    return result;
}

// ===========================================================================
// 3. utilities
// ===========================================================================
extern "C" int lz4mtHipGenSynthetic(void* d_dst, uint64_t n, uint64_t seed, void* stream) {
    if (!have_device()) return -1;
    return launch_gen_synthetic(static_cast<uint8_t*>(d_dst), n, seed, static_cast<hipStream_t>(stream)) == hipSuccess
               ? 0 : -1;
}

extern "C" uint32_t lz4mtHipXxh32(const void* d_src, uint64_t len, void* stream) {
    if (!have_device()) return 0;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    uint32_t* d = reinterpret_cast<uint32_t*>(small_dev());
    uint32_t h = 0;
    if (!d) return 0;
    if (launch_xxh32_stream(static_cast<const uint8_t*>(d_src), len, d, st) == hipSuccess &&
        hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, st) == hipSuccess)
        hipStreamSynchronize(st);
    return h;
}

extern "C" int lz4mtHipXxh32Chunks(const void* d_src, uint64_t len, uint32_t chunkBytes, uint32_t* d_digests,
                                   void* stream) {
    if (!have_device() || chunkBytes == 0 || (len && (!d_src || !d_digests))) return -1;
    return launch_xxh32_chunks(static_cast<const uint8_t*>(d_src), len, chunkBytes, d_digests,
                               static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -1;
}

namespace lz4mt {
void release_slot_cache();
}

extern "C" void lz4mtHipReleaseCaches(void) {
    release_slot_cache();
    decode_cache().release();
    scratch_pool().clear();
}

extern "C" int lz4mtHipDeviceCount(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" void lz4mtHipSetTiming(int enable) {
    g_timing.enabled = enable != 0;
    g_timing.valid = false;
}

extern "C" int lz4mtHipGetTimings(float* ms4) {
    if (!g_timing.valid || !ms4) return -1;
    for (int i = 0; i < 5; ++i)
        if (!g_timing.ev[i]) return -1;
    if (hipEventSynchronize(g_timing.ev[4]) != hipSuccess) return -1;
    float a = 0, b = 0, c = 0, d = 0;
    hipEventElapsedTime(&a, g_timing.ev[0], g_timing.ev[1]);
    hipEventElapsedTime(&b, g_timing.ev[1], g_timing.ev[2]);
    hipEventElapsedTime(&c, g_timing.ev[2], g_timing.ev[3]);
    hipEventElapsedTime(&d, g_timing.ev[0], g_timing.ev[4]);
    ms4[0] = a; ms4[1] = b; ms4[2] = c; ms4[3] = d;
    return 0;
}

// ===========================================================================
// 4. diagnostics: phase cycle counts of the encode / decode kernels
// ===========================================================================
// The frame path's block encoder (launch_encode: the kernel LZ4MT_AMD_ENC /
// the block size select) over n bytes in blocks of ANY size 65 547 B .. 4 MiB
// -- also sizes no frame uses (512 KiB, 2 MiB): what one stream of a split
// parse costs per byte at full occupancy (tools/occ_sweep.py).  d_slots:
// nb x blockSize + 64 bytes, d_csize: nb int32.  Asynchronous; timing only.
extern "C" int lz4mtHipDebugEncode(const void* d_src, uint64_t n, uint32_t blockSize, void* d_slots, void* d_csize,
                                   void* stream) {
    if (!have_device() || blockSize < 65547u || blockSize > (4u << 20) || !d_src || !d_slots || !d_csize) return -1;
    const uint64_t nb = (n + blockSize - 1) / blockSize;
    return launch_encode(static_cast<const uint8_t*>(d_src), n, blockSize, (uint32_t)nb, static_cast<uint8_t*>(d_slots),
                         blockSize, 0xFFFFFFFFu, static_cast<int32_t*>(d_csize), static_cast<hipStream_t>(stream)) ==
                   hipSuccess ? 0 : -1;
}

// The parse work of a split parse of n bytes into streams of S bytes, each
// parsed from ov bytes before its start (k_encode_overlap): d_slots nb x
// (S + ov) + 64 bytes, d_csize nb int32; p17 selects the 3-byte table.
// Asynchronous; timing only (tools/occ_sweep.py --overlap).
extern "C" int lz4mtHipDebugEncodeOverlap(const void* d_src, uint64_t n, uint32_t S, uint32_t ov, int p17,
                                          void* d_slots, void* d_csize, void* stream) {
    if (!have_device() || S == 0 || (uint64_t)S + ov > (4u << 20) || !d_src || !d_slots || !d_csize) return -1;
    return launch_encode_overlap(static_cast<const uint8_t*>(d_src), n, S, ov, p17 != 0, static_cast<uint8_t*>(d_slots),
                                 static_cast<int32_t*>(d_csize), static_cast<hipStream_t>(stream)) == hipSuccess
               ? 0 : -1;
}

namespace {
// k_encode_stats over [d_src, d_src + n); per-block counters (16 words per
// block) into perBlock when given, their sums into stats16 when given
int encode_stats(const void* d_src, uint64_t n, uint32_t blockSize, uint64_t* stats16, uint64_t* perBlock,
                 void* stream) {
    if (!have_device() || blockSize == 0) return -1;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t nb = (n + blockSize - 1) / blockSize;
    uint8_t* slots = nullptr;
    int32_t* cs = nullptr;
    uint64_t* dst = nullptr;
    int rc = -1;
    if (hipMalloc(reinterpret_cast<void**>(&slots), nb * blockSize + 64) == hipSuccess &&
        hipMalloc(reinterpret_cast<void**>(&cs), nb * 4 + 4) == hipSuccess &&
        hipMalloc(reinterpret_cast<void**>(&dst), nb * 128 + 64) == hipSuccess &&
        launch_encode_stats(static_cast<const uint8_t*>(d_src), n, blockSize, (uint32_t)nb, slots, cs, dst, st) ==
            hipSuccess) {
        std::vector<uint64_t> h(nb * 16);
        if (hipMemcpyAsync(h.data(), dst, nb * 128, hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipStreamSynchronize(st) == hipSuccess) {
            if (stats16) {
                for (int i = 0; i < 16; ++i) stats16[i] = 0;
                for (uint64_t b = 0; b < nb; ++b)
                    for (int i = 0; i < 16; ++i) stats16[i] += h[b * 16 + i];
            }
            if (perBlock) std::copy(h.begin(), h.end(), perBlock);
            rc = 0;
        }
    }
    hipFree(slots); hipFree(cs); hipFree(dst);
    return rc;
}
}  // namespace

extern "C" int lz4mtHipDebugEncodeStats(const void* d_src, uint64_t n, uint32_t blockSize, uint64_t* stats16,
                                        void* stream) {
    return encode_stats(d_src, n, blockSize, stats16, nullptr, stream);
}

extern "C" int lz4mtHipDebugEncodeBlockStats(const void* d_src, uint64_t n, uint32_t blockSize, uint64_t* perBlock16,
                                             void* stream) {
    return perBlock16 ? encode_stats(d_src, n, blockSize, nullptr, perBlock16, stream) : -1;
}

extern "C" int lz4mtHipDebugDecodeStats(const void* d_frame, uint64_t frameSize, uint64_t* stats16, void* stream) {
    if (!have_device()) return -1;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const uint8_t* f = static_cast<const uint8_t*>(d_frame);
    uint8_t h[kMaxHeader + 8] = {0};
    const uint64_t avail = std::min<uint64_t>(sizeof(h), frameSize);
    if (hipMemcpyAsync(h, f, avail, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return -1;
    Lz4MtStreamDescriptor sd;
    int hb = 0;
    if (get32(h) != kMagic || parse_header(h + 4, avail - 4, &sd, &hb) != LZ4MT_RESULT_OK) return -1;
    const uint32_t bm = (uint32_t)block_max_bytes(sd.bd.blockMaximumSize);
    DecodeBuffers B;
    WalkInfo wi{};
    if (walk_frame(f, frameSize, 4 + hb, bm, sd.flg.blockChecksum, B, wi, st) != LZ4MT_RESULT_OK) return -1;
    uint8_t* out = nullptr;
    uint64_t* dst = nullptr;
    int rc = -1;
    const uint64_t nb = wi.nBlocks;
    if (hipMalloc(reinterpret_cast<void**>(&out), nb * bm + 64) == hipSuccess &&
        hipMalloc(reinterpret_cast<void**>(&dst), nb * 128 + 64) == hipSuccess &&
        launch_decode_stats(f, B.recs, (uint32_t)nb, bm, out, nb * bm, B.dsize, dst, st) == hipSuccess) {
        std::vector<uint64_t> hs(nb * 16);
        if (hipMemcpyAsync(hs.data(), dst, nb * 128, hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipStreamSynchronize(st) == hipSuccess) {
            for (int i = 0; i < 16; ++i) stats16[i] = 0;
            for (uint64_t b = 0; b < nb; ++b)
                for (int i = 0; i < 16; ++i) stats16[i] += hs[b * 16 + i];
            rc = 0;
        }
    }
    hipFree(out); hipFree(dst);
    return rc;
}
