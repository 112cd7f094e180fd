// lz4mt_frame.cpp — the drop-in lz4mt.h API over callbacks.
//
// lz4mtCompress / lz4mtDecompress keep the reference's contract
// (src/lz4mt.cpp:851-1011): header via makeHeader, blocks in order, EOS,
// optional content checksum; first error wins; read/readEof/readSeek/
// readSkippable only on the calling thread; write strictly in block order;
// the codec callbacks may run concurrently.  Two schedulers sit behind it:
//
//   PARALLEL / SEQUENTIAL  — host pipeline calling ctx->compress /
//       ctx->decompress per block (a bounded ring of nPool = workers + 1
//       blocks, worker threads, one in-order writer thread that also owns the
//       serial content checksum).  Null codec callbacks default to the GPU
//       block operators of lz4mt_hip.h.
//   DEVICE (extension bit) — batched MI355X engine: blocks are read into a
//       pinned batch, copied to HBM, encoded/decoded by one kernel launch per
//       batch (wave per block), and written back in order; the serial
//       content checksum runs on the host while the GPU works.
//
// Deliberate fixes vs the reference (documented in DESIGN.md): non-magic
// bytes after a frame end the stream with OK (the reference loops forever,
// src/lz4mt.cpp:971-979); skippable frames are skipped by reading when
// readSkippable is null (the CLI leaves it null and segfaults,
// src/main.cpp:767-775); the futures vector race (src/lz4mt.cpp:408,448) has
// no counterpart.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/lz4mt.h"
#include "../../include/lz4mt_hip.h"
#include "lz4mt_device.h"
#include "lz4mt_host.h"

namespace lz4mt {
Lz4MtResult device_compress_body(const uint8_t* src, uint64_t n, uint32_t bm, int blockChecksum, uint8_t* ws,
                                 uint8_t* body, uint32_t hdrLen, hipStream_t st, uint64_t** d_recOffOut,
                                 const AuxStream* aux, const LinkState* link, int level);
uint64_t compress_ws_bytes(uint64_t n, uint32_t bm, int level, int bd = 0);
}  // namespace lz4mt

using namespace lz4mt;

namespace {

// ---------------------------------------------------------------------------
// Context wrapper: first-error-wins result (reference Ctx, src/lz4mt.cpp:163-271)
// ---------------------------------------------------------------------------
class Session {
public:
    explicit Session(Lz4MtContext* c) : c_(c) {}

    Lz4MtResult set(Lz4MtResult r) {
        std::lock_guard<std::mutex> g(mu_);
        if (c_->result == LZ4MT_RESULT_OK || c_->result == LZ4MT_RESULT_ERROR) c_->result = r;
        return c_->result;
    }
    Lz4MtResult result() {
        std::lock_guard<std::mutex> g(mu_);
        return c_->result;
    }
    bool error() { return result() != LZ4MT_RESULT_OK; }
    Lz4MtResult quit(Lz4MtResult r) {
        set(r);
        quit_ = true;
        return r;
    }
    bool quitting() const { return quit_.load(); }

    int read(void* d, int n) {
        if (!c_->read) return 0;
        const int r = c_->read(c_, d, n);
        if (r < n) eofHint_ = true;
        return r < 0 ? 0 : (r > n ? n : r);   // (a callback claiming more than it was given n bytes for)
    }
    bool readEof() { return c_->readEof ? c_->readEof(c_) != 0 : eofHint_; }
    // readU32: a short read sets ERROR (reference Ctx::readU32)
    bool readU32(uint32_t* v) {
        if (error()) return false;
        if (!peekU32(v)) { set(LZ4MT_RESULT_ERROR); return false; }
        return true;
    }
    // the same read without touching the result: the DEVICE engine records
    // the code and applies it after the blocks already batched are written
    bool peekU32(uint32_t* v) {
        uint8_t b[4];
        if (read(b, 4) != 4) return false;
        *v = get32(b);
        return true;
    }
    bool write(const void* p, int n) {  // reference Ctx::writeBin
        if (error()) return false;
        if (!c_->write || c_->write(c_, p, n) != n) { set(LZ4MT_RESULT_ERROR); return false; }
        return true;
    }
    bool writeU32(uint32_t v) {
        uint8_t b[4];
        put32(b, v);
        return write(b, 4);
    }
    bool skip(uint32_t magic, uint32_t size) {
        if (c_->readSkippable) return c_->readSkippable(c_, magic, size) >= 0;
        std::vector<uint8_t> sink(std::min<uint32_t>(size, 1u << 20));
        uint32_t left = size;
        while (left) {
            const int take = (int)std::min<uint32_t>(left, (uint32_t)sink.size());
            const int got = read(sink.data(), take);
            if (got <= 0) break;  // like fseek past EOF: not an error
            left -= (uint32_t)got;
        }
        return true;
    }
    int compress(const char* s, char* d, int n, int cap) {
        Lz4MtCompress fn = c_->compress ? c_->compress : lz4mtHipCompressBlock;
        return fn(s, d, n, cap, c_->compressionLevel);
    }
    int decompress(const char* s, char* d, int n, int cap) {
        Lz4MtDecompress fn = c_->decompress ? c_->decompress : lz4mtHipDecompressBlock;
        return fn(s, d, n, cap);
    }
    Lz4MtMode mode() const { return c_->mode; }
    int level() const { return c_->compressionLevel; }
    void clearEofHint() { eofHint_ = false; }

private:
    Lz4MtContext* c_;
    std::mutex mu_;
    std::atomic<bool> quit_{false};
    bool eofHint_ = false;
};

unsigned worker_count(const Session& s) {
    if (s.mode() & LZ4MT_MODE_SEQUENTIAL) return 0;
    const unsigned hw = std::thread::hardware_concurrency();
    return hw ? hw : 1;
}

// ---------------------------------------------------------------------------
// A small ordered pipeline: jobs are produced in order by the caller thread,
// processed by W workers, and consumed strictly in order by one writer.
// With W == 0 everything runs inline on the caller thread (SEQUENTIAL).
// ---------------------------------------------------------------------------
struct Job {
    std::vector<char> in, out;
    int n = 0;          // input bytes
    int res = 0;        // codec result
    bool raw = false;
    uint32_t ck = 0;    // block checksum (compress: computed; decompress: expected)
    bool ckbad = false; // decompress: stored checksum mismatched
    bool skip = false;  // an earlier error: nothing to do
    bool ready = false;
};

class Pipeline {
public:
    Pipeline(unsigned workers, unsigned slots, std::function<void(Job&)> work, std::function<void(Job&)> emit)
        : work_(std::move(work)), emit_(std::move(emit)), jobs_(slots) {
        for (unsigned i = 0; i < workers; ++i) threads_.emplace_back([this] { worker(); });
        if (workers) writer_ = std::thread([this] { writer(); });
        inline_ = workers == 0;
    }
    ~Pipeline() { finish(); }

    // Returns the next free job slot (blocks while the ring is full).
    Job& acquire() {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return produced_ - written_ < jobs_.size(); });
        Job& j = jobs_[produced_ % jobs_.size()];
        j.ready = false;
        return j;
    }
    void submit() {
        if (inline_) {
            Job& j = jobs_[produced_ % jobs_.size()];
            ++produced_;
            work_(j);
            emit_(j);
            ++written_;
            return;
        }
        std::lock_guard<std::mutex> g(mu_);
        queue_.push_back(produced_++);
        cv_.notify_all();
    }
    // Waits until every submitted job has been written.
    void drain() {
        if (inline_) return;
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return written_ == produced_; });
    }
    void finish() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
            cv_.notify_all();
        }
        for (auto& t : threads_) t.join();
        threads_.clear();
        if (writer_.joinable()) writer_.join();
    }

private:
    void worker() {
        for (;;) {
            uint64_t id;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || !queue_.empty(); });
                if (queue_.empty()) return;
                id = queue_.front();
                queue_.pop_front();
            }
            Job& j = jobs_[id % jobs_.size()];
            work_(j);
            std::lock_guard<std::mutex> g(mu_);
            j.ready = true;
            cv_.notify_all();
        }
    }
    void writer() {
        for (;;) {
            Job* j;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return (written_ < produced_ && jobs_[written_ % jobs_.size()].ready) ||
                                         (stop_ && written_ == produced_); });
                if (written_ == produced_) return;
                j = &jobs_[written_ % jobs_.size()];
            }
            emit_(*j);
            std::lock_guard<std::mutex> g(mu_);
            ++written_;
            cv_.notify_all();
        }
    }

    std::function<void(Job&)> work_, emit_;
    std::vector<Job> jobs_;
    std::vector<std::thread> threads_;
    std::thread writer_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<uint64_t> queue_;
    uint64_t produced_ = 0, written_ = 0;
    bool stop_ = false, inline_ = false;
};

// ---------------------------------------------------------------------------
// compress: host scheduler (reference compress(), src/lz4mt.cpp:372-457)
// ---------------------------------------------------------------------------
void compress_host(Session& s, const Lz4MtStreamDescriptor* sd, HostXxh32& xs) {
    const int bm = block_max_bytes(sd->bd.blockMaximumSize);
    const bool bck = sd->flg.blockChecksum, sck = sd->flg.streamChecksum;
    const unsigned W = worker_count(s);
    auto work = [&](Job& j) {
        j.skip = s.error() || s.quitting();
        if (j.skip) return;
        j.out.resize((size_t)bm + 64);
        j.res = s.compress(j.in.data(), j.out.data(), j.n, j.n);  // cap = srcSize (src/lz4mt.cpp:391)
        j.raw = j.res <= 0;
        if (bck) j.ck = j.raw ? HostXxh32::oneshot(j.in.data(), (size_t)j.n) : HostXxh32::oneshot(j.out.data(), (size_t)j.res);
    };
    auto emit = [&](Job& j) {
        if (j.skip || s.error() || s.quitting()) return;
        if (sck) xs.update(j.in.data(), (size_t)j.n);
        if (j.raw) {
            s.writeU32((uint32_t)j.n | kRawBit);
            s.write(j.in.data(), j.n);
        } else {
            s.writeU32((uint32_t)j.res);
            s.write(j.out.data(), j.res);
        }
        if (bck) s.writeU32(j.ck);
    };
    Pipeline pipe(W, W + 1, work, emit);
    for (;;) {
        if (s.error() || s.quitting()) break;
        Job& j = pipe.acquire();
        j.in.resize((size_t)bm);
        j.n = s.read(j.in.data(), bm);
        if (j.n <= 0) break;
        pipe.submit();
    }
    pipe.drain();
}

// ---------------------------------------------------------------------------
// DEVICE engine: batch slots.  Each slot owns pinned host staging, device
// buffers and its own stream; several slots are in flight at once, so the
// host's read() of batch i+1, the H2D/kernels/D2H of batches i-k..i and the
// in-order write() of batch i-k-1 overlap, and the GPU sees several batches'
// blocks at once (one wavefront per block needs many blocks to fill the
// chip).  Slots are cached per thread across calls (pinning is expensive),
// sized by the largest batch seen; they are reused in FIFO order, which is
// the block order the writes must keep.
// ---------------------------------------------------------------------------
constexpr int kSlots = 8;   // slots allocated (at most); slot_count() are used
// LZ4MT_AMD_SLOTS / LZ4MT_AMD_BATCH_MIB override the defaults (tuning runs)
int env_int(const char* name, int dflt, int lo, int hi) {
    const char* e = getenv(name);
    const int v = e ? atoi(e) : dflt;
    return v < lo ? lo : (v > hi ? hi : v);
}
// Pipeline shape per direction.  An encode batch of any size takes about one
// block latency (~150-190 ms for 4 MiB blocks), so compress
// needs GiBs in flight to approach the kernel rate: 4 slots of up to 4 GiB.
// Decode latency is ~6x shorter: 8 slots of up to 1 GiB.  Batches start at
// 256 MiB and double per fill, so small inputs stage little.
struct PipeShape {
    int slots;
    uint64_t maxBatch;   // bytes of uncompressed data per batch
};
PipeShape pipe_shape(bool compress) {
    const int dS = compress ? 4 : 8, dM = compress ? 4096 : 1024;
    return PipeShape{env_int("LZ4MT_AMD_SLOTS", dS, 1, kSlots),
                     (uint64_t)env_int("LZ4MT_AMD_BATCH_MIB", dM, 1, 16384) << 20};
}
// blocks of batch number `i` (0, 1, ...): first << i, capped, >= 1 block
// (first = 256 MiB, LZ4MT_AMD_BATCH0_MIB overrides)
uint64_t batch_blocks(const PipeShape& P, uint32_t bm, uint64_t i) {
    const uint64_t first = (uint64_t)env_int("LZ4MT_AMD_BATCH0_MIB", 256, 1, 16384) << 20;
    const uint64_t want = std::min<uint64_t>(P.maxBatch, first << std::min<uint64_t>(i, 16));
    return std::max<uint64_t>(1, want / bm);
}

struct Slot {
    hipStream_t st = nullptr;
    // one pinned host buffer per slot: hOut aliases hIn (a batch's H2D is
    // stream-ordered before its D2H, and the host is done with its input
    // before the D2H is issued)
    uint8_t *hIn = nullptr, *hOut = nullptr, *dIn = nullptr, *dOut = nullptr, *dWs = nullptr;
    uint64_t hCap = 0, inCap = 0, outCap = 0, wsCap = 0;
    // per-batch metadata, pinned so it can travel asynchronously
    uint64_t* hMeta = nullptr;                // [0] = compressed body size
    BlockRec* hRecs = nullptr;                // decompress: block records
    int32_t *hDs = nullptr, *hSt = nullptr;   // decompress: decoded sizes, verify status
    BlockRec* dRecs = nullptr;
    int32_t *dDs = nullptr, *dSt = nullptr;
    uint32_t* dDig = nullptr;
    uint64_t metaCap = 0;                     // blocks the metadata arrays hold
    // the batch in flight
    bool busy = false;
    uint64_t total = 0, nb = 0;

    void release() {
        if (st) hipStreamSynchronize(st);
        hipHostFree(hIn); hipHostFree(hMeta); hipHostFree(hRecs); hipHostFree(hDs);
        hipHostFree(hSt);
        hipFree(dIn); hipFree(dOut); hipFree(dWs); hipFree(dRecs); hipFree(dDs); hipFree(dSt); hipFree(dDig);
        if (st) hipStreamDestroy(st);
        *this = Slot();
    }
    // grows the buffers (contents are not kept); 0 sizes leave a buffer alone
    bool ensure(uint64_t in, uint64_t out, uint64_t ws, uint64_t blocks) {
        if (!st && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return false;
        const uint64_t h = std::max(in, out);
        if (h > hCap) {
            hipHostFree(hIn);
            hIn = hOut = nullptr; hCap = 0;
            if (hipHostMalloc(reinterpret_cast<void**>(&hIn), h + 64, 0) != hipSuccess) return false;
            hOut = hIn;
            hCap = h;
        }
        if (in > inCap) {
            hipFree(dIn);
            dIn = nullptr; inCap = 0;
            if (hipMalloc(reinterpret_cast<void**>(&dIn), in + 64) != hipSuccess) return false;
            inCap = in;
        }
        if (out > outCap) {
            hipFree(dOut);
            dOut = nullptr; outCap = 0;
            if (hipMalloc(reinterpret_cast<void**>(&dOut), out + 64) != hipSuccess) return false;
            outCap = out;
        }
        if (ws > wsCap) {
            hipFree(dWs);
            dWs = nullptr; wsCap = 0;
            if (hipMalloc(reinterpret_cast<void**>(&dWs), ws + 64) != hipSuccess) return false;
            wsCap = ws;
        }
        if (blocks > metaCap || !hMeta) {
            hipHostFree(hMeta); hipHostFree(hRecs); hipHostFree(hDs); hipHostFree(hSt);
            hipFree(dRecs); hipFree(dDs); hipFree(dSt); hipFree(dDig);
            hMeta = nullptr; hRecs = nullptr; hDs = nullptr; hSt = nullptr;
            dRecs = nullptr; dDs = nullptr; dSt = nullptr; dDig = nullptr; metaCap = 0;
            const uint64_t k = std::max<uint64_t>(blocks, 2);   // >= 2: the linked decoder's status pair
            if (hipHostMalloc(reinterpret_cast<void**>(&hMeta), 64, 0) != hipSuccess ||
                hipHostMalloc(reinterpret_cast<void**>(&hRecs), k * sizeof(BlockRec), 0) != hipSuccess ||
                hipHostMalloc(reinterpret_cast<void**>(&hDs), k * 4, 0) != hipSuccess ||
                hipHostMalloc(reinterpret_cast<void**>(&hSt), k * 4, 0) != hipSuccess ||
                hipMalloc(reinterpret_cast<void**>(&dRecs), k * sizeof(BlockRec)) != hipSuccess ||
                hipMalloc(reinterpret_cast<void**>(&dDs), k * 4) != hipSuccess ||
                hipMalloc(reinterpret_cast<void**>(&dSt), k * 4) != hipSuccess ||
                hipMalloc(reinterpret_cast<void**>(&dDig), k * 4) != hipSuccess)
                return false;
            metaCap = k;
        }
        return true;
    }
};

struct SlotCache {
    Slot slot[kSlots];
    ~SlotCache() {
        for (Slot& s : slot) s.release();
    }
    void release() {
        for (Slot& s : slot) s.release();
    }
    // a call that ends early (error) may leave batches in flight: drain them
    void quiesce() {
        for (Slot& s : slot) {
            if (s.st) hipStreamSynchronize(s.st);
            s.busy = false;
        }
    }
};
thread_local SlotCache g_slots;

// The slot pipeline: the calling thread fills and launches batches (all
// read() calls stay on it, as the reference requires); one writer thread
// completes them in FIFO order (D2H, in-order write(); the reference also
// writes from a worker thread).  fill(S) returns false when there is no
// more input (S not launched) and sets *stop to end after a launched batch;
// finish(S) returns false to stop the frame (later batches are drained
// without writes).
// LZ4MT_AMD_PIPE_TRACE=1: one stderr line per batch (ms since the call
// began: fill start / launched, finish start / done) -- the e2e timeline
bool pipe_trace() {
    static const bool on = getenv("LZ4MT_AMD_PIPE_TRACE") && atoi(getenv("LZ4MT_AMD_PIPE_TRACE")) != 0;
    return on;
}
double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

template <class Fill, class Finish>
void run_slot_pipeline(Session& s, int nSlots, Fill fill, Finish finish) {
    const auto t0 = std::chrono::steady_clock::now();
    const bool tr = pipe_trace();
    std::vector<double> tFill0(kSlots), tFill1(kSlots);
    int seqNo = 0;
    std::vector<int> slotSeq(kSlots);
    SlotCache& C = g_slots;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<int> q;
    bool done = false, failed = false;
    std::thread writer([&] {
        for (;;) {
            int i;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !q.empty() || done; });
                if (q.empty()) return;
                i = q.front();
                q.pop_front();
            }
            Slot& S = C.slot[i];
            bool okS;
            {
                bool f;
                { std::lock_guard<std::mutex> g(mu); f = failed; }
                const double a = tr ? ms_since(t0) : 0;
                if (f) { hipStreamSynchronize(S.st); okS = false; }
                else okS = finish(S);
                if (tr)
                    fprintf(stderr, "pipe batch %d blocks %llu: fill %.1f-%.1f ms, finish %.1f-%.1f ms\n", slotSeq[i],
                            (unsigned long long)S.nb, tFill0[i], tFill1[i], a, ms_since(t0));
            }
            {
                std::lock_guard<std::mutex> g(mu);
                if (!okS) failed = true;
                S.busy = false;
            }
            cv.notify_all();
        }
    });
    int head = 0;
    for (;;) {
        Slot& S = C.slot[head];
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return !S.busy || failed; });
            if (failed) break;
        }
        if (s.error()) break;
        bool stop = false;
        if (tr) tFill0[head] = ms_since(t0);
        if (!fill(S, &stop)) break;
        if (tr) { tFill1[head] = ms_since(t0); slotSeq[head] = seqNo++; }
        {
            std::lock_guard<std::mutex> g(mu);
            S.busy = true;
            q.push_back(head);
        }
        cv.notify_all();
        head = (head + 1) % nSlots;
        if (stop) break;
    }
    {
        std::lock_guard<std::mutex> g(mu);
        done = true;
    }
    cv.notify_all();
    writer.join();
    C.quiesce();
    // The pinned staging (up to slots x batch bytes) stays cached per thread
    // only for callers that opted into LZ4MT_MODE_DEVICE (repeated calls pay
    // no re-pinning; lz4mtHipReleaseCaches() frees it).  A relinked default
    // PARALLEL caller gets it freed at the end of every call.
    if (!(s.mode() & LZ4MT_MODE_DEVICE)) C.release();
}

// Blocks per batch: ~512 MiB of input (at least one block); kSlots batches
// in flight keep up to 3 GiB of blocks on the GPU at once.


// device buffer owned by one call (freed on return; hipFree waits for the device)
struct CallBuf {
    void* p = nullptr;
    ~CallBuf() { if (p) hipFree(p); }
    bool alloc(size_t n) { return hipMalloc(&p, n) == hipSuccess; }
};

// ---------------------------------------------------------------------------
// Streamed DEVICE compress (independent 1 / 4 MiB blocks, levels 0..2):
// k_encode_stream (lz4mt_kernels.hip) is launched once, before the first
// read(); the calling thread reads block after block into a ring of
// coherent pinned staging slots and publishes each one; the persistent grid
// encodes each block as soon as it is published and pushes its record's
// payload into a ring of coherent pinned output slots; a writer thread
// writes the records in block order as they appear.  So encoding overlaps
// the reads (no batch waits for its last block, no batch-sized copy after
// the last read) and the writes overlap the encodes.
// LZ4MT_AMD_STREAM=0 keeps the batch pipeline below.
// ---------------------------------------------------------------------------
bool stream_enabled() {
    const char* e = getenv("LZ4MT_AMD_STREAM");
    return !e || atoi(e) != 0;
}

struct StreamBufs {
    uint8_t *hIn = nullptr, *hOut = nullptr, *dIn = nullptr, *dSlot = nullptr;
    uint32_t* hCtl = nullptr;       // g[8] | in[4 Rin] | out[4 Rout]  (coherent pinned)
    uint32_t* dNext = nullptr;      // the grid's block counter
    uint32_t* dPend = nullptr;      // per wave: a block parked on its output slot {b + 1, word, sum, 0}
    uint32_t bm = 0, waves = 0, Rin = 0, Rout = 0;
    hipStream_t st = nullptr;
    int dev = -1;
    // (DEVICE-mode calls keep the rings per thread; a thread's exit frees them)
    ~StreamBufs() { release(); }
    void release() {
        if (st) hipStreamSynchronize(st);
        hipHostFree(hIn); hipHostFree(hOut); hipHostFree(hCtl);
        hipFree(dIn); hipFree(dSlot); hipFree(dNext); hipFree(dPend);
        if (st) hipStreamDestroy(st);
        hIn = hOut = dIn = dSlot = nullptr;
        hCtl = dNext = dPend = nullptr;
        bm = waves = Rin = Rout = 0;
        st = nullptr;
        dev = -1;
    }
    bool ensure(uint32_t bm_, uint32_t waves_, uint32_t rin, uint32_t rout) {
        int d = -1;
        if (hipGetDevice(&d) != hipSuccess) return false;
        if (hIn && bm == bm_ && waves == waves_ && Rin == rin && Rout == rout && dev == d) return true;
        release();
        bm = bm_; waves = waves_; Rin = rin; Rout = rout; dev = d;
        const unsigned hf = hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&hIn), (uint64_t)Rin * bm + 64, hf) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&hOut), (uint64_t)Rout * bm + 64, hf) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&hCtl), 4ull * (8 + 4ull * Rin + 4ull * Rout), hf) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&dIn), (uint64_t)waves * (bm + 64)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&dSlot), (uint64_t)waves * (bm + 64)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&dNext), 64) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&dPend), 16ull * waves) != hipSuccess) {
            (void)hipGetLastError();
            release();
            return false;
        }
        return true;
    }
};
thread_local StreamBufs g_stream;

// Waves of the streamed grids: LZ4MT_AMD_STREAM_WAVES_PER_CU (1..8) per CU.
// Every wave owns two bm-byte HBM buffers (its block's input and output), so
// this sets the engine's HBM footprint: waves x 2 x (bm + 64) per calling
// thread.
uint32_t stream_waves(int cus) {
    return (uint32_t)cus * (uint32_t)env_int("LZ4MT_AMD_STREAM_WAVES_PER_CU", 4, 1, 8);
}

inline uint32_t ld_acq(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void st_rel(uint32_t* p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

// spins briefly, then sleeps in 20 us steps, until pred() or stop()
template <class P, class Q>
bool host_wait(P pred, Q stop) {
    for (int i = 0;; ++i) {
        if (pred()) return true;
        if (stop()) return false;
        if (i < 64) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// A wave of the streamed grids gives up a wait after LZ4MT_AMD_STREAM_TIMEOUT_S
// seconds without progress (so a stuck host never pins the GPU); waiting on the
// user's read() / write() is progress: while any callback runs, the monitor
// thread bumps the liveness word g[5] every 100 ms (a stalled pipe upstream
// or downstream is not a hang).
// Parking: a grid holds the LDS of every CU it runs on for as long as it
// runs.  When one read() or one write() has been blocked for
// LZ4MT_AMD_STREAM_PARK_MS (200 ms by default), the monitor sets the park
// word g[7] and the grid leaves the device: a wave waiting for a block that
// is not published leaves (it re-reads the block's word after seeing the
// park, so a block published before the park is always taken); a wave whose
// block is encoded (decoded) but whose output slot is still taken leaves its
// block in its own HBM buffers with a descriptor in dPend; waves working on
// a block finish it and then do one of the two.  While parked the reader
// publishes nothing (publish() below, under the mutex the park is set
// under), so every block below the reader's next one was taken.  Other work
// on the device -- a callback's own GPU calls included -- can then run.
// Within 10 ms of no callback being stalled any more, the monitor waits for
// the parked grid to drain and launches it again at the reader's next block;
// each wave first finishes the block it parked with.  The callbacks
// themselves only stamp their start and end (atomics): the reader's one
// publish per block is the only lock on the data path.
uint64_t stream_wait_ticks() {
    return (uint64_t)env_int("LZ4MT_AMD_STREAM_TIMEOUT_S", 60, 1, 86400) * 100000000ull;   // 100 MHz
}
class StreamMonitor {
  public:
    template <class Launch>
    StreamMonitor(StreamBufs& B, uint32_t* g, Launch launch)
        : B_(B), g_(g), launch_(launch),
          parkAfter_(std::chrono::milliseconds(env_int("LZ4MT_AMD_STREAM_PARK_MS", 200, 1, 86400000))),
          th_([this] { run(); }) {}
    ~StreamMonitor() { stop(); }
    // no relaunch after this (the call's blocks are all out, or it stops)
    void stop() {
        { std::lock_guard<std::mutex> lk(mu_); stop_ = true; }
        cv_.notify_all();
        if (th_.joinable()) th_.join();
    }
    // one callback in progress for the scope's lifetime (the reader's or the
    // writer's: each is timed for parking)
    class Scope {
      public:
        Scope(StreamMonitor& k, bool reader) : k_(k), since_(reader ? k.readSince_ : k.writeSince_) {
            k_.busy_.fetch_add(1, std::memory_order_relaxed);
            since_.store(now_ns(), std::memory_order_release);
        }
        ~Scope() {
            since_.store(-1, std::memory_order_release);
            k_.busy_.fetch_sub(1, std::memory_order_relaxed);
        }

      private:
        StreamMonitor& k_;
        std::atomic<int64_t>& since_;
    };
    // The reader publishes block b through fn() -- never while the grid is
    // parked (it waits for the relaunch).  false: the call is stopping
    // (abort, GPU error, failed relaunch).
    template <class F, class Stop>
    bool publish(uint32_t b, F fn, Stop stop) {
        for (;;) {
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (!parked_) {
                    fn();
                    nextPub_ = b + 1;
                    return true;
                }
            }
            if (stop() || failed()) return false;
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }
    bool failed() const { return failed_.load(std::memory_order_acquire); }

  private:
    static int64_t now_ns() {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    // which callback has run for at least parkAfter_ (nullptr: none)
    const char* stalled() const {
        const int64_t t = now_ns(), lim = std::chrono::duration_cast<std::chrono::nanoseconds>(parkAfter_).count();
        const int64_t r = readSince_.load(std::memory_order_acquire), w = writeSince_.load(std::memory_order_acquire);
        return (r >= 0 && t - r >= lim) ? "read()" : (w >= 0 && t - w >= lim) ? "write()" : nullptr;
    }
    // (mu_ held: nothing is published meanwhile) waits for the parked grid
    // to drain -- every wave leaves by itself -- and launches it again at the
    // reader's next block
    bool relaunch_locked() {
        if (hipStreamSynchronize(B_.st) != hipSuccess || __atomic_load_n(g_ + 4, __ATOMIC_ACQUIRE) != 0 ||
            __atomic_load_n(g_ + 1, __ATOMIC_ACQUIRE) != 0) {
            (void)hipGetLastError();
            return false;
        }
        __atomic_store_n(g_ + 7, 0u, __ATOMIC_RELEASE);
        parked_ = false;
        if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(B_.dNext), (int)nextPub_, 1, B_.st) != hipSuccess ||
            launch_() != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (const char* t = getenv("LZ4MT_AMD_PIPE_TRACE"); t && atoi(t) != 0)   // (read per event: rare)
            fprintf(stderr, "lz4mt_amd: streamed grid parked while a %s stalled; relaunched at block %u\n",
                    why_, nextPub_);
        return true;
    }
    void run() {
        std::unique_lock<std::mutex> lk(mu_);
        uint32_t beat = 1;
        for (uint32_t tick = 0; !cv_.wait_for(lk, std::chrono::milliseconds(10), [this] { return stop_; }); ++tick) {
            if (tick % 10 == 0 && busy_.load(std::memory_order_relaxed) > 0)
                __atomic_store_n(g_ + 5, beat++, __ATOMIC_RELEASE);
            if (failed()) continue;
            const char* why = stalled();
            if (!parked_ && why) {
                why_ = why;
                __atomic_store_n(g_ + 7, 1u, __ATOMIC_RELEASE);
                parked_ = true;
            } else if (parked_ && !why && !relaunch_locked()) {
                failed_.store(true, std::memory_order_release);
                __atomic_store_n(g_ + 1, 1u, __ATOMIC_RELEASE);   // abort: the grid, the reader and the writer stop
            }
        }
    }
    StreamBufs& B_;
    uint32_t* g_;
    std::function<hipError_t()> launch_;
    std::chrono::steady_clock::duration parkAfter_;
    std::atomic<int> busy_{0};
    std::atomic<int64_t> readSince_{-1}, writeSince_{-1};   // start of the running read() / write(), -1: none
    std::atomic<bool> failed_{false};                        // a relaunch failed
    std::mutex mu_;
    std::condition_variable cv_;
    // (under mu_)
    bool stop_ = false, parked_ = false;
    uint32_t nextPub_ = 0;
    const char* why_ = "read()";
    std::thread th_;   // last: started once the members above exist
};

// every block size of independent blocks at levels < 3 (64 KiB blocks on
// the byU16 stream kernel); LZ4-HC levels keep the batch engine
bool stream_eligible(const Session& s, const Lz4MtStreamDescriptor* sd) {
    return stream_enabled() && sd->flg.blockIndependence && s.level() < 3;
}

// Ring slots: LZ4MT_AMD_STREAM_IN / _OUT, else 1 GiB / 2 GiB of pinned
// memory whatever the block size (256 / 512 slots of 4 MiB; 64 KiB blocks
// get 16384 / 32768 slots, so as many bytes stay in flight)
uint32_t stream_slots(const char* var, uint64_t bytes, uint32_t bm) {
    const uint64_t def = std::min<uint64_t>(65536, std::max<uint64_t>(8, bytes / bm));
    return (uint32_t)env_int(var, (int)def, 8, 65536);
}

// false: the engine could not start (its buffers, the device): nothing was
// read, and the caller takes the batch engine instead
bool compress_streamed(Session& s, const Lz4MtStreamDescriptor* sd, HostXxh32& xs) {
    const uint32_t bm = (uint32_t)block_max_bytes(sd->bd.blockMaximumSize);
    const bool bck = sd->flg.blockChecksum, sck = sd->flg.streamChecksum;
    int cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess || cus <= 0)
        return false;
    // the staging ring only has to stay ahead of the pulls (~1 ms per
    // block), the output ring behind the writer
    const uint32_t waves = stream_waves(cus);
    const uint32_t Rin = stream_slots("LZ4MT_AMD_STREAM_IN", 1ull << 30, bm);
    const uint32_t Rout = stream_slots("LZ4MT_AMD_STREAM_OUT", 2ull << 30, bm);
    StreamBufs& B = g_stream;
    if (!B.ensure(bm, waves, Rin, Rout)) return false;
    uint32_t* g = B.hCtl;
    uint32_t* inC = g + 8;
    uint32_t* outC = inC + 4ull * Rin;
    memset(g, 0, 4ull * (8 + 4ull * Rin + 4ull * Rout));
    g[0] = 0xFFFFFFFFu;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const uint64_t ticks = stream_wait_ticks();
    auto launch = [&] {
        return launch_encode_stream(B.hIn, B.hOut, inC, outC, g, B.dNext, B.dPend, B.dIn, B.dSlot, bm, Rin, Rout,
                                    waves, bck ? 1 : 0, ticks, B.st);
    };
    if (hipMemsetAsync(B.dNext, 0, 4, B.st) != hipSuccess || hipMemsetAsync(B.dPend, 0, 16ull * waves, B.st) !=
        hipSuccess || launch() != hipSuccess) {
        (void)hipGetLastError();
        hipStreamSynchronize(B.st);
        return false;
    }
    std::atomic<uint32_t> total{0xFFFFFFFFu};   // blocks in the stream, once known
    std::atomic<bool> wfail{false};
    bool relaunchFail = false;
    auto gpuFailed = [&] { return ld_acq(g + 4) != 0; };
    auto stopped = [&] { return gpuFailed() || ld_acq(g + 1) != 0; };
    StreamMonitor ka(B, g, launch);
    std::thread writer([&] {
        for (uint32_t b = 0;; ++b) {
            uint32_t* o = outC + 4ull * (b % Rout);
            const bool ok = host_wait([&] { return ld_acq(o) == b + 1 || b >= total.load(); }, stopped);
            if (!ok || (b >= total.load() && ld_acq(o) != b + 1)) {
                if (!ok) wfail = true;
                return;
            }
            const uint32_t word = ld_acq(o + 1), len = word & ~kRawBit, sum = ld_acq(o + 2);
            const uint8_t* payload = B.hOut + (uint64_t)(b % Rout) * bm;
            bool wok;
            {
                StreamMonitor::Scope cb(ka, false);
                wok = s.writeU32(word) && s.write(payload, (int)len) && (!bck || s.writeU32(sum));
            }
            if (!wok) {
                wfail = true;
                st_rel(g + 1, 1u);   // abort: the grid and the reader stop
                return;
            }
            st_rel(o + 3, b + 1);   // the slot may take block b + Rout
            st_rel(g + 3, b + 1);   // heartbeat
        }
    });
    // the content checksum (FLG.2) is one serial XXH32 chain: a hasher
    // thread runs it over the staged blocks in order, beside the reads (a
    // staging slot is refilled only once it is both pulled and hashed)
    std::atomic<uint32_t> hashed{0};
    std::thread hasher;
    if (sck) {
        hasher = std::thread([&] {
            for (uint32_t h = 0;; ++h) {
                const uint32_t* ic = inC + 4ull * (h % Rin);
                if (!host_wait([&] { return ld_acq(ic) == h + 1 || h >= total.load(); }, stopped) ||
                    ld_acq(ic) != h + 1)
                    return;
                xs.update(B.hIn + (uint64_t)(h % Rin) * bm, ld_acq(ic + 1));
                hashed.store(h + 1, std::memory_order_release);
            }
        });
    }
    // the reader: every read() on this thread, one block per read (a short
    // read is a short block; 0 ends the stream: src/lz4mt.cpp:434-447)
    uint32_t b = 0;
    for (;; ++b) {
        uint32_t* ic = inC + 4ull * (b % Rin);
        if (b >= Rin && !host_wait([&] { return ld_acq(ic + 2) == b - Rin + 1 &&
                                                (!sck || hashed.load(std::memory_order_acquire) > b - Rin); },
                                   stopped))
            break;
        if (stopped()) break;   // the writer or the grid stopped
        uint8_t* dst = B.hIn + (uint64_t)(b % Rin) * bm;
        int n;
        {
            StreamMonitor::Scope rs(ka, true);
            n = s.read(dst, (int)bm);
        }
        if (n <= 0) break;
        // never while the grid is parked (a read() or write() stalled): the
        // reader relaunches it at b first, or waits for the writer to
        if (!ka.publish(b, [&] {
                st_rel(ic + 1, (uint32_t)n);
                st_rel(ic, b + 1);
                st_rel(g + 2, b + 1);   // heartbeat
            }, stopped)) {
            if (!stopped()) relaunchFail = true;
            st_rel(g + 1, 1u);
            break;
        }
    }
    total = b;
    st_rel(g, b);   // waves waiting for a block >= b leave
    // (a grid parked by the last read() holds blocks that still go out: the
    // monitor relaunches it; it stops once the writer is done)
    if (hasher.joinable()) hasher.join();
    writer.join();
    ka.stop();
    if (ka.failed()) relaunchFail = true;
    if (wfail || gpuFailed()) st_rel(g + 1, 1u);
    const hipError_t e = hipStreamSynchronize(B.st);
    if (e != hipSuccess || gpuFailed() || ((wfail || relaunchFail) && !s.error())) s.quit(LZ4MT_RESULT_ERROR);
    if (!(s.mode() & LZ4MT_MODE_DEVICE)) B.release();
    return true;
}

void compress_device(Session& s, const Lz4MtStreamDescriptor* sd, HostXxh32& xs) {
    if (lz4mtHipDeviceCount() <= 0) { s.quit(LZ4MT_RESULT_ERROR); return; }
    if (stream_eligible(s, sd) && compress_streamed(s, sd, xs)) return;
    // LZ4-HC on independent blocks: levels 3..9 the hashChain parser, 10..12
    // (and above, clamped) the optimal parser.  Block-dependent frames at any
    // level >= 3 are the reference's HC stream, at level 9 (HcBdSim).
    const int level = s.level() >= 3 ? s.level() : 0;
    const uint32_t bm = (uint32_t)block_max_bytes(sd->bd.blockMaximumSize);
    const bool bck = sd->flg.blockChecksum, sck = sd->flg.streamChecksum;
    // Block-dependent frames (compressBlockDependency, src/lz4mt.cpp:460-538)
    // are one serial stream: one slot (batches in order on one stream), each
    // batch's input preceded by the 64 KiB before it (`hist`), the lz4
    // stream table carried in `table`, the per-block lz4 modes from BdSim.
    const bool linked = !sd->flg.blockIndependence;
    const uint64_t pre = linked ? 65536 : 0;
    PipeShape P = pipe_shape(true);
    if (linked) P.slots = 1;
    const bool refBytes = linked && bd_reference_bytes();
    BdSim sim(sd->bd.blockMaximumSize, refBytes);
    HcBdSim hsim(sd->bd.blockMaximumSize);   // level >= 3
    std::vector<uint8_t> hist(linked ? 65536 : 0, 0);
    std::vector<LinkPlan> plan;
    std::vector<uint64_t> segAbs;
    std::vector<uint8_t> packed;
    CallBuf table, dplan, rounds;
    if (linked && !table.alloc(4096 * 4)) { s.quit(LZ4MT_RESULT_ERROR); return; }
    uint64_t batch = 0, planCap = 0, roundCap = 0, streamPos = 0;
    auto fill = [&](Slot& S, bool* stop) -> bool {
        const uint64_t K = batch_blocks(P, bm, batch++), inCap = K * bm;
        if (!S.ensure(pre + inCap, inCap + K * 8 + 64, compress_ws_bytes(inCap, bm, level), 0)) {
            s.quit(LZ4MT_RESULT_ERROR);
            return false;
        }
        uint8_t* in = S.hIn + pre;
        // One read() per block, as the reference does (src/lz4mt.cpp:435-450):
        // a read of 0 ends the input; a short read is a short block, which
        // closes this batch (a batch is blocks of bm bytes plus at most one
        // short last block) -- the next batch carries on reading.
        uint64_t total = 0;
        for (uint64_t j = 0; j < K; ++j) {
            const int n = s.read(in + total, (int)bm);
            if (n <= 0) { *stop = true; break; }
            total += (uint64_t)n;
            if ((uint32_t)n < bm) break;
        }
        if (total == 0) return false;
        uint64_t* dRecOff = nullptr;
        const uint64_t nb = (total + bm - 1) / bm;
        LinkState ls{};
        if (linked && level) {   // the HC stream's segments over (hist ++ this input)
            memcpy(S.hIn, hist.data(), 65536);
            segAbs.resize(nb);
            for (uint64_t b = 0; b < nb; ++b) segAbs[b] = hsim.next((uint32_t)std::min<uint64_t>(bm, total - b * bm));
            ls.nSeg = hc_bd_pack(segAbs.data(), nb, streamPos, total, 65536, packed, bm, &ls.hcPerBlock);
            if (packed.size() + 64 > planCap * sizeof(LinkPlan)) {
                if (dplan.p) { hipStreamSynchronize(S.st); hipFree(dplan.p); dplan.p = nullptr; }
                planCap = (packed.size() + 64 + sizeof(LinkPlan) - 1) / sizeof(LinkPlan);
                if (!dplan.alloc(planCap * sizeof(LinkPlan))) { s.quit(LZ4MT_RESULT_ERROR); return false; }
            }
            if (hipMemcpyAsync(dplan.p, packed.data(), packed.size(), hipMemcpyHostToDevice, S.st) != hipSuccess) {
                s.quit(LZ4MT_RESULT_ERROR);
                return false;
            }
            ls.hcSegs = static_cast<const uint8_t*>(dplan.p);
        } else if (linked) {
            memcpy(S.hIn, hist.data(), 65536);
            plan.resize(nb);
            bool xh = false;
            for (uint64_t b = 0; b < nb; ++b) {
                plan[b].shift = 0;
                sim.next((uint32_t)std::min<uint64_t>(bm, total - b * bm), &plan[b].lowIn, &plan[b].lowDict,
                         &plan[b].candLow, refBytes ? &plan[b].shift : nullptr);
                xh = xh || plan[b].shift != 0;
            }
            if (sim.bad) { s.quit(LZ4MT_RESULT_ERROR); return false; }
            if (nb > planCap) {
                if (dplan.p) { hipStreamSynchronize(S.st); hipFree(dplan.p); dplan.p = nullptr; }
                if (!dplan.alloc(nb * sizeof(LinkPlan))) { s.quit(LZ4MT_RESULT_ERROR); return false; }
                planCap = nb;
            }
            // the plan buffer is reused by the next batch: same stream, in order
            if (hipMemcpyAsync(dplan.p, plan.data(), nb * sizeof(LinkPlan), hipMemcpyHostToDevice, S.st) != hipSuccess) {
                s.quit(LZ4MT_RESULT_ERROR);
                return false;
            }
            if (nb > roundCap) {   // the parallel rounds' entry / exit tables
                if (rounds.p) { hipStreamSynchronize(S.st); hipFree(rounds.p); rounds.p = nullptr; }
                if (!rounds.alloc(link_round_bytes(nb))) { s.quit(LZ4MT_RESULT_ERROR); return false; }
                roundCap = nb;
            }
            ls = LinkState{static_cast<LinkPlan*>(dplan.p), static_cast<uint32_t*>(table.p), batch == 1,
                           static_cast<uint32_t*>(rounds.p)};
            ls.xh = xh;
        }
        if (linked) {   // the history of the next batch: the last 64 KiB of (hist ++ this input)
            if (total >= 65536) memcpy(hist.data(), in + total - 65536, 65536);
            else {
                memmove(hist.data(), hist.data() + total, 65536 - total);
                memcpy(hist.data() + 65536 - total, in, total);
            }
        }
        streamPos += total;
        if (hipMemcpyAsync(S.dIn, S.hIn, pre + total, hipMemcpyHostToDevice, S.st) != hipSuccess ||
            device_compress_body(S.dIn + pre, total, bm, bck, S.dWs, S.dOut, 0, S.st, &dRecOff, nullptr,
                                 linked ? &ls : nullptr, level) != LZ4MT_RESULT_OK ||
            hipMemcpyAsync(S.hMeta, dRecOff + nb, 8, hipMemcpyDeviceToHost, S.st) != hipSuccess) {
            s.quit(LZ4MT_RESULT_ERROR);
            return false;
        }
        S.total = total;
        S.nb = nb;
        if (sck) xs.update(in, total);   // serial content checksum overlaps the kernels
        return true;
    };
    // the body size, D2H of the body, then write() per record in the
    // reference's pieces: size word, payload, [block checksum]
    // (src/lz4mt.cpp:418-428), so a bounded sink sees the same calls
    auto finish = [&](Slot& S) -> bool {
        if (hipStreamSynchronize(S.st) != hipSuccess) { s.quit(LZ4MT_RESULT_ERROR); return false; }
        const uint64_t bodySize = S.hMeta[0];
        if (hipMemcpyAsync(S.hOut, S.dOut, bodySize, hipMemcpyDeviceToHost, S.st) != hipSuccess ||
            hipStreamSynchronize(S.st) != hipSuccess) {
            s.quit(LZ4MT_RESULT_ERROR);
            return false;
        }
        for (uint64_t o = 0, b = 0; b < S.nb; ++b) {
            const uint32_t len = get32(S.hOut + o) & ~kRawBit;
            if (o + 4 + len + (bck ? 4 : 0) > bodySize) { s.quit(LZ4MT_RESULT_ERROR); return false; }
            if (!s.write(S.hOut + o, 4) || !s.write(S.hOut + o + 4, (int)len) ||
                (bck && !s.write(S.hOut + o + 4 + len, 4)))
                return false;
            o += 4 + (uint64_t)len + (bck ? 4 : 0);
        }
        return true;
    };
    run_slot_pipeline(s, P.slots, fill, finish);
}

// ---------------------------------------------------------------------------
// decompress: host scheduler (reference decompress(), src/lz4mt.cpp:593-734)
// Returns true when the EOS mark was reached.
// ---------------------------------------------------------------------------
bool decompress_host(Session& s, const Lz4MtStreamDescriptor* sd, HostXxh32& xs) {
    const int bm = block_max_bytes(sd->bd.blockMaximumSize);
    const bool bck = sd->flg.blockChecksum, sck = sd->flg.streamChecksum;
    const unsigned W = worker_count(s);
    auto work = [&](Job& j) {
        j.skip = s.error() || s.quitting();
        if (j.skip) return;
        j.ckbad = bck && HostXxh32::oneshot(j.in.data(), (size_t)j.n) != j.ck;
        if (j.raw) { j.res = j.n; return; }
        j.out.resize((size_t)bm + 64);
        j.res = s.decompress(j.in.data(), j.out.data(), j.n, bm);   // cap = blockMax (src/lz4mt.cpp:645)
    };
    auto emit = [&](Job& j) {   // reference worker tail, src/lz4mt.cpp:619-681
        if (j.skip || s.error() || s.quitting()) return;
        if (!j.raw && j.res < 0) { s.quit(LZ4MT_RESULT_DECOMPRESS_FAIL); return; }
        const char* p = j.raw ? j.in.data() : j.out.data();
        if (sck) xs.update(p, (size_t)j.res);
        if (!s.write(p, j.res)) {
            s.quit(j.raw ? LZ4MT_RESULT_CANNOT_WRITE_DATA_BLOCK : LZ4MT_RESULT_CANNOT_WRITE_DECODED_BLOCK);
            return;
        }
        if (j.ckbad) s.quit(LZ4MT_RESULT_BLOCK_CHECKSUM_MISMATCH);
    };
    Pipeline pipe(W, W + 1, work, emit);
    bool eos = false;
    while (!eos && !s.quitting() && !s.error() && !s.readEof()) {
        uint32_t bits = 0;
        if (!s.readU32(&bits)) { s.quit(LZ4MT_RESULT_CANNOT_READ_BLOCK_SIZE); break; }
        if (bits == 0) { eos = true; break; }
        const int n = (int)(bits & ~kRawBit);
        if (n > bm) { s.quit(LZ4MT_RESULT_INVALID_BLOCK_SIZE); break; }
        Job& j = pipe.acquire();
        j.in.resize((size_t)n + 64);
        if (s.read(j.in.data(), n) != n || s.error()) { s.quit(LZ4MT_RESULT_CANNOT_READ_BLOCK_DATA); break; }
        j.n = n;
        j.raw = (bits & kRawBit) != 0;
        j.ck = 0;
        if (bck && !s.readU32(&j.ck)) { s.quit(LZ4MT_RESULT_CANNOT_READ_BLOCK_CHECKSUM); break; }
        pipe.submit();
    }
    pipe.drain();
    return eos;
}

// ---------------------------------------------------------------------------
// Streamed DEVICE decompress (independent 1 / 4 MiB blocks): k_decode_stream
// is launched once, before the first record is read; the calling thread
// reads record after record (size word, stored bytes, block checksum) into
// the staging ring, the persistent grid decodes each one as soon as it is
// published and pushes the decoded bytes into the output ring, a writer
// thread writes them in block order and a hasher thread runs the content
// checksum (FLG.2) over them beside it.  Errors keep the batch engine's
// order: a block that fails to decode stops the frame before it is written,
// a block checksum mismatch after it is written, and a read error found
// while reading applies once every record before it is written.
// LZ4MT_AMD_STREAM=0 keeps the batch engine below.
// ---------------------------------------------------------------------------
// false: the engine could not start (nothing was read); *eos: the EOS mark
// was reached
bool decompress_streamed(Session& s, const Lz4MtStreamDescriptor* sd, HostXxh32& xs, bool* eosOut) {
    const uint32_t bm = (uint32_t)block_max_bytes(sd->bd.blockMaximumSize);
    const bool bck = sd->flg.blockChecksum, sck = sd->flg.streamChecksum;
    int cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess || cus <= 0)
        return false;
    const uint32_t waves = stream_waves(cus);
    const uint32_t Rin = stream_slots("LZ4MT_AMD_STREAM_IN", 1ull << 30, bm);
    const uint32_t Rout = stream_slots("LZ4MT_AMD_STREAM_OUT", 2ull << 30, bm);
    StreamBufs& B = g_stream;
    if (!B.ensure(bm, waves, Rin, Rout)) return false;
    uint32_t* g = B.hCtl;
    uint32_t* inC = g + 8;
    uint32_t* outC = inC + 4ull * Rin;
    memset(g, 0, 4ull * (8 + 4ull * Rin + 4ull * Rout));
    g[0] = 0xFFFFFFFFu;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const uint64_t ticks = stream_wait_ticks();
    auto launch = [&] {
        return launch_decode_stream(B.hIn, B.hOut, inC, outC, g, B.dNext, B.dPend, B.dIn, B.dSlot, bm, Rin, Rout,
                                    waves, bck ? 1 : 0, ticks, B.st);
    };
    if (hipMemsetAsync(B.dNext, 0, 4, B.st) != hipSuccess || hipMemsetAsync(B.dPend, 0, 16ull * waves, B.st) !=
        hipSuccess || launch() != hipSuccess) {
        (void)hipGetLastError();
        hipStreamSynchronize(B.st);
        return false;
    }
    std::atomic<uint32_t> total{0xFFFFFFFFu};
    std::atomic<bool> wfail{false};
    bool relaunchFail = false;
    std::atomic<uint32_t> hashed{0};
    auto gpuFailed = [&] { return ld_acq(g + 4) != 0; };
    auto stopped = [&] { return gpuFailed() || ld_acq(g + 1) != 0; };
    StreamMonitor ka(B, g, launch);
    // the content checksum over the decoded blocks, in order, beside the writer
    std::thread hasher;
    if (sck) {
        hasher = std::thread([&] {
            for (uint32_t h = 0;; ++h) {
                const uint32_t* o = outC + 4ull * (h % Rout);
                if (!host_wait([&] { return ld_acq(o) == h + 1 || h >= total.load(); }, stopped) || ld_acq(o) != h + 1)
                    return;
                const int32_t n = (int32_t)ld_acq(o + 1);
                if (n < 0 || (ld_acq(o + 2) & 0xFFu) == 18u) return;   // the frame stops at this block
                xs.update(B.hOut + (uint64_t)(h % Rout) * bm, (size_t)n);
                hashed.store(h + 1, std::memory_order_release);
            }
        });
    }
    std::thread writer([&] {
        for (uint32_t b = 0;; ++b) {
            uint32_t* o = outC + 4ull * (b % Rout);
            const bool ok = host_wait([&] { return ld_acq(o) == b + 1 || b >= total.load(); }, stopped);
            if (!ok || (b >= total.load() && ld_acq(o) != b + 1)) {
                if (!ok) wfail = true;
                return;
            }
            const int32_t n = (int32_t)ld_acq(o + 1);
            const uint32_t st = ld_acq(o + 2);
            if ((st & 0xFFu) == 18u || n < 0) {   // decode failure: stop before writing the block
                s.quit(LZ4MT_RESULT_DECOMPRESS_FAIL);
                st_rel(g + 1, 1u);
                return;
            }
            if (sck && !host_wait([&] { return hashed.load(std::memory_order_acquire) > b; }, stopped)) {
                wfail = true;
                return;
            }
            bool wok;
            {
                StreamMonitor::Scope cb(ka, false);
                wok = s.write(B.hOut + (uint64_t)(b % Rout) * bm, n);
            }
            if (!wok) {
                s.quit((st & 0x100u) ? LZ4MT_RESULT_CANNOT_WRITE_DATA_BLOCK : LZ4MT_RESULT_CANNOT_WRITE_DECODED_BLOCK);
                st_rel(g + 1, 1u);
                return;
            }
            if (st & 16u) {   // checksum mismatch: after the block is written
                s.quit(LZ4MT_RESULT_BLOCK_CHECKSUM_MISMATCH);
                st_rel(g + 1, 1u);
                return;
            }
            st_rel(o + 3, b + 1);   // the slot may take block b + Rout
            st_rel(g + 3, b + 1);   // heartbeat
        }
    });
    // the reader: every read on this thread (the batch engine's record checks)
    bool eos = false;
    Lz4MtResult pending = LZ4MT_RESULT_OK;
    uint32_t b = 0;
    for (;; ++b) {
        uint32_t* ic = inC + 4ull * (b % Rin);
        if (b >= Rin && !host_wait([&] { return ld_acq(ic + 3) == b - Rin + 1; }, stopped)) break;
        if (stopped() || s.quitting()) break;
        uint32_t bits = 0, ck = 0;
        {
            StreamMonitor::Scope rs(ka, true);   // the record's read() calls
            if (s.readEof()) break;
            if (!s.peekU32(&bits)) { pending = LZ4MT_RESULT_CANNOT_READ_BLOCK_SIZE; break; }
            if (bits == 0) { eos = true; break; }
            const uint32_t n = bits & ~kRawBit;
            if (n > bm) { pending = LZ4MT_RESULT_INVALID_BLOCK_SIZE; break; }
            if (s.read(B.hIn + (uint64_t)(b % Rin) * bm, (int)n) != (int)n) {
                pending = LZ4MT_RESULT_CANNOT_READ_BLOCK_DATA;
                break;
            }
            if (bck && !s.peekU32(&ck)) { pending = LZ4MT_RESULT_CANNOT_READ_BLOCK_CHECKSUM; break; }
        }
        if (!ka.publish(b, [&] {
                st_rel(ic + 1, bits);
                st_rel(ic + 2, ck);
                st_rel(ic, b + 1);
                st_rel(g + 2, b + 1);   // heartbeat
            }, stopped)) {
            if (!stopped()) relaunchFail = true;
            st_rel(g + 1, 1u);
            break;
        }
    }
    total = b;
    st_rel(g, b);   // waves waiting for a block >= b leave
    // (a grid parked by the last read() holds blocks that still go out: the
    // monitor relaunches it; it stops once the writer is done)
    writer.join();
    if (hasher.joinable()) {
        if (s.error() || s.quitting() || wfail) st_rel(g + 1, 1u);
        hasher.join();
    }
    ka.stop();
    if (ka.failed()) relaunchFail = true;
    if (wfail || gpuFailed()) st_rel(g + 1, 1u);
    const hipError_t e = hipStreamSynchronize(B.st);
    if (e != hipSuccess || gpuFailed() || ((wfail || relaunchFail) && !s.error())) s.quit(LZ4MT_RESULT_ERROR);
    if (!(s.mode() & LZ4MT_MODE_DEVICE)) B.release();
    if (pending != LZ4MT_RESULT_OK && !s.error()) s.quit(pending);
    *eosOut = eos;
    return true;
}

bool stream_eligible_dec(const Lz4MtStreamDescriptor* sd) {
    return stream_enabled() && sd->flg.blockIndependence;
}

// ---------------------------------------------------------------------------
// decompress: DEVICE batch engine (the same slot pipeline as compress)
// ---------------------------------------------------------------------------
bool decompress_device(Session& s, const Lz4MtStreamDescriptor* sd, HostXxh32& xs) {
    if (lz4mtHipDeviceCount() <= 0) { s.quit(LZ4MT_RESULT_ERROR); return false; }
    if (bool eos = false; stream_eligible_dec(sd) && decompress_streamed(s, sd, xs, &eos)) return eos;
    const uint32_t bm = (uint32_t)block_max_bytes(sd->bd.blockMaximumSize);
    const bool bck = sd->flg.blockChecksum, sck = sd->flg.streamChecksum;
    // Block-dependent frames (decompressBlockDependency, src/lz4mt.cpp:
    // 737-845): one slot, one wave decoding the blocks in order, the 64 KiB
    // history carried from batch to batch in `hist` (zeros at the start).
    const bool linked = !sd->flg.blockIndependence;
    PipeShape P = pipe_shape(false);
    if (linked) P.slots = 1;
    CallBuf hist, slotScratch;
    const bool serialBd = bd_serial();
    uint64_t scratchCap = 0;   // blocks the linked scratch holds
    if (linked && (!hist.alloc(65536) || hipMemset(hist.p, 0, 65536) != hipSuccess)) {
        s.quit(LZ4MT_RESULT_ERROR);
        return false;
    }
    uint64_t batch = 0;
    bool eos = false;
    Lz4MtResult pending = LZ4MT_RESULT_OK;   // a read error found while filling a batch
    auto fill = [&](Slot& S, bool* stop) -> bool {
        if (eos || pending != LZ4MT_RESULT_OK || s.readEof()) return false;
        const uint64_t K = batch_blocks(P, bm, batch++);
        if (!S.ensure(K * bm + 16 * K, K * bm, 0, K)) { s.quit(LZ4MT_RESULT_ERROR); return false; }
        uint64_t used = 0, nb = 0;
        while (nb < K) {
            uint32_t bits = 0;
            if (s.readEof()) break;
            if (!s.peekU32(&bits)) { pending = LZ4MT_RESULT_CANNOT_READ_BLOCK_SIZE; break; }
            if (bits == 0) { eos = true; break; }
            const uint32_t n = bits & ~kRawBit;
            if (n > bm) { pending = LZ4MT_RESULT_INVALID_BLOCK_SIZE; break; }
            if (s.read(S.hIn + used, (int)n) != (int)n) { pending = LZ4MT_RESULT_CANNOT_READ_BLOCK_DATA; break; }
            uint32_t ck = 0;
            if (bck && !s.peekU32(&ck)) { pending = LZ4MT_RESULT_CANNOT_READ_BLOCK_CHECKSUM; break; }
            S.hRecs[nb++] = BlockRec{used, bits, ck};
            used = (used + n + 15) & ~15ull;
        }
        *stop = eos || pending != LZ4MT_RESULT_OK;
        if (nb == 0) return false;
        if (linked) {
            // scratch: the parallel rounds' slots (one slot for the serial kernel);
            // one slot pipeline, so the previous batch is done with it
            const uint64_t need = serialBd ? 65536 + (uint64_t)bm + 64 : dlink_scratch_bytes(nb, bm);
            if (need > scratchCap) {
                if (slotScratch.p) { hipStreamSynchronize(S.st); hipFree(slotScratch.p); slotScratch.p = nullptr; }
                if (!slotScratch.alloc(need)) { s.quit(LZ4MT_RESULT_ERROR); return false; }
                scratchCap = need;
            }
            uint8_t* const scr = static_cast<uint8_t*>(slotScratch.p);
            uint8_t* const hst = static_cast<uint8_t*>(hist.p);
            if (hipMemcpyAsync(S.dIn, S.hIn, used, hipMemcpyHostToDevice, S.st) != hipSuccess ||
                hipMemcpyAsync(S.dRecs, S.hRecs, nb * sizeof(BlockRec), hipMemcpyHostToDevice, S.st) != hipSuccess ||
                (bck && launch_xxh32_frame_blocks(S.dIn, S.dRecs, (uint32_t)nb, S.dDig, S.st) != hipSuccess) ||
                (serialBd ? launch_decode_linked(S.dIn, S.dRecs, (uint32_t)nb, bm, S.dOut, nb * bm, scr, hst, S.dDig,
                                                 bck, S.dDs, S.dSt, S.st)
                          : launch_decode_linked_par(S.dIn, S.dRecs, (uint32_t)nb, bm, S.dOut, nb * bm, hst, S.dDig,
                                                     bck, S.dDs, S.dSt, scr, env_rounds(), S.st)) != hipSuccess ||
                hipMemcpyAsync(S.hDs, S.dDs, nb * 4, hipMemcpyDeviceToHost, S.st) != hipSuccess ||
                hipMemcpyAsync(S.hSt, S.dSt, 8, hipMemcpyDeviceToHost, S.st) != hipSuccess ||
                hipMemcpyAsync(S.hOut, S.dOut, nb * bm, hipMemcpyDeviceToHost, S.st) != hipSuccess) {
                s.quit(LZ4MT_RESULT_ERROR);
                return false;
            }
            S.nb = nb;
            return true;
        }
        if (hipMemcpyAsync(S.dIn, S.hIn, used, hipMemcpyHostToDevice, S.st) != hipSuccess ||
            hipMemcpyAsync(S.dRecs, S.hRecs, nb * sizeof(BlockRec), hipMemcpyHostToDevice, S.st) != hipSuccess ||
            launch_decode(S.dIn, S.dRecs, (uint32_t)nb, bm, S.dOut, nb * bm, S.dDs, S.st) != hipSuccess ||
            (bck && launch_xxh32_frame_blocks(S.dIn, S.dRecs, (uint32_t)nb, S.dDig, S.st) != hipSuccess) ||
            launch_block_verify(S.dRecs, (uint32_t)nb, S.dDig, S.dDs, bm, bck, S.dSt, S.st) != hipSuccess ||
            hipMemcpyAsync(S.hDs, S.dDs, nb * 4, hipMemcpyDeviceToHost, S.st) != hipSuccess ||
            hipMemcpyAsync(S.hSt, S.dSt, nb * 4, hipMemcpyDeviceToHost, S.st) != hipSuccess ||
            hipMemcpyAsync(S.hOut, S.dOut, nb * bm, hipMemcpyDeviceToHost, S.st) != hipSuccess) {
            s.quit(LZ4MT_RESULT_ERROR);
            return false;
        }
        S.nb = nb;
        return true;
    };
    // statuses, then the blocks in order; the first failing block stops the
    // frame (reference precedence: a decode failure before writing)
    auto finish = [&](Slot& S) -> bool {
        if (hipStreamSynchronize(S.st) != hipSuccess) { s.quit(LZ4MT_RESULT_ERROR); return false; }
        if (linked) {   // blocks [0, done) are decoded back to back; a failing block is not written
            const int32_t done = S.hSt[0], code = S.hSt[1];
            const uint8_t* p = S.hOut;
            for (int32_t i = 0; i < done; ++i) {
                const int n = S.hDs[i];
                if (sck) xs.update(p, (size_t)n);
                if (!s.write(p, n)) { s.quit(LZ4MT_RESULT_CANNOT_WRITE_DATA_BLOCK); return false; }
                p += n;
            }
            if (code) {
                s.quit(code == 16 ? LZ4MT_RESULT_BLOCK_CHECKSUM_MISMATCH
                                  : code == 18 ? LZ4MT_RESULT_DECOMPRESS_FAIL : LZ4MT_RESULT_ERROR);
                return false;
            }
            return true;
        }
        for (uint64_t i = 0; i < S.nb; ++i) {
            const bool raw = (S.hRecs[i].bits & kRawBit) != 0;
            const int32_t st = S.hSt[i];
            if (st == 18 || st == 1) {
                s.quit(st == 18 ? LZ4MT_RESULT_DECOMPRESS_FAIL : LZ4MT_RESULT_ERROR);
                return false;
            }
            const uint8_t* p = S.hOut + i * bm;
            const int n = S.hDs[i];
            if (sck) xs.update(p, (size_t)n);
            if (!s.write(p, n)) {
                s.quit(raw ? LZ4MT_RESULT_CANNOT_WRITE_DATA_BLOCK : LZ4MT_RESULT_CANNOT_WRITE_DECODED_BLOCK);
                return false;
            }
            if (st == 16) { s.quit(LZ4MT_RESULT_BLOCK_CHECKSUM_MISMATCH); return false; }
        }
        return true;
    };
    run_slot_pipeline(s, P.slots, fill, finish);
    // a read failure found while filling comes after every batched block in
    // stream order: it applies once they are written (a block's own failure
    // wins); the reference sets ERROR and then this code (src/lz4mt.cpp:687-717)
    if (pending != LZ4MT_RESULT_OK) s.quit(pending);
    return eos;
}

}  // namespace

// Frees this thread's cached DEVICE-engine slots (pinned staging, device
// buffers, streams); called by lz4mtHipReleaseCaches.
namespace lz4mt {
void release_slot_cache() { g_slots.release(); g_stream.release(); }
}  // namespace lz4mt

// ===========================================================================
// public API
// ===========================================================================
extern "C" Lz4MtContext lz4mtInitContext(void) {
    Lz4MtContext c;
    memset(&c, 0, sizeof(c));
    c.result = LZ4MT_RESULT_OK;
    c.mode = LZ4MT_MODE_PARALLEL;
    c.compressionLevel = 0;
    return c;
}

extern "C" Lz4MtStreamDescriptor lz4mtInitStreamDescriptor(void) {
    Lz4MtStreamDescriptor d;
    memset(&d, 0, sizeof(d));
    d.flg.streamChecksum = 1;
    d.flg.blockIndependence = 1;
    d.flg.versionNumber = 1;
    d.bd.blockMaximumSize = 7;
    return d;
}

// The batched device engine runs for LZ4MT_MODE_DEVICE, and also for the
// reference's default PARALLEL mode when the codec callback of that
// direction is null -- i.e. when every block would go to this library's GPU
// block operator one launch at a time (a relinked lz4mt caller).  Same
// frames, same callback protocol (LZ4-HC included: levels 3..9).
bool use_device_engine(const Lz4MtContext* ctx, bool compress) {
    if (ctx->mode & LZ4MT_MODE_DEVICE) return true;
    if (ctx->mode != LZ4MT_MODE_PARALLEL) return false;
    return compress ? !ctx->compress : !ctx->decompress;
}

extern "C" Lz4MtResult lz4mtCompress(Lz4MtContext* ctx, const Lz4MtStreamDescriptor* sd) {
    if (!ctx || !sd) return LZ4MT_RESULT_BAD_ARG;
    Session s(ctx);
    // header (makeHeader, src/lz4mt.cpp:335-369)
    const Lz4MtResult v = validate_sd(sd);
    if (v != LZ4MT_RESULT_OK) return s.quit(v);
    uint8_t hdr[kMaxHeader];
    const int hl = build_header(sd, hdr);
    if (!ctx->write || ctx->write(ctx, hdr, hl) != hl) return s.quit(LZ4MT_RESULT_CANNOT_WRITE_HEADER);
    HostXxh32 xs(0);
    // block-dependent frames: the reference calls lz4's streaming API
    // directly, not ctx->compress (src/lz4mt.cpp:295-332): the device engine
    if (!sd->flg.blockIndependence || use_device_engine(ctx, true)) compress_device(s, sd, xs);
    else compress_host(s, sd, xs);
    if (s.result() != LZ4MT_RESULT_OK) return s.result();
    if (!s.writeU32(0)) return s.quit(LZ4MT_RESULT_CANNOT_WRITE_EOS);
    if (sd->flg.streamChecksum && !s.writeU32(xs.digest())) return s.quit(LZ4MT_RESULT_CANNOT_WRITE_STREAM_CHECKSUM);
    return LZ4MT_RESULT_OK;
}

extern "C" Lz4MtResult lz4mtDecompress(Lz4MtContext* ctx, Lz4MtStreamDescriptor* sd) {
    if (!ctx || !sd) return LZ4MT_RESULT_BAD_ARG;
    Session s(ctx);
    bool seen = false;
    s.set(LZ4MT_RESULT_OK);
    while (!s.quitting() && !s.error() && !s.readEof()) {
        uint32_t magic = 0;
        if (!s.readU32(&magic)) {
            // end of input between frames is the normal end (src/lz4mt.cpp:951-957)
            s.set(s.readEof() ? LZ4MT_RESULT_OK : LZ4MT_RESULT_INVALID_HEADER);
            break;
        }
        if (magic != kMagic) {
            if (magic >= kSkippableMin && magic <= kSkippableMax) {
                uint32_t size = 0;
                if (!s.readU32(&size)) { s.set(LZ4MT_RESULT_INVALID_HEADER_SKIPPABLE_SIZE_UNREADABLE); break; }
                if (!s.skip(magic, size) || s.error()) { s.set(LZ4MT_RESULT_INVALID_HEADER_CANNOT_SKIP_SKIPPABLE_AREA); break; }
                s.clearEofHint();
                continue;
            }
            if (!seen) s.set(LZ4MT_RESULT_INVALID_MAGIC_NUMBER);
            break;   // trailing non-frame data ends the stream
        }
        seen = true;
        // readHeader (src/lz4mt.cpp:541-590)
        uint8_t h[kMaxHeader];
        if (s.read(h, 2) != 2) { s.quit(LZ4MT_RESULT_INVALID_HEADER); break; }
        Lz4MtStreamDescriptor tmp = *sd;
        parse_flg(h[0], &tmp.flg);
        parse_bd(h[1], &tmp.bd);
        const Lz4MtResult vr = validate_sd(&tmp);
        if (vr != LZ4MT_RESULT_OK) { *sd = tmp; s.quit(vr); break; }
        const int nex = (tmp.flg.streamSize ? 8 : 0) + (tmp.flg.presetDictionary ? 4 : 0) + 1;
        if (s.read(h + 2, nex) != nex) { *sd = tmp; s.quit(LZ4MT_RESULT_INVALID_HEADER); break; }
        int hb = 0;
        const Lz4MtResult hr = parse_header(h, (size_t)(2 + nex), &tmp, &hb);
        *sd = tmp;
        if (hr != LZ4MT_RESULT_OK) { s.quit(hr); break; }
        HostXxh32 xs(0);
        // block-dependent frames: LZ4_decompress_safe_withPrefix64k, not
        // ctx->decompress, in the reference (src/lz4mt.cpp:813-818)
        const bool eos = (!sd->flg.blockIndependence || use_device_engine(ctx, false)) ? decompress_device(s, sd, xs)
                                                                                       : decompress_host(s, sd, xs);
        if (s.error() || s.quitting()) break;
        if (!eos) { s.quit(LZ4MT_RESULT_CANNOT_READ_BLOCK_SIZE); break; }
        if (sd->flg.streamChecksum) {
            uint32_t want = 0;
            if (!s.readU32(&want)) { s.set(LZ4MT_RESULT_CANNOT_READ_STREAM_CHECKSUM); break; }
            if (xs.digest() != want) { s.set(LZ4MT_RESULT_STREAM_CHECKSUM_MISMATCH); break; }
        }
    }
    return s.result();
}

// A caller may pass any int (the reference's table answers "Unknown code"):
// take the argument's bits without an enum-typed load of a value outside the
// enumeration's range (UB in C++; UBSan -fsanitize=enum).
static int result_bits(const Lz4MtResult* r) {
    int v;
    std::memcpy(&v, r, sizeof v);
    return v;
}

extern "C" const char* lz4mtResultToString(Lz4MtResult r) {
    // Exactly the reference's table (src/lz4mt_result.cpp:4-89): it has no
    // case for BLOCK_CHECKSUM_MISMATCH (16), INVALID_HEADER_SKIPPABLE_SIZE_
    // UNREADABLE (24) or INVALID_HEADER_CANNOT_SKIP_SKIPPABLE_AREA (25), so
    // those print "Unknown code" there and here.
    static const char* const names[] = {
        "OK", "ERROR", "INVALID_MAGIC_NUMBER", "INVALID_HEADER", "PRESET_DICTIONARY_IS_NOT_SUPPORTED_YET",
        "BLOCK_DEPENDENCE_IS_NOT_SUPPORTED_YET", "INVALID_VERSION", "INVALID_HEADER_CHECKSUM",
        "INVALID_BLOCK_MAXIMUM_SIZE", "CANNOT_WRITE_HEADER", "CANNOT_WRITE_EOS", "CANNOT_WRITE_STREAM_CHECKSUM",
        "CANNOT_READ_BLOCK_SIZE", "CANNOT_READ_BLOCK_DATA", "CANNOT_READ_BLOCK_CHECKSUM",
        "CANNOT_READ_STREAM_CHECKSUM", nullptr, "STREAM_CHECKSUM_MISMATCH", "DECOMPRESS_FAIL",
        "BAD_ARG", "INVALID_BLOCK_SIZE", "INVALID_HEADER_RESERVED1", "INVALID_HEADER_RESERVED2",
        "INVALID_HEADER_RESERVED3", nullptr, nullptr, "CANNOT_WRITE_DATA_BLOCK", "CANNOT_WRITE_DECODED_BLOCK"};
    const unsigned i = (unsigned)result_bits(&r);
    const char* s = i < sizeof(names) / sizeof(names[0]) ? names[i] : nullptr;
    return s ? s : "Unknown code";
}

extern "C" int lz4mtResultToLz4cExitCode(Lz4MtResult r) {
    // lz4c exit codes per result (reference src/lz4mt_result.cpp:92-270)
    switch (result_bits(&r)) {
        case LZ4MT_RESULT_OK: return 0;
        case LZ4MT_RESULT_INVALID_MAGIC_NUMBER: return 44;
        case LZ4MT_RESULT_INVALID_HEADER_SKIPPABLE_SIZE_UNREADABLE: return 42;
        case LZ4MT_RESULT_INVALID_HEADER_CANNOT_SKIP_SKIPPABLE_AREA: return 43;
        case LZ4MT_RESULT_CANNOT_WRITE_HEADER: return 32;
        case LZ4MT_RESULT_CANNOT_WRITE_EOS:
        case LZ4MT_RESULT_CANNOT_WRITE_STREAM_CHECKSUM: return 37;
        case LZ4MT_RESULT_INVALID_HEADER: return 61;
        case LZ4MT_RESULT_INVALID_VERSION: return 62;
        case LZ4MT_RESULT_INVALID_HEADER_RESERVED1: return 65;
        case LZ4MT_RESULT_PRESET_DICTIONARY_IS_NOT_SUPPORTED_YET: return 66;
        case LZ4MT_RESULT_INVALID_HEADER_RESERVED2:
        case LZ4MT_RESULT_INVALID_HEADER_RESERVED3: return 67;
        case LZ4MT_RESULT_INVALID_BLOCK_MAXIMUM_SIZE: return 68;
        case LZ4MT_RESULT_INVALID_HEADER_CHECKSUM: return 69;
        case LZ4MT_RESULT_CANNOT_READ_BLOCK_SIZE: return 71;
        case LZ4MT_RESULT_INVALID_BLOCK_SIZE: return 72;
        case LZ4MT_RESULT_CANNOT_READ_BLOCK_DATA: return 73;
        case LZ4MT_RESULT_CANNOT_READ_BLOCK_CHECKSUM:
        case LZ4MT_RESULT_CANNOT_READ_STREAM_CHECKSUM: return 74;
        case LZ4MT_RESULT_BLOCK_CHECKSUM_MISMATCH:
        case LZ4MT_RESULT_STREAM_CHECKSUM_MISMATCH: return 75;
        case LZ4MT_RESULT_CANNOT_WRITE_DATA_BLOCK: return 76;
        case LZ4MT_RESULT_DECOMPRESS_FAIL: return 77;
        case LZ4MT_RESULT_CANNOT_WRITE_DECODED_BLOCK: return 78;
        default: return 1;
    }
}

// Diagnostics (host only, no device needed): the per-block lz4 stream plan
// BdSim derives for a -BD frame of nBlocks blocks of the given sizes --
// lowIn, lowDict, candLow, shift per block into plan4[4 * b] -- with the
// reference's input buffer replayed for every block size (refBuffer = 1, as
// LZ4MT_AMD_BD_REFERENCE does at 1 / 4 MiB) or only where lz4mt's buffer
// keeps the history contiguous.  Returns 0, -1 on a bad id, 1 if the plan
// needs a history that is neither (BdSim.bad).  tests/test_abi.py pins it
// against a restatement of the reference's buffer loop.
extern "C" int lz4mtDebugBdPlan(int blockMaxId, int refBuffer, const uint32_t* sizes, uint64_t nBlocks,
                                uint32_t* plan4) {
    if (blockMaxId < 4 || blockMaxId > 7 || (!sizes && nBlocks) || (!plan4 && nBlocks)) return -1;
    lz4mt::BdSim sim(blockMaxId, refBuffer != 0);
    for (uint64_t b = 0; b < nBlocks; ++b) {
        uint32_t* p = plan4 + 4 * b;
        p[3] = 0;
        sim.next(sizes[b], &p[0], &p[1], &p[2], refBuffer ? &p[3] : nullptr);
    }
    return sim.bad ? 1 : 0;
}
