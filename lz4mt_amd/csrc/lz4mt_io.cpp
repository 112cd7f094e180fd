// lz4mt_io.cpp — FILE* and memory callbacks for Lz4MtContext.
// FILE* side mirrors reference src/lz4mt_io_cstdio.cpp:75-175 (fread/fwrite/
// fseek/feof; "stdin"/"stdout" names; null sink = writeCtx == ctx).
//
// Large transfers (>= 2 MiB: the DEVICE engine reads and writes whole
// blocks) are split over a small copy pool, so one calling thread is not
// held to one core's memcpy/page-cache rate (~6.5 GB/s into pinned memory).
// The callbacks keep the reference's contract: they are still called from
// one thread at a time per stream and return only when the bytes are there.
#include <cerrno>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/lz4mt_io.h"

namespace {
// LZ4MT_AMD_COPY_THREADS / LZ4MT_AMD_COPY_PIECE_KIB / LZ4MT_AMD_COPY_MIN_KIB:
// the copy pool's width (caller included), the smallest piece a transfer is
// split into, and the smallest transfer that is split at all (smaller ones
// stay on the caller).  512 KiB / 256 KiB: 1 MiB-block records split 4-8
// ways (e2e B6 decompress 27-31 GiB/s vs 18-23 at 2 MiB / 1 MiB, B7 35 vs
// 31-33); 256 KiB / 128 KiB costs B5 a quarter (profiles/r06/r06n_copy_split_ab.txt)
size_t env_size(const char* name, size_t dflt, size_t lo, size_t hi) {
    const char* e = getenv(name);
    const long long v = e ? atoll(e) : (long long)dflt;
    return v < (long long)lo ? lo : ((size_t)v > hi ? hi : (size_t)v);
}
const size_t kPiece = env_size("LZ4MT_AMD_COPY_PIECE_KIB", 256, 64, 1 << 20) << 10;
const size_t kParMin = env_size("LZ4MT_AMD_COPY_MIN_KIB", 512, 64, 1 << 20) << 10;

// Persistent helper threads; run(n, f) calls f(0..n-1) on the helpers and
// the caller and returns when all are done.  Safe for concurrent callers
// (the DEVICE engine reads on the calling thread while its writer writes).
class CopyPool {
    struct Job {
        std::function<void(int)> fn;
        int n = 0;
        std::atomic<int> next{0};
        std::atomic<int> done{0};
        std::mutex m;
        std::condition_variable cv;
        void work() {
            for (int i; (i = next.fetch_add(1)) < n;) {
                fn(i);
                if (done.fetch_add(1) + 1 == n) {
                    std::lock_guard<std::mutex> g(m);
                    cv.notify_all();
                }
            }
        }
    };
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<Job>> q_;
    std::vector<std::thread> th_;
    bool stop_ = false;

    CopyPool() {
        const unsigned hw = std::thread::hardware_concurrency();
        const unsigned want = (unsigned)env_size("LZ4MT_AMD_COPY_THREADS", 8, 1, 64);
        const unsigned nt = std::min(want - 1, hw > 1 ? hw - 1 : 0u);
        for (unsigned i = 0; i < nt; ++i) th_.emplace_back([this] { loop(); });
    }
    ~CopyPool() {
        { std::lock_guard<std::mutex> g(m_); stop_ = true; }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void loop() {
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || !q_.empty(); });
                if (stop_) return;
                j = std::move(q_.front());
                q_.pop_front();
            }
            j->work();
        }
    }

public:
    static CopyPool& get() { static CopyPool p; return p; }
    int width() const { return (int)th_.size() + 1; }
    void run(int n, std::function<void(int)> fn) {
        if (n <= 1 || th_.empty()) {
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        auto j = std::make_shared<Job>();
        j->fn = std::move(fn);
        j->n = n;
        {
            std::lock_guard<std::mutex> g(m_);
            for (int k = 1; k < std::min(n, width()); ++k) q_.push_back(j);
        }
        cv_.notify_all();
        j->work();
        std::unique_lock<std::mutex> g(j->m);
        j->cv.wait(g, [&] { return j->done.load() == j->n; });
    }
};

int pieces(size_t n) { return (int)std::min<size_t>((size_t)CopyPool::get().width(), n / kPiece); }

// a piece of n split k ways, page-aligned: ceil(n / k) rounded up to 4 KiB
// (rounding floor(n / k) up dropped the last n % k bytes whenever n / k was
// already a multiple of 4 KiB, e.g. n = 4 MiB + 3 over 4 pieces)
size_t piece_len(size_t n, int k) { return ((n + (size_t)k - 1) / (size_t)k + 4095) & ~(size_t)4095; }

void par_copy(void* dst, const void* src, size_t n) {
    if (n < kParMin) { memcpy(dst, src, n); return; }
    const int k = pieces(n);
    const size_t per = piece_len(n, k);
    CopyPool::get().run(k, [=](int i) {
        const size_t o = (size_t)i * per;
        if (o < n) memcpy(static_cast<char*>(dst) + o, static_cast<const char*>(src) + o, std::min(per, n - o));
    });
}

// pread/pwrite of [off, off + n) split over the pool; returns bytes moved
// from the start (stops at the first short piece, like one big call)
size_t par_pio(int fd, void* buf, size_t n, off_t off, bool wr) {
    const int k = pieces(n);
    const size_t per = piece_len(n, k);
    std::vector<size_t> got((size_t)k, 0);
    CopyPool::get().run(k, [&](int i) {
        const size_t o = (size_t)i * per;
        if (o >= n) return;
        const size_t len = std::min(per, n - o);
        size_t d = 0;
        while (d < len) {
            char* p = static_cast<char*>(buf) + o + d;
            const ssize_t r = wr ? pwrite(fd, p, len - d, off + (off_t)(o + d)) : pread(fd, p, len - d, off + (off_t)(o + d));
            if (r < 0 && errno == EINTR) continue;   // interrupted, not the end of the file
            if (r <= 0) break;
            d += (size_t)r;
        }
        got[(size_t)i] = d;
    });
    size_t total = 0;
    for (int i = 0; i < k; ++i) {
        total += got[(size_t)i];
        if (got[(size_t)i] < std::min(per, n - std::min(n, (size_t)i * per))) break;
    }
    return total;
}

bool regular(FILE* fp) {
    struct stat st;
    return fstat(fileno(fp), &st) == 0 && S_ISREG(st.st_mode);
}

FILE* in_fp(const Lz4MtContext* c) { return static_cast<FILE*>(c->readCtx); }
FILE* out_fp(const Lz4MtContext* c) { return static_cast<FILE*>(c->writeCtx); }
bool is_null_sink(const Lz4MtContext* c) { return c->writeCtx == static_cast<const void*>(c); }
}  // namespace

extern "C" int lz4mtIoOpenIstream(Lz4MtContext* ctx, const char* filename) {
    FILE* fp = strcmp(filename, "stdin") == 0 ? stdin : fopen(filename, "rb");
    ctx->readCtx = fp;
    return fp != nullptr;
}

extern "C" int lz4mtIoOpenOstream(Lz4MtContext* ctx, const char* filename, int nullWrite) {
    if (nullWrite) {
        ctx->writeCtx = ctx;
        return 1;
    }
    FILE* fp = strcmp(filename, "stdout") == 0 ? stdout : fopen(filename, "wb");
    ctx->writeCtx = fp;
    return fp != nullptr;
}

extern "C" void lz4mtIoCloseIstream(Lz4MtContext* ctx) {
    FILE* fp = in_fp(ctx);
    if (fp && fp != stdin) fclose(fp);
    ctx->readCtx = nullptr;
}

extern "C" void lz4mtIoCloseOstream(Lz4MtContext* ctx) {
    if (!is_null_sink(ctx)) {
        FILE* fp = out_fp(ctx);
        if (fp && fp != stdout) fclose(fp);
    }
    ctx->writeCtx = nullptr;
}

extern "C" int lz4mtIoRead(Lz4MtContext* ctx, void* dst, int dstSize) {
    FILE* fp = in_fp(ctx);
    if (!fp) return 0;
    if (dstSize >= (int)kParMin && regular(fp)) {   // parallel pread at the stream position
        const off_t off = ftello(fp);
        if (off >= 0) {
            const size_t got = par_pio(fileno(fp), dst, (size_t)dstSize, off, false);
            fseeko(fp, off + (off_t)got, SEEK_SET);
            if (got < (size_t)dstSize) {   // short: leave the stream at EOF like fread
                const int c = fgetc(fp);
                if (c != EOF) ungetc(c, fp);
            }
            return (int)got;
        }
    }
    return (int)fread(dst, 1, (size_t)dstSize, fp);
}

extern "C" int lz4mtIoReadSkippable(const Lz4MtContext* ctx, uint32_t, size_t size) {
    FILE* fp = in_fp(ctx);
    return fp ? fseek(fp, (long)size, SEEK_CUR) : -1;
}

extern "C" int lz4mtIoReadSeek(const Lz4MtContext* ctx, int offset) {
    FILE* fp = in_fp(ctx);
    return fp ? fseek(fp, offset, SEEK_CUR) : -1;
}

extern "C" int lz4mtIoReadEof(const Lz4MtContext* ctx) {
    FILE* fp = in_fp(ctx);
    return fp ? feof(fp) : 1;
}

extern "C" int lz4mtIoWrite(const Lz4MtContext* ctx, const void* src, int srcSize) {
    if (is_null_sink(ctx)) return srcSize;
    FILE* fp = out_fp(ctx);
    if (!fp) return 0;
    // One fwrite (glibc hands a large buffer to write(2) directly).  Buffered
    // writes into one file serialise on its inode lock, so splitting them
    // over the copy pool only adds contention: 8 GiB into tmpfs, 6.0 GiB/s
    // from one thread vs 4.9-5.2 from 8 pwrite threads (tools/e2e.py --file,
    // profiles/r02_e2e_file.txt).  Reads stay parallel (no such lock).
    return (int)fwrite(src, 1, (size_t)srcSize, fp);
}

extern "C" uint64_t lz4mtIoGetFilesize(const char* filename) {
    struct stat st;
    if (stat(filename, &st) != 0 || !S_ISREG(st.st_mode)) return 0;
    return (uint64_t)st.st_size;
}

extern "C" void lz4mtIoBindCstdio(Lz4MtContext* ctx) {
    ctx->read = lz4mtIoRead;
    ctx->readSkippable = lz4mtIoReadSkippable;
    ctx->readSeek = lz4mtIoReadSeek;
    ctx->readEof = lz4mtIoReadEof;
    ctx->write = lz4mtIoWrite;
}

// ---- memory-backed callbacks ----------------------------------------------
namespace {
Lz4MtMemIo* mem(const Lz4MtContext* c) { return static_cast<Lz4MtMemIo*>(c->readCtx); }

int mem_read(Lz4MtContext* ctx, void* dst, int n) {
    Lz4MtMemIo* io = mem(ctx);
    if (n <= 0) return 0;
    const uint64_t rem = io->inSize - io->inPos;
    const uint64_t got = (uint64_t)n < rem ? (uint64_t)n : rem;
    if ((uint64_t)n > rem) io->eof = 1;
    par_copy(dst, io->in + io->inPos, got);
    io->inPos += got;
    return (int)got;
}
int mem_skip(const Lz4MtContext* ctx, uint32_t, size_t size) {
    Lz4MtMemIo* io = mem(ctx);
    io->eof = 0;   // fseek clears EOF
    const uint64_t rem = io->inSize - io->inPos;
    io->inPos += size < rem ? size : rem;
    return 0;
}
int mem_seek(const Lz4MtContext* ctx, int off) {
    Lz4MtMemIo* io = mem(ctx);
    const int64_t p = (int64_t)io->inPos + off;
    if (p < 0) return -1;
    io->inPos = (uint64_t)p > io->inSize ? io->inSize : (uint64_t)p;
    io->eof = 0;
    return 0;
}
int mem_eof(const Lz4MtContext* ctx) { return mem(ctx)->eof; }
int mem_write(const Lz4MtContext* ctx, const void* src, int n) {
    Lz4MtMemIo* io = static_cast<Lz4MtMemIo*>(ctx->writeCtx);
    if (n < 0) return 0;
    if (io->out) {
        if (io->outPos + (uint64_t)n > io->outCap) return 0;
        par_copy(io->out + io->outPos, src, (size_t)n);
    }
    io->outPos += (uint64_t)n;
    return n;
}
}  // namespace

extern "C" void lz4mtMemBind(Lz4MtContext* ctx, Lz4MtMemIo* io) {
    ctx->readCtx = io;
    ctx->writeCtx = io;
    ctx->read = mem_read;
    ctx->readSkippable = mem_skip;
    ctx->readSeek = mem_seek;
    ctx->readEof = mem_eof;
    ctx->write = mem_write;
}
