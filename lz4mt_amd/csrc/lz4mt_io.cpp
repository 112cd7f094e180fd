// lz4mt_io.cpp — FILE* and memory callbacks for Lz4MtContext.
// FILE* side mirrors reference src/lz4mt_io_cstdio.cpp:75-175 (fread/fwrite/
// fseek/feof; "stdin"/"stdout" names; null sink = writeCtx == ctx).
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>

#include "../../include/lz4mt_io.h"

namespace {
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
    return fp ? (int)fread(dst, 1, (size_t)dstSize, fp) : 0;
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
    return fp ? (int)fwrite(src, 1, (size_t)srcSize, fp) : 0;
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
    memcpy(dst, io->in + io->inPos, got);
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
        memcpy(io->out + io->outPos, src, (size_t)n);
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
