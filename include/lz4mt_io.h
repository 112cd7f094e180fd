/*
 * lz4mt_io.h — I/O callback adapters for Lz4MtContext (liblz4mt_amd.so).
 *
 * FILE*-backed callbacks: the C-ABI counterpart of the reference's
 * Lz4Mt::Cstdio namespace (src/lz4mt_io_cstdio.h:1-33,
 * src/lz4mt_io_cstdio.cpp:75-175), with the same conventions: the file name
 * "stdin"/"stdout" selects the standard streams, and a null sink is marked
 * by writeCtx == ctx (src/lz4mt_io_cstdio.cpp:19-21, 86-97, 147-156).
 *
 * Memory-backed callbacks (extension): bind a caller-owned Lz4MtMemIo as
 * both read and write context; reads follow fread/feof semantics (EOF is
 * reported after a read came up short), writes fail once outCap is full.
 */
#ifndef LZ4MT_AMD_LZ4MT_IO_H
#define LZ4MT_AMD_LZ4MT_IO_H

#include "lz4mt.h"

#ifdef __cplusplus
extern "C" {
#endif

int lz4mtIoOpenIstream(Lz4MtContext* ctx, const char* filename);
int lz4mtIoOpenOstream(Lz4MtContext* ctx, const char* filename, int nullWrite);
void lz4mtIoCloseIstream(Lz4MtContext* ctx);
void lz4mtIoCloseOstream(Lz4MtContext* ctx);
/* Installs the five FILE* callbacks (read, readSkippable, readSeek, readEof, write). */
void lz4mtIoBindCstdio(Lz4MtContext* ctx);
int lz4mtIoRead(Lz4MtContext* ctx, void* dst, int dstSize);
int lz4mtIoReadSkippable(const Lz4MtContext* ctx, uint32_t magicNumber, size_t size);
int lz4mtIoReadSeek(const Lz4MtContext* ctx, int offset);
int lz4mtIoReadEof(const Lz4MtContext* ctx);
int lz4mtIoWrite(const Lz4MtContext* ctx, const void* src, int srcSize);
uint64_t lz4mtIoGetFilesize(const char* filename);

typedef struct Lz4MtMemIo {
    const uint8_t* in;   /* input bytes */
    uint64_t inSize;
    uint64_t inPos;
    int      eof;        /* set once a read came up short */
    uint8_t* out;        /* output buffer (NULL: count only, a null sink) */
    uint64_t outCap;
    uint64_t outPos;
} Lz4MtMemIo;

/* Points ctx's callbacks at `io` (readCtx = writeCtx = io). */
void lz4mtMemBind(Lz4MtContext* ctx, Lz4MtMemIo* io);

#ifdef __cplusplus
}
#endif
#endif
