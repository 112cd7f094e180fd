/*
 * lz4mt.h — drop-in C ABI of the MI355X LZ4 frame codec.
 *
 * Names, enum values and struct layouts are those of the reference
 * public header (t-mat/lz4mt src/lz4mt.h:1-170), so code written against
 * the reference links against liblz4mt_amd.so unchanged.  Verified x86-64
 * layout: Lz4MtContext = 96 B, Lz4MtStreamDescriptor = 32 B, enums 4 B
 * (tests/test_abi.py checks every offset).
 *
 * Differences from the reference header, all ABI-neutral:
 *   - `struct Lz4MtContext` is forward-declared so the header is valid C
 *     (the reference first names it inside the callback parameter lists,
 *     src/lz4mt.h:14-39);
 *   - one extra mode bit, LZ4MT_MODE_DEVICE, selects the batched HIP
 *     frame engine (see lz4mt_hip.h); PARALLEL (0) and SEQUENTIAL (1)
 *     keep their values (src/lz4mt.h:61-66).
 */
#ifndef LZ4MT_AMD_LZ4MT_H
#define LZ4MT_AMD_LZ4MT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct Lz4MtContext;

/* I/O plugin points (reference src/lz4mt.h:14-39). */
/* read: returns bytes read into dst, 0 at end of input. */
typedef int (*Lz4MtRead)(struct Lz4MtContext* ctx, void* dst, int dstSize);
/* readSeek: relative seek of the input, 0 on success. */
typedef int (*Lz4MtReadSeek)(const struct Lz4MtContext* ctx, int offset);
/* readEof: nonzero once the input is exhausted. */
typedef int (*Lz4MtReadEof)(const struct Lz4MtContext* ctx);
/* readSkippable: skip `size` bytes of a skippable frame, 0 on success. */
typedef int (*Lz4MtReadSkippable)(const struct Lz4MtContext* ctx,
                                  uint32_t magicNumber, size_t size);
/* write: must return srcSize, anything else is an error. */
typedef int (*Lz4MtWrite)(const struct Lz4MtContext* ctx, const void* src,
                          int srcSize);

/* Block codec operator API (reference src/lz4mt.h:41-58).
 * compress: > 0 = compressed size; <= 0 = store the block raw.
 * decompress: >= 0 = decoded size; < 0 = malformed block. */
typedef int (*Lz4MtCompress)(const char* src, char* dst, int isize,
                             int maxOutputSize, int compressionLevel);
typedef int (*Lz4MtCompressBound)(int isize);
typedef int (*Lz4MtDecompress)(const char* src, char* dst, int isize,
                               int maxOutputSize);

enum Lz4MtMode {
    LZ4MT_MODE_DEFAULT    = 0,
    LZ4MT_MODE_PARALLEL   = 0,        /* host worker pool, callbacks per block */
    LZ4MT_MODE_SEQUENTIAL = 1 << 0,   /* one block at a time on the caller thread */
    LZ4MT_MODE_DEVICE     = 1 << 1    /* extension: batched MI355X frame engine */
};
typedef enum Lz4MtMode Lz4MtMode;

/* Result codes, in the reference's declaration order (src/lz4mt.h:69-98). */
enum Lz4MtResult {
    LZ4MT_RESULT_OK = 0,
    LZ4MT_RESULT_ERROR,                                       /*  1 */
    LZ4MT_RESULT_INVALID_MAGIC_NUMBER,                        /*  2 */
    LZ4MT_RESULT_INVALID_HEADER,                              /*  3 */
    LZ4MT_RESULT_PRESET_DICTIONARY_IS_NOT_SUPPORTED_YET,      /*  4 */
    LZ4MT_RESULT_BLOCK_DEPENDENCE_IS_NOT_SUPPORTED_YET,       /*  5 */
    LZ4MT_RESULT_INVALID_VERSION,                             /*  6 */
    LZ4MT_RESULT_INVALID_HEADER_CHECKSUM,                     /*  7 */
    LZ4MT_RESULT_INVALID_BLOCK_MAXIMUM_SIZE,                  /*  8 */
    LZ4MT_RESULT_CANNOT_WRITE_HEADER,                         /*  9 */
    LZ4MT_RESULT_CANNOT_WRITE_EOS,                            /* 10 */
    LZ4MT_RESULT_CANNOT_WRITE_STREAM_CHECKSUM,                /* 11 */
    LZ4MT_RESULT_CANNOT_READ_BLOCK_SIZE,                      /* 12 */
    LZ4MT_RESULT_CANNOT_READ_BLOCK_DATA,                      /* 13 */
    LZ4MT_RESULT_CANNOT_READ_BLOCK_CHECKSUM,                  /* 14 */
    LZ4MT_RESULT_CANNOT_READ_STREAM_CHECKSUM,                 /* 15 */
    LZ4MT_RESULT_BLOCK_CHECKSUM_MISMATCH,                     /* 16 */
    LZ4MT_RESULT_STREAM_CHECKSUM_MISMATCH,                    /* 17 */
    LZ4MT_RESULT_DECOMPRESS_FAIL,                             /* 18 */
    LZ4MT_RESULT_BAD_ARG,                                     /* 19 */
    LZ4MT_RESULT_INVALID_BLOCK_SIZE,                          /* 20 */
    LZ4MT_RESULT_INVALID_HEADER_RESERVED1,                    /* 21 */
    LZ4MT_RESULT_INVALID_HEADER_RESERVED2,                    /* 22 */
    LZ4MT_RESULT_INVALID_HEADER_RESERVED3,                    /* 23 */
    LZ4MT_RESULT_INVALID_HEADER_SKIPPABLE_SIZE_UNREADABLE,    /* 24 */
    LZ4MT_RESULT_INVALID_HEADER_CANNOT_SKIP_SKIPPABLE_AREA,   /* 25 */
    LZ4MT_RESULT_CANNOT_WRITE_DATA_BLOCK,                     /* 26 */
    LZ4MT_RESULT_CANNOT_WRITE_DECODED_BLOCK                   /* 27 */
};
typedef enum Lz4MtResult Lz4MtResult;

/* FLG byte, one char per bit field (reference src/lz4mt.h:102-111). */
struct Lz4MtFlg {
    char presetDictionary;   /* bit 0 */
    char reserved1;          /* bit 1 */
    char streamChecksum;     /* bit 2 */
    char streamSize;         /* bit 3 */
    char blockChecksum;      /* bit 4 */
    char blockIndependence;  /* bit 5 */
    char versionNumber;      /* bits 6-7 */
};
typedef struct Lz4MtFlg Lz4MtFlg;

/* BD byte (reference src/lz4mt.h:114-119). */
struct Lz4MtBd {
    char reserved3;          /* bits 0-3 */
    char blockMaximumSize;   /* bits 4-6: 4..7 => 64 KiB .. 4 MiB */
    char reserved2;          /* bit 7 */
};
typedef struct Lz4MtBd Lz4MtBd;

struct Lz4MtStreamDescriptor {
    Lz4MtFlg flg;            /* offset 0 */
    Lz4MtBd  bd;             /* offset 7 */
    uint64_t streamSize;     /* offset 16 */
    uint32_t dictId;         /* offset 24 */
};
typedef struct Lz4MtStreamDescriptor Lz4MtStreamDescriptor;

struct Lz4MtContext {
    Lz4MtResult        result;           /* offset  0 */
    void*              readCtx;          /* offset  8 */
    Lz4MtRead          read;             /* offset 16 */
    Lz4MtReadSkippable readSkippable;    /* offset 24 */
    Lz4MtReadSeek      readSeek;         /* offset 32 */
    Lz4MtReadEof       readEof;          /* offset 40 */
    void*              writeCtx;         /* offset 48 */
    Lz4MtWrite         write;            /* offset 56 */
    Lz4MtCompress      compress;         /* offset 64 */
    Lz4MtCompressBound compressBound;    /* offset 72 */
    Lz4MtDecompress    decompress;       /* offset 80 */
    Lz4MtMode          mode;             /* offset 88 */
    int                compressionLevel; /* offset 92 */
};
typedef struct Lz4MtContext Lz4MtContext;

/* Reference src/lz4mt.cpp:851-871: all callbacks null, PARALLEL, level 0. */
Lz4MtContext lz4mtInitContext(void);
/* Reference src/lz4mt.cpp:874-895: stream checksum on, independent blocks,
 * version 1, block maximum size id 7 (4 MiB). */
Lz4MtStreamDescriptor lz4mtInitStreamDescriptor(void);
/* Reference src/lz4mt_result.cpp:4-89. */
const char* lz4mtResultToString(Lz4MtResult result);
/* Reference src/lz4mt_result.cpp:92-270. */
int lz4mtResultToLz4cExitCode(Lz4MtResult result);
/* Reference src/lz4mt.cpp:898-935. */
Lz4MtResult lz4mtCompress(Lz4MtContext* ctx, const Lz4MtStreamDescriptor* sd);
/* Reference src/lz4mt.cpp:938-1011; `sd` receives each frame's descriptor. */
Lz4MtResult lz4mtDecompress(Lz4MtContext* ctx, Lz4MtStreamDescriptor* sd);

#ifdef __cplusplus
}
#endif

#endif /* LZ4MT_AMD_LZ4MT_H */
