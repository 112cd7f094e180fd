/*
 * lz4_oracle.c — CPU restatement of the lz4mt hot path (TEST INFRASTRUCTURE
 * ONLY; see lz4_oracle.h).  Plain C11 + pthreads, built by oracle/Makefile
 * into oracle/liblz4mt_oracle.so.
 *
 * Citations: "ref" = /root/reference (t-mat/lz4mt); "lz4 1.9.3" = the
 * un-vendored lz4 submodule's algorithm at the version pinned by this image
 * (liblz4.so.1.9.3), restated from its published source structure.
 */
#include "lz4_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ===================================================================== */
/* XXH32 (xxhash; seed 0 in lz4mt, ref src/lz4mt.cpp:23, 359, 399, 414)   */
/* ===================================================================== */
#define P1 2654435761u
#define P2 2246822519u
#define P3 3266489917u
#define P4 668265263u
#define P5 374761393u

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
static inline void wr32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static inline uint32_t xround(uint32_t acc, uint32_t w) { return rotl32(acc + w * P2, 13) * P1; }

static uint32_t xxh32_finish(uint32_t h, const uint8_t* p, size_t len) {
    while (len >= 4) { h = rotl32(h + rd32(p) * P3, 17) * P4; p += 4; len -= 4; }
    while (len > 0) { h = rotl32(h + (*p) * P5, 11) * P1; p++; len--; }
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

uint32_t orc_xxh32(const void* in, size_t len, uint32_t seed) {
    const uint8_t* p = (const uint8_t*)in;
    size_t rem = len;
    uint32_t h;
    if (len >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        while (rem >= 16) {
            v1 = xround(v1, rd32(p)); v2 = xround(v2, rd32(p + 4));
            v3 = xround(v3, rd32(p + 8)); v4 = xround(v4, rd32(p + 12));
            p += 16; rem -= 16;
        }
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    return xxh32_finish(h, p, rem);
}

void orc_xxh32_reset(orc_xxh32_state* s, uint32_t seed) {
    memset(s, 0, sizeof(*s));
    s->seed = seed;
    s->v[0] = seed + P1 + P2; s->v[1] = seed + P2; s->v[2] = seed; s->v[3] = seed - P1;
}

void orc_xxh32_update(orc_xxh32_state* s, const void* in, size_t len) {
    const uint8_t* p = (const uint8_t*)in;
    s->total += len;
    if (s->memSize + len < 16) { memcpy(s->mem + s->memSize, p, len); s->memSize += (uint32_t)len; return; }
    if (s->memSize) {
        size_t fill = 16 - s->memSize;
        memcpy(s->mem + s->memSize, p, fill);
        for (int i = 0; i < 4; i++) s->v[i] = xround(s->v[i], rd32(s->mem + 4 * i));
        p += fill; len -= fill; s->memSize = 0;
    }
    {   /* lanes in locals: s->v stores would alias the byte pointer */
        uint32_t v1 = s->v[0], v2 = s->v[1], v3 = s->v[2], v4 = s->v[3];
        while (len >= 16) {
            v1 = xround(v1, rd32(p)); v2 = xround(v2, rd32(p + 4));
            v3 = xround(v3, rd32(p + 8)); v4 = xround(v4, rd32(p + 12));
            p += 16; len -= 16;
        }
        s->v[0] = v1; s->v[1] = v2; s->v[2] = v3; s->v[3] = v4;
    }
    memcpy(s->mem, p, len); s->memSize = (uint32_t)len;
}

uint32_t orc_xxh32_digest(const orc_xxh32_state* s) {
    uint32_t h;
    if (s->total >= 16)
        h = rotl32(s->v[0], 1) + rotl32(s->v[1], 7) + rotl32(s->v[2], 12) + rotl32(s->v[3], 18);
    else
        h = s->seed + P5;
    h += (uint32_t)s->total;
    return xxh32_finish(h, s->mem, s->memSize);
}

/* ===================================================================== */
/* LZ4 1.9.3 fast compressor, acceleration 1.         */
/* lz4mt calls it as LZ4_compress_limitedOutput(src, dst, n, n)          */
/* (ref src/main.cpp:749-751; src/lz4mt.cpp:248-250, 391).               */
/* ===================================================================== */
#define MINMATCH 4
#define LASTLITERALS 5
#define MFLIMIT 12
#define MIN_LENGTH 13
#define DIST_MAX 65535u
#define LIMIT_64K 65547
#define MAX_INPUT 0x7E000000

int orc_lz4_compress_bound(int isize) {
    return ((unsigned)isize > (unsigned)MAX_INPUT) ? 0 : isize + isize / 255 + 16;
}

/* byU16 (n < 65547): hash4, 13-bit; byU32: hash5, 12-bit. */
static inline uint32_t hpos(const uint8_t* p, int u16) {
    if (u16) return (rd32(p) * 2654435761u) >> 19;
    return (uint32_t)(((rd64(p) << 24) * 889523592379ull) >> 52);
}

int orc_lz4_compress(const uint8_t* src, uint8_t* dst, int n, int cap) {
    if ((unsigned)n > (unsigned)MAX_INPUT) return 0;
    const int limited = cap < orc_lz4_compress_bound(n);
    if (n == 0) {
        if (limited && cap <= 0) return 0;
        dst[0] = 0;
        return 1;
    }
    const int u16 = n < LIMIT_64K;
    uint32_t* T = (uint32_t*)calloc(8192, sizeof(uint32_t));
    const uint32_t mflimitP1 = (uint32_t)n - MFLIMIT + 1;
    const uint32_t matchlimit = (uint32_t)n - LASTLITERALS;
    uint32_t anchor = 0, ip = 0, cand = 0, fh, token;
    size_t op = 0;
    int result = 0;

    if (n < MIN_LENGTH) goto last_literals;
    T[hpos(src, u16)] = 0;
    ip = 1;
    fh = hpos(src + 1, u16);

    for (;;) {
        /* Find a match: probe schedule of step 1 for 64 probes, then +1
         * every 64 probes (searchMatchNb >> skipTrigger). */
        {
            uint32_t fip = ip, step = 1, nb = 64;
            for (;;) {
                const uint32_t h = fh, cur = fip;
                cand = T[h];
                ip = fip;
                fip += step;
                step = nb++ >> 6;
                if (fip > mflimitP1) goto last_literals;
                fh = hpos(src + fip, u16);
                T[h] = cur;
                if (!u16 && cand + DIST_MAX < cur) continue;
                if (rd32(src + cand) == rd32(src + ip)) break;
            }
        }
        /* Catch up (index 0 of a fresh table is a valid candidate). */
        while (ip > anchor && cand > 0 && src[ip - 1] == src[cand - 1]) { ip--; cand--; }
        {
            const uint32_t lit = ip - anchor;
            token = (uint32_t)op++;
            if (limited && op + lit + 8 + lit / 255 > (size_t)cap) goto fail;
            if (lit >= 15) {
                uint32_t len = lit - 15;
                dst[token] = 15 << 4;
                for (; len >= 255; len -= 255) dst[op++] = 255;
                dst[op++] = (uint8_t)len;
            } else {
                dst[token] = (uint8_t)(lit << 4);
            }
            memcpy(dst + op, src + anchor, lit);
            op += lit;
        }
    next_match:
        {
            const uint32_t off = ip - cand;
            dst[op++] = (uint8_t)off;
            dst[op++] = (uint8_t)(off >> 8);
            uint32_t mc = 0;
            while (ip + MINMATCH + mc < matchlimit && src[ip + MINMATCH + mc] == src[cand + MINMATCH + mc]) mc++;
            ip += mc + MINMATCH;
            if (limited && op + 6 + (mc + 240) / 255 > (size_t)cap) goto fail;
            if (mc >= 15) {
                dst[token] += 15;
                mc -= 15;
                for (; mc >= 255; mc -= 255) dst[op++] = 255;
                dst[op++] = (uint8_t)mc;
            } else {
                dst[token] += (uint8_t)mc;
            }
        }
        anchor = ip;
        if (ip >= mflimitP1) break;
        T[hpos(src + ip - 2, u16)] = ip - 2;
        {
            const uint32_t h = hpos(src + ip, u16);
            cand = T[h];
            T[h] = ip;
            if ((u16 || cand + DIST_MAX >= ip) && rd32(src + cand) == rd32(src + ip)) {
                token = (uint32_t)op++;
                dst[token] = 0;
                goto next_match;
            }
        }
        ip++;
        fh = hpos(src + ip, u16);
    }

last_literals:
    {
        const size_t run = (size_t)n - anchor;
        if (limited && op + run + 1 + (run + 240) / 255 > (size_t)cap) goto fail;
        if (run >= 15) {
            size_t acc = run - 15;
            dst[op++] = 15 << 4;
            for (; acc >= 255; acc -= 255) dst[op++] = 255;
            dst[op++] = (uint8_t)acc;
        } else {
            dst[op++] = (uint8_t)(run << 4);
        }
        memcpy(dst + op, src + anchor, run);
        op += run;
    }
    result = (int)op;
fail:
    free(T);
    return result;
}

/* ===================================================================== */
/* LZ4 1.9.3 LZ4_decompress_safe (endOnInputSize, full block, noDict,    */
/* LZ4_FAST_DEC_LOOP=1 as built for x86-64).  lz4mt calls it with        */
/* cap = blockMax (ref src/lz4mt.cpp:644-646; src/main.cpp:774).         */
/* Positions are signed byte offsets so pointer-before-buffer compares   */
/* behave like the C original; copies are exact LZ77 (the original's     */
/* wild-copy overrun bytes lie past the returned size).                  */
/* ===================================================================== */
typedef long long sll;

static void lz77_copy(uint8_t* dst, sll op, sll match, sll len) {
    if (match == op) { memset(dst + op, 0, (size_t)len); return; } /* offset 0 => zeros */
    uint8_t* d = dst + op;
    const uint8_t* s = dst + match;
    const sll off = op - match;
    if (off >= len) { memcpy(d, s, (size_t)len); return; }   /* no overlap */
    sll i = 0;
    if (off >= 8) /* 8-byte pieces: each piece's source lies before its target */
        for (; i + 8 <= len; i += 8) memcpy(d + i, s + i, 8);
    for (; i < len; i++) d[i] = s[i];                         /* short-period runs */
}

/* read_variable_length(): returns -1 initial error, -2 loop error. */
static int rvl(const uint8_t* src, sll srcSize, sll* ip, sll lencheck, int loopCheck, int initialCheck,
               size_t* length) {
    *length = 0;
    if (initialCheck && *ip >= lencheck) return -1;
    unsigned s;
    do {
        s = (*ip >= 0 && *ip < srcSize) ? src[*ip] : 0;
        (*ip)++;
        *length += s;
        if (loopCheck && *ip >= lencheck) return -2;
    } while (s == 255);
    return 0;
}

static inline unsigned in8(const uint8_t* src, sll n, sll i) { return (i >= 0 && i < n) ? src[i] : 0; }

/* lowP = lowest output position a match may read: 0 for
 * LZ4_decompress_safe (lowPrefix = dst), -65536 for
 * LZ4_decompress_safe_withPrefix64k (lowPrefix = dst - 64 KB; then no offset
 * can point before it, and the fast-copy test `dict == withPrefix64k ||
 * match >= lowPrefix` is the same comparison). */
static int decompress_generic(const uint8_t* src, uint8_t* dst, int srcSize, int outputSize, sll lowP) {
    if (src == NULL) return -1;
    const sll N = srcSize;
    sll ip = 0, op = 0, cpy, match;
    const sll iend = N, oend = outputSize;
    const sll shortiend = iend - 14 - 2, shortoend = oend - 14 - 18;
    unsigned token;
    size_t length, offset;
    int e;

    if (outputSize == 0) return (srcSize == 1 && src[0] == 0) ? 0 : -1;
    if (srcSize == 0) return -1;

    if (oend - op < 64) goto safe_decode;
    for (;;) { /* fast loop */
        token = in8(src, N, ip++);
        length = token >> 4;
        if (length == 15) {
            size_t ext;
            e = rvl(src, N, &ip, iend - 15, 1, 1, &ext);
            length += ext;
            if (e == -1) goto output_error;
            cpy = op + (sll)length;
            if (cpy > oend - 32 || ip + (sll)length > iend - 32) goto safe_literal_copy;
            memcpy(dst + op, src + ip, length);
            ip += (sll)length; op = cpy;
        } else {
            cpy = op + (sll)length;
            if (ip > iend - 17) goto safe_literal_copy;
            memcpy(dst + op, src + ip, length);
            ip += (sll)length; op = cpy;
        }
        offset = in8(src, N, ip) | (in8(src, N, ip + 1) << 8);
        ip += 2;
        match = op - (sll)offset;
        length = token & 15;
        if (length == 15) {
            size_t ext;
            if (match < lowP) goto output_error;
            e = rvl(src, N, &ip, iend - LASTLITERALS + 1, 1, 0, &ext);
            length += ext;
            if (e != 0) goto output_error;
            length += MINMATCH;
            if (op + (sll)length >= oend - 64) goto safe_match_copy;
        } else {
            length += MINMATCH;
            if (op + (sll)length >= oend - 64) goto safe_match_copy;
            if (match >= lowP && offset >= 8) {
                lz77_copy(dst, op, match, (sll)length);
                op += (sll)length;
                continue;
            }
        }
        if (match < lowP) goto output_error;
        cpy = op + (sll)length;
        lz77_copy(dst, op, match, (sll)length);
        op = cpy;
    }

safe_decode:
    for (;;) {
        token = in8(src, N, ip++);
        length = token >> 4;
        if (length != 15 && ip < shortiend && op <= shortoend) {
            memcpy(dst + op, src + ip, length);
            op += (sll)length; ip += (sll)length;
            length = token & 15;
            offset = in8(src, N, ip) | (in8(src, N, ip + 1) << 8);
            ip += 2;
            match = op - (sll)offset;
            if (length != 15 && offset >= 8 && match >= lowP) {
                lz77_copy(dst, op, match, (sll)length + MINMATCH);
                op += (sll)length + MINMATCH;
                continue;
            }
            goto copy_match;
        }
        if (length == 15) {
            size_t ext;
            e = rvl(src, N, &ip, iend - 15, 1, 1, &ext);
            length += ext;
            if (e == -1) goto output_error;
        }
        cpy = op + (sll)length;
    safe_literal_copy:
        if (cpy > oend - MFLIMIT || ip + (sll)length > iend - (2 + 1 + LASTLITERALS)) {
            /* must be the last sequence */
            if (ip + (sll)length != iend || cpy > oend) goto output_error;
            memmove(dst + op, src + ip, length);
            ip += (sll)length;
            op += (sll)length;
            break;
        }
        memcpy(dst + op, src + ip, length);
        ip += (sll)length; op = cpy;

        offset = in8(src, N, ip) | (in8(src, N, ip + 1) << 8);
        ip += 2;
        match = op - (sll)offset;
        length = token & 15;
    copy_match:
        if (length == 15) {
            size_t ext;
            e = rvl(src, N, &ip, iend - LASTLITERALS + 1, 1, 0, &ext);
            length += ext;
            if (e != 0) goto output_error;
        }
        length += MINMATCH;
    safe_match_copy:
        if (match < lowP) goto output_error;
        cpy = op + (sll)length;
        if (cpy > oend - 12 && cpy > oend - LASTLITERALS) goto output_error;
        lz77_copy(dst, op, match, (sll)length);
        op = cpy;
    }
    return (int)op;

output_error:
    return (int)(-ip) - 1;
}

int orc_lz4_decompress_safe(const uint8_t* src, uint8_t* dst, int srcSize, int outputSize) {
    return decompress_generic(src, dst, srcSize, outputSize, 0);
}

/* LZ4_decompress_safe_withPrefix64k (lz4 1.9.3): the 64 KiB before dst are
 * readable history (ref src/lz4mt.cpp:813-818, block-dependent frames). */
int orc_lz4_decompress_safe_prefix64k(const uint8_t* src, uint8_t* dst, int srcSize, int outputSize) {
    return decompress_generic(src, dst, srcSize, outputSize, -65536);
}

/* ===================================================================== */
/* Minimal parallel-for over pthreads                                    */
/* ===================================================================== */
typedef void (*pf_fn)(void* arg, size_t i);
typedef struct { pf_fn fn; void* arg; size_t n; size_t next; pthread_mutex_t mu; } pf_ctx;

static void* pf_worker(void* p) {
    pf_ctx* c = (pf_ctx*)p;
    for (;;) {
        pthread_mutex_lock(&c->mu);
        size_t i = c->next++;
        pthread_mutex_unlock(&c->mu);
        if (i >= c->n) return NULL;
        c->fn(c->arg, i);
    }
}

static void parallel_for(size_t n, int nthreads, pf_fn fn, void* arg) {
    if (nthreads <= 1 || n <= 1) { for (size_t i = 0; i < n; i++) fn(arg, i); return; }
    pf_ctx c = { fn, arg, n, 0, PTHREAD_MUTEX_INITIALIZER };
    pthread_t th[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, pf_worker, &c);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* ===================================================================== */
/* lz4mt frame writer (ref src/lz4mt.cpp:335-369 makeHeader,             */
/* 372-457 compress(), 898-935 lz4mtCompress).                           */
/* ===================================================================== */
#define MAGIC 0x184D2204u
#define SKIP_MIN 0x184D2A50u
#define SKIP_MAX 0x184D2A5Fu
#define RAW_BIT 0x80000000u

static size_t block_max(int id) { return (size_t)1 << (8 + 2 * id); }

size_t orc_frame_bound(size_t n, const orc_frame_params* p) {
    const size_t bm = block_max(p->blockMaxId);
    const size_t nb = (n + bm - 1) / bm;
    return 19 + n + nb * 8 + 8;
}

static size_t write_header(uint8_t* d, const orc_frame_params* p) {
    size_t o = 0;
    wr32(d, MAGIC); o = 4;
    const uint8_t flg = (uint8_t)((1u << 6) | (1u << 5) | ((p->blockChecksum & 1) << 4) |
                                  ((p->streamSizeFlag & 1) << 3) | ((p->streamChecksum & 1) << 2));
    d[o++] = flg;
    d[o++] = (uint8_t)((p->blockMaxId & 7) << 4);
    if (p->streamSizeFlag) { wr32(d + o, (uint32_t)p->streamSize); wr32(d + o + 4, (uint32_t)(p->streamSize >> 32)); o += 8; }
    d[o] = (uint8_t)((orc_xxh32(d + 4, o - 4, 0) >> 8) & 0xFF);
    return o + 1;
}

typedef struct { const uint8_t* src; size_t n, bm; uint8_t* tmp; int* csz; } cjob;

static void cjob_fn(void* a, size_t i) {
    cjob* j = (cjob*)a;
    size_t off = i * j->bm, len = j->n - off < j->bm ? j->n - off : j->bm;
    j->csz[i] = orc_lz4_compress(j->src + off, j->tmp + off, (int)len, (int)len);
}

size_t orc_frame_compress(const uint8_t* src, size_t n, uint8_t* dst, const orc_frame_params* p, int nthreads) {
    if (p->blockMaxId < 4 || p->blockMaxId > 7) return 0;
    const size_t bm = block_max(p->blockMaxId);
    const size_t nb = (n + bm - 1) / bm;
    size_t o = write_header(dst, p);
    cjob j = { src, n, bm, (uint8_t*)malloc(n ? n : 1), (int*)malloc((nb ? nb : 1) * sizeof(int)) };
    parallel_for(nb, nthreads, cjob_fn, &j);
    for (size_t i = 0; i < nb; i++) {
        const size_t off = i * bm, len = n - off < bm ? n - off : bm;
        const uint8_t* stored;
        size_t slen;
        if (j.csz[i] <= 0) { /* incompressible: raw, size | bit 31 (ref src/lz4mt.cpp:392-394,418-420) */
            wr32(dst + o, (uint32_t)len | RAW_BIT);
            stored = src + off; slen = len;
        } else {
            wr32(dst + o, (uint32_t)j.csz[i]);
            stored = j.tmp + off; slen = (size_t)j.csz[i];
        }
        o += 4;
        memcpy(dst + o, stored, slen);
        o += slen;
        if (p->blockChecksum) { wr32(dst + o, orc_xxh32(stored, slen, 0)); o += 4; }
    }
    wr32(dst + o, 0); o += 4; /* EOS (ref src/lz4mt.cpp:923) */
    if (p->streamChecksum) { wr32(dst + o, orc_xxh32(src, n, 0)); o += 4; }
    free(j.tmp); free(j.csz);
    return o;
}

/* ===================================================================== */
/* lz4mt frame reader (ref src/lz4mt.cpp:541-590 readHeader, 593-734     */
/* decompress(), 938-1011 lz4mtDecompress) over a memory stream with     */
/* FILE-like end-of-file semantics (ref src/lz4mt_io_cstdio.cpp:112-145). */
/* Deterministic: blocks of one frame are checked in order, so the first */
/* failing block's code is the result (the reference's first-error-wins  */
/* is racy in PARALLEL mode).  Two reference bugs are NOT reproduced:    */
/* trailing non-magic bytes end the stream with OK instead of spinning   */
/* (ref 971-979), and skippable frames are skipped instead of calling a  */
/* null readSkippable (ref src/main.cpp:767-775).                        */
/* ===================================================================== */
enum { R_OK = 0, R_ERROR = 1, R_MAGIC = 2, R_HEADER = 3, R_DICT = 4, R_DEP = 5, R_VERSION = 6, R_HC = 7,
       R_BMAX = 8, R_RD_BSIZE = 12, R_RD_BDATA = 13, R_RD_BCK = 14, R_RD_SCK = 15, R_BCK = 16, R_SCK = 17,
       R_DECOMP = 18, R_BSIZE = 20, R_RES1 = 21, R_RES2 = 22, R_RES3 = 23, R_SKIP_SIZE = 24, R_SKIP = 25 };

typedef struct { const uint8_t* p; size_t n, pos; int eof; } mstream;

static size_t ms_read(mstream* s, void* d, size_t k) {
    size_t rem = s->n - s->pos, got = k < rem ? k : rem;
    if (k > rem) s->eof = 1;
    memcpy(d, s->p + s->pos, got);
    s->pos += got;
    return got;
}

typedef struct { const uint8_t* src; int len; uint8_t* out; int raw; uint32_t bck; int hasBck; int bm; int res; int dsz; } djob;
static void djob_fn(void* a, size_t i) {
    djob* j = ((djob*)a) + i;
    if (j->raw) { memcpy(j->out, j->src, (size_t)j->len); j->dsz = j->len; j->res = R_OK; }
    else {
        j->dsz = orc_lz4_decompress_safe(j->src, j->out, j->len, j->bm);
        j->res = j->dsz < 0 ? R_DECOMP : R_OK;
    }
    if (j->res == R_OK && j->hasBck && orc_xxh32(j->src, (size_t)j->len, 0) != j->bck) j->res = R_BCK;
}

int orc_frame_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t outCap, size_t* outSize, int nthreads) {
    mstream s = { src, n, 0, 0 };
    size_t out = 0;
    int result = R_OK, seen = 0;
    uint8_t b[16];
    *outSize = 0;
    while (result == R_OK && !s.eof) {
        if (ms_read(&s, b, 4) != 4) { result = s.eof ? R_OK : R_HEADER; break; }
        const uint32_t magic = rd32(b);
        if (magic != MAGIC) {
            if (magic >= SKIP_MIN && magic <= SKIP_MAX) {
                if (ms_read(&s, b, 4) != 4) { result = R_SKIP_SIZE; break; }
                const size_t sk = rd32(b), rem = s.n - s.pos;
                s.pos += sk < rem ? sk : rem; /* fseek past EOF succeeds */
                continue;
            }
            result = seen ? R_OK : R_MAGIC;
            break;
        }
        seen = 1;
        /* readHeader */
        if (ms_read(&s, b, 2) != 2) { result = R_HEADER; break; }
        const uint8_t flg = b[0], bd = b[1];
        if (((flg >> 6) & 3) != 1) { result = R_VERSION; break; }
        if (flg & 1) { result = R_DICT; break; }
        if ((flg >> 1) & 1) { result = R_RES1; break; }
        const int bid = (bd >> 4) & 7;
        if (bid < 4 || bid > 7) { result = R_BMAX; break; }
        if (bd & 15) { result = R_RES3; break; }
        if (bd >> 7) { result = R_RES2; break; }
        const int hasSize = (flg >> 3) & 1, sck = (flg >> 2) & 1, bck = (flg >> 4) & 1, indep = (flg >> 5) & 1;
        const size_t nex = (hasSize ? 8 : 0) + 1;
        if (ms_read(&s, b + 2, nex) != nex) { result = R_HEADER; break; }
        if ((uint8_t)((orc_xxh32(b, 2 + (hasSize ? 8 : 0), 0) >> 8) & 0xFF) != b[2 + (hasSize ? 8 : 0)]) {
            result = R_HC; break;
        }
        const size_t bm = block_max(bid);
        /* scan blocks */
        size_t cap = 64, nb = 0;
        djob* jobs = (djob*)malloc(cap * sizeof(djob));
        int eos = 0;
        const size_t frameOut = out;
        while (!eos && result == R_OK && !s.eof) {
            if (ms_read(&s, b, 4) != 4) { result = R_RD_BSIZE; break; }
            const uint32_t bits = rd32(b);
            if (bits == 0) { eos = 1; break; }
            const size_t len = bits & 0x7FFFFFFFu;
            if (len > bm) { result = R_BSIZE; break; }
            if (s.n - s.pos < len) { s.pos = s.n; s.eof = 1; result = R_RD_BDATA; break; }
            const uint8_t* bp = s.p + s.pos;
            s.pos += len;
            uint32_t ck = 0;
            if (bck) {
                if (ms_read(&s, b, 4) != 4) { result = R_RD_BCK; break; }
                ck = rd32(b);
            }
            /* a compressed block decodes into a full blockMax slot (cap = blockMax) */
            if (out + ((bits & RAW_BIT) ? len : bm) > outCap) { result = R_ERROR; break; }
            if (nb == cap) { cap *= 2; jobs = (djob*)realloc(jobs, cap * sizeof(djob)); }
            djob* j = &jobs[nb++];
            j->src = bp; j->len = (int)len; j->out = dst + out; j->raw = (bits & RAW_BIT) != 0;
            j->bck = ck; j->hasBck = bck; j->bm = (int)bm; j->res = R_OK; j->dsz = 0;
            out += j->raw ? len : bm; /* provisional slot; compacted below */
        }
        if (!indep) {
            /* decompressBlockDependency (ref src/lz4mt.cpp:737-845): blocks in
               order, each checked BEFORE it is decoded or written, decoded
               with LZ4_decompress_safe_withPrefix64k against a history of 64
               KiB of zeros (the zero-filled MemPool buffer) followed by all
               of this frame's output so far */
            /* the blocks read before a read error are still decoded and
               written (the reference handles each block as it is read); a
               block's own failure comes first in stream order */
            uint8_t* hist = (uint8_t*)calloc(65536 + bm, 1);
            size_t w = frameOut;
            int bres = R_OK;
            for (size_t i = 0; i < nb && bres == R_OK; i++) {
                djob* j = &jobs[i];
                if (j->hasBck && orc_xxh32(j->src, (size_t)j->len, 0) != j->bck) { bres = R_BCK; break; }
                const size_t have = w - frameOut, keep = have < 65536 ? have : 65536;
                memset(hist, 0, 65536);
                memcpy(hist + 65536 - keep, dst + w - keep, keep);
                int d;
                if (j->raw) { memcpy(hist + 65536, j->src, (size_t)j->len); d = j->len; }
                else d = orc_lz4_decompress_safe_prefix64k(j->src, hist + 65536, j->len, (int)bm);
                if (d < 0) { bres = R_DECOMP; break; }
                if (w + (size_t)d > outCap) { bres = R_ERROR; break; }
                memcpy(dst + w, hist + 65536, (size_t)d);
                w += (size_t)d;
            }
            if (bres != R_OK && (result == R_OK || result == R_ERROR)) result = bres;
            free(hist);
            free(jobs);
            out = w;
            if (result != R_OK) break;
            if (!eos) { result = R_RD_BSIZE; break; }
            if (sck) {
                if (ms_read(&s, b, 4) != 4) { result = R_RD_SCK; break; }
                if (orc_xxh32(dst + frameOut, out - frameOut, 0) != rd32(b)) { result = R_SCK; break; }
            }
            if (s.pos == s.n) break;
            continue;
        }
        /* decode (in parallel), then compact slots in block order */
        parallel_for(nb, nthreads, djob_fn, jobs);
        size_t w = frameOut;
        for (size_t i = 0; i < nb; i++) {
            if (jobs[i].res != R_OK) {
                /* a checksum mismatch is found after the block was written
                   (ref src/lz4mt.cpp:665-681); a decode failure before */
                if (jobs[i].res == R_BCK) {
                    if (dst + w != jobs[i].out) memmove(dst + w, jobs[i].out, (size_t)jobs[i].dsz);
                    w += (size_t)jobs[i].dsz;
                }
                if (result == R_OK || result == R_ERROR) result = jobs[i].res;
                break;
            }
            if (dst + w != jobs[i].out) memmove(dst + w, jobs[i].out, (size_t)jobs[i].dsz);
            w += (size_t)jobs[i].dsz;
        }
        free(jobs);
        out = w;
        if (result != R_OK) break;
        if (!eos) { result = R_RD_BSIZE; break; }
        if (sck) {
            if (ms_read(&s, b, 4) != 4) { result = R_RD_SCK; break; }
            if (orc_xxh32(dst + frameOut, out - frameOut, 0) != rd32(b)) { result = R_SCK; break; }
        }
        if (s.pos == s.n) break; /* clean end: the next 4-byte read would hit EOF */
    }
    *outSize = out;
    return result;
}

/* ===================================================================== */
/* Synthetic input: independent 64 KiB segments of     */
/* splitmix64-driven literal runs (1..16 of 'a'..'z') and back-copies     */
/* (length 4..67, offset 1..min(pos,65535), probability 76/256).          */
/* ===================================================================== */
#define GOLDEN 0x9E3779B97F4A7C15ull
static inline uint64_t sm_next(uint64_t* s) {
    uint64_t z = (*s += GOLDEN);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef struct { uint8_t* dst; uint64_t n, seed; } gjob;
static void gen_seg(void* a, size_t i) {
    gjob* g = (gjob*)a;
    uint8_t buf[65536 + 80];
    uint64_t s = g->seed + (uint64_t)i * GOLDEN;
    uint32_t len = 0;
    while (len < 65536) {
        const uint64_t r = sm_next(&s);
        if (len >= 64 && (r & 255) < 76) {
            const uint32_t L = 4 + (uint32_t)((r >> 8) & 63);
            const uint32_t lim = len < 65535 ? len : 65535;
            const uint32_t off = 1 + (uint32_t)((r >> 16) % lim);
            for (uint32_t k = 0; k < L; k++, len++) buf[len] = buf[len - off];
        } else {
            const uint32_t cnt = (uint32_t)((r >> 8) & 15) + 1;
            for (uint32_t k = 0; k < cnt; k++) buf[len++] = (uint8_t)(97 + (sm_next(&s) >> 40) % 26);
        }
    }
    const uint64_t off = (uint64_t)i * 65536;
    const uint64_t take = g->n - off < 65536 ? g->n - off : 65536;
    memcpy(g->dst + off, buf, take);
}

void orc_gen_synthetic(uint8_t* dst, uint64_t n, uint64_t seed) {
    gjob g = { dst, n, seed };
    parallel_for((size_t)((n + 65535) / 65536), 8, gen_seg, &g);
}

void orc_gen_random(uint8_t* dst, uint64_t n, uint64_t seed) {
    uint64_t s = seed;
    for (uint64_t i = 0; i < n; i += 8) {
        const uint64_t z = sm_next(&s);
        for (int k = 0; k < 8 && i + k < n; k++) dst[i + k] = (uint8_t)(z >> (8 * k));
    }
}

/* ===================================================================== */
/* lz4mt-shaped CPU pipeline (the bench's cpu_baseline "port"):           */
/* worker pool with nPool = nthreads + 1 blocks in flight (ref            */
/* src/lz4mt.cpp:281,375-376), in-order writer to a null sink with block  */
/* and stream XXH32 (ref 396-432), then the mirror decompress (593-734).  */
/* ===================================================================== */
typedef struct {
    const uint8_t* src; size_t n, bm, nb; const orc_frame_params* p; int decode;
    orc_codec_fn cfn, dfn;
    uint8_t** out; int* res; int* done; uint8_t** cin; int* clen; int* craw;
    size_t next, written; pthread_mutex_t mu; pthread_cond_t cv; size_t npool;
    orc_xxh32_state sx; size_t frameBytes; int err; int writing;
} pipe_ctx;

static void* pipe_worker(void* a) {
    pipe_ctx* c = (pipe_ctx*)a;
    for (;;) {
        pthread_mutex_lock(&c->mu);
        while (c->next < c->nb && c->next >= c->written + c->npool) pthread_cond_wait(&c->cv, &c->mu);
        if (c->next >= c->nb) { pthread_mutex_unlock(&c->mu); return NULL; }
        size_t i = c->next++;
        pthread_mutex_unlock(&c->mu);
        const size_t off = i * c->bm, len = c->n - off < c->bm ? c->n - off : c->bm;
        /* the worker: codec and block XXH32 (ref src/lz4mt.cpp:390-401 compress,
         * 629-650 decompress: the checksum is verified before the decode) */
        if (!c->decode) {
            c->res[i] = c->cfn((const char*)c->src + off, (char*)c->out[i % c->npool], (int)len, (int)len);
            const int cs = c->res[i];
            if (c->p->blockChecksum)
                (void)orc_xxh32(cs > 0 ? c->out[i % c->npool] : c->src + off, cs > 0 ? (size_t)cs : len, 0);
        } else {
            if (c->p->blockChecksum) (void)orc_xxh32(c->cin[i], (size_t)c->clen[i], 0);
            if (c->craw[i]) { memcpy(c->out[i % c->npool], c->cin[i], (size_t)c->clen[i]); c->res[i] = c->clen[i]; }
            else c->res[i] = c->dfn((const char*)c->cin[i], (char*)c->out[i % c->npool], c->clen[i], (int)c->bm);
        }
        /* in-order write chain: ONE writer at a time (the reference's
         * futures[i-1].wait() chain), the stream XXH32 inside it */
        pthread_mutex_lock(&c->mu);
        c->done[i] = 1;
        if (!c->writing) {
            c->writing = 1;
            while (c->written < c->nb && c->done[c->written]) {
                const size_t k = c->written;
                const size_t ko = k * c->bm, klen = c->n - ko < c->bm ? c->n - ko : c->bm;
                pthread_mutex_unlock(&c->mu);
                if (!c->decode) {
                    const int cs = c->res[k];
                    const size_t slen = cs > 0 ? (size_t)cs : klen;
                    if (c->p->streamChecksum) orc_xxh32_update(&c->sx, c->src + ko, klen);
                    c->frameBytes += 4 + slen + (c->p->blockChecksum ? 4 : 0);
                } else {
                    if (c->res[k] < 0) c->err = 1;
                    if (c->p->streamChecksum && c->res[k] > 0)
                        orc_xxh32_update(&c->sx, c->out[k % c->npool], (size_t)c->res[k]);
                }
                pthread_mutex_lock(&c->mu);
                c->written++;
                pthread_cond_broadcast(&c->cv);
            }
            c->writing = 0;
        }
        pthread_mutex_unlock(&c->mu);
    }
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void pipe_run(pipe_ctx* c, int nthreads) {
    pthread_t th[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, pipe_worker, c);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

static int own_compress(const char* s, char* d, int n, int cap) {
    return orc_lz4_compress((const uint8_t*)s, (uint8_t*)d, n, cap);
}
static int own_decompress(const char* s, char* d, int n, int cap) {
    return orc_lz4_decompress_safe((const uint8_t*)s, (uint8_t*)d, n, cap);
}

int orc_pipeline_roundtrip(const uint8_t* src, size_t n, const orc_frame_params* p, int nthreads, double* secs,
                           size_t* frameSize) {
    return orc_pipeline_roundtrip_codec(src, n, p, nthreads, secs, frameSize, NULL, NULL);
}

int orc_pipeline_roundtrip_codec(const uint8_t* src, size_t n, const orc_frame_params* p, int nthreads,
                                 double* secs, size_t* frameSize, orc_codec_fn cfn, orc_codec_fn dfn) {
    const size_t bm = block_max(p->blockMaxId), nb = (n + bm - 1) / bm;
    const size_t npool = (size_t)nthreads + 1;
    pipe_ctx c;
    memset(&c, 0, sizeof(c));
    c.src = src; c.n = n; c.bm = bm; c.nb = nb; c.p = p; c.npool = npool;
    c.cfn = cfn ? cfn : own_compress;
    c.dfn = dfn ? dfn : own_decompress;
    c.out = (uint8_t**)malloc(npool * sizeof(uint8_t*));
    for (size_t i = 0; i < npool; i++) c.out[i] = (uint8_t*)malloc(bm);
    c.res = (int*)calloc(nb + 1, sizeof(int));
    c.done = (int*)calloc(nb + 1, sizeof(int));
    pthread_mutex_init(&c.mu, NULL);
    pthread_cond_init(&c.cv, NULL);
    /* compress leg */
    orc_xxh32_reset(&c.sx, 0);
    c.frameBytes = 7 + 4 + (p->streamChecksum ? 4 : 0);
    double t0 = now_s();
    pipe_run(&c, nthreads);
    if (p->streamChecksum) (void)orc_xxh32_digest(&c.sx);
    secs[0] = now_s() - t0;
    *frameSize = c.frameBytes;
    /* decompress leg: pre-compressed block list built outside the timing */
    c.cin = (uint8_t**)malloc(nb * sizeof(uint8_t*) + 1);
    c.clen = (int*)malloc(nb * sizeof(int) + 4);
    c.craw = (int*)malloc(nb * sizeof(int) + 4);
    uint8_t* tmp = (uint8_t*)malloc(bm);
    for (size_t i = 0; i < nb; i++) {
        const size_t off = i * bm, len = n - off < bm ? n - off : bm;
        const int cs = c.cfn((const char*)src + off, (char*)tmp, (int)len, (int)len);
        c.craw[i] = cs <= 0;
        c.clen[i] = cs > 0 ? cs : (int)len;
        c.cin[i] = (uint8_t*)malloc((size_t)c.clen[i] + 1);
        memcpy(c.cin[i], cs > 0 ? tmp : src + off, (size_t)c.clen[i]);
    }
    free(tmp);
    memset(c.done, 0, (nb + 1) * sizeof(int));
    c.next = 0; c.written = 0; c.decode = 1; c.err = 0; c.writing = 0;
    orc_xxh32_reset(&c.sx, 0);
    t0 = now_s();
    pipe_run(&c, nthreads);
    if (p->streamChecksum) (void)orc_xxh32_digest(&c.sx);
    secs[1] = now_s() - t0;
    for (size_t i = 0; i < nb; i++) free(c.cin[i]);
    for (size_t i = 0; i < npool; i++) free(c.out[i]);
    free(c.cin); free(c.clen); free(c.craw); free(c.out); free(c.res); free(c.done);
    return c.err;
}

/* ===================================================================== */
/* Known answers for large configs, streamed (no whole-input buffer):     */
/* the App. F input of n bytes (seed), framed as lz4mt writes it          */
/* (orc_frame_compress, ref src/lz4mt.cpp:898-935), batch by batch.       */
/* Reports the frame size, XXH32 of the frame and of the content, and a   */
/* "checksum of checksums" for each: XXH32 over the little-endian u32     */
/* XXH32 digests of consecutive `chunk`-byte pieces (the last one short). */
/* ===================================================================== */
typedef struct { orc_xxh32_state whole, piece, list; uint64_t fill, chunk, count; } chunked_hash;

static void ch_reset(chunked_hash* h, uint64_t chunk) {
    orc_xxh32_reset(&h->whole, 0); orc_xxh32_reset(&h->piece, 0); orc_xxh32_reset(&h->list, 0);
    h->fill = 0; h->chunk = chunk; h->count = 0;
}
static void ch_close_piece(chunked_hash* h) {
    uint8_t b[4];
    wr32(b, orc_xxh32_digest(&h->piece));
    orc_xxh32_update(&h->list, b, 4);
    orc_xxh32_reset(&h->piece, 0);
    h->fill = 0; h->count++;
}
static void ch_update(chunked_hash* h, const uint8_t* p, size_t len) {
    orc_xxh32_update(&h->whole, p, len);
    while (len) {
        size_t take = (size_t)(h->chunk - h->fill);
        if (take > len) take = len;
        orc_xxh32_update(&h->piece, p, take);
        h->fill += take; p += take; len -= take;
        if (h->fill == h->chunk) ch_close_piece(h);
    }
}
static void ch_finish(chunked_hash* h) { if (h->fill) ch_close_piece(h); }

int orc_stream_known_answer(uint64_t n, uint64_t seed, const orc_frame_params* p, int nthreads, uint64_t chunk,
                            orc_known_answer* ka) {
    if (p->blockMaxId < 4 || p->blockMaxId > 7 || chunk == 0) return -1;
    const size_t bm = block_max(p->blockMaxId);
    const size_t batchBlocks = (256u << 20) / bm;          /* 256 MiB of input per batch */
    const size_t batch = batchBlocks * bm;
    uint8_t* in = (uint8_t*)malloc(batch);
    uint8_t* tmp = (uint8_t*)malloc(batch);
    uint8_t* rec = (uint8_t*)malloc(batch + batchBlocks * 8 + 64);
    int* csz = (int*)malloc(batchBlocks * sizeof(int));
    if (!in || !tmp || !rec || !csz) { free(in); free(tmp); free(rec); free(csz); return -1; }
    chunked_hash fh, chh;
    ch_reset(&fh, chunk); ch_reset(&chh, chunk);
    uint8_t hdr[32];
    const size_t hl = write_header(hdr, p);
    ch_update(&fh, hdr, hl);
    uint64_t frameSize = hl;
    for (uint64_t off = 0; off < n; off += batch) {
        const size_t len = (size_t)(n - off < batch ? n - off : batch);
        /* segment i of the stream starts from seed + i*G (App. F), so a batch
           at a 64 KiB-aligned offset is generated on its own */
        orc_gen_synthetic(in, len, seed + (off >> 16) * GOLDEN);
        ch_update(&chh, in, len);
        const size_t nb = (len + bm - 1) / bm;
        cjob j = { in, len, bm, tmp, csz };
        parallel_for(nb, nthreads, cjob_fn, &j);
        size_t o = 0;
        for (size_t i = 0; i < nb; i++) {
            const size_t bo = i * bm, bl = len - bo < bm ? len - bo : bm;
            const uint8_t* stored = csz[i] <= 0 ? in + bo : tmp + bo;
            const size_t slen = csz[i] <= 0 ? bl : (size_t)csz[i];
            wr32(rec + o, csz[i] <= 0 ? (uint32_t)bl | RAW_BIT : (uint32_t)csz[i]); o += 4;
            memcpy(rec + o, stored, slen); o += slen;
            if (p->blockChecksum) { wr32(rec + o, orc_xxh32(stored, slen, 0)); o += 4; }
        }
        ch_update(&fh, rec, o);
        frameSize += o;
    }
    ch_finish(&chh);
    uint8_t tail[8];
    size_t tl = 4;
    wr32(tail, 0);
    if (p->streamChecksum) { wr32(tail + 4, orc_xxh32_digest(&chh.whole)); tl = 8; }
    ch_update(&fh, tail, tl);
    frameSize += tl;
    ch_finish(&fh);
    ka->frameSize = frameSize;
    ka->frameXxh32 = orc_xxh32_digest(&fh.whole);
    ka->frameChunks = orc_xxh32_digest(&fh.list);
    ka->contentXxh32 = orc_xxh32_digest(&chh.whole);
    ka->contentChunks = orc_xxh32_digest(&chh.list);
    free(in); free(tmp); free(rec); free(csz);
    return 0;
}
