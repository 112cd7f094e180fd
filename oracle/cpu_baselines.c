/* cpu_baselines.c -- TEST / MEASUREMENT INFRASTRUCTURE ONLY (bench.py's
 * cpu_baseline leg; never linked or loaded by the product library).
 *
 * The reference's CPU path for the two non-default codecs, driven through
 * the codec the reference links (liblz4 function pointers handed in by the
 * caller; the oracle's own restatements when liblz4 is absent):
 *
 *   orc_hc_codec_set / orc_hc_compress_tramp
 *       LZ4-HC as lz4mt binds it for level >= 3: ctx.compress =
 *       LZ4_compressHC2_limitedOutput(src, dst, n, cap, level)
 *       (reference src/main.cpp:778-785).  The trampoline gives it the
 *       4-argument codec signature of orc_pipeline_roundtrip_codec, so the
 *       lz4mt-shaped pipeline times it like the fast codec.
 *
 *   orc_bd_roundtrip
 *       -BD frames: compressBlockDependency / decompressBlockDependency
 *       (reference src/lz4mt.cpp:460-538, 737-845) are single-threaded; one
 *       LZ4 stream, LZ4_compress_fast_continue per block (cap = n - 1,
 *       acceleration 1; hc: an HC stream at its default level 9,
 *       LZ4_compress_HC_continue, the reference's level >= 3 path
 *       src/lz4mt.cpp:295-332), block / stream XXH32, then the blocks decoded in
 *       order against the 64 KiB before them (LZ4_decompress_safe_usingDict
 *       over the contiguous output).  The reference's 1088 KiB input buffer
 *       and its slides change which bytes the dictionary holds, not the
 *       work per byte, so the timing uses one contiguous buffer.
 */
#include "lz4_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef int (*orc_hc_fn)(const char* src, char* dst, int n, int cap, int level);
static orc_hc_fn g_hc_fn;
static int g_hc_level = 9;

void orc_hc_codec_set(void* fn, int level) {
    g_hc_fn = (orc_hc_fn)fn;
    g_hc_level = level;
}

int orc_hc_compress_tramp(const char* src, char* dst, int n, int cap) {
    if (g_hc_fn) return g_hc_fn(src, dst, n, cap, g_hc_level);
    return orc_lz4hc_compress((const uint8_t*)src, (uint8_t*)dst, n, cap, g_hc_level);
}

typedef void* (*lz_create_fn)(void);
typedef int (*lz_free_fn)(void*);
typedef int (*lz_cont_fn)(void* stream, const char* src, char* dst, int n, int cap, int accel);
typedef int (*lz_dec_dict_fn)(const char* src, char* dst, int csize, int cap, const char* dict, int dictSize);
typedef int (*lz_hc_cont_fn)(void* stream, const char* src, char* dst, int n, int cap);

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* returns 0 on success (round trip verified), -1 on a decode or checksum error */
int orc_bd_roundtrip(const uint8_t* src, size_t n, int blockMaxId, int sck, int bck, void* create, void* freefn,
                     void* cont, void* decdict, int hc, double* secs, size_t* frameSize) {
    const size_t bm = (size_t)1 << (8 + 2 * blockMaxId), nb = (n + bm - 1) / bm;
    lz_create_fn cr = (lz_create_fn)create;
    lz_free_fn fr = (lz_free_fn)freefn;
    lz_cont_fn cf = (lz_cont_fn)cont;
    lz_hc_cont_fn hf = (lz_hc_cont_fn)cont;
    lz_dec_dict_fn df = (lz_dec_dict_fn)decdict;
    if (!cr || !fr || !cf || !df) return -1;
    uint8_t* body = (uint8_t*)malloc(n + 16 * nb + 64);
    size_t* boff = (size_t*)malloc((nb + 1) * sizeof(size_t));
    int* blen = (int*)malloc((nb + 1) * sizeof(int));
    int* braw = (int*)malloc((nb + 1) * sizeof(int));
    uint32_t* bsum = (uint32_t*)malloc((nb + 1) * sizeof(uint32_t));
    uint8_t* out = (uint8_t*)malloc(n + 64);
    int err = 0;
    /* compress leg */
    orc_xxh32_state sx;
    orc_xxh32_reset(&sx, 0);
    double t0 = now_s();
    void* st = cr();
    size_t pos = 0;
    for (size_t b = 0; b < nb; ++b) {
        const size_t off = b * bm, len = n - off < bm ? n - off : bm;
        const int cs = hc ? hf(st, (const char*)src + off, (char*)body + pos, (int)len, (int)len - 1)
                          : cf(st, (const char*)src + off, (char*)body + pos, (int)len, (int)len - 1, 1);
        braw[b] = cs <= 0;
        blen[b] = cs > 0 ? cs : (int)len;
        if (cs <= 0) memcpy(body + pos, src + off, len);
        boff[b] = pos;
        if (bck) bsum[b] = orc_xxh32(body + pos, (size_t)blen[b], 0);
        if (sck) orc_xxh32_update(&sx, src + off, len);
        pos += (size_t)blen[b];
    }
    if (sck) (void)orc_xxh32_digest(&sx);
    fr(st);
    secs[0] = now_s() - t0;
    *frameSize = 7 + pos + 4 * nb + (bck ? 4 * nb : 0) + 4 + (sck ? 4 : 0);
    /* decompress leg */
    orc_xxh32_reset(&sx, 0);
    t0 = now_s();
    for (size_t b = 0; b < nb && !err; ++b) {
        const size_t off = b * bm;
        if (bck && orc_xxh32(body + boff[b], (size_t)blen[b], 0) != bsum[b]) { err = -1; break; }
        int d;
        if (braw[b]) {
            memcpy(out + off, body + boff[b], (size_t)blen[b]);
            d = blen[b];
        } else {
            const size_t ds = off < 65536 ? off : 65536;
            d = df((const char*)body + boff[b], (char*)out + off, blen[b], (int)bm, (const char*)out + off - ds,
                   (int)ds);
        }
        if (d < 0) { err = -1; break; }
        if (sck) orc_xxh32_update(&sx, out + off, (size_t)d);
    }
    if (sck) (void)orc_xxh32_digest(&sx);
    secs[1] = now_s() - t0;
    if (!err && memcmp(out, src, n) != 0) err = -1;
    free(body); free(boff); free(blen); free(braw); free(bsum); free(out);
    return err;
}
