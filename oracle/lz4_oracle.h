/*
 * lz4_oracle.h — CPU restatement of the lz4mt hot path.  TEST INFRASTRUCTURE
 * ONLY: linked by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker.  The product (lz4mt_amd/) never links,
 * loads or calls anything in oracle/.
 *
 * What it restates (see lz4_oracle.c for per-function citations):
 *   - LZ4 1.9.3 LZ4_compress_limitedOutput / LZ4_compress_default
 *     (acceleration 1, fresh state) — the codec lz4mt binds through
 *     ctx.compress (reference src/main.cpp:749-751,776-785).  The lz4
 *     submodule is absent from the reference (.gitmodules:1-4); the pinned
 *     version is the lz4 1.9.3 shipped in this image (liblz4.so.1,
 *     LZ4_versionNumber() == 10903), see DESIGN.md "Oracle".
 *   - LZ4 1.9.3 LZ4_decompress_safe including its fast/safe loop split, so
 *     accept/reject decisions and negative return values match exactly.
 *   - XXH32 (xxhash, seed 0 everywhere in lz4mt: src/lz4mt.cpp:23).
 *   - The lz4mt frame writer/reader for independent blocks
 *     (src/lz4mt.cpp:335-457, 541-734, 898-1011).
 *   - The pinned synthetic input generator.
 *
 * Parity pins: tests/test_oracle.py checks every function against liblz4
 * 1.9.3 (ctypes), python-xxhash, the lz4 1.9.3 CLI and the known answers
 * in SURVEY.md App. F (produced by the reference build in the survey).
 */
#ifndef LZ4MT_ORACLE_H
#define LZ4MT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- XXH32 ------------------------------------------------------------ */
typedef struct {
    uint64_t total;
    uint32_t v[4];
    uint32_t seed;
    uint8_t  mem[16];
    uint32_t memSize;
} orc_xxh32_state;

uint32_t orc_xxh32(const void* p, size_t len, uint32_t seed);
void     orc_xxh32_reset(orc_xxh32_state* s, uint32_t seed);
void     orc_xxh32_update(orc_xxh32_state* s, const void* p, size_t len);
uint32_t orc_xxh32_digest(const orc_xxh32_state* s);

/* ---- LZ4 block codec -------------------------------------------------- */
int orc_lz4_compress_bound(int isize);
/* Returns compressed size, or 0 when the output does not fit `cap` under
 * LZ4 1.9.3's conservative limitedOutput margins. */
int orc_lz4_compress(const uint8_t* src, uint8_t* dst, int n, int cap);
/* LZ4_decompress_safe 1.9.3: decoded size, or -(error position)-1. */
int orc_lz4_decompress_safe(const uint8_t* src, uint8_t* dst, int srcSize,
                            int cap);

/* LZ4-HC 1.9.3 LZ4_compress_HC (= LZ4_compressHC2_limitedOutput, lz4mt's
 * codec for levels >= 3): levels 1..9 (hash chain); -1 for 10..12. */
int orc_lz4hc_compress(const uint8_t* src, uint8_t* dst, int n, int cap, int level);
/* -BD frame body at level >= 3 (the legacy HC stream, level 9); returns its size. */
int64_t orc_bd_hc_body(const uint8_t* src, size_t n, int blockMaxId, int bck, uint8_t* out);

/* LZ4_decompress_safe_withPrefix64k 1.9.3: dst[-65536..-1] is history. */
int orc_lz4_decompress_safe_prefix64k(const uint8_t* src, uint8_t* dst,
                                      int srcSize, int cap);

/* ---- lz4mt frame ------------------------------------------------------- */
typedef struct {
    int      streamChecksum;   /* FLG bit 2 */
    int      blockChecksum;    /* FLG bit 4 */
    int      blockMaxId;       /* BD bits 4-6, 4..7 */
    int      streamSizeFlag;   /* FLG bit 3 */
    uint64_t streamSize;
} orc_frame_params;

/* Worst-case frame size for n input bytes. */
size_t orc_frame_bound(size_t n, const orc_frame_params* p);
/* Writes one frame; returns its size (0 on bad params).  `nthreads` > 1
 * compresses blocks on that many pthreads (output is identical). */
size_t orc_frame_compress(const uint8_t* src, size_t n, uint8_t* dst,
                          const orc_frame_params* p, int nthreads);
/* Decodes a byte stream of concatenated frames the way lz4mtDecompress
 * does, block-dependent (-BD) frames included (decompressBlockDependency).  Returns an Lz4MtResult code; *outSize receives decoded bytes.
 * `outCap` bounds the output; exceeding it returns LZ4MT_RESULT_ERROR. */
int orc_frame_decompress(const uint8_t* src, size_t n, uint8_t* dst,
                         size_t outCap, size_t* outSize, int nthreads);

/* ---- synthetic input ------------------------------- */
void orc_gen_synthetic(uint8_t* dst, uint64_t n, uint64_t seed);
/* Incompressible control: splitmix64 bytes. */
void orc_gen_random(uint8_t* dst, uint64_t n, uint64_t seed);

/* ---- lz4mt-shaped CPU frame pipeline for the baseline ----------------- */
/* Times one compress + one decompress of `src` with `nthreads` workers
 * (nPool = nthreads + 1 blocks in flight, in-order writer, block and
 * stream XXH32 as flags say).  Returns 0 on success; seconds in out[0..1],
 * frame size in *frameSize. */
int orc_pipeline_roundtrip(const uint8_t* src, size_t n,
                           const orc_frame_params* p, int nthreads,
                           double* secs, size_t* frameSize);
/* The same pipeline over a caller-supplied block codec with the LZ4
 * signatures lz4mt binds (LZ4_compress_limitedOutput / LZ4_decompress_safe,
 * e.g. dlopen'd from liblz4.so.1); NULL = this restatement. */
typedef int (*orc_codec_fn)(const char* src, char* dst, int n, int cap);
int orc_pipeline_roundtrip_codec(const uint8_t* src, size_t n,
                                 const orc_frame_params* p, int nthreads,
                                 double* secs, size_t* frameSize,
                                 orc_codec_fn compress, orc_codec_fn decompress);

/* cpu_baselines.c: the reference's CPU path for LZ4-HC (through the
 * pipeline, via a trampoline fixing the level) and for -BD (single thread,
 * one LZ4 stream), over liblz4 function pointers (bench.py cpu_baseline) */
void orc_hc_codec_set(void* fn, int level);
int orc_hc_compress_tramp(const char* src, char* dst, int n, int cap);
int orc_bd_roundtrip(const uint8_t* src, size_t n, int blockMaxId, int sck, int bck, void* create, void* freefn,
                     void* cont, void* decdict, int hc, double* secs, size_t* frameSize);

/* ---- streamed known answers for large configs ------------------------- */
typedef struct {
    uint64_t frameSize;
    uint32_t frameXxh32, frameChunks;      /* XXH32 of the frame; of its chunk digests */
    uint32_t contentXxh32, contentChunks;  /* the same for the content */
} orc_known_answer;
/* Frames the App. F input of n bytes (seed) batch by batch without holding
 * it whole.  "Chunks" = XXH32 over the LE u32 XXH32 digests of consecutive
 * `chunk`-byte pieces (the last one short).  Returns 0 on success. */
int orc_stream_known_answer(uint64_t n, uint64_t seed, const orc_frame_params* p,
                            int nthreads, uint64_t chunk, orc_known_answer* ka);

#ifdef __cplusplus
}
#endif
#endif
