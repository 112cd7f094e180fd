/*
 * lz4mt_hip.h — MI355X extensions to the lz4mt C ABI (liblz4mt_amd.so).
 *
 * Three layers, all plain C types (pointers, sizes, an opaque stream):
 *
 * 1. Block operators with exactly the reference's plugin signatures
 *    (typedefs Lz4MtCompress / Lz4MtCompressBound / Lz4MtDecompress,
 *    reference src/lz4mt.h:41-58).  Assign them to ctx.compress /
 *    ctx.compressBound / ctx.decompress and the reference-shaped host
 *    scheduler (lz4mtCompress in PARALLEL/SEQUENTIAL mode) runs every block
 *    on the GPU.  Host pointers; each call stages through device memory.
 *    They replace LZ4_compress_limitedOutput / LZ4_compressBound /
 *    LZ4_decompress_safe as wired in reference src/main.cpp:749-751,767-785.
 *
 * 2. Device-resident frame engine: one call compresses or decompresses a
 *    whole lz4mt frame whose input and output already live in HBM
 *    (the performance path; used by lz4mtCompress/lz4mtDecompress in
 *    LZ4MT_MODE_DEVICE and by bench.py).
 *
 * 3. Utilities: synthetic input generator, XXH32, device info.
 *
 * Streams are hipStream_t passed as void* (NULL = default stream).
 * Every function fails loudly (returns LZ4MT_RESULT_ERROR / a negative
 * value) when no HIP device is present; nothing falls back to the CPU.
 */
#ifndef LZ4MT_AMD_LZ4MT_HIP_H
#define LZ4MT_AMD_LZ4MT_HIP_H

#include "lz4mt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- 1. block operators (reference plugin signatures) ------------------ */
/* LZ4_compress_limitedOutput semantics (lz4 1.9.3, acceleration 1):
 * returns the compressed size, or 0 when it does not fit maxOutputSize.
 * compressionLevel >= 3: LZ4_compressHC2_limitedOutput, the codec the
 * reference wires for those levels (src/main.cpp:778-785): 3..9 LZ4-HC
 * 1.9.3's hash-chain parser, 10..12 its optimal parser
 * (LZ4HC_compress_optimal); levels above 12 are clamped to 12 as lz4hc
 * does. */
int lz4mtHipCompressBlock(const char* src, char* dst, int isize, int maxOutputSize, int compressionLevel);
/* LZ4_compressBound. */
int lz4mtHipCompressBound(int isize);
/* LZ4_decompress_safe semantics: decoded size, or a negative value. */
int lz4mtHipDecompressBlock(const char* src, char* dst, int isize, int maxOutputSize);

/* ---- 2. device-resident frame engine ----------------------------------- */
/* Upper bound of a frame for srcSize input bytes under `sd`. */
uint64_t lz4mtHipFrameBound(uint64_t srcSize, const Lz4MtStreamDescriptor* sd);
/* Scratch bytes lz4mtHipCompressFrame needs for srcSize (slots + tables). */
uint64_t lz4mtHipCompressWorkspaceSize(uint64_t srcSize, const Lz4MtStreamDescriptor* sd);
/* Compresses d_src[0..srcSize) into one frame at d_frame (device memory).
 * d_workspace may be NULL (the library then allocates and frees scratch).
 * *frameSize (host) receives the frame length; the call synchronises the
 * stream once at the end to read it.  blockIndependence = 0 writes a
 * block-dependent (-BD) frame: one wavefront encodes the blocks in order,
 * each against the 64 KiB before it (lz4's streaming compressor, as the
 * reference's compressBlockDependency calls it).  The plan, table and
 * round scratch of -BD frames live in the workspace, so size it with
 * lz4mtHipCompressWorkspaceSize for the same `sd`. */
Lz4MtResult lz4mtHipCompressFrame(const void* d_src, uint64_t srcSize, void* d_frame, uint64_t frameCap,
                                  uint64_t* frameSize, const Lz4MtStreamDescriptor* sd,
                                  void* d_workspace, uint64_t workspaceSize, void* stream);
/* Asynchronous variant: *d_frameSize is device memory, nothing is
 * synchronised (the stream carries the dependency). */
Lz4MtResult lz4mtHipCompressFrameAsync(const void* d_src, uint64_t srcSize, void* d_frame, uint64_t frameCap,
                                       uint64_t* d_frameSize, const Lz4MtStreamDescriptor* sd,
                                       void* d_workspace, uint64_t workspaceSize, void* stream);

/* The same with a compression level: 0..2 fast LZ4, 3..9 LZ4-HC hash
 * chain, 10..12 (and above, clamped to 12) LZ4-HC's optimal parser (the
 * workspace then holds 2 more bytes per input byte: use
 * lz4mtHipCompressWorkspaceSizeEx).  Block-dependent frames at any level
 * >= 3 are the reference's HC stream, which runs at lz4hc's level 9. */
uint64_t lz4mtHipCompressWorkspaceSizeEx(uint64_t srcSize, const Lz4MtStreamDescriptor* sd, int level);
Lz4MtResult lz4mtHipCompressFrameEx(const void* d_src, uint64_t srcSize, void* d_frame, uint64_t frameCap,
                                    uint64_t* frameSize, const Lz4MtStreamDescriptor* sd, int level,
                                    void* d_workspace, uint64_t workspaceSize, void* stream);
Lz4MtResult lz4mtHipCompressFrameAsyncEx(const void* d_src, uint64_t srcSize, void* d_frame, uint64_t frameCap,
                                         uint64_t* d_frameSize, const Lz4MtStreamDescriptor* sd, int level,
                                         void* d_workspace, uint64_t workspaceSize, void* stream);

/* Parses the frame header at d_frame (one small device->host copy) and
 * reports its descriptor, header length and an upper bound of the decoded
 * size (blocks x blockMax, from a device walk of the block size words). */
Lz4MtResult lz4mtHipFrameInfo(const void* d_frame, uint64_t frameSize, Lz4MtStreamDescriptor* sd,
                              uint64_t* decodedBound, uint64_t* nBlocks, void* stream);
/* Decompresses every frame in d_frame[0..frameSize) (concatenated frames
 * and skippable frames included) into d_out.  outCap must hold
 * (blocks x blockMax) bytes of the last frame (see lz4mtHipFrameInfo).
 * *outSize receives the decoded length; `sd` the last frame's descriptor.
 * Result codes follow lz4mtDecompress (reference src/lz4mt.cpp:938-1011). */
Lz4MtResult lz4mtHipDecompressFrame(const void* d_frame, uint64_t frameSize, void* d_out, uint64_t outCap,
                                    uint64_t* outSize, Lz4MtStreamDescriptor* sd, void* stream);

/* Upper bound of the decoded size of every frame in d_frame[0..frameSize)
 * (concatenated and skippable frames included): the out capacity
 * lz4mtHipDecompressFrame needs.  Walks each frame's size words. */
Lz4MtResult lz4mtHipStreamBound(const void* d_frame, uint64_t frameSize, uint64_t* decodedBound, void* stream);
/* Record table of the single frame at d_frame: recordStart[i] = frame
 * offset of block i's size word (i < *nBlocks), recordStart[*nBlocks] = the
 * EOS word; *hdrLen = header bytes incl. magic.  `cap` entries of host
 * memory (>= blocks + 1; recordStart NULL = count only).  The device walk of
 * lz4mtHipDecompressFrame; used to cut a frame into per-GPU sub-frames of
 * whole records (the multi-GPU decompress scatter). */
Lz4MtResult lz4mtHipFrameRecords(const void* d_frame, uint64_t frameSize, uint64_t* recordStart, uint64_t cap,
                                 uint64_t* nBlocks, int* hdrLen, Lz4MtStreamDescriptor* sd, void* stream);

/* ---- 3. utilities ------------------------------------------------------- */
/* SURVEY.md App. F generator, bit-identical to the CPU oracle. */
int lz4mtHipGenSynthetic(void* d_dst, uint64_t n, uint64_t seed, void* stream);
/* XXH32 (seed 0) of device memory; synchronises the stream.  One serial
 * chain (one wavefront): use it for small ranges. */
uint32_t lz4mtHipXxh32(const void* d_src, uint64_t len, void* stream);
/* XXH32 of each consecutive chunkBytes piece of d_src (the last one short)
 * into d_digests[ceil(len / chunkBytes)] (device memory), in parallel;
 * asynchronous.  Returns 0, or -1 without a device / on bad arguments. */
int lz4mtHipXxh32Chunks(const void* d_src, uint64_t len, uint32_t chunkBytes, uint32_t* d_digests, void* stream);
/* Number of HIP devices visible (0 = none: every compute entry point errors). */
int lz4mtHipDeviceCount(void);
/* Frees the calling thread's cached engine memory (the DEVICE mode's pinned
 * staging slots and device buffers, the decode scratch) and the idle
 * scratch of the block operators.  LZ4MT_MODE_DEVICE callers keep their
 * slots between calls (no re-pinning); relinked default-PARALLEL callers
 * have them freed at the end of every call. */
void lz4mtHipReleaseCaches(void);

/* Per-stage device timings (ms, hipEvents) of the last frame call on this
 * thread: [0] encode/decode kernel, [1] checksum kernel(s), [2] scan +
 * assemble / walk + verify, [3] whole call.  Enabled by
 * lz4mtHipSetTiming(1) (adds event records, no synchronisation). */
void lz4mtHipSetTiming(int enable);
int lz4mtHipGetTimings(float* ms4);

/* ---- 4. block-sharded multi-GPU compress, gather streamed beside the encode
 * (lz4mt_amd/dist.py drives it over RCCL).  A shard is a
 * contiguous block range of one -Sx stream (FLG.2 and FLG.3 off: they do not
 * shard).  The sending rank launches its encode once, then packs rounds of
 * whatever the encoder has published so far (each round one contiguous
 * buffer: header, a descriptor per block, payload) and sends them while the
 * encode runs; the root unpacks them into a mirror of that shard's slots and,
 * once every shard is complete, assembles each shard's records into the one
 * frame.  Replaces nothing in the reference (it has no multi-device path);
 * the frame is the one lz4mtCompress writes for the whole stream
 * (src/lz4mt.cpp:898-935). ------------------------------------------------ */
/* Bytes of a shard workspace, and of the root's mirror of a shard (same
 * layout); 0 for a descriptor that cannot shard. */
uint64_t lz4mtHipShardWorkspaceSize(uint64_t n, const Lz4MtStreamDescriptor* sd);
/* Largest pack one round can produce with at most perBlockCap bytes per block. */
uint64_t lz4mtHipShardPackBound(uint64_t n, const Lz4MtStreamDescriptor* sd, uint32_t perBlockCap);
/* The frame header lz4mtCompress writes for `sd` (magic .. header checksum)
 * into out[19]; returns its length, -1 on a bad descriptor. */
int lz4mtHipFrameHeader(const Lz4MtStreamDescriptor* sd, uint8_t* out);
/* Zeroes the workspace's round state (published, packed and hashed counts)
 * on `stream`.  Required before every encode into the workspace, and it must
 * be stream-ordered before the encode AND before the call's first pack (the
 * two usually run on different streams: reset on a stream both wait on). */
Lz4MtResult lz4mtHipShardReset(uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_ws, uint64_t wsSize, void* stream);
/* Launches the shard's encode (+ block checksums) on `stream`; 1 and 4 MiB
 * blocks publish their progress as they go.  Asynchronous.  The workspace
 * must have been reset (lz4mtHipShardReset) after its previous use. */
Lz4MtResult lz4mtHipShardEncode(const void* d_src, uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_ws,
                                uint64_t wsSize, void* stream);
/* Forgets the call-order state kept for the workspace at d_ws (its next use
 * needs lz4mtHipShardReset first).  Call it when the workspace is freed, so
 * that a new allocation at the same address starts unknown. */
void lz4mtHipShardRelease(const void* d_ws);
/* One round into d_pack (capacity >= lz4mtHipShardPackBound): final = 0 while
 * the encode may still run (stream-ordered anywhere), final = 1 once it is
 * done (stream-ordered after it; repeat until the header's flags bit 0 is
 * set).  Header (64 B, little-endian): u64 magic, u64 payload bytes, u64
 * bytes still to send, u64 bytes of this pack, u32 blocks, u32 flags
 * (1 = shard complete), u64 the shard's record bytes (when complete). */
Lz4MtResult lz4mtHipShardPack(const void* d_src, uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_ws,
                              uint64_t wsSize, void* d_pack, uint64_t packCap, uint32_t perBlockCap, int final,
                              void* stream);
/* Root: one received pack of an n-byte shard into its mirror (a buffer of
 * lz4mtHipShardWorkspaceSize bytes). */
Lz4MtResult lz4mtHipShardUnpack(const void* d_pack, uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_mirror,
                                uint64_t mirrorSize, void* stream);
/* The shard's records (size word, payload, [checksum]) into d_body, as they
 * stand in the frame of the whole stream.  d_ws: a complete mirror, or the
 * shard workspace itself after its encode; d_src: the shard's source for the
 * latter (incompressible blocks), NULL for a mirror.  Body bytes = the
 * complete pack's record bytes. */
Lz4MtResult lz4mtHipShardAssemble(const void* d_src, uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_ws,
                                  uint64_t wsSize, void* d_body, uint64_t bodyCap, void* stream);
/* The root's receive buffers for the copy-engine push of packs: allocate
 * (hipMalloc) and export an IPC handle (64 bytes); open / close another
 * process's buffer (mapped for the calling thread's device); free; and an
 * asynchronous device-to-device copy (a mapped peer buffer included).
 * 0 on success, -1 otherwise. */
int lz4mtHipIpcAlloc(uint64_t bytes, void** d_ptr, void* handle64);
/* The same, choosing the memory kind (*kind receives it): 2 uncached device
 * memory (hipDeviceMallocUncached: no L2 line of it is ever held, so a peer
 * copy engine's writes are what every later read sees), 1 fine-grained,
 * 0 plain hipMalloc -- the best kind <= want that allocates and exports an
 * IPC handle.  lz4mtHipShardUnpack starts with a system-scope acquire in
 * every case. */
int lz4mtHipIpcAllocKind(uint64_t bytes, void** d_ptr, void* handle64, int want, int* kind);
/* PCI bus id ("dddd:bb:dd.f", len >= 13) of device `dev`; the ordinal of the
 * visible device with that bus id (-1: not visible); hipDeviceCanAccessPeer
 * (1 yes, 0 no, -1 error).  The IPC setup identifies the root's GPU by bus id
 * so that processes that number devices differently agree. */
int lz4mtHipDevicePciBusId(int dev, char* buf, int len);
int lz4mtHipDeviceByPciBusId(const char* busId);
int lz4mtHipCanAccessPeer(int dev, int peer);
int lz4mtHipIpcOpen(const void* handle64, void** d_ptr);
int lz4mtHipIpcClose(void* d_ptr);
int lz4mtHipFree(void* d_ptr);
int lz4mtHipCopyAsync(void* d_dst, const void* d_src, uint64_t n, void* stream);
/* Record bytes of a complete shard workspace (or mirror): synchronises the
 * stream; UINT64_MAX on bad arguments or a device error. */
uint64_t lz4mtHipShardBodyBytes(uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_ws, uint64_t wsSize, void* stream);

/* ---- 5. diagnostics ----------------------------------------------------- */
/* Runs s_memtime-stamped twins of the encode / decode kernels (never the
 * product launch) and sums per-phase shader cycles over all blocks.
 * encode (16 slots): [hash, table+dedup, candidate check, round issue,
 * literal staging, round wait, table writes, count, emit, loop overhead,
 * windows, tag aliases, tag-candidate winners, -, -, -];
 * decode (16 slots): [batch parse, serial literal copy, serial match copy
 * / batch dependent copies, batch group + far copies, batches, total,
 * matches, far matches, batch sequences, serial-path sequences, -...]. */
int lz4mtHipDebugEncodeStats(const void* d_src, uint64_t n, uint32_t blockSize, uint64_t* stats16, void* stream);
/* The same counters per block, unsummed: perBlock16 holds ceil(n /
 * blockSize) x 16 words (block b at 16 b).  0, or -1. */
int lz4mtHipDebugEncodeBlockStats(const void* d_src, uint64_t n, uint32_t blockSize, uint64_t* perBlock16,
                                  void* stream);
/* The frame path's block encoder alone over blocks of any size 65 547 B ..
 * 4 MiB (frames use 64 KiB .. 4 MiB by 4x steps; the others are timing
 * points of a split parse, tools/occ_sweep.py).  d_slots: nb x blockSize +
 * 64 bytes, d_csize: nb int32.  Asynchronous; 0, or -1 on bad arguments. */
int lz4mtHipDebugEncode(const void* d_src, uint64_t n, uint32_t blockSize, void* d_slots, void* d_csize, void* stream);
/* 1 when the current device applies one wave's same-address LDS exchanges
 * in ascending lane order (what the block encoders' exchange probe relies
 * on; checked once per device before the first encode), 0 when it does not
 * (the encoders then run their read-back probe: same bytes, no ordering
 * assumed), -1 without a device or when the check could not run. */
int lz4mtHipCheckEncoderOrder(void);
/* The table probe the block encoders use on the current device: 1 the LDS
 * exchange, 0 the read-back probe (the order check failed, or
 * LZ4MT_AMD_ENC_PROBE=readback), -1 without a device / on a HIP error.  A
 * call whose stream is being captured into a graph before this device was
 * checked also takes the read-back probe (the check synchronises). */
int lz4mtHipEncoderProbe(void);
/* The parse work of a split parse: n bytes in streams of S bytes, stream b
 * parsed from ov bytes before its start (the overlap a join needs), S + ov
 * <= 4 MiB, into d_slots (nb x (S + ov) + 64 bytes), sizes into d_csize;
 * p17 = 1 selects the 3-byte table.  Timing only; 0, or -1 on bad args. */
int lz4mtHipDebugEncodeOverlap(const void* d_src, uint64_t n, uint32_t S, uint32_t ov, int p17, void* d_slots,
                               void* d_csize, void* stream);
int lz4mtHipDebugDecodeStats(const void* d_frame, uint64_t frameSize, uint64_t* stats16, void* stream);
/* FETCH_SIZE calibration (tools/fetch_cal.py): reads n bytes of d_buf exactly
 * once with `width`-byte loads per lane (1, 4, 8 or 16); d_out4: 4 bytes of
 * device scratch.  Asynchronous; 0, or -1 on a bad width. */
/* The per-block lz4 stream plan of a -BD frame (host only): for blocks of
 * sizes[0..nBlocks), plan4[4b..4b+3] = catch-up bound for candidates in the
 * block, in the history, the dictSmall limit (block coordinates: the block
 * at 65536) and where the history bytes stand (0 = before the block; else
 * the block's own bytes from shift - 65536: the reference's buffer,
 * refBuffer = 1).  0 on success, 1 if a history would be neither, -1 on a
 * bad id. */
int lz4mtDebugBdPlan(int blockMaxId, int refBuffer, const uint32_t* sizes, uint64_t nBlocks, uint32_t* plan4);
int lz4mtHipDebugFetchCal(const void* d_buf, uint64_t n, int width, void* d_out4, void* stream);

#ifdef __cplusplus
}
#endif
#endif
