// lz4mt_device.h — shared declarations between the HIP kernels
// (lz4mt_kernels.hip) and the host engine (lz4mt_engine.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace lz4mt {

// LZ4 1.9.3 constants.
constexpr int kMinMatch = 4;
constexpr int kLastLiterals = 5;
constexpr int kMfLimit = 12;
constexpr int kMinLength = 13;
constexpr uint32_t kDistMax = 65535;
constexpr int kLimit64K = 65547;

// Decoder status codes beyond LZ4_decompress_safe's own negative values.
constexpr int kDecodeOutputTooSmall = INT32_MIN;   // physical slot smaller than the decoded block

// Per-block record of a parsed frame (device-resident, one per block).
struct BlockRec {
    uint64_t offset;     // payload offset inside the frame
    uint32_t bits;       // size word: stored size | 0x80000000 if raw
    uint32_t checksum;   // block XXH32 read from the frame (if FLG.4)
};

// Per-block lz4 stream state of a block-dependent (-BD) frame's encode
// (see k_encode_linked): catch-up lower bounds for candidates in the block /
// in the history and the dictSmall limit, in coordinates where the block
// starts at 65536 and its 64 KiB history is [0, 65536).
// shift: where the history bytes stand (BdSim): 0 = the 64 KiB before the
// block; else position p < 65536 reads the block's own byte p - 65536 + shift
// (the reference's 1 / 4 MiB buffer, LZ4MT_AMD_BD_REFERENCE=1).
struct LinkPlan {
    uint32_t lowIn, lowDict, candLow, shift;
};

// Device state of a block-dependent encode: per-block plans, the carried table.
struct LinkState {
    LinkPlan* plan;
    uint32_t* table;
    bool fresh;
    uint32_t* rounds;    // parallel rounds' scratch, link_round_bytes(nBlocks) (null: the serial kernel)
    // level >= 3: the HC stream's segments (hc_bd_pack's layout on the device)
    const uint8_t* hcSegs = nullptr;
    uint32_t nSeg = 0;
    bool hcPerBlock = false;   // every block starts its own segment (1 / 4 MiB blocks)
    bool xh = false;           // some plan has a shift: the encoder variant that reads such histories
};

// Frame-walk summary written by the walk kernel.
struct WalkInfo {
    uint64_t endPos;     // position just after the EOS word
    uint32_t nBlocks;
    int32_t  result;     // Lz4MtResult code (0 = OK)
};

// Scratch of the parallel frame walk (launch_frame_walk_count/_path): the
// frame is scanned in 64 KiB chunks for candidate record offsets.
constexpr int kWalkChunkLog = 16;
struct WalkScratch {
    uint32_t* count;     // nChunks: candidates per chunk
    uint64_t* base;      // nChunks + 1: exclusive scan of count, M at [nChunks]
    uint64_t* pos;       // M: node -> frame offset (ascending)
    uint32_t* Ja;        // M + 1: successor tables (node M = DEAD)
    uint32_t* Jb;
    uint32_t* P;         // maxBlocks + 1 (path)
};

// A side stream + two events (per thread, re-made when the device changes)
// for work that can run beside the main stream.
struct AuxStream {
    hipStream_t st = nullptr;
    hipEvent_t evIn = nullptr, evMid = nullptr, evOut = nullptr;
    int dev = -1;
    bool ensure();
    void release();
    ~AuxStream() { release(); }
};

// ---- kernel launchers (lz4mt_kernels.hip) ----
// once per device, before the first block-encoder launch: the LDS exchange
// order the encoder's table probe relies on (k_xchg_order)
hipError_t encoder_ready(hipStream_t st);
hipError_t launch_encode_overlap(const uint8_t* src, uint64_t srcSize, uint32_t S, uint32_t ov, bool p17,
                                 uint8_t* slots, int32_t* csize, hipStream_t st);
hipError_t launch_encode(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                         uint8_t* slots, uint64_t slotStride, uint32_t capOverride, int32_t* csize,
                         hipStream_t st);
// k_encode with per-block progress publishing (pub[b]: bytes of slot b final;
// slot stride = blockSize), for the block-sharded streamed gather
hipError_t launch_encode_pub(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                             uint8_t* slots, int32_t* csize, uint32_t* pub, hipStream_t st);
hipError_t launch_decode(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t blockMax,
                         uint8_t* out, uint64_t outCap, int32_t* dsize, hipStream_t st);
// the serial frame walk fused with the decode (k_decode_walk): records are
// decoded as the walk publishes them.  ctl: 8 zeroed device words.
hipError_t launch_decode_walk(const uint8_t* frame, uint64_t frameSize, uint64_t bodyPos, uint32_t blockMax,
                              int blockChecksum, uint32_t maxBlocks, BlockRec* recs, WalkInfo* info, uint32_t* ctl,
                              uint8_t* out, uint64_t outCap, int32_t* dsize, uint32_t waves, hipStream_t st);
// beside it: the block checksums as the walk publishes them, and the verify
// with the walk's block count read on the device
hipError_t launch_xxh32_walked(const uint8_t* frame, const BlockRec* recs, uint32_t* ctl, uint32_t* digest,
                               uint32_t waves, hipStream_t st);
hipError_t launch_block_verify_walked(const BlockRec* recs, const WalkInfo* info, const uint32_t* digest,
                                      const int32_t* dsize, int blockChecksum, int32_t* status, uint32_t maxBlocks,
                                      hipStream_t st);
// the streamed compress's persistent encoder (lz4mt_kernels.hip, k_encode_stream);
// ticks: a wait's limit without progress (s_memrealtime, 100 MHz); pend:
// 4 words per wave, a block parked on its output slot (zeroed before the
// first launch of a call; a relaunch finishes those blocks first)
hipError_t launch_encode_stream(const uint8_t* hin, uint8_t* hout, uint32_t* inCtl, uint32_t* outCtl, uint32_t* g,
                                uint32_t* next, uint32_t* pend, uint8_t* dIn, uint8_t* dSlot, uint32_t bm, uint32_t Rin,
                                uint32_t Rout, uint32_t waves, int bck, uint64_t ticks, hipStream_t st);
// the streamed decompress's persistent decoder (lz4mt_kernels.hip, k_decode_stream)
hipError_t launch_decode_stream(const uint8_t* hin, uint8_t* hout, uint32_t* inCtl, uint32_t* outCtl, uint32_t* g,
                                uint32_t* next, uint32_t* pend, uint8_t* dIn, uint8_t* dSlot, uint32_t bm, uint32_t Rin,
                                uint32_t Rout, uint32_t waves, int bck, uint64_t ticks, hipStream_t st);
hipError_t launch_xxh32_stored(const uint8_t* src, const uint8_t* slots, uint64_t srcSize, uint32_t blockSize,
                               uint32_t nBlocks, const int32_t* csize, uint32_t* digest, hipStream_t st);
// block checksums while k_encode_pub runs (on another stream; pub / xdone
// zeroed before both), and the fix-up of blocks it did not finish
hipError_t launch_xxh32_follow(const uint8_t* src, const uint8_t* slots, uint64_t srcSize, uint32_t blockSize,
                               uint32_t nBlocks, uint32_t* pub, uint32_t* digest, uint32_t* xdone, hipStream_t st);
hipError_t launch_xxh32_fixup(const uint8_t* src, const uint8_t* slots, uint64_t srcSize, uint32_t blockSize,
                              uint32_t nBlocks, const int32_t* csize, uint32_t* digest, const uint32_t* xdone,
                              hipStream_t st);
hipError_t launch_xxh32_frame_blocks(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t* digest,
                                     hipStream_t st);
hipError_t launch_xxh32_stream(const uint8_t* p, uint64_t len, uint32_t* digest, hipStream_t st);
hipError_t launch_xxh32_chunks(const uint8_t* p, uint64_t len, uint32_t chunk, uint32_t* digest, hipStream_t st);
hipError_t launch_frame_scan(const int32_t* csize, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                             int blockChecksum, uint64_t* recOff, hipStream_t st);
hipError_t launch_frame_assemble(const uint8_t* src, const uint8_t* slots, uint64_t srcSize, uint32_t blockSize,
                                 uint32_t nBlocks, const int32_t* csize, const uint32_t* bsum,
                                 const uint64_t* recOff, int blockChecksum, uint8_t* frame, uint32_t hdrLen,
                                 hipStream_t st);
// blockChecksum for launch_frame_assemble: 0 none, 1 write the words, 2 leave
// them to launch_frame_sums
hipError_t launch_frame_sums(const int32_t* csize, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                             const uint32_t* bsum, const uint64_t* recOff, uint8_t* frame, uint32_t hdrLen,
                             hipStream_t st);
hipError_t launch_frame_finalize(uint8_t* frame, const uint8_t* hdr, uint32_t hdrLen, const uint64_t* recOff,
                                 uint32_t nBlocks, const uint32_t* streamSum, uint64_t* frameSize,
                                 hipStream_t st);
hipError_t launch_frame_walk(const uint8_t* frame, uint64_t frameSize, uint64_t bodyPos, uint32_t blockMax,
                             int blockChecksum, uint32_t maxBlocks, BlockRec* recs, WalkInfo* info,
                             hipStream_t st);
uint64_t frame_walk_par_chunks(uint64_t frameSize);
hipError_t launch_frame_walk_count(const uint8_t* frame, uint64_t frameSize, uint64_t bodyPos, uint32_t blockMax,
                                   int blockChecksum, const WalkScratch& ws, hipStream_t st);
hipError_t launch_frame_walk_path(const uint8_t* frame, uint64_t frameSize, uint64_t bodyPos, uint32_t blockMax,
                                  int blockChecksum, uint32_t maxBlocks, uint32_t M, const WalkScratch& ws,
                                  BlockRec* recs, WalkInfo* info, hipStream_t st);
hipError_t launch_block_verify(const BlockRec* recs, uint32_t nBlocks, const uint32_t* digest, const int32_t* dsize,
                               uint32_t blockMax, int blockChecksum, int32_t* status, hipStream_t st);
hipError_t launch_encode_stats(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                               uint8_t* slots, int32_t* csize, uint64_t* stats, hipStream_t st);
hipError_t launch_decode_stats(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t blockMax,
                               uint8_t* out, uint64_t outCap, int32_t* dsize, uint64_t* stats, hipStream_t st);
hipError_t launch_gen_synthetic(uint8_t* dst, uint64_t n, uint64_t seed, hipStream_t st);
// LZ4-HC (lz4mt_hc.hip): level 1..9 (lz4 1.9.3 hash chain); `delta` is
// scratch of 2 bytes per input byte.  hipErrorInvalidValue for levels > 9.
// capOverride: 0xFFFFFFFF = n (lz4mt), 0xFFFFFFFE = n - 1 (-BD), else the cap.
// splitWs (hc_split_bytes, or null): blocks of at least 2 x hc_split_sub()
// bytes are parsed by several waves and spliced (slotStride >= blockSize).
hipError_t launch_encode_hc(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                            uint8_t* slots, uint64_t slotStride, uint32_t capOverride, int level, uint16_t* delta,
                            int32_t* csize, hipStream_t st, uint8_t* splitWs = nullptr);
uint32_t hc_split_sub();
uint64_t hc_split_bytes(uint64_t nBlocks, uint32_t blockSize);
uint64_t hc_ws_bytes(uint64_t nBlocks, uint32_t blockSize, int level);   // splitWs size for a level
uint32_t hc_attempts(int level);   // lz4hc nbSearches of a level (> 12 = 12)
// -BD at level >= 3: segments [begin[k], end[k]) of src (begin >= -64 KiB),
// blockSeg[b] = block b's segment; delta0 = chain scratch for src[0], with
// 64 Ki entries before it.
hipError_t launch_encode_hc_bd(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                               uint8_t* slots, const int64_t* segBegin, const int64_t* segEnd, uint32_t nSeg,
                               const uint32_t* blockSeg, uint16_t* delta0, int32_t* csize, hipStream_t st);
hipError_t launch_encode_linked(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                                uint8_t* slots, const LinkPlan* plan, uint32_t* table, bool fresh, bool xh, int32_t* csize,
                                hipStream_t st);
// The block-dependent encode as parallel fixed-point rounds
// (k_encode_linked_round / k_link_settle; the serial kernel finishes from
// the first unsettled block if kLinkRounds rounds do not settle).
constexpr int kLinkRounds = 32;
uint64_t link_round_bytes(uint64_t nBlocks);   // scratch: entry + exit tables, round control words
hipError_t launch_encode_linked_par(const uint8_t* src, uint64_t srcSize, uint32_t blockSize, uint32_t nBlocks,
                                    uint8_t* slots, const LinkPlan* plan, uint32_t* table, bool fresh, bool xh,
                                    uint32_t* scratch, int32_t* csize, int rounds, hipStream_t st);
hipError_t launch_decode_linked(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t blockMax,
                                uint8_t* out, uint64_t outCap, uint8_t* slot, uint8_t* hist, const uint32_t* digest,
                                int blockChecksum, int32_t* dsize, int32_t* status, hipStream_t st);
// The same contract as launch_decode_linked (status, dsize, out, hist in/out),
// decoded in parallel fixed-point rounds (k_dlink_*; serial finish if
// `rounds` do not settle).  scratch: dlink_scratch_bytes(nBlocks, blockMax).
uint64_t dlink_scratch_bytes(uint64_t nBlocks, uint32_t blockMax);
// LZ4MT_AMD_BD_ROUNDS=k caps the -BD encode's parallel rounds (tests: the
// serial finish from the first unsettled block); default kLinkRounds
inline int env_rounds() {
    const char* e = getenv("LZ4MT_AMD_BD_ROUNDS");
    return e ? atoi(e) : kLinkRounds;
}
// LZ4MT_AMD_BD_REFERENCE=1: -BD frames with 1 and 4 MiB blocks written byte
// for byte as the reference writes them (its input buffer replayed by BdSim:
// each block after the first read over its own dictionary, frames that do
// not decode back -- DESIGN.md §1).  Off by default: the decodable stream.
inline bool bd_reference_bytes() {
    const char* e = getenv("LZ4MT_AMD_BD_REFERENCE");
    return e && e[0] == '1';
}
// LZ4MT_AMD_BD_SERIAL=1: the one-wave -BD kernels only (A/B and tests)
inline bool bd_serial() {
    const char* e = getenv("LZ4MT_AMD_BD_SERIAL");
    return e && e[0] == '1';
}
hipError_t launch_decode_linked_par(const uint8_t* frame, const BlockRec* recs, uint32_t nBlocks, uint32_t blockMax,
                                    uint8_t* out, uint64_t outCap, uint8_t* hist, const uint32_t* digest,
                                    int blockChecksum, int32_t* dsize, int32_t* status, uint8_t* scratch, int rounds,
                                    hipStream_t st);

}  // namespace lz4mt
