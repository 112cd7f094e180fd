// lz4mt_shard.hip — the block-sharded streamed gather.
//
// Multi-GPU compress of ONE frame: rank r owns a contiguous block range
// (blocks are independent, FLG bit 5, reference src/lz4mt.cpp:914-918,
// 991-995).  Gathering each rank's finished record run only after its
// encode (dist.gather_frame) leaves the whole transfer -- (G-1)/G of the
// compressed bytes into the root's inbound xGMI links -- behind the encode,
// because every block of a shard finishes at about the same time (2048
// serial parses running side by side).  Here the transfer runs DURING the
// encode instead:
//
//   k_encode_pub (lz4mt_kernels.hip)   the frame encoder that, every 64 KiB of
//                                      a block's output, releases the bytes
//                                      written so far and publishes the count
//                                      (pub[b])
//   k_shard_plan  + k_shard_pack       one round on the sending rank: what was
//                                      published since the last round (at most
//                                      perBlockCap bytes per block), packed
//                                      into one contiguous buffer with a
//                                      descriptor per block -- one RCCL send
//   k_shard_unpack                     the root puts a received pack into its
//                                      mirror of that rank's slots
//   frame scan + assemble              once every rank is done, the root lays
//                                      each shard's records into the frame
//
// The last round (after a rank's encode) also carries the block tails,
// incompressible blocks as source bytes, the stored sizes and the block
// checksums.  The pack layout is the wire format between ranks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "../../include/lz4mt_hip.h"
#include "lz4mt_device.h"
#include "lz4mt_host.h"

namespace lz4mt {
namespace shard {

typedef const __attribute__((address_space(1))) uint8_t g_cu8;
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef const __attribute__((address_space(1))) uint32_t g_cu32;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_u4;

__device__ __forceinline__ g_cu8* gp(const uint8_t* p) { return (g_cu8*)p; }
__device__ __forceinline__ g_u8* gp(uint8_t* p) { return (g_u8*)p; }

constexpr uint64_t kMagic = 0x44485354344D5A4Cull;   // "LZ4MTSHD"
constexpr uint32_t kRawBit = 0x80000000u;            // desc.lo / sent: source bytes (incompressible block)
constexpr uint32_t kFlagFinal = 1u;                  // csize / bsum valid: the shard is complete

struct PackHdr {              // 64 bytes at the start of a pack
    uint64_t magic;
    uint64_t dataBytes;       // payload bytes in this pack
    uint64_t remaining;       // bytes still to send after this pack (final rounds)
    uint64_t packedBytes;     // bytes of the whole pack (header .. end of payload)
    uint32_t nb, flags;
    uint64_t bodyBytes;       // kFlagFinal: the shard's record bytes (its frame body)
    uint64_t pad[2];
};
static_assert(sizeof(PackHdr) == 64, "pack header");
struct Desc {                 // per block: bytes [lo, lo + len) of its slot (or source)
    uint32_t lo, len;
    uint64_t off;             // payload offset of those bytes in this pack
};
static_assert(sizeof(Desc) == 16, "desc");

__host__ __device__ inline uint64_t al256(uint64_t v) { return (v + 255) & ~255ull; }
__host__ __device__ inline uint64_t desc_off() { return sizeof(PackHdr); }
__host__ __device__ inline uint64_t csize_off(uint64_t nb) { return desc_off() + 16 * nb; }
__host__ __device__ inline uint64_t bsum_off(uint64_t nb) { return csize_off(nb) + 4 * nb; }
__host__ __device__ inline uint64_t data_off(uint64_t nb) { return al256(bsum_off(nb) + 4 * nb); }

// Shard workspace (and the root's mirror of a shard: same layout)
struct ShardWs {
    uint8_t* slots;    // nb x bm (+64): block b's encoded bytes at b * bm
    int32_t* csize;    // nb + 1: stored size, <= 0 = raw
    uint32_t* bsum;    // nb + 1: block XXH32 of the stored bytes
    uint64_t* recOff;  // nb + 1: record offsets (assembly)
    uint32_t* pub;     // nb: published bytes (k_encode_pub)
    uint32_t* sent;    // nb: bytes already packed (| kRawBit: source bytes)
    uint32_t* xdone;   // nb: block checksum finished by k_xxh32_follow
    uint64_t bytes;
};
inline ShardWs carve(uint8_t* base, uint64_t nb, uint64_t bm) {
    ShardWs w{};
    uint64_t o = 0;
    auto take = [&](uint64_t n) { uint8_t* p = base ? base + o : nullptr; o = al256(o + n); return p; };
    w.slots = take(nb * bm + 64);
    w.csize = reinterpret_cast<int32_t*>(take((nb + 1) * 4));
    w.bsum = reinterpret_cast<uint32_t*>(take((nb + 1) * 4));
    w.recOff = reinterpret_cast<uint64_t*>(take((nb + 1) * 8));
    w.pub = reinterpret_cast<uint32_t*>(take(nb * 4 + 4));
    w.sent = reinterpret_cast<uint32_t*>(take(nb * 4 + 4));
    w.xdone = reinterpret_cast<uint32_t*>(take(nb * 4 + 4));
    w.bytes = o;
    return w;
}

// Copies L bytes from S to D (any alignment of either) with one workgroup:
// unaligned head / tail bytes, and 16-B aligned destination chunks gathered
// from 4-B aligned source words in between.  Reads at most 3 bytes before S
// and 3 past S + L (inside the slots / pack buffers, which carry slack).
__device__ __forceinline__ void wg_copy(g_u8* D, g_cu8* S, uint64_t L, uint32_t t, uint32_t nt) {
    const uintptr_t Da = reinterpret_cast<uintptr_t>(D);
    const uintptr_t A0 = (Da + 15) & ~uintptr_t(15);
    const uintptr_t E0 = (Da + L) & ~uintptr_t(15);
    if (A0 >= E0) {
        for (uint64_t i = t; i < L; i += nt) D[i] = S[i];
        return;
    }
    const uint64_t head = A0 - Da, tailStart = E0 - Da;
    for (uint64_t i = t; i < head; i += nt) D[i] = S[i];
    for (uint64_t i = tailStart + t; i < L; i += nt) D[i] = S[i];
    const uintptr_t Sa = reinterpret_cast<uintptr_t>(S);
    const uint32_t sm = (uint32_t)(Sa & 3);
    g_cu32* base = (g_cu32*)(Sa - sm);
    const uint64_t nchunks = (E0 - A0) >> 4;
    for (uint64_t j = t; j < nchunks; j += nt) {
        const uint64_t so = head + 16 * j + sm;   // byte offset from `base`
        g_cu32* q = base + (so >> 2);
        const uint32_t s3 = (uint32_t)(so & 3);
        const uint32_t a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
        const uint32_t a4 = s3 ? q[4] : 0u;
        v4u v;
        v.x = __builtin_amdgcn_alignbyte(a1, a0, s3);
        v.y = __builtin_amdgcn_alignbyte(a2, a1, s3);
        v.z = __builtin_amdgcn_alignbyte(a3, a2, s3);
        v.w = __builtin_amdgcn_alignbyte(a4, a3, s3);
        *(g_u4*)(D + head + 16 * j) = v;
    }
}

// One round's plan, ONE wave and no LDS (while the encode runs, every CU's
// LDS is taken by its 8 encoder waves: a kernel that needs LDS would wait for
// the encode to end): per block the bytes to send now, their payload offsets
// (a wave scan through lane shuffles), the header.  Non-final rounds read
// the encoder's published counts (relaxed agent-scope loads: the encoder is
// still running); final rounds (stream-ordered after the encode) the stored
// sizes, and incompressible blocks switch to their source bytes.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
    const uint32_t L = __lane_id();
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(v, d, 64);
        if (L >= d) v += u;
    }
    return v;
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
    for (uint32_t d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

__global__ void __launch_bounds__(64) k_shard_plan(uint32_t* pub, uint32_t* __restrict__ sent,
                                                   const int32_t* __restrict__ csize,
                                                   const uint32_t* __restrict__ bsum, uint64_t srcSize, uint32_t bm,
                                                   uint32_t nb, int final, uint32_t cap, int bck,
                                                   uint8_t* __restrict__ pack) {
    Desc* desc = reinterpret_cast<Desc*>(pack + desc_off());
    int32_t* pcs = reinterpret_cast<int32_t*>(pack + csize_off(nb));
    uint32_t* pbs = reinterpret_cast<uint32_t*>(pack + bsum_off(nb));
    const uint32_t t = __lane_id();
    const uint32_t per = (nb + 63) / 64;
    const uint32_t lo0 = min(nb, t * per), hi0 = min(nb, lo0 + per);
    uint64_t sum = 0, rsum = 0, bsz = 0;
    for (uint32_t b = lo0; b < hi0; ++b) {
        const uint32_t n = (uint32_t)min<uint64_t>(bm, srcSize - (uint64_t)b * bm);
        uint32_t s = sent[b], lo, hi;
        bool raw = false;
        if (final) {
            const int32_t cs = csize[b];
            if (cs > 0) {
                hi = (uint32_t)cs;
            } else {
                if (!(s & kRawBit)) s = kRawBit;   // restart from the block's source bytes
                raw = true;
                hi = n;
            }
            bsz += 4ull + (cs > 0 ? (uint64_t)cs : n) + (bck ? 4ull : 0ull);
            pcs[b] = cs;
            pbs[b] = bck ? bsum[b] : 0u;
        } else {
            // while encoding: bytes final so far; once done: the stored size
            // (or kPubRaw: the final round sends the source bytes instead)
            const uint32_t pv = __hip_atomic_load(pub + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            hi = (pv & 0x40000000u) ? 0u : (pv & 0x3FFFFFFFu);
        }
        // never past the block's slot (its stored bytes are at most n), never
        // from past what is available: a workspace whose round state was not
        // reset then packs nothing wrong-sized instead of
        // reading outside the slots
        hi = min(hi, n);
        lo = min(s & ~kRawBit, hi);
        const uint32_t avail = hi > lo ? hi - lo : 0u;
        const uint32_t len = min(avail, cap);
        desc[b] = Desc{lo | (raw ? kRawBit : 0u), len, 0};
        sent[b] = (raw ? kRawBit : 0u) | (lo + len);
        sum += len;
        rsum += avail - len;
    }
    const uint64_t incl = wave_incl_scan(sum);
    uint64_t run = incl - sum;
    for (uint32_t b = lo0; b < hi0; ++b) {
        desc[b].off = run;
        run += desc[b].len;
    }
    const uint64_t total = __shfl(incl, 63, 64);
    const uint64_t remT = wave_sum(rsum), bodyT = wave_sum(bsz);
    if (t == 0) {
        PackHdr* h = reinterpret_cast<PackHdr*>(pack);
        h->magic = kMagic;
        h->dataBytes = total;
        h->remaining = remT;
        h->packedBytes = data_off(nb) + total;
        h->nb = nb;
        h->flags = (final && remT == 0) ? kFlagFinal : 0u;
        h->bodyBytes = final ? bodyT : 0;
        h->pad[0] = h->pad[1] = 0;
    }
}

// Copies each block's planned bytes into the pack (a new launch after the
// plan: its start is the agent-scope acquire that makes the released bytes
// visible here, whichever XCD wrote them).
__global__ void __launch_bounds__(256) k_shard_pack(const uint8_t* __restrict__ src, const uint8_t* __restrict__ slots,
                                                    uint32_t bm, uint32_t nb, uint8_t* __restrict__ pack) {
    const uint32_t b = blockIdx.x;
    const Desc d = reinterpret_cast<const Desc*>(pack + desc_off())[b];
    if (d.len == 0) return;
    const bool raw = d.lo & kRawBit;
    const uint64_t at = (uint64_t)b * bm + (d.lo & ~kRawBit);
    wg_copy(gp(pack) + data_off(nb) + d.off, raw ? gp(src) + at : gp(slots) + at, d.len, threadIdx.x, 256);
}

// Root: a received pack into the mirror of that shard's slots (source bytes
// of an incompressible block land in its slot too: the assembly reads raw
// blocks from the mirror).
// The pack may have been written into this device's memory by ANOTHER
// device's copy engine (IpcPushTransport): no XCD L2 here saw those writes,
// and this workgroup's L2 may still hold lines of the same buffer from the
// round that used it two rounds ago.  The receive buffers are allocated
// uncached where the runtime allows (lz4mtHipIpcAllocKind), and every
// workgroup starts with a system-scope acquire (buffer_inv sc0 sc1: L1 and
// the non-coherent L2 lines invalidated) before its first read of the pack.
__global__ void __launch_bounds__(256) k_shard_unpack(const uint8_t* __restrict__ pack, uint32_t bm, uint32_t nb,
                                                      uint8_t* __restrict__ mirror, int32_t* __restrict__ csize,
                                                      uint32_t* __restrict__ bsum) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint32_t b = blockIdx.x;
    const PackHdr* h = reinterpret_cast<const PackHdr*>(pack);
    if ((h->flags & kFlagFinal) && threadIdx.x == 0) {
        csize[b] = reinterpret_cast<const int32_t*>(pack + csize_off(nb))[b];
        bsum[b] = reinterpret_cast<const uint32_t*>(pack + bsum_off(nb))[b];
    }
    const Desc d = reinterpret_cast<const Desc*>(pack + desc_off())[b];
    if (d.len == 0) return;
    wg_copy(gp(mirror) + (uint64_t)b * bm + (d.lo & ~kRawBit), gp(pack) + data_off(nb) + d.off, d.len, threadIdx.x,
            256);
}

}  // namespace shard
}  // namespace lz4mt

using namespace lz4mt;
using namespace lz4mt::shard;

namespace {

#define SHCHK(x)                                          \
    do {                                                  \
        if ((x) != hipSuccess) return LZ4MT_RESULT_ERROR; \
    } while (0)

// A shardable descriptor: independent blocks, no content checksum (one
// serial chain over the whole stream), no content size (it would describe
// one shard), block size 64 KiB .. 4 MiB.
Lz4MtResult shard_sd(const Lz4MtStreamDescriptor* sd, uint32_t* bm) {
    if (!sd) return LZ4MT_RESULT_BAD_ARG;
    const Lz4MtResult v = validate_sd(sd);
    if (v != LZ4MT_RESULT_OK) return v;
    if (!sd->flg.blockIndependence || sd->flg.streamChecksum || sd->flg.streamSize) return LZ4MT_RESULT_BAD_ARG;
    *bm = (uint32_t)block_max_bytes(sd->bd.blockMaximumSize);
    return LZ4MT_RESULT_OK;
}

}  // namespace
bool follow_enabled();   // lz4mt_engine.hip: LZ4MT_AMD_FOLLOW=1
namespace {

bool use_pub(uint32_t bm) {   // k_encode_pub's v5 path: 1 and 4 MiB blocks (64 / 256 KiB keep their own kernels)
    return bm >= (1u << 20) && bm <= (4u << 20);
}

// The call order a shard workspace must follow: Reset, then
// Encode, then Packs -- kept per workspace address on the host, so that an
// Encode into a workspace whose round state was not reset since its last
// encode, or a Pack from one never encoded since its reset, returns BAD_ARG
// instead of packing from stale (or, on a fresh buffer, arbitrary) counts.
enum class WsState { kReset, kEncoded };
std::mutex g_ws_mu;
std::unordered_map<const void*, WsState> g_ws_state;
bool ws_advance(const void* ws, WsState need, WsState next) {
    std::lock_guard<std::mutex> g(g_ws_mu);
    auto it = g_ws_state.find(ws);
    if (it == g_ws_state.end() || it->second != need) return false;
    it->second = next;
    return true;
}
void ws_forget(const void* ws) {
    std::lock_guard<std::mutex> g(g_ws_mu);
    g_ws_state.erase(ws);
}
bool ws_is(const void* ws, WsState st) {
    std::lock_guard<std::mutex> g(g_ws_mu);
    auto it = g_ws_state.find(ws);
    return it != g_ws_state.end() && it->second == st;
}

}  // namespace

extern "C" uint64_t lz4mtHipShardWorkspaceSize(uint64_t n, const Lz4MtStreamDescriptor* sd) {
    uint32_t bm = 0;
    if (shard_sd(sd, &bm) != LZ4MT_RESULT_OK) return 0;
    return carve(nullptr, (n + bm - 1) / bm, bm).bytes;
}

extern "C" uint64_t lz4mtHipShardPackBound(uint64_t n, const Lz4MtStreamDescriptor* sd, uint32_t perBlockCap) {
    uint32_t bm = 0;
    if (shard_sd(sd, &bm) != LZ4MT_RESULT_OK) return 0;
    const uint64_t nb = (n + bm - 1) / bm;
    return data_off(nb) + nb * (uint64_t)std::min(perBlockCap, bm) + 64;
}

extern "C" int lz4mtHipFrameHeader(const Lz4MtStreamDescriptor* sd, uint8_t* out) {
    if (!sd || !out || validate_sd(sd) != LZ4MT_RESULT_OK) return -1;
    return build_header(sd, out);
}

// The round state (published / packed / hashed counts) of a workspace back to
// zero.  Separate from the encode: the encode and the rounds' packs run on
// two streams, and both must be ordered after the reset -- a pack that read
// `sent` or `pub` while another stream still zeroed them could pack from a
// stale (or, on a fresh buffer, arbitrary) offset.
extern "C" Lz4MtResult lz4mtHipShardReset(uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_ws, uint64_t wsSize,
                                          void* stream) {
    uint32_t bm = 0;
    const Lz4MtResult v = shard_sd(sd, &bm);
    if (v != LZ4MT_RESULT_OK) return v;
    const uint64_t nb = (n + bm - 1) / bm;
    if (!d_ws || wsSize < carve(nullptr, nb, bm).bytes || nb > 0xFFFFFFFFull) return LZ4MT_RESULT_BAD_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return LZ4MT_RESULT_ERROR;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const ShardWs w = carve(static_cast<uint8_t*>(d_ws), nb, bm);
    SHCHK(hipMemsetAsync(w.pub, 0, nb * 4 + 4, st));
    SHCHK(hipMemsetAsync(w.sent, 0, nb * 4 + 4, st));
    SHCHK(hipMemsetAsync(w.xdone, 0, nb * 4 + 4, st));
    std::lock_guard<std::mutex> g(g_ws_mu);
    g_ws_state[d_ws] = WsState::kReset;
    return LZ4MT_RESULT_OK;
}

namespace {
Lz4MtResult shard_encode_launches(const uint8_t* src, uint64_t n, const Lz4MtStreamDescriptor* sd, const ShardWs& w,
                                  uint32_t bm, uint64_t nb, hipStream_t st);
}  // namespace

extern "C" Lz4MtResult lz4mtHipShardEncode(const void* d_src, uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_ws,
                                           uint64_t wsSize, void* stream) {
    uint32_t bm = 0;
    const Lz4MtResult v = shard_sd(sd, &bm);
    if (v != LZ4MT_RESULT_OK) return v;
    const uint64_t nb = (n + bm - 1) / bm;
    if ((!d_src && n) || !d_ws || wsSize < carve(nullptr, nb, bm).bytes || nb > 0xFFFFFFFFull)
        return LZ4MT_RESULT_BAD_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return LZ4MT_RESULT_ERROR;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const ShardWs w = carve(static_cast<uint8_t*>(d_ws), nb, bm);
    const uint8_t* src = static_cast<const uint8_t*>(d_src);
    if (!ws_is(d_ws, WsState::kReset)) return LZ4MT_RESULT_BAD_ARG;   // not reset
    // encoded only once every launch went in: a failed launch
    // forgets the workspace, so only a new reset makes it usable again
    const Lz4MtResult r = shard_encode_launches(src, n, sd, w, bm, nb, st);
    if (r == LZ4MT_RESULT_OK) ws_advance(d_ws, WsState::kReset, WsState::kEncoded);
    else ws_forget(d_ws);
    return r;
}

namespace {
Lz4MtResult shard_encode_launches(const uint8_t* src, uint64_t n, const Lz4MtStreamDescriptor* sd, const ShardWs& w,
                                  uint32_t bm, uint64_t nb, hipStream_t st) {
    if (nb == 0) return LZ4MT_RESULT_OK;
    // block checksums hashed beside the encode (k_xxh32_follow on a side
    // stream; `stream` waits for it, so the shard is complete on `stream`)
    thread_local AuxStream aux;
    const bool follow = use_pub(bm) && sd->flg.blockChecksum && follow_enabled() && aux.ensure();
    if (follow) SHCHK(hipEventRecord(aux.evIn, st));
    SHCHK(use_pub(bm) ? launch_encode_pub(src, n, bm, (uint32_t)nb, w.slots, w.csize, w.pub, st)
                      : launch_encode(src, n, bm, (uint32_t)nb, w.slots, bm, 0xFFFFFFFFu, w.csize, st));
    if (follow) {   // launched after the encoder (one shared hardware queue would only serialise them)
        SHCHK(hipStreamWaitEvent(aux.st, aux.evIn, 0));
        SHCHK(launch_xxh32_follow(src, w.slots, n, bm, (uint32_t)nb, w.pub, w.bsum, w.xdone, aux.st));
        SHCHK(hipEventRecord(aux.evMid, st));
        SHCHK(hipStreamWaitEvent(aux.st, aux.evMid, 0));
        SHCHK(launch_xxh32_fixup(src, w.slots, n, bm, (uint32_t)nb, w.csize, w.bsum, w.xdone, aux.st));
        SHCHK(hipEventRecord(aux.evOut, aux.st));
        SHCHK(hipStreamWaitEvent(st, aux.evOut, 0));
    } else if (sd->flg.blockChecksum) {
        SHCHK(launch_xxh32_stored(src, w.slots, n, bm, (uint32_t)nb, w.csize, w.bsum, st));
    }
    return LZ4MT_RESULT_OK;
}
}  // namespace

// Forgets a workspace's call-order state: a freed workspace
// whose address a new allocation reuses must not inherit "encoded".  The
// Python binding calls it when the workspace tensor is freed; a forgotten
// workspace needs a reset before its next encode.
extern "C" void lz4mtHipShardRelease(const void* d_ws) { ws_forget(d_ws); }

extern "C" Lz4MtResult lz4mtHipShardPack(const void* d_src, uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_ws,
                                         uint64_t wsSize, void* d_pack, uint64_t packCap, uint32_t perBlockCap,
                                         int final, void* stream) {
    uint32_t bm = 0;
    const Lz4MtResult v = shard_sd(sd, &bm);
    if (v != LZ4MT_RESULT_OK) return v;
    const uint64_t nb = (n + bm - 1) / bm;
    if ((!d_src && n) || !d_ws || !d_pack || wsSize < carve(nullptr, nb, bm).bytes || perBlockCap == 0 ||
        packCap < lz4mtHipShardPackBound(n, sd, perBlockCap))
        return LZ4MT_RESULT_BAD_ARG;
    if (!ws_is(d_ws, WsState::kEncoded)) return LZ4MT_RESULT_BAD_ARG;   // no encode since the last reset
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const ShardWs w = carve(static_cast<uint8_t*>(d_ws), nb, bm);
    uint8_t* pack = static_cast<uint8_t*>(d_pack);
    hipLaunchKernelGGL(k_shard_plan, dim3(1), dim3(64), 0, st, w.pub, w.sent, w.csize, w.bsum, n, bm,
                       (uint32_t)nb, final ? 1 : 0, std::min(perBlockCap, bm), (int)sd->flg.blockChecksum, pack);
    SHCHK(hipGetLastError());
    if (nb) {
        hipLaunchKernelGGL(k_shard_pack, dim3((uint32_t)nb), dim3(256), 0, st, static_cast<const uint8_t*>(d_src),
                           w.slots, bm, (uint32_t)nb, pack);
        SHCHK(hipGetLastError());
    }
    return LZ4MT_RESULT_OK;
}

extern "C" Lz4MtResult lz4mtHipShardUnpack(const void* d_pack, uint64_t n, const Lz4MtStreamDescriptor* sd,
                                           void* d_mirror, uint64_t mirrorSize, void* stream) {
    uint32_t bm = 0;
    const Lz4MtResult v = shard_sd(sd, &bm);
    if (v != LZ4MT_RESULT_OK) return v;
    const uint64_t nb = (n + bm - 1) / bm;
    if (!d_pack || !d_mirror || mirrorSize < carve(nullptr, nb, bm).bytes) return LZ4MT_RESULT_BAD_ARG;
    if (nb == 0) return LZ4MT_RESULT_OK;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const ShardWs w = carve(static_cast<uint8_t*>(d_mirror), nb, bm);
    hipLaunchKernelGGL(k_shard_unpack, dim3((uint32_t)nb), dim3(256), 0, st, static_cast<const uint8_t*>(d_pack), bm,
                       (uint32_t)nb, w.slots, w.csize, w.bsum);
    SHCHK(hipGetLastError());
    return LZ4MT_RESULT_OK;
}

extern "C" Lz4MtResult lz4mtHipShardAssemble(const void* d_src, uint64_t n, const Lz4MtStreamDescriptor* sd,
                                             void* d_ws, uint64_t wsSize, void* d_body, uint64_t bodyCap,
                                             void* stream) {
    uint32_t bm = 0;
    const Lz4MtResult v = shard_sd(sd, &bm);
    if (v != LZ4MT_RESULT_OK) return v;
    const uint64_t nb = (n + bm - 1) / bm;
    if (!d_ws || wsSize < carve(nullptr, nb, bm).bytes || (!d_body && nb)) return LZ4MT_RESULT_BAD_ARG;
    if (nb == 0) return LZ4MT_RESULT_OK;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const ShardWs w = carve(static_cast<uint8_t*>(d_ws), nb, bm);
    // raw blocks: from the caller's source (the shard's own rank) or from the
    // mirror, whose slot holds the source bytes the last round carried
    const uint8_t* rawSrc = d_src ? static_cast<const uint8_t*>(d_src) : w.slots;
    const int bck = sd->flg.blockChecksum;
    SHCHK(launch_frame_scan(w.csize, n, bm, (uint32_t)nb, bck, w.recOff, st));
    // the records must fit: one small readback (a shard is assembled once)
    uint64_t body = 0;
    SHCHK(hipMemcpyAsync(&body, w.recOff + nb, 8, hipMemcpyDeviceToHost, st));
    SHCHK(hipStreamSynchronize(st));
    if (body > bodyCap) return LZ4MT_RESULT_BAD_ARG;
    SHCHK(launch_frame_assemble(rawSrc, w.slots, n, bm, (uint32_t)nb, w.csize, w.bsum, w.recOff, bck,
                                static_cast<uint8_t*>(d_body), 0, st));
    return LZ4MT_RESULT_OK;
}

extern "C" uint64_t lz4mtHipShardBodyBytes(uint64_t n, const Lz4MtStreamDescriptor* sd, void* d_ws, uint64_t wsSize,
                                          void* stream) {
    uint32_t bm = 0;
    if (shard_sd(sd, &bm) != LZ4MT_RESULT_OK) return UINT64_MAX;
    const uint64_t nb = (n + bm - 1) / bm;
    if (!d_ws || wsSize < carve(nullptr, nb, bm).bytes) return UINT64_MAX;
    if (nb == 0) return 0;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const ShardWs w = carve(static_cast<uint8_t*>(d_ws), nb, bm);
    uint64_t body = 0;
    if (launch_frame_scan(w.csize, n, bm, (uint32_t)nb, sd->flg.blockChecksum, w.recOff, st) != hipSuccess ||
        hipMemcpyAsync(&body, w.recOff + nb, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return UINT64_MAX;
    return body;
}

// ---- the root's receive buffers, shared with the senders (copy-engine push)
// Kinds, best first: 2 uncached device memory (hipDeviceMallocUncached: no
// XCD L2 ever holds a line of it, so a peer's copy-engine writes are what
// every later read sees), 1 fine-grained (its L2 lines are invalidated by
// the unpack's system-scope acquire), 0 plain hipMalloc (coarse-grained: the
// acquire still invalidates the reading CU's L1; the setup's pattern check
// is then the proof).  The first kind that allocates AND exports an IPC
// handle is taken; `want` caps the kind (2 = best available).
extern "C" int lz4mtHipIpcAllocKind(uint64_t bytes, void** d_ptr, void* handle64, int want, int* kind) {
    if (!d_ptr || !handle64) return -1;
    static_assert(sizeof(hipIpcMemHandle_t) <= 64, "ipc handle");
    const unsigned flags[3] = {0u, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
    const char* tr = getenv("LZ4MT_AMD_IPC_TRACE");
    const bool trace = tr && atoi(tr) != 0;
    const uint64_t n = bytes ? bytes : 1;
    for (int k = std::min(want, 2); k >= 0; --k) {
        // each kind at the size asked for, then rounded up to 2 MiB (whole
        // large pages of its own, never a sub-allocation of a shared chunk)
        const uint64_t sizes[2] = {n, (n + (2ull << 20) - 1) & ~((2ull << 20) - 1)};
        for (const uint64_t sz : sizes) {
            void* p = nullptr;
            const hipError_t e = k == 0 ? hipMalloc(&p, sz) : hipExtMallocWithFlags(&p, sz, flags[k]);
            hipError_t x = hipErrorUnknown;
            if (e == hipSuccess && p) {
                hipIpcMemHandle_t h;
                x = hipIpcGetMemHandle(&h, p);
                if (x == hipSuccess) {
                    memset(handle64, 0, 64);
                    memcpy(handle64, &h, sizeof(h));
                    *d_ptr = p;
                    if (kind) *kind = k;
                    return 0;
                }
                (void)hipFree(p);
            }
            (void)hipGetLastError();
            if (trace)
                fprintf(stderr, "lz4mt_amd: IPC receive buffer kind %d, %llu B: alloc %d, export %d\n", k,
                        (unsigned long long)sz, (int)e, (int)x);
        }
    }
    *d_ptr = nullptr;
    return -1;
}

// Plain hipMalloc memory, as before lz4mtHipIpcAllocKind existed (ADVICE r05:
// a caller that computes on the buffer keeps its L2); the push transport asks
// for uncached memory through lz4mtHipIpcAllocKind.
extern "C" int lz4mtHipIpcAlloc(uint64_t bytes, void** d_ptr, void* handle64) {
    return lz4mtHipIpcAllocKind(bytes, d_ptr, handle64, 0, nullptr);
}

// PCI bus id ("dddd:bb:dd.f") of device `dev`, and the ordinal of the visible
// device with a given bus id (-1: not visible here): the IPC setup names the
// root's GPU by bus id, which every process resolves to its own ordinal.
extern "C" int lz4mtHipDevicePciBusId(int dev, char* buf, int len) {
    if (!buf || len < 13) return -1;
    return hipDeviceGetPCIBusId(buf, len, dev) == hipSuccess ? 0 : -1;
}

extern "C" int lz4mtHipDeviceByPciBusId(const char* busId) {
    int dev = -1;
    if (!busId || hipDeviceGetByPCIBusId(&dev, busId) != hipSuccess) { (void)hipGetLastError(); return -1; }
    return dev;
}

extern "C" int lz4mtHipCanAccessPeer(int dev, int peer) {
    int ok = 0;
    if (dev == peer) return 1;
    return hipDeviceCanAccessPeer(&ok, dev, peer) == hipSuccess ? (ok ? 1 : 0) : -1;
}

extern "C" int lz4mtHipIpcOpen(const void* handle64, void** d_ptr) {
    if (!handle64 || !d_ptr) return -1;
    hipIpcMemHandle_t h;
    memcpy(&h, handle64, sizeof(h));
    if (hipIpcOpenMemHandle(d_ptr, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) { *d_ptr = nullptr; return -1; }
    return 0;
}

extern "C" int lz4mtHipIpcClose(void* d_ptr) { return hipIpcCloseMemHandle(d_ptr) == hipSuccess ? 0 : -1; }

extern "C" int lz4mtHipFree(void* d_ptr) { return hipFree(d_ptr) == hipSuccess ? 0 : -1; }

// device-to-device copy (another device's memory mapped by lz4mtHipIpcOpen
// included: the runtime moves it with a copy engine or a blit, no LDS)
extern "C" int lz4mtHipCopyAsync(void* d_dst, const void* d_src, uint64_t n, void* stream) {
    if (!n) return 0;
    return hipMemcpyAsync(d_dst, d_src, n, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)) == hipSuccess
               ? 0 : -1;
}

// ---------------------------------------------------------------------------
// Diagnostics: FETCH_SIZE calibration (tools/fetch_cal.py).  Reads n bytes
// exactly once, every lane `width` bytes per load (1, 4, 8 or 16: the
// encoder's byte, gld4u, gld8u loads and a dwordx4 stream), 64 x width
// contiguous bytes per wave instruction, consecutive loads of one lane
// 64 x width apart (so they stay separate instructions).  The XOR of every
// word is stored only if it equals `never` (a run-time argument the host
// picks so that it cannot match): the loads stay, with no store per load.
// ---------------------------------------------------------------------------
namespace lz4mt { namespace shard {
template <int W>
__global__ void __launch_bounds__(256) k_fetch_cal(const uint8_t* __restrict__ p, uint64_t n,
                                                   uint32_t* __restrict__ out, uint32_t never) {
    const uint64_t waves = (uint64_t)gridDim.x * 4;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t L = threadIdx.x & 63;
    const uint64_t step = 64ull * W;
    uint32_t acc = 0;
    for (uint64_t c = wave * step; c + step <= n; c += waves * step) {
        g_cu8* q = gp(p) + c + (uint64_t)L * W;
        if constexpr (W == 1) acc ^= *q;
        else if constexpr (W == 4) acc ^= *(g_cu32*)q;
        else if constexpr (W == 8) {
            const uint64_t v = *(const __attribute__((address_space(1))) uint64_t*)q;
            acc ^= (uint32_t)v ^ (uint32_t)(v >> 32);
        } else {
            const v4u v = *(const __attribute__((address_space(1))) v4u*)q;
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == never) out[0] = acc;
}
}}  // namespace lz4mt::shard

extern "C" int lz4mtHipDebugFetchCal(const void* d_buf, uint64_t n, int width, void* d_out4, void* stream) {
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 g(256 * 16), b(256);
    const uint8_t* p = static_cast<const uint8_t*>(d_buf);
    uint32_t* o = static_cast<uint32_t*>(d_out4);
    switch (width) {
        case 1: hipLaunchKernelGGL(k_fetch_cal<1>, g, b, 0, st, p, n, o, 0xFFFFFFFFu); break;
        case 4: hipLaunchKernelGGL(k_fetch_cal<4>, g, b, 0, st, p, n, o, 0xFFFFFFFFu); break;
        case 8: hipLaunchKernelGGL(k_fetch_cal<8>, g, b, 0, st, p, n, o, 0xFFFFFFFFu); break;
        case 16: hipLaunchKernelGGL(k_fetch_cal<16>, g, b, 0, st, p, n, o, 0xFFFFFFFFu); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
