/* split_sim.c -- how far two LZ4 1.9.3 greedy parses of one 4 MiB block must
 * run before they agree for good (the overlap a split parse of the block
 * needs).  Analysis tool, not product.
 *
 * parse(): lz4 1.9.3 LZ4_compress_generic, byU32 table (4096 entries, hash5),
 * no dictionary, acceleration 1 -- the parse k_encode reproduces (SURVEY.md
 * App. A) -- started at position s with anchor = s and every table entry out
 * of range (s = 0: the real block parse, whose fresh entries are position 0).
 * It records, per sequence, the probe that hit (before the catch-up) and the
 * match end; the match ends are the loop tops where the parse state is
 * (ip = anchor, table).  Two parses that pass the same loop top and then hit
 * the same probes with the same match ends for 64 KiB have written the same
 * table entries for every position that can still be a candidate, so they
 * agree from there on.
 * build: gcc -O2 -shared -fPIC -o /tmp/split_sim.so tools/split_sim.c */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t hash5(const uint8_t* p) {
    return (uint32_t)(((rd64(p) << 24) * 889523592379ULL) >> (64 - 12));
}
static inline uint32_t count(const uint8_t* a, const uint8_t* b, const uint8_t* lim) {
    const uint8_t* s = a;
    while (a < lim && *a == *b) { a++; b++; }
    return (uint32_t)(a - s);
}

/* returns the number of sequences; hit[i] = probe position that found
 * sequence i's match, end[i] = its match end (positions relative to src) */
int parse(const uint8_t* src, uint32_t n, uint32_t s, uint32_t* hit, uint32_t* end, int cap, uint32_t* start) {
    uint32_t T[4096];
    const uint32_t INV = 0x80000000u;   /* out of range for every probe */
    for (int i = 0; i < 4096; ++i) T[i] = s == 0 ? 0u : INV;
    const uint8_t* base = src;
    const uint8_t* iend = src + n;
    const uint8_t* mflimitP1 = iend - 12 + 1;
    const uint8_t* matchlimit = iend - 5;
    const uint8_t* ip = src + s;
    const uint8_t* anchor = ip;
    int k = 0;
    if (n - s < 13) return 0;
    T[hash5(ip)] = (uint32_t)(ip - base);
    ip++;
    uint32_t fh = hash5(ip);
    for (;;) {
        const uint8_t* match;
        const uint8_t* fip = ip;
        uint32_t step = 1, nb = 1u << 6;
        for (;;) {
            const uint32_t h = fh, cur = (uint32_t)(fip - base), mi = T[h];
            ip = fip;
            fip += step;
            step = nb++ >> 6;
            if (fip > mflimitP1) return k;
            match = base + (mi == INV ? 0 : mi);
            fh = hash5(fip);
            T[h] = cur;
            if (mi == INV || mi + 65535u < cur) continue;
            if (rd32(match) == rd32(ip)) break;
        }
        uint32_t hp = (uint32_t)(ip - base);
        while (ip > anchor && match > src && ip[-1] == match[-1]) { ip--; match--; }
        for (;;) {   /* _next_match */
            const uint32_t mstart = (uint32_t)(ip - base);
            ip += 4 + count(ip + 4, match + 4, matchlimit);
            anchor = ip;
            if (k < cap) { hit[k] = hp; end[k] = (uint32_t)(ip - base); if (start) start[k] = mstart; }
            k++;
            if (ip >= mflimitP1) return k;
            T[hash5(ip - 2)] = (uint32_t)(ip - 2 - base);
            const uint32_t h = hash5(ip), cur = (uint32_t)(ip - base), mi = T[h];
            T[h] = cur;
            if (mi != INV && mi + 65535u >= cur && rd32(base + mi) == rd32(ip)) {
                match = base + mi;
                hp = cur;   /* the TEST hit: the next sequence's probe is ip itself */
                continue;
            }
            break;
        }
        fh = hash5(++ip);
    }
}

/* False candidates a tag must filter: lz4 1.9.3's search loop on one block
 * (byU16 table, hash4, 8192 entries, blocks below 65 547 B; or byU32 as
 * parse() above), counting the probes whose table entry is a usable
 * candidate whose 4 bytes differ from ip's -- each costs the encoder a
 * round trip whenever its tag happens to match (probability 2^-tagbits).
 * Returns the number of sequences; *probes / *falseCand accumulate. */
static inline uint32_t hash4(const uint8_t* p) { return (rd32(p) * 2654435761U) >> (32 - 13); }
int false_cands(const uint8_t* src, uint32_t n, int u16, uint64_t* probes, uint64_t* falseCand) {
    static uint32_t T[8192];
    memset(T, 0, sizeof(T));
    const uint8_t* base = src;
    const uint8_t* iend = src + n;
    const uint8_t* mflimitP1 = iend - 12 + 1;
    const uint8_t* matchlimit = iend - 5;
    const uint8_t* ip = src;
    const uint8_t* anchor = ip;
    int k = 0;
    if (n < 13) return 0;
#define HSH(p) (u16 ? hash4(p) : hash5(p))
    T[HSH(ip)] = 0;
    ip++;
    uint32_t fh = HSH(ip);
    for (;;) {
        const uint8_t* match;
        const uint8_t* fip = ip;
        uint32_t step = 1, nb = 1u << 6;
        for (;;) {
            const uint32_t h = fh, cur = (uint32_t)(fip - base), mi = T[h];
            ip = fip;
            fip += step;
            step = nb++ >> 6;
            if (fip > mflimitP1) return k;
            match = base + mi;
            fh = HSH(fip);
            T[h] = cur;
            ++*probes;
            if (!u16 && mi + 65535u < cur) continue;
            if (rd32(match) == rd32(ip)) break;
            ++*falseCand;
        }
        while (ip > anchor && match > src && ip[-1] == match[-1]) { ip--; match--; }
        for (;;) {
            ip += 4 + count(ip + 4, match + 4, matchlimit);
            anchor = ip;
            k++;
            if (ip >= mflimitP1) return k;
            T[HSH(ip - 2)] = (uint32_t)(ip - 2 - base);
            const uint32_t h = HSH(ip), cur = (uint32_t)(ip - base), mi = T[h];
            T[h] = cur;
            ++*probes;
            if ((u16 || mi + 65535u >= cur) && rd32(base + mi) == rd32(ip)) { match = base + mi; continue; }
            if (u16 || mi + 65535u >= cur) ++*falseCand;
            break;
        }
        fh = HSH(++ip);
    }
#undef HSH
}
