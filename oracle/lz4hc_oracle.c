/*
 * lz4hc_oracle.c — CPU restatement of LZ4-HC 1.9.3 as lz4mt calls it
 * (TEST INFRASTRUCTURE ONLY; see lz4_oracle.h).
 *
 * lz4mt selects LZ4_compressHC2_limitedOutput(src, dst, n, cap = n, level)
 * for compression levels >= 3 (ref src/main.cpp:778-785; the reference
 * then stores the block raw when it returns <= 0, src/lz4mt.cpp:391-394).
 * In lz4 1.9.3 that is LZ4_compress_HC on a fresh state: levels 1..9 run
 * LZ4HC_compress_hashChain with maxNbAttempts = 2,2,2,4,8,16,32,64,128,256
 * (clTable), pattern analysis from 256 attempts (level 9), no chain swap,
 * favorCompressionRatio.  Levels 10..12 (and above, clamped to 12: the
 * CLI's -A asks for 17) run LZ4HC_compress_optimal: nbSearches 96 / 512 /
 * 16384, target length 64 / 128 / LZ4_OPT_NUM, full update at 12, pattern
 * analysis and chain swap in every search.
 *
 * Positions are indices from src; lz4hc's own indices are these + 64 KiB
 * (LZ4HC_init_internal: startingOffset = 64 KB), which only matters for the
 * zero-initialised tables: hash entry 0 and chain delta 0 of a fresh state.
 * Pinned against liblz4 1.9.3's LZ4_compress_HC by tests/test_oracle.py.
 */
#include "lz4_oracle.h"

#include <stdlib.h>
#include <string.h>

#define HC_MINMATCH 4
#define HC_LASTLITERALS 5
#define HC_MFLIMIT 12
#define HC_MIN_LENGTH 13
#define HC_DIST_MAX 65535u
#define HC_HASH_LOG 15
#define HC_OPTIMAL_ML 18          /* (ML_MASK - 1) + MINMATCH */
#define HC_BASE 65536u            /* index of src[0] (startingOffset) */

typedef struct {
    const uint8_t* s;   /* src */
    int n;
    uint32_t* hashTable;   /* 32768 entries, indices (0 = never set) */
    uint16_t* chainTable;  /* 65536 deltas */
    uint32_t nextToUpdate; /* index */
} hc_ctx;

static inline uint32_t hc_rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint32_t hc_rd16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
static inline uint32_t hc_hash(uint32_t v) { return (v * 2654435761u) >> (32 - HC_HASH_LOG); }
/* byte at index i (index space, i >= HC_BASE) */
#define AT(c, i) ((c)->s + ((i) - HC_BASE))

/* LZ4HC_Insert */
static void hc_insert(hc_ctx* c, uint32_t target) {
    uint32_t idx = c->nextToUpdate;
    while (idx < target) {
        const uint32_t h = hc_hash(hc_rd32(AT(c, idx)));
        uint32_t delta = idx - c->hashTable[h];
        if (delta > HC_DIST_MAX) delta = HC_DIST_MAX;
        c->chainTable[(uint16_t)idx] = (uint16_t)delta;
        c->hashTable[h] = idx;
        idx++;
    }
    c->nextToUpdate = target;
}

/* LZ4_count: equal bytes of [a, limit) and [b, ...) */
static unsigned hc_count(const uint8_t* a, const uint8_t* b, const uint8_t* limit) {
    const uint8_t* s = a;
    while (a < limit && *a == *b) { a++; b++; }
    return (unsigned)(a - s);
}

/* LZ4HC_countBack: how far both sides extend backwards (<= 0) */
static int hc_count_back(const uint8_t* ip, const uint8_t* match, const uint8_t* iMin, const uint8_t* mMin) {
    int back = 0;
    const int min = (int)((iMin - ip) > (mMin - match) ? (iMin - ip) : (mMin - match));
    while (back > min && ip[back - 1] == match[back - 1]) back--;
    return back;
}

/* LZ4HC_countPattern / LZ4HC_reverseCountPattern for a one-byte pattern
 * (the only kind pattern analysis confirms): run length forward up to
 * iEnd, backward down to iLow. */
static unsigned hc_count_run(const uint8_t* ip, const uint8_t* iEnd, uint8_t b) {
    const uint8_t* s = ip;
    while (ip < iEnd && *ip == b) ip++;
    return (unsigned)(ip - s);
}
static unsigned hc_rcount_run(const uint8_t* ip, const uint8_t* iLow, uint8_t b) {
    const uint8_t* s = ip;
    while (ip > iLow && ip[-1] == b) ip--;
    return (unsigned)(s - ip);
}

/* LZ4HC_InsertAndGetWiderMatch (noDictCtx, single segment: every candidate
 * is in the prefix, dictLimit = lowLimit = HC_BASE; chainSwap on for the
 * optimal parser only). */
static int hc_wider_match(hc_ctx* c, const uint8_t* ip, const uint8_t* iLowLimit, const uint8_t* iHighLimit,
                          int longest, const uint8_t** matchpos, const uint8_t** startpos, int maxNbAttempts,
                          int patternAnalysis, int chainSwap) {
    const uint32_t ipIndex = (uint32_t)(ip - c->s) + HC_BASE;
    const uint32_t lowestMatchIndex = (HC_BASE + HC_DIST_MAX + 1 > ipIndex) ? HC_BASE : ipIndex - HC_DIST_MAX;
    const uint8_t* const lowPrefixPtr = c->s;
    const int lookBackLength = (int)(ip - iLowLimit);
    int nbAttempts = maxNbAttempts;
    const uint32_t pattern = hc_rd32(ip);
    int repeat = 0;   /* 0 untested, 1 confirmed, 2 not */
    size_t srcPatternLength = 0;

    uint32_t matchChainPos = 0;
    hc_insert(c, ipIndex);
    uint32_t matchIndex = c->hashTable[hc_hash(pattern)];
    while (matchIndex >= lowestMatchIndex && nbAttempts > 0) {
        int matchLength = 0;
        nbAttempts--;
        {
            const uint8_t* const matchPtr = AT(c, matchIndex);
            if (hc_rd16(iLowLimit + longest - 1) == hc_rd16(matchPtr - lookBackLength + longest - 1)) {
                if (hc_rd32(matchPtr) == pattern) {
                    const int back = lookBackLength ? hc_count_back(ip, matchPtr, iLowLimit, lowPrefixPtr) : 0;
                    matchLength = HC_MINMATCH + (int)hc_count(ip + HC_MINMATCH, matchPtr + HC_MINMATCH, iHighLimit);
                    matchLength -= back;
                    if (matchLength > longest) {
                        longest = matchLength;
                        *matchpos = matchPtr + back;
                        *startpos = ip + back;
                    }
                }
            }
        }
        if (chainSwap && matchLength == longest) {   /* better match => select a better chain */
            if (matchIndex + (uint32_t)longest <= ipIndex) {
                const int kTrigger = 4;
                uint32_t distanceToNextMatch = 1;
                const int end = longest - HC_MINMATCH + 1;
                int step = 1;
                int accel = 1 << kTrigger;
                for (int pos = 0; pos < end; pos += step) {
                    const uint32_t candidateDist = c->chainTable[(uint16_t)(matchIndex + (uint32_t)pos)];
                    step = (accel++ >> kTrigger);
                    if (candidateDist > distanceToNextMatch) {
                        distanceToNextMatch = candidateDist;
                        matchChainPos = (uint32_t)pos;
                        accel = 1 << kTrigger;
                    }
                }
                if (distanceToNextMatch > 1) {
                    if (distanceToNextMatch > matchIndex) break;   /* avoid overflow */
                    matchIndex -= distanceToNextMatch;
                    continue;
                }
            }
        }
        {
            const uint32_t distNextMatch = c->chainTable[(uint16_t)matchIndex];
            if (patternAnalysis && distNextMatch == 1 && matchChainPos == 0) {
                const uint32_t matchCandidateIdx = matchIndex - 1;
                if (repeat == 0) {
                    if (((pattern & 0xFFFF) == (pattern >> 16)) & ((pattern & 0xFF) == (pattern >> 24))) {
                        repeat = 1;
                        srcPatternLength = hc_count_run(ip + 4, iHighLimit, (uint8_t)pattern) + 4;
                    } else {
                        repeat = 2;
                    }
                }
                /* LZ4HC_protectDictEnd(dictLimit, idx) holds for every idx >= lowest here */
                if (repeat == 1 && matchCandidateIdx >= lowestMatchIndex &&
                    (uint32_t)((HC_BASE - 1) - matchCandidateIdx) >= 3) {
                    const uint8_t* const matchPtr = AT(c, matchCandidateIdx);
                    if (hc_rd32(matchPtr) == pattern) {   /* good candidate */
                        const size_t forwardPatternLength =
                            hc_count_run(matchPtr + 4, iHighLimit, (uint8_t)pattern) + 4;
                        size_t backLength = hc_rcount_run(matchPtr, lowPrefixPtr, (uint8_t)pattern);
                        {
                            const uint32_t lo = matchCandidateIdx - (uint32_t)backLength;
                            backLength = matchCandidateIdx - (lo > lowestMatchIndex ? lo : lowestMatchIndex);
                        }
                        const size_t currentSegmentLength = backLength + forwardPatternLength;
                        if (currentSegmentLength >= srcPatternLength && forwardPatternLength <= srcPatternLength) {
                            matchIndex = matchCandidateIdx + (uint32_t)forwardPatternLength - (uint32_t)srcPatternLength;
                        } else {
                            matchIndex = matchCandidateIdx - (uint32_t)backLength;
                            if (lookBackLength == 0) {   /* no back possible */
                                const size_t maxML =
                                    currentSegmentLength < srcPatternLength ? currentSegmentLength : srcPatternLength;
                                if ((size_t)longest < maxML) {
                                    if (ipIndex - matchIndex > HC_DIST_MAX) break;
                                    longest = (int)maxML;
                                    *matchpos = AT(c, matchIndex);
                                    *startpos = ip;
                                }
                                {
                                    const uint32_t distToNextPattern = c->chainTable[(uint16_t)matchIndex];
                                    if (distToNextPattern > matchIndex) break;
                                    matchIndex -= distToNextPattern;
                                }
                            }
                        }
                        continue;
                    }
                }
            }
        }
        matchIndex -= c->chainTable[(uint16_t)(matchIndex + matchChainPos)];   /* follow the current chain */
    }
    return longest;
}

/* LZ4HC_encodeSequence; returns 1 on output overflow (limitedOutput) */
static int hc_encode(const uint8_t** ip, uint8_t** op, const uint8_t** anchor, int matchLength, const uint8_t* match,
                     int limit, const uint8_t* oend) {
    uint8_t* token = (*op)++;
    size_t length = (size_t)(*ip - *anchor);
    if (limit && (*op + (length / 255) + length + (2 + 1 + HC_LASTLITERALS)) > oend) return 1;
    if (length >= 15) {
        size_t len = length - 15;
        *token = (uint8_t)(15 << 4);
        for (; len >= 255; len -= 255) *(*op)++ = 255;
        *(*op)++ = (uint8_t)len;
    } else {
        *token = (uint8_t)(length << 4);
    }
    memcpy(*op, *anchor, length);
    *op += length;
    {
        const uint32_t off = (uint32_t)(*ip - match);
        (*op)[0] = (uint8_t)off;
        (*op)[1] = (uint8_t)(off >> 8);
        *op += 2;
    }
    length = (size_t)matchLength - HC_MINMATCH;
    if (limit && (*op + (length / 255) + (1 + HC_LASTLITERALS) > oend)) return 1;
    if (length >= 15) {
        *token += 15;
        length -= 15;
        for (; length >= 510; length -= 510) { *(*op)++ = 255; *(*op)++ = 255; }
        if (length >= 255) { length -= 255; *(*op)++ = 255; }
        *(*op)++ = (uint8_t)length;
    } else {
        *token += (uint8_t)length;
    }
    *ip += matchLength;
    *anchor = *ip;
    return 0;
}

/* LZ4HC_compress_hashChain over the n bytes at ip0 (inside c->s: the bytes
 * of c->s before ip0 are the prefix the stream has already seen, every
 * position of it inserted as LZ4HC_Insert does); 0 = does not fit cap. */
static int hc_compress_range(hc_ctx* c, const uint8_t* ip0, uint8_t* dst, int n, int cap, int maxNbAttempts,
                             int patternAnalysis) {
    const int limit = cap < orc_lz4_compress_bound(n);
    const uint8_t* ip = ip0;
    const uint8_t* anchor = ip;
    const uint8_t* const iend = ip + n;
    const uint8_t* const mflimit = iend - HC_MFLIMIT;
    const uint8_t* const matchlimit = iend - HC_LASTLITERALS;
    uint8_t* op = dst;
    const uint8_t* const oend = dst + cap;
    int ml0, ml, ml2, ml3;
    const uint8_t *start0, *ref0, *ref = NULL, *start2 = NULL, *ref2 = NULL, *start3 = NULL, *ref3 = NULL;
    int result = 0;

    if (n < HC_MIN_LENGTH) goto last_literals;
    while (ip <= mflimit) {
        {
            const uint8_t* useless = ip;
            ml = hc_wider_match(c, ip, ip, matchlimit, HC_MINMATCH - 1, &ref, &useless, maxNbAttempts,
                                patternAnalysis, 0);
        }
        if (ml < HC_MINMATCH) { ip++; continue; }
        start0 = ip; ref0 = ref; ml0 = ml;
    search2:
        if (ip + ml <= mflimit)
            ml2 = hc_wider_match(c, ip + ml - 2, ip, matchlimit, ml, &ref2, &start2, maxNbAttempts, patternAnalysis, 0);
        else
            ml2 = ml;
        if (ml2 == ml) {   /* no better match: encode ML1 */
            if (hc_encode(&ip, &op, &anchor, ml, ref, limit, oend)) goto overflow;
            continue;
        }
        if (start0 < ip && start2 < ip + ml0) { ip = start0; ref = ref0; ml = ml0; }   /* restore initial ML1 */
        if ((start2 - ip) < 3) {   /* first match too small: removed */
            ml = ml2; ip = start2; ref = ref2;
            goto search2;
        }
    search3:
        if ((start2 - ip) < HC_OPTIMAL_ML) {
            int new_ml = ml;
            if (new_ml > HC_OPTIMAL_ML) new_ml = HC_OPTIMAL_ML;
            if (ip + new_ml > start2 + ml2 - HC_MINMATCH) new_ml = (int)(start2 - ip) + ml2 - HC_MINMATCH;
            const int correction = new_ml - (int)(start2 - ip);
            if (correction > 0) { start2 += correction; ref2 += correction; ml2 -= correction; }
        }
        if (start2 + ml2 <= mflimit)
            ml3 = hc_wider_match(c, start2 + ml2 - 3, start2, matchlimit, ml2, &ref3, &start3, maxNbAttempts,
                                 patternAnalysis, 0);
        else
            ml3 = ml2;
        if (ml3 == ml2) {   /* no better match: encode ML1 and ML2 */
            if (start2 < ip + ml) ml = (int)(start2 - ip);
            if (hc_encode(&ip, &op, &anchor, ml, ref, limit, oend)) goto overflow;
            ip = start2;
            if (hc_encode(&ip, &op, &anchor, ml2, ref2, limit, oend)) goto overflow;
            continue;
        }
        if (start3 < ip + ml + 3) {   /* not enough space for match 2: remove it */
            if (start3 >= ip + ml) {  /* can write Seq1 immediately: Seq2 removed, Seq3 becomes Seq1 */
                if (start2 < ip + ml) {
                    const int correction = (int)(ip + ml - start2);
                    start2 += correction; ref2 += correction; ml2 -= correction;
                    if (ml2 < HC_MINMATCH) { start2 = start3; ref2 = ref3; ml2 = ml3; }
                }
                if (hc_encode(&ip, &op, &anchor, ml, ref, limit, oend)) goto overflow;
                ip = start3; ref = ref3; ml = ml3;
                start0 = start2; ref0 = ref2; ml0 = ml2;
                goto search2;
            }
            start2 = start3; ref2 = ref3; ml2 = ml3;
            goto search3;
        }
        /* three ascending matches: write ML1, ML2 becomes ML1, ML3 becomes ML2 */
        if (start2 < ip + ml) {
            if ((start2 - ip) < HC_OPTIMAL_ML) {
                if (ml > HC_OPTIMAL_ML) ml = HC_OPTIMAL_ML;
                if (ip + ml > start2 + ml2 - HC_MINMATCH) ml = (int)(start2 - ip) + ml2 - HC_MINMATCH;
                const int correction = ml - (int)(start2 - ip);
                if (correction > 0) { start2 += correction; ref2 += correction; ml2 -= correction; }
            } else {
                ml = (int)(start2 - ip);
            }
        }
        if (hc_encode(&ip, &op, &anchor, ml, ref, limit, oend)) goto overflow;
        ip = start2; ref = ref2; ml = ml2;
        start2 = start3; ref2 = ref3; ml2 = ml3;
        goto search3;
    }
last_literals:
    {
        const size_t lastRunSize = (size_t)(iend - anchor);
        const size_t llAdd = (lastRunSize + 255 - 15) / 255;
        const size_t totalSize = 1 + llAdd + lastRunSize;
        if (limit && op + totalSize > oend) goto overflow;
        if (lastRunSize >= 15) {
            size_t acc = lastRunSize - 15;
            *op++ = (uint8_t)(15 << 4);
            for (; acc >= 255; acc -= 255) *op++ = 255;
            *op++ = (uint8_t)acc;
        } else {
            *op++ = (uint8_t)(lastRunSize << 4);
        }
        memcpy(op, anchor, lastRunSize);
        op += lastRunSize;
    }
    result = (int)(op - dst);
overflow:
    return result;
}

/* ---- the optimal parser (levels 10..12: LZ4HC_compress_optimal 1.9.3) ---- */
#define HC_OPT_NUM 4096           /* LZ4_OPT_NUM */
#define HC_TRAILING_LITERALS 3

typedef struct { int price, off, mlen, litlen; } hc_opt_t;

/* LZ4HC_literalsPrice / LZ4HC_sequencePrice: bytes */
static int hc_lit_price(int litlen) {
    int price = litlen;
    if (litlen >= 15) price += 1 + (litlen - 15) / 255;
    return price;
}
static int hc_seq_price(int litlen, int mlen) {
    int price = 1 + 2 + hc_lit_price(litlen);
    if (mlen >= 15 + HC_MINMATCH) price += 1 + (mlen - (15 + HC_MINMATCH)) / 255;
    return price;
}

/* LZ4HC_FindLongerMatch: a match longer than minLen at ip (no look-back,
 * pattern analysis and chain swap on); len 0 if none */
static void hc_longer_match(hc_ctx* c, const uint8_t* ip, const uint8_t* iHighLimit, int minLen, int nbSearches,
                            int* len, int* off) {
    const uint8_t* matchPtr = NULL;
    const uint8_t* start = ip;
    const int ml = hc_wider_match(c, ip, ip, iHighLimit, minLen, &matchPtr, &start, nbSearches, 1, 1);
    if (ml <= minLen) { *len = 0; *off = 0; return; }
    *len = ml;
    *off = (int)(start - matchPtr);
}

/* LZ4HC_compress_optimal (favorCompressionRatio, noDictCtx); 0 = does not fit cap */
static int hc_compress_optimal(hc_ctx* c, const uint8_t* src, uint8_t* dst, int n, int cap, int nbSearches,
                               int sufficient_len, int fullUpdate, hc_opt_t* opt) {
    const int limit = cap < orc_lz4_compress_bound(n);
    const uint8_t* ip = src;
    const uint8_t* anchor = ip;
    const uint8_t* const iend = ip + n;
    const uint8_t* const mflimit = iend - HC_MFLIMIT;
    const uint8_t* const matchlimit = iend - HC_LASTLITERALS;
    uint8_t* op = dst;
    const uint8_t* const oend = dst + cap;
    if (sufficient_len >= HC_OPT_NUM) sufficient_len = HC_OPT_NUM - 1;

    while (ip <= mflimit) {
        const int llen = (int)(ip - anchor);
        int best_mlen, best_off, cur, last_match_pos = 0;
        int fmLen, fmOff;
        hc_longer_match(c, ip, matchlimit, HC_MINMATCH - 1, nbSearches, &fmLen, &fmOff);
        if (fmLen == 0) { ip++; continue; }
        if (fmLen > sufficient_len) {   /* good enough: immediate encoding */
            if (hc_encode(&ip, &op, &anchor, fmLen, ip - fmOff, limit, oend)) return 0;
            continue;
        }
        for (int rPos = 0; rPos < HC_MINMATCH; rPos++) {   /* literals at the first positions */
            opt[rPos].mlen = 1;
            opt[rPos].off = 0;
            opt[rPos].litlen = llen + rPos;
            opt[rPos].price = hc_lit_price(llen + rPos);
        }
        for (int mlen = HC_MINMATCH; mlen <= fmLen; mlen++) {   /* the first match */
            opt[mlen].mlen = mlen;
            opt[mlen].off = fmOff;
            opt[mlen].litlen = llen;
            opt[mlen].price = hc_seq_price(llen, mlen);
        }
        last_match_pos = fmLen;
        for (int addLit = 1; addLit <= HC_TRAILING_LITERALS; addLit++) {
            opt[last_match_pos + addLit].mlen = 1;
            opt[last_match_pos + addLit].off = 0;
            opt[last_match_pos + addLit].litlen = addLit;
            opt[last_match_pos + addLit].price = opt[last_match_pos].price + hc_lit_price(addLit);
        }
        for (cur = 1; cur < last_match_pos; cur++) {
            const uint8_t* const curPtr = ip + cur;
            int nmLen, nmOff;
            if (curPtr > mflimit) break;
            if (fullUpdate) {
                if (opt[cur + 1].price <= opt[cur].price && opt[cur + HC_MINMATCH].price < opt[cur].price + 3) continue;
            } else {
                if (opt[cur + 1].price <= opt[cur].price) continue;
            }
            if (fullUpdate)
                hc_longer_match(c, curPtr, matchlimit, HC_MINMATCH - 1, nbSearches, &nmLen, &nmOff);
            else
                hc_longer_match(c, curPtr, matchlimit, last_match_pos - cur, nbSearches, &nmLen, &nmOff);
            if (!nmLen) continue;
            if (nmLen > sufficient_len || nmLen + cur >= HC_OPT_NUM) {   /* immediate encoding */
                best_mlen = nmLen;
                best_off = nmOff;
                last_match_pos = cur + 1;
                goto encode;
            }
            {   /* before the match: literals after the path to cur */
                const int baseLitlen = opt[cur].litlen;
                for (int litlen = 1; litlen < HC_MINMATCH; litlen++) {
                    const int price = opt[cur].price - hc_lit_price(baseLitlen) + hc_lit_price(baseLitlen + litlen);
                    const int pos = cur + litlen;
                    if (price < opt[pos].price) {
                        opt[pos].mlen = 1;
                        opt[pos].off = 0;
                        opt[pos].litlen = baseLitlen + litlen;
                        opt[pos].price = price;
                    }
                }
            }
            for (int ml = HC_MINMATCH; ml <= nmLen; ml++) {   /* the match at cur */
                const int pos = cur + ml;
                int price, ll;
                if (opt[cur].mlen == 1) {
                    ll = opt[cur].litlen;
                    price = ((cur > ll) ? opt[cur - ll].price : 0) + hc_seq_price(ll, ml);
                } else {
                    ll = 0;
                    price = opt[cur].price + hc_seq_price(0, ml);
                }
                if (pos > last_match_pos + HC_TRAILING_LITERALS || price <= opt[pos].price) {
                    if (ml == nmLen && last_match_pos < pos) last_match_pos = pos;
                    opt[pos].mlen = ml;
                    opt[pos].off = nmOff;
                    opt[pos].litlen = ll;
                    opt[pos].price = price;
                }
            }
            for (int addLit = 1; addLit <= HC_TRAILING_LITERALS; addLit++) {
                opt[last_match_pos + addLit].mlen = 1;
                opt[last_match_pos + addLit].off = 0;
                opt[last_match_pos + addLit].litlen = addLit;
                opt[last_match_pos + addLit].price = opt[last_match_pos].price + hc_lit_price(addLit);
            }
        }
        best_mlen = opt[last_match_pos].mlen;
        best_off = opt[last_match_pos].off;
        cur = last_match_pos - best_mlen;
    encode:
        {   /* reverse traversal: the shortest path's sequences */
            int candidate_pos = cur;
            int selected_matchLength = best_mlen;
            int selected_offset = best_off;
            for (;;) {
                const int next_matchLength = opt[candidate_pos].mlen;
                const int next_offset = opt[candidate_pos].off;
                opt[candidate_pos].mlen = selected_matchLength;
                opt[candidate_pos].off = selected_offset;
                selected_matchLength = next_matchLength;
                selected_offset = next_offset;
                if (next_matchLength > candidate_pos) break;
                candidate_pos -= next_matchLength;
            }
        }
        {
            int rPos = 0;
            while (rPos < last_match_pos) {
                const int ml = opt[rPos].mlen;
                const int offset = opt[rPos].off;
                if (ml == 1) { ip++; rPos++; continue; }
                rPos += ml;
                if (hc_encode(&ip, &op, &anchor, ml, ip - offset, limit, oend)) return 0;
            }
        }
    }
    {   /* last literals */
        const size_t lastRunSize = (size_t)(iend - anchor);
        const size_t llAdd = (lastRunSize + 255 - 15) / 255;
        const size_t totalSize = 1 + llAdd + lastRunSize;
        if (limit && op + totalSize > oend) return 0;
        if (lastRunSize >= 15) {
            size_t acc = lastRunSize - 15;
            *op++ = (uint8_t)(15 << 4);
            for (; acc >= 255; acc -= 255) *op++ = 255;
            *op++ = (uint8_t)acc;
        } else {
            *op++ = (uint8_t)(lastRunSize << 4);
        }
        memcpy(op, anchor, lastRunSize);
        op += lastRunSize;
    }
    return (int)(op - dst);
}

static void hc_ctx_init(hc_ctx* c, const uint8_t* s, int n) {
    c->s = s;
    c->n = n;
    memset(c->hashTable, 0, (1u << HC_HASH_LOG) * sizeof(uint32_t));
    memset(c->chainTable, 0, 65536 * sizeof(uint16_t));
    c->nextToUpdate = HC_BASE;
}

int orc_lz4hc_compress(const uint8_t* src, uint8_t* dst, int n, int cap, int level) {
    static const int kAttempts[13] = {2, 2, 2, 4, 8, 16, 32, 64, 128, 256, 96, 512, 16384};   /* clTable */
    static const int kTarget[13] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 64, 128, HC_OPT_NUM};
    if ((unsigned)n > 0x7E000000u) return 0;
    if (level < 1) level = 9;   /* LZ4HC_CLEVEL_DEFAULT */
    if (level > 12) level = 12; /* LZ4HC_CLEVEL_MAX */
    hc_ctx c;
    c.hashTable = (uint32_t*)malloc((1u << HC_HASH_LOG) * sizeof(uint32_t));
    c.chainTable = (uint16_t*)malloc(65536 * sizeof(uint16_t));
    hc_ctx_init(&c, src, n);
    int r;
    if (level <= 9) {
        r = hc_compress_range(&c, src, dst, n, cap, kAttempts[level], kAttempts[level] > 128);
    } else {
        hc_opt_t* opt = (hc_opt_t*)malloc(sizeof(hc_opt_t) * (HC_OPT_NUM + HC_TRAILING_LITERALS));
        r = hc_compress_optimal(&c, src, dst, n, cap, kAttempts[level], kTarget[level], level == 12, opt);
        free(opt);
    }
    free(c.hashTable);
    free(c.chainTable);
    return r;
}

/* -BD at level >= 3: compressBlockDependency over the legacy HC stream
 * (reference src/lz4mt.cpp:295-332, 460-538, lz4 1.9.3): the input buffer
 * of max(blockMax + 64 KiB, 1088 KiB) bytes; LZ4_resetStreamStateHC leaves
 * the stream at the default level 9; each block is
 * LZ4_compressHC_limitedOutput_continue (cap = inSize - 1) over the blocks
 * before it in the buffer; when the next block would not fit,
 * LZ4_slideInputBufferHC resets the stream (a new segment, no dictionary).
 * Writes the frame body (records: size word, payload, [block XXH32]) to
 * out (n + 8 * blocks bytes at most) and returns its size. */
int64_t orc_bd_hc_body(const uint8_t* src, size_t n, int blockMaxId, int bck, uint8_t* out) {
    const size_t bm = (size_t)1 << (8 + 2 * blockMaxId);
    const size_t bufSize = bm + 65536 > (size_t)(1024 + 64) * 1024 ? bm + 65536 : (size_t)(1024 + 64) * 1024;
    hc_ctx c;
    c.hashTable = (uint32_t*)malloc((1u << HC_HASH_LOG) * sizeof(uint32_t));
    c.chainTable = (uint16_t*)malloc(65536 * sizeof(uint16_t));
    size_t inStart = 0, seg = 0, op = 0;
    for (size_t pos = 0; pos < n;) {
        const size_t len = n - pos < bm ? n - pos : bm;
        if (pos == 0 || inStart + bm > bufSize) {   /* translate(): a fresh stream */
            inStart = 0;
            seg = pos;
            hc_ctx_init(&c, src + seg, 0);
        }
        uint8_t* rec = out + op;
        int cs = hc_compress_range(&c, src + pos, rec + 4, (int)len, (int)len - 1, 256, 1);
        if (cs <= 0) {
            memcpy(rec + 4, src + pos, len);
            cs = (int)len;
            rec[0] = (uint8_t)len; rec[1] = (uint8_t)(len >> 8); rec[2] = (uint8_t)(len >> 16);
            rec[3] = (uint8_t)((len >> 24) | 0x80);
        } else {
            rec[0] = (uint8_t)cs; rec[1] = (uint8_t)(cs >> 8); rec[2] = (uint8_t)(cs >> 16); rec[3] = (uint8_t)(cs >> 24);
        }
        op += 4 + (size_t)cs;
        if (bck) {
            const uint32_t h = orc_xxh32(rec + 4, (size_t)cs, 0);
            out[op] = (uint8_t)h; out[op + 1] = (uint8_t)(h >> 8); out[op + 2] = (uint8_t)(h >> 16);
            out[op + 3] = (uint8_t)(h >> 24);
            op += 4;
        }
        inStart += len;
        pos += len;
    }
    free(c.hashTable);
    free(c.chainTable);
    return (int64_t)op;
}
