"""Lane-level Python model of the v5 encoder window loop (encode_block_v5 in
lz4mt_kernels.hip) for debugging on the CPU: runs the same window algorithm
with 64 explicit lanes and compares against the oracle.

usage: python tools/enc_model.py            (fuzz cases of tests/test_gpu.py)
"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402

POSB = 22
MASK = (1 << POSB) - 1


def rd32(s, i):
    return int.from_bytes(s[i:i + 4].ljust(4, b"\0"), "little")


def rd64(s, i):
    return int.from_bytes(s[i:i + 8].ljust(8, b"\0"), "little")


def h5(v8):
    return (((v8 << 24) & 0xFFFFFFFFFFFFFFFF) * 889523592379 & 0xFFFFFFFFFFFFFFFF) >> 52


def tag(w0):
    return ((w0 * 0x85EBCA77) & 0xFFFFFFFF) >> POSB


def poff(k):
    if k == 0:
        return 0
    q, r = (k - 1) >> 6, (k - 1) & 63
    return 1 + 32 * q * (q + 1) + r * (q + 1)


def ext_len(v):
    return (v - 15) // 255 + 1 if v >= 15 else 0


def encode(s, cap, last_lane_wins=True, xchg=False):
    """xchg=True: the exchange probe of encode_block_v5 (LZ4MT_ENC_XCHG):
    lanes exchange their entries in ascending lane order, so each gets its
    in-window predecessor's entry or the table's; no read-back, no
    predecessor resolution; lanes past the stop undo their inserts (the
    first of each bucket puts back what it displaced)."""
    if xchg:
        return encode_xchg(s, cap)
    n = len(s)
    assert 65547 <= n <= 1 << 22
    bound = n + n // 255 + 16
    limited = cap < bound
    T = [(tag(rd32(s, 0)) << POSB)] * 4096 + [0] * 64
    mfl = n - 12 + 1
    matchlimit = n - 5
    anchor = op = 0
    out = bytearray()
    insOn, testOn = True, False
    insPos = testPos = 0
    sPos, k0 = 1, 0
    while True:
        p, step = [0] * 64, [1] * 64
        for L in range(64):
            k = k0 + L - 2
            if L >= 2:
                p[L] = sPos + poff(k)
                step[L] = 1 if k == 0 else (63 + k) >> 6
        p[0], p[1] = insPos, testPos
        live = [(p[L] <= mfl) if L >= 2 else (insOn if L == 0 else testOn) for L in range(64)]
        term = [L >= 2 and live[L] and p[L] + step[L] > mfl for L in range(64)]
        w0 = [rd32(s, min(p[L], n - 8)) for L in range(64)]
        h = [h5(rd64(s, min(p[L], n - 8))) for L in range(64)]
        mark = [(p[L] | (tag(w0[L]) << POSB)) & 0xFFFFFFFF for L in range(64)]
        ti = [h[L] if live[L] else 4096 + L for L in range(64)]
        told = [T[ti[L]] for L in range(64)]
        order = range(64) if last_lane_wins else range(63, -1, -1)
        for L in order:
            T[ti[L]] = mark[L]
        sv = [T[ti[L]] for L in range(64)]
        pend = [sv[L] != mark[L] for L in range(64)]
        cand = [told[L] & MASK for L in range(64)]
        cok = [live[L] and L != 0 and not term[L] and cand[L] + 65535 >= p[L] for L in range(64)]
        maybe = [cok[L] and (told[L] >> POSB) == (mark[L] >> POSB) for L in range(64)]
        sm = [maybe[L] or term[L] for L in range(64)]
        mm = list(maybe)
        dd = False
        gmask = [{L} for L in range(64)]
        aliased = set()
        while True:
            w = next((L for L in range(64) if sm[L]), 64)
            collide = any(pend[L] for L in range(min(w, 63) + 1))
            if not dd and collide:
                dd = True
                pred = [-1] * 64
                for L in range(64):
                    if live[L]:
                        grp = [j for j in range(64) if live[j] and h[j] == h[L]]
                        gmask[L] = set(grp)
                        below = [j for j in grp if j < L]
                        pred[L] = below[-1] if below else -1
                ok = [False] * 64
                for L in range(64):
                    if pred[L] >= 0:
                        pp, pw = p[pred[L]], w0[pred[L]]
                        ok[L] = live[L] and L != 0 and not term[L] and pp + 65535 >= p[L] and pw == w0[L]
                        maybe[L] = False
                        cand[L] = pp
                mm = list(maybe)
                sm = [(ok[L] or maybe[L] or term[L]) and L not in aliased for L in range(64)]
                continue
            wTerm = w < 64 and term[w]
            if w == 64 or wTerm:
                break
            ip, cd = p[w], cand[w]
            if mm[w] and rd32(s, cd) != w0[w]:
                sm[w] = False
                aliased.add(w)
                continue
            break
        wlim = 63 if w == 64 else (w - 1 if wTerm else w)
        for L in range(64):
            if live[L] and L > wlim:
                T[h[L]] = told[L]
        if any(pend):
            for L in order:
                le = L <= wlim
                lastM = (not dd) or not any(j > L and j <= wlim for j in gmask[L])
                if live[L] and le and lastM:
                    T[h[L]] = mark[L]
        if w == 64:
            k0 += 62
            insOn = testOn = False
            continue
        if wTerm:
            break
        maxb = 0 if w == 1 else min(ip - anchor, cd)
        back = 0
        while back < maxb and s[ip - back - 1] == s[cd - back - 1]:
            back += 1
        lim = matchlimit - (ip + 4)
        mc = 0
        while mc < lim and s[ip + 4 + mc] == s[cd + 4 + mc]:
            mc += 1
        lit = ip - anchor - back
        mcf = mc + back
        litExt, mlExt = ext_len(lit), ext_len(mcf)
        if limited:
            if w != 1 and op + 1 + lit + 8 + lit // 255 > cap:
                return b""
            if op + 1 + litExt + lit + 2 + 6 + (mcf + 240) // 255 > cap:
                return b""
        tok = (min(lit, 15) << 4) | min(mcf, 15)
        seq = bytearray([tok])
        if lit >= 15:
            seq += b"\xff" * (litExt - 1) + bytes([(lit - 15) % 255])
        seq += s[anchor:anchor + lit]
        off = ip - cd
        seq += bytes([off & 255, off >> 8])
        if mcf >= 15:
            seq += b"\xff" * (mlExt - 1) + bytes([(mcf - 15) % 255])
        out += seq
        op += len(seq)
        ipe = ip + 4 + mc
        anchor = ipe
        if ipe >= mfl:
            break
        insOn = testOn = True
        insPos, testPos, sPos, k0 = ipe - 2, ipe, ipe + 1, 0
    run = n - anchor
    if limited and op + run + 1 + (run + 240) // 255 > cap:
        return b""
    out.append(min(run, 15) << 4)
    if run >= 15:
        out += b"\xff" * (ext_len(run) - 1) + bytes([(run - 15) % 255])
    out += s[anchor:]
    return bytes(out)


def tag_ht(w0):
    """the hash-product tag (LZ4MT_ENC_HTAG): bits 42..51 of hash5's product"""
    return ((((w0 << 24) * 889523592379) & 0xFFFFFFFFFFFFFFFF) >> (52 - (32 - POSB))) & ((1 << (32 - POSB)) - 1)


def encode_xchg(s, cap):
    n = len(s)
    assert 65547 <= n <= 1 << 22
    bound = n + n // 255 + 16
    limited = cap < bound
    T = [(tag_ht(rd32(s, 0)) << POSB)] * 4096 + [0] * 64
    mfl = n - 12 + 1
    matchlimit = n - 5
    anchor = op = 0
    out = bytearray()
    mode = 2            # 2: INSERT 0 only; 1: INSERT + TEST after a match; 0: continuation
    sPos, k0 = 1, 0
    while True:
        p, step = [0] * 64, [1] * 64
        for L in range(2, 64):
            k = k0 + L - 2
            p[L] = sPos + poff(k)
            step[L] = 1 if k == 0 else (63 + k) >> 6
        p[0] = 0 if mode == 2 else sPos - 3
        p[1] = sPos - 1
        live = [p[L] <= mfl if L >= 2 else (mode != 0 if L == 0 else mode == 1) for L in range(64)]
        term = [L >= 2 and live[L] and p[L] + step[L] > mfl for L in range(64)]
        w0 = [rd32(s, min(p[L], n - 8)) for L in range(64)]
        h = [h5(rd64(s, min(p[L], n - 8))) for L in range(64)]
        mark = [(p[L] | (tag_ht(w0[L]) << POSB)) & 0xFFFFFFFF for L in range(64)]
        told = [0] * 64
        for L in range(64):   # the exchanges, in ascending lane order
            i = h[L] if live[L] else 4096 + L
            told[L] = T[i]
            T[i] = mark[L]
        cand = [told[L] & MASK for L in range(64)]
        maybe = [live[L] and L != 0 and not term[L] and cand[L] + 65535 >= p[L] and
                 (told[L] >> POSB) == (mark[L] >> POSB) for L in range(64)]
        aliased = set()
        redo = False

        def table_writes(wlim):
            if redo:   # re-insert the lanes up to the stop, in lane order
                for L in range(64):
                    if live[L] and L <= wlim:
                        T[h[L]] = mark[L]
            past = [L for L in range(64) if live[L] and L > wlim]
            # the first lane of each bucket past the stop restores: lanes are in
            # position order, so "displaced by no lane past the stop" is "the
            # displaced entry's position is at most lane wlim's" (the kernel's
            # table_writes; no mask scan for the first lane past the stop)
            pB = p[wlim] if wlim >= 0 else -1
            for L in past:
                if (told[L] & MASK) <= pB:
                    T[h[L]] = told[L]

        while True:
            w = next((L for L in range(64) if (maybe[L] or term[L]) and L not in aliased), 64)
            wTerm = w < 64 and term[w]
            if w < 64 and not wTerm and rd32(s, cand[w]) != w0[w]:
                aliased.add(w)     # tag alias: the stop moves on
                table_writes(w)    # (the kernel writes in the round trip's shadow, then redoes)
                redo = True
                continue
            break
        wlim = 63 if w == 64 else (w - 1 if wTerm else w)
        table_writes(wlim)
        if w == 64:   # (probe offsets poff(k) count from the sequence's first search position)
            k0 += 62
            mode = 0
            continue
        if wTerm:
            break
        ip, cd = p[w], cand[w]
        maxb = 0 if w == 1 else min(ip - anchor, cd)
        back = 0
        while back < maxb and s[ip - back - 1] == s[cd - back - 1]:
            back += 1
        lim = matchlimit - (ip + 4)
        mc = 0
        while mc < lim and s[ip + 4 + mc] == s[cd + 4 + mc]:
            mc += 1
        lit = ip - anchor - back
        mcf = mc + back
        litExt, mlExt = ext_len(lit), ext_len(mcf)
        if limited:
            if w != 1 and op + 1 + lit + 8 + lit // 255 > cap:
                return b""
            if op + 1 + litExt + lit + 2 + 6 + (mcf + 240) // 255 > cap:
                return b""
        tok = (min(lit, 15) << 4) | min(mcf, 15)
        seq = bytearray([tok])
        if lit >= 15:
            seq += b"\xff" * (litExt - 1) + bytes([(lit - 15) % 255])
        seq += s[anchor:anchor + lit]
        off = ip - cd
        seq += bytes([off & 255, off >> 8])
        if mcf >= 15:
            seq += b"\xff" * (mlExt - 1) + bytes([(mcf - 15) % 255])
        out += seq
        op += len(seq)
        ipe = ip + 4 + mc
        anchor = ipe
        if ipe >= mfl:
            break
        mode = 1
        sPos, k0 = ipe + 1, 0
    run = n - anchor
    if limited and op + run + 1 + (run + 240) // 255 > cap:
        return b""
    out.append(min(run, 15) << 4)
    if run >= 15:
        out += b"\xff" * (ext_len(run) - 1) + bytes([(run - 15) % 255])
    out += s[anchor:]
    return bytes(out)


def fuzz_cases():
    rnd = random.Random(3)
    syn = oracle.gen_synthetic(1 << 20)
    for t in range(80):
        n = rnd.choice([1, 7, 12, 13, 14, 20, 64, 100, 1000, 4095, 65535, 65546, 65547, 65548, 100_000, 262_144])
        kind = t % 5
        if kind == 0:
            d = syn[:n]
        elif kind == 1:
            d = bytes(rnd.randrange(3) for _ in range(n))
        elif kind == 2:
            d = oracle.gen_random(n, t)
        elif kind == 3:
            d = (bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 70))) * (n + 1))[:n]
        else:
            d = bytes(n)
        yield t, d


if __name__ == "__main__":
    for t, d in fuzz_cases():
        if len(d) < 65547:
            continue
        for cap in (len(d), len(d) + len(d) // 255 + 16):
            for llw in (True, False, "xchg"):
                got = encode(d, cap, xchg=True) if llw == "xchg" else encode(d, cap, llw)
                want = oracle.compress_block(d, cap)
                if got != want:
                    i = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), None)
                    print(f"MISMATCH t={t} n={len(d)} cap={cap} lastLaneWins={llw} first diff at {i}")
                else:
                    print(f"ok t={t} n={len(d)} cap={cap} llw={llw}")
