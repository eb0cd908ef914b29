#!/usr/bin/env python3
"""CPU simulator of one decode chunk's lane logic (hg_decode.hip).

Mirrors, lane for lane: the header filter, per-lane guesses, lane walks, the
relaxation seeding (chain lanes + max-scan) and rounds.  Used to debug the
algorithm on the CPU before spending GPU time; not part of the product.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHUNK, THREADS, SEG = 16384, 256, 64
NO_GUESS = 0xFFFFFFFF
FAR = (1 << 64) - 1


def hdr(buf, p):
    return int.from_bytes(buf[p:p + 8].tobytes(), "little"), \
        int.from_bytes(buf[p + 8:p + 16].tobytes(), "little")


class Lane:
    __slots__ = ("g", "exit", "cnt", "dead", "pos")

    def __init__(self):
        self.g, self.exit, self.cnt, self.dead, self.pos = NO_GUESS, 0, 0, True, []


def lane_walk(data, base, L, x, segend, w):
    w.cnt, w.dead, w.pos = 0, False, []
    cur = x
    for _ in range(4):
        if cur >= segend:
            break
        a = base + cur
        if a + 16 > L:
            w.dead = True
            break
        kl, vl = hdr(data, cur)
        if kl + vl > (1 << 64) - 1 or kl + vl > L - a - 16 or (kl >> 32) or (vl >> 32):
            w.dead = True
            break
        w.pos.append(cur)
        w.cnt += 1
        cur += 16 + kl + vl
    w.exit = base + cur


def strong_candidates(data, base, L, clen, rem, hz):
    """Per lane: strong candidates (filter + bound + one-step look-ahead)
    with their one-step next position."""
    plim = rem - 16 if rem >= 16 else -1
    cand = np.zeros(CHUNK, bool)
    for p in range(clen):
        if p > plim:
            break
        if (not data[p + 8 - hz:p + 8].any()) and (not data[p + 16 - hz:p + 16].any()):
            cand[p] = True
    strong = []
    for t in range(THREADS):
        lst = []
        for p in range(t * SEG, t * SEG + SEG):
            if p >= CHUNK or not cand[p]:
                continue
            kl, vl = hdr(data, p)
            if (kl >> 32) or (vl >> 32) or kl + vl > rem - p - 16:
                continue
            nx = p + 16 + kl + vl
            if nx < clen and not cand[nx]:
                continue
            lst.append((p, nx))
        strong.append(lst)
    return strong


def chunk_setup(sst, k, L, mode="backed"):
    base = k * CHUNK
    rem = L - base
    clen = min(CHUNK, rem)
    data = np.zeros(CHUNK + 64, np.uint8)
    n = min(CHUNK + 16, rem)
    data[:n] = sst[base:base + n]
    nb = 0
    x = L
    while x:
        nb += 1
        x >>= 8
    hz = 8 - nb
    strong = strong_candidates(data, base, L, clen, rem, hz)
    backed = set(nx for lst in strong for _, nx in lst if nx < clen)
    lanes = []
    for t in range(THREADS):
        w = Lane()
        segend = min(t * SEG + SEG, clen)
        for p, nx in strong[t]:
            if mode == "first" or p in backed:
                w.g = p
                break
        if w.g != NO_GUESS:
            lane_walk(data, base, L, w.g, segend, w)
        lanes.append(w)
    # chunk-entry guess: first strong candidate whose next is a lane guess,
    # else the strong candidate with the shortest record
    guesses = set(w.g for w in lanes if w.g != NO_GUESS)
    entry = None
    for lst in strong:
        for p, nx in lst:
            if nx < clen and nx in guesses:
                entry = p
                break
        if entry is not None:
            break
    if entry is None:
        allc = [(nx - p, p) for lst in strong for p, nx in lst]
        entry = min(allc)[1] if allc else None
    return data, base, clen, lanes, (None if entry is None else base + entry)


def relax(data, base, L, clen, lanes, X, max_rounds=24):
    je = THREADS if X >= base + clen else (X - base) // SEG
    if je < THREADS:
        w = lanes[je]
        if w.g == NO_GUESS or base + w.g != X:
            w.g = X - base
            lane_walk(data, base, L, w.g, min((je + 1) * SEG, clen), w)
    valid = [w.g != NO_GUESS and not w.dead for w in lanes]
    sg = [w.g if v else NO_GUESS for w, v in zip(lanes, valid)]
    sx0 = [w.exit if v else FAR for w, v in zip(lanes, valid)]
    tgt = [0] * THREADS
    for t, w in enumerate(lanes):
        if t >= je and valid[t] and w.exit < base + clen:
            u = (w.exit - base) // SEG
            if sg[u] == w.exit - base:
                tgt[u] = 1
    seed = []
    c = -1
    for t in range(THREADS):
        if t >= je and (t == je or (valid[t] and tgt[t])):
            c = t
        seed.append((sx0[c] if c >= 0 else FAR) if t >= je else 0)
    cur = seed
    passes = [False] * THREADS
    for r in range(1, max_rounds + 1):
        nxt = [0] * THREADS
        changed = False
        for t in range(THREADS):
            if t < je:
                continue
            w = lanes[t]
            segend = min((t + 1) * SEG, clen)
            ein = X if t == je else cur[t - 1]
            if ein >= base + segend:
                passes[t] = True
                val = ein
            else:
                passes[t] = False
                if w.g == NO_GUESS or ein != base + w.g:
                    w.g = ein - base
                    lane_walk(data, base, L, w.g, segend, w)
                val = FAR if w.dead else w.exit
            changed |= val != cur[t]
            nxt[t] = val
        cur = nxt
        if not changed:
            cnt = [0 if (t < je or passes[t]) else lanes[t].cnt for t in range(THREADS)]
            dead = any(t >= je and not passes[t] and lanes[t].dead for t in range(THREADS))
            return True, r, sum(cnt), cur[THREADS - 1], dead
    return False, max_rounds, None, None, None


def true_starts(sst):
    L = sst.size
    out, p = [], 0
    while p < L:
        out.append(p)
        kl, vl = hdr(sst, p)
        p += 16 + kl + vl
    return np.array(out, dtype=np.int64)


def evaluate(name, sst, chunks):
    L = sst.size
    starts = true_starts(sst)
    stats = {"entry_ok": 0, "conv": 0, "rounds": [], "n": 0}
    for k in chunks:
        base = k * CHUNK
        if base >= L:
            break
        i = np.searchsorted(starts, base)
        X = int(starts[i]) if i < starts.size else L
        data, base, clen, lanes, guess = chunk_setup(sst, k, L)
        stats["n"] += 1
        stats["entry_ok"] += int(guess == X)
        ok, r, cnt, ex, dead = relax(data, base, L, clen, lanes, X)
        stats["conv"] += int(ok)
        stats["rounds"].append(r)
        if ok and X >= base + clen:
            ex = X
        if ok:
            j = np.searchsorted(starts, base + clen)
            want_cnt = j - i
            want_exit = int(starts[j]) if j < starts.size else L
            if X >= base + clen:
                want_cnt, want_exit = 0, X
            assert cnt == want_cnt and (ex == want_exit), (name, k, cnt, want_cnt, ex, want_exit)
    rr = np.array(stats["rounds"])
    print(f"{name:28s} chunks={stats['n']:3d} entry_ok={stats['entry_ok']:3d} "
          f"conv={stats['conv']:3d} rounds p50={np.median(rr):.0f} max={rr.max()}")


def main():
    from horreum_amd import synth
    from tests import corpus
    from oracle import oracle
    sst = synth.host_fixed_sst(6000, 16, 100, seed=2)
    evaluate("cfg2 16/100", sst, range(1, 40))
    for name in ["fixed_32_256", "fixed_tomb", "mixed_small", "tiny", "empty_keys_tombs",
                 "zero_values", "mixed_4k", "large_values", "zero_large"]:
        _, _, data, _ = corpus.make(name)
        evaluate(name, data, range(0, 24))


if __name__ == "__main__":
    main()
