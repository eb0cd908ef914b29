import numpy as np, sys
PIECE, T, SEG = 16384, 256, 64
FAR = 8192
rng = np.random.default_rng(4)
m = 400_000
kl = rng.integers(0, 24, m); vl = rng.integers(0, 64, m); vl[rng.random(m) < 0.05] = 0
offs = np.concatenate([[0], np.cumsum(16 + kl + vl)])
buf = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
hdr = np.stack([kl, vl], axis=1).astype("<u8").view(np.uint8).reshape(m, 16)
for i in range(16): buf[offs[:-1] + i] = hdr[:, i]
L = len(buf); nb = 0; x = L
while x: nb += 1; x >>= 8
hz = 8 - nb
starts = set(offs[:-1].tolist())
def H(p):
    return int.from_bytes(buf[p:p+8].tobytes(),'little'), int.from_bytes(buf[p+8:p+16].tobytes(),'little')
def cand(p):
    if p + 16 > L: return False
    return all(buf[p+8-hz:p+8] == 0) and all(buf[p+16-hz:p+16] == 0)
tot_rounds = []; wrong = []
for piece in range(5, 25):
    base = piece * PIECE; clen = PIECE
    rem = L - base
    C = [cand(base + j) for j in range(clen)]
    g = [None]*T
    for t in range(T):
        for j in range(t*SEG, t*SEG+SEG):
            if not C[j]: continue
            if j + 1 < clen and C[j+1]: continue   # not the end of a run of candidates
            k, v = H(base+j)
            body = k + v
            if k >> 32 or v >> 32 or body >= FAR or body > rem - j - 16: continue
            nx = j + 16 + body
            if nx < clen:
                if not C[nx]: continue
                if nx + 16 <= clen:
                    a, b = H(base+nx); nbd = a + b
                    if a >> 32 or b >> 32 or nbd > rem - nx - 16: continue
                    nx2 = nx + 16 + nbd
                    if nx2 < clen and not C[nx2]: continue
            g[t] = j; break
    truth = [s - base for s in starts if base <= s < base + clen]
    first_true = [None]*T
    for s in sorted(truth, reverse=True): first_true[s // SEG] = s
    nw = sum(1 for t in range(T) if g[t] != first_true[t])
    wrong.append(nw)
print("wrong guesses per piece:", wrong)
# classify for the last piece
kinds = {}
for t in range(T):
    if g[t] == first_true[t]: continue
    if first_true[t] is None: kind = 'guess_but_no_start'
    elif g[t] is None: kind = 'no_guess_but_start'
    elif g[t] < first_true[t]: kind = 'guess_before_true'
    else: kind = 'guess_after_true'
    kinds[kind] = kinds.get(kind, 0) + 1
    if kind in ('guess_before_true','no_guess_but_start') and kinds[kind] <= 3:
        j = first_true[t]; k, v = H(base + j)
        print(kind, 't', t, 'g', g[t], 'true', j, 'true hdr', k, v, 'shift', (g[t]-j) if g[t] is not None else None)
        if g[t] is not None: print('   guess hdr', H(base+g[t]))
print(kinds)
