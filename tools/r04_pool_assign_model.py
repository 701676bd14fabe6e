"""Model of k_dsmp's pool (round 4): the free slot-to-lane assignment of the kernel
against a bank-conflict-free one in which lane l only takes slots s = l (mod 16)
(every ds_read_b128 lane group of 16 then reads 16 distinct 16-B bank groups).
Op streams from the ref10 slide of random scalars; step costs DBL 1070 / mixed
1500 VALU (the round-3 pool model).  usage: python tools/r04_pool_assign_model.py [n]"""
import numpy as np, sys
rng = np.random.default_rng(1)
L = 2**252 + 27742317777372353535851937790883648493
def slide(a):
    r = [(a >> i) & 1 for i in range(256)]
    for i in range(256):
        if r[i]:
            for b in range(1, 7):
                if i + b >= 256: break
                if r[i+b]:
                    if r[i] + (r[i+b] << b) <= 15:
                        r[i] += r[i+b] << b; r[i+b] = 0
                    elif r[i] - (r[i+b] << b) >= -15:
                        r[i] -= r[i+b] << b
                        for k in range(i+b, 256):
                            if not r[k]: r[k] = 1; break
                            r[k] = 0
                    else: break
    return r
def ops(h, s):
    a, b = slide(h), slide(s)
    top = max([i for i in range(256) if a[i] or b[i]] or [0])
    o = []
    for i in range(top, -1, -1):
        o.append(0)
        if a[i]: o.append(1)
        if b[i]: o.append(2)
    return o
NS = int(sys.argv[1]) if len(sys.argv) > 1 else 600
import random
random.seed(1)
streams = [ops(random.getrandbits(512) % L, random.getrandbits(512) % L) for _ in range(NS)]
print("mean ops", np.mean([len(x) for x in streams]), file=sys.stderr)
P = 112
CD, CM = 1070, 1500
def sim(policy):
    q = list(range(NS)); cur = [None]*P; pos = [0]*P
    valu = 0; steps = 0; lanes = 0
    while True:
        for sl in range(P):
            if cur[sl] is None and q:
                cur[sl] = q.pop(); pos[sl] = 0
        live = [sl for sl in range(P) if cur[sl] is not None]
        if not live: break
        cls = {sl: (0 if streams[cur[sl]][pos[sl]] == 0 else 1) for sl in live}
        D = [sl for sl in live if cls[sl] == 0]; A = [sl for sl in live if cls[sl] == 1]
        if policy == "free":
            if len(D) >= 64 or not A:
                sel = D[:64]; cost = CD
            else:
                sel = (A + D)[:64]; cost = CM
        else:
            # residue classes: lane l only takes slots s = l mod 16 (4 lanes per residue, 7 slots)
            byr = {r: ([s for s in D if s % 16 == r], [s for s in A if s % 16 == r]) for r in range(16)}
            dfull = all(len(byr[r][0]) >= 4 for r in range(16))
            if dfull or not A:
                sel = [s for r in range(16) for s in byr[r][0][:4]]; cost = CD
            else:
                sel = [s for r in range(16) for s in (byr[r][1] + byr[r][0])[:4]]; cost = CM
        valu += cost; steps += 1; lanes += len(sel)
        for sl in sel:
            pos[sl] += 1
            if pos[sl] == len(streams[cur[sl]]): cur[sl] = None
    return valu / NS, steps, lanes / steps
for pol in ("free", "residue"):
    v, st, fill = sim(pol)
    print(pol, "VALU/sig %.0f steps %d fill %.3f" % (v, st, fill / 64))
