"""Model (round 5): can a pooled DSM body raise the streaming tile's rate?
Op streams from the ref10 slide of random scalars (tools/r04_pool_assign_model.py),
step costs of the round-3 pool model (pure DBL step 1070 VALU, mixed step 1500),
k_dsm's per-lane step 1450.  Compares, in VALU per signature:
  per-lane body     the tile today: a 64-frag chunk costs 1450 x its longest op stream
  fixed pool        two chunks (128 signatures) pooled together, no refill
  chunk-admitted    a pool of P slots that admits a whole chunk (64) when 64 slots are free
  continuous        k_dsmp: refill as slots free up (P = 112)
usage: python tools/r05_tile_pool_model.py [signatures]"""
import random
import sys
import os

src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "r04_pool_assign_model.py")).read()
ns = {}
exec(src[:src.index("NS = int(")], ns)
ops, L = ns["ops"], ns["L"]
random.seed(7)
NS = int(sys.argv[1]) if len(sys.argv) > 1 else 1536
streams = [ops(random.getrandbits(512) % L, random.getrandbits(512) % L) for _ in range(NS)]
CD, CM, CL = 1070, 1500, 1450


def step(cur, pos, live):
    D = [sl for sl in live if streams[cur[sl]][pos[sl]] == 0]
    A = [sl for sl in live if streams[cur[sl]][pos[sl]] != 0]
    if len(D) >= 64:
        return D[:64], CD
    rem = lambda sl: len(streams[cur[sl]]) - pos[sl]   # noqa: E731
    return (sorted(A, key=rem, reverse=True) + sorted(D, key=rem, reverse=True))[:64], CM


def pool(sigs, P, admit):
    q = list(sigs); cur = [None] * P; pos = [0] * P; cost = 0
    while True:
        free = [sl for sl in range(P) if cur[sl] is None]
        if q and len(free) >= admit:
            for sl in free[:admit if admit > 1 else len(free)]:
                if q:
                    cur[sl] = q.pop(); pos[sl] = 0
        live = [sl for sl in range(P) if cur[sl] is not None]
        if not live:
            return cost
        sel, c = step(cur, pos, live)
        cost += c
        for sl in sel:
            pos[sl] += 1
            if pos[sl] >= len(streams[cur[sl]]):
                cur[sl] = None


lane = sum(CL * max(len(streams[i]) for i in range(k, k + 64)) for k in range(0, NS, 64)) / NS
print("signatures %d, mean ops %.1f" % (NS, sum(map(len, streams)) / NS))
print("per-lane body (64 per chunk)          %6.0f VALU/sig  1.000" % lane)
fx = sum(pool(range(k, k + 128), 128, 128) for k in range(0, NS, 128)) / NS
print("fixed pool of two chunks (128)        %6.0f           %.3f" % (fx, fx / lane))
for P in (112, 128, 160, 192):
    v = pool(range(NS), P, 64) / NS
    print("chunk-admitted pool P=%-3d             %6.0f           %.3f" % (P, v, v / lane))
v = pool(range(NS), 112, 1) / NS
print("continuous refill P=112 (k_dsmp)      %6.0f           %.3f" % (v, v / lane))
