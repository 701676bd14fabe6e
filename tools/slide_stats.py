"""Op-count spread of the double-scalar multiply across signatures: per
signature, (top digit position + 1) doublings + the nonzero sliding-window
digits of h and s (ref10 slide, the digit rule of fd_ed25519_ge.c's
ge_slide); and the lane utilisation a chunk of 64 (or 16) signatures gets when
every lane runs until the chunk's longest op stream ends.  Pure Python, 4096
random scalars mod L.

usage: python tools/slide_stats.py
"""
import random
L = 2**252 + 27742317777372353535851937790883648493
def slide(a):
    r = [(a >> i) & 1 for i in range(256)]
    for i in range(256):
        if r[i]:
            b = 1
            while b <= 6 and i + b < 256:
                if r[i+b]:
                    if r[i] + (r[i+b] << b) <= 15:
                        r[i] += r[i+b] << b; r[i+b] = 0
                    elif r[i] - (r[i+b] << b) >= -15:
                        r[i] -= r[i+b] << b
                        for k in range(i+b, 256):
                            if not r[k]: r[k] = 1; break
                            r[k] = 0
                    else: break
                b += 1
    return r
random.seed(1)
steps = []
for _ in range(4096):
    h = random.getrandbits(512) % L; s = random.getrandbits(512) % L
    a = slide(h); b = slide(s)
    top = max(i for i in range(256) if a[i] or b[i])
    n = (top + 1) + sum(1 for x in a if x) + sum(1 for x in b if x)
    steps.append(n)
import statistics
m = statistics.mean(steps); sd = statistics.pstdev(steps)
chunks = [max(steps[i:i+64]) for i in range(0, len(steps), 64)]
util = sum(steps) / (64 * sum(chunks))
print("mean %.1f sd %.2f  mean max/64 %.1f  lane util %.4f" % (m, sd, statistics.mean(chunks), util))
ch16 = [max(steps[i:i+16]) for i in range(0, len(steps), 16)]
print("16-chunk util %.4f" % (sum(steps) / (16 * sum(ch16))))
