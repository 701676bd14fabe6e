"""Pure-Python restatement of fd_ed25519_ge_slide (src/ballet/ed25519/
avx/fd_ed25519_ge.c:378-400) and of h = SHA-512(R||A||M) mod L
(fd_ed25519_user.c:411-414) -- small-case checker for the k_prep digits."""
import hashlib

L = 2**252 + 27742317777372353535851937790883648493


def slide(a):
    r = [(a >> i) & 1 for i in range(256)]
    for i in range(256):
        if not r[i]:
            continue
        for b in range(1, 7):
            if i + b >= 256:
                break
            if not r[i + b]:
                continue
            if r[i] + (r[i + b] << b) <= 15:
                r[i] += r[i + b] << b
                r[i + b] = 0
            elif r[i] - (r[i + b] << b) >= -15:
                r[i] -= r[i + b] << b
                for k in range(i + b, 256):
                    if not r[k]:
                        r[k] = 1
                        break
                    r[k] = 0
            else:
                break
    return r


def h_scalar(sig, pub, msg):
    return int.from_bytes(hashlib.sha512(bytes(sig[:32]) + bytes(pub) + bytes(msg)).digest(), "little") % L
