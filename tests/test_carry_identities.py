"""The carry-chain rewrites used by the HIP field kernels give the
reference's limbs (avx/fd_ed25519_fe_avx_inl.h:568-584) on every input:
the biased chain (fe_carry_b), the carry-folded chain (fe_sq_fold,
fe_mul_fold2w, fe_carry_fold_out) and the folded chain with
an independent column 9 (fe_mul_fold1), all in
firedancer_amd/csrc/fd_ed25519_dev.h, modelled here
with Python integers (int64 semantics checked) over random and extreme
column sums.  CPU only."""
import random

M64 = 1 << 64


def i64(x):
    x %= M64
    return x - M64 if x >= 1 << 63 else x


def i32(x):
    x %= 1 << 32
    return x - (1 << 32) if x >= 1 << 31 else x


def ref_carry(h):
    h = list(h)
    def c(k, w, nxt, mul=1):
        cc = (h[k] + (1 << (w - 1))) >> w
        h[nxt] += cc * mul
        h[k] -= cc << w
    c(0, 26, 1); c(4, 26, 5); c(1, 25, 2); c(5, 25, 6); c(2, 26, 3); c(6, 26, 7)
    c(3, 25, 4); c(7, 25, 8); c(4, 26, 5); c(8, 26, 9); c(9, 25, 0, 19); c(0, 26, 1)
    return [i32(v) for v in h]


def biased_carry(h):
    b = [1 << 25 if k % 2 == 0 else 1 << 24 for k in range(10)]
    h = [h[k] + b[k] for k in range(10)]
    M26, M25 = (1 << 26) - 1, (1 << 25) - 1
    h[1] += h[0] >> 26; h[5] += h[4] >> 26; h[2] += h[1] >> 25; h[6] += h[5] >> 25
    h[3] += h[2] >> 26; h[7] += h[6] >> 26
    t4 = (h[4] & M26) + (h[3] >> 25)
    h[8] += h[7] >> 25
    c4b = t4 >> 26
    h[9] += h[8] >> 26
    t0 = (h[0] & M26) + (h[9] >> 25) * 19
    c0b = t0 >> 26
    return fold_limbs(h, t0, t4, c0b, c4b)


def fold_limbs(h, t0, t4, c0b, c4b):
    m26, m25 = (1 << 26) - 1, (1 << 25) - 1
    r = [0] * 10
    r[0] = (t0 & m26) - (1 << 25)
    r[1] = (h[1] & m25) - (1 << 24) + c0b
    r[2] = (h[2] & m26) - (1 << 25)
    r[3] = (h[3] & m25) - (1 << 24)
    r[4] = (t4 & m26) - (1 << 25)
    r[5] = (h[5] & m25) - (1 << 24) + c4b
    for k in (6, 8):
        r[k] = (h[k] & m26) - (1 << 25)
    for k in (7, 9):
        r[k] = (h[k] & m25) - (1 << 24)
    return [i32(v) for v in r]


def folded_carry(s):
    """s = the unbiased column sums; the chains of 1,3,5,7,9 start from the
    previous even column's carry, even columns from K = 2^25 + 2^50."""
    K = (1 << 25) + (1 << 50)
    h = [0] * 10
    for k in (0, 4, 2, 6, 8):
        h[k] = i64(K + s[k])
    h[1] = i64((h[0] >> 26) + s[1])
    h[5] = i64((h[4] >> 26) + s[5])
    h[2] = i64(h[2] + (h[1] >> 25))
    h[6] = i64(h[6] + (h[5] >> 25))
    h[3] = i64((h[2] >> 26) + s[3])
    h[7] = i64((h[6] >> 26) + s[7])
    h[8] = i64(h[8] + (h[7] >> 25))
    h[9] = i64((h[8] >> 26) + s[9])
    M26 = (1 << 26) - 1
    t4 = (h[4] & M26) + (h[3] >> 25)
    c4b = t4 >> 26
    t0 = (h[0] & M26) + (h[9] >> 25) * 19
    c0b = t0 >> 26
    return fold_limbs(h, t0, t4, c0b, c4b)


def folded_carry_k9(s):
    """fe_mul_fold1: as folded_carry, but column 9 starts from its own bias
    2^24 (it runs beside columns 3 and 7), column 8 from 2^25 alone, and
    column 8's carry reaches 9 through an add."""
    K = (1 << 25) + (1 << 50)
    h = [0] * 10
    for k in (0, 4, 2, 6):
        h[k] = i64(K + s[k])
    h[8] = i64((1 << 25) + s[8])
    h[1] = i64((h[0] >> 26) + s[1])
    h[5] = i64((h[4] >> 26) + s[5])
    h[2] = i64(h[2] + (h[1] >> 25))
    h[6] = i64(h[6] + (h[5] >> 25))
    h[3] = i64((h[2] >> 26) + s[3])
    h[7] = i64((h[6] >> 26) + s[7])
    h[9] = i64((1 << 24) + s[9])
    h[8] = i64(h[8] + (h[7] >> 25))
    h[9] = i64(h[9] + (h[8] >> 26))
    M26 = (1 << 26) - 1
    t4 = (h[4] & M26) + (h[3] >> 25)
    c4b = t4 >> 26
    t0 = (h[0] & M26) + (h[9] >> 25) * 19
    c0b = t0 >> 26
    return fold_limbs(h, t0, t4, c0b, c4b)


def test_carry_rewrites_match_reference_chain():
    rng = random.Random(7)
    bound = 1 << 61                  # |column sum| < 2^61.8 for the kernels' operand ranges
    cases = [[0] * 10, [bound - 1] * 10, [-bound] * 10,
             [(1 << 25) * (k % 2 + 1) for k in range(10)], [-(1 << 24)] * 10]
    for _ in range(20000):
        mode = rng.random()
        if mode < 0.5:
            s = [rng.randrange(-bound, bound) for _ in range(10)]
        elif mode < 0.8:
            s = [rng.randrange(-(1 << 54), 1 << 54) for _ in range(10)]
        else:                        # exact rounding-boundary sums
            s = [rng.randrange(-1000, 1000) * (1 << 26) + rng.choice([1 << 25, (1 << 25) - 1, -(1 << 25), 1 << 24])
                 for _ in range(10)]
        cases.append(s)
    for s in cases:
        r = ref_carry(s)
        assert biased_carry(s) == r, s
        assert folded_carry(s) == r, s
        assert folded_carry_k9(s) == r, s


# ---- squares: the column sums of fe_sq_fold2w / sq_term (fd_ed25519_dev.h) ----

def _mul_cols(f, g):
    """Column sums of fe_mul( f, g ): term (i, j) weighted x2 when i and j
    are both odd and x19 when i + j >= 10 (avx/fd_ed25519_fe_avx_inl.h)."""
    h = [0] * 10
    for i in range(10):
        for j in range(10):
            h[(i + j) % 10] += (2 if (i & 1 and j & 1) else 1) * (19 if i + j >= 10 else 1) * f[i] * g[j]
    return h


def _sq_cols(f, d2):
    """sq_term's 55 products: pair (i <= j) of column K with its power of two
    as a shift of f_i and the 19 on f_j; every operand must fit int32."""
    h = [0] * 10
    for K in range(10):
        for i in range(10):
            j = (K - i + 10) % 10
            if i > j:
                continue
            c2 = (i != j) + (1 if (i & 1 and j & 1) else 0) + (1 if d2 else 0)
            lhs = f[i] << c2
            rhs = 19 * f[j] if i + j >= 10 else f[j]
            assert -(1 << 31) <= lhs < (1 << 31) and -(1 << 31) <= rhs < (1 << 31)
            h[K] += lhs * rhs
    return h


def test_square_columns_equal_mul_columns():
    """fe_sq_fold2w<D2> computes exactly the column sums of fe_mul( f, f )
    (resp. fe_mul( f, f+f )), without wrapping an operand, for the input
    ranges k_dsmp feeds it: |limb| <= 2^26 (X+Y of carried limbs) and
    |limb| <= 2^25 for the sq2 input Z -- so it gives the same limbs as the
    general product the reference's sq / sq2 equal."""
    rng = random.Random(2025)
    cases = [[(1 << 26)] * 10, [-(1 << 26)] * 10, [(1 << 26) * (-1) ** k for k in range(10)]]
    cases += [[rng.randint(-(1 << 26), 1 << 26) for _ in range(10)] for _ in range(3000)]
    for f in cases:
        assert _sq_cols(f, False) == _mul_cols(f, f)
        z = [max(-(1 << 25), min(1 << 25, v >> 1)) for v in f]
        assert _sq_cols(z, True) == _mul_cols(z, [2 * v for v in z])
    # and the sums stay inside int64 with the fold's 2^25 + 2^50 start value
    for f in cases[:3]:
        for v in _sq_cols(f, False):
            assert abs(v) + (1 << 25) + (1 << 50) < (1 << 63)
