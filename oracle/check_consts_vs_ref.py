#!/usr/bin/env python3
"""TEST INFRASTRUCTURE (build container only): check that the constants
regenerated from first principles by tools/gen_consts.py equal, limb for
limb, the tables the reference ships.  Reads the reference sources as TEXT
(numbers only); nothing is copied into the repo.  Exits 0 (and prints
"skipped") when /root/reference is absent, e.g. on the GPU box.

Checked:
  * src/ballet/ed25519/table/fd_ed25519_ge_bi_precomp.c       Bi[8] rows
  * src/ballet/ed25519/table/fd_ed25519_ge_bi_precomp_avx.c   same, lane form
    [1, y-x, y+x, 2dxy] stored zero-extended (uint32) per limb
  * d / 2d / sqrt(-1) limbs in src/ballet/ed25519/avx/fd_ed25519_ge.c
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tools"))
import gen_consts as g  # noqa: E402

REF = "/root/reference/src/ballet/ed25519"


def ints(text):
    return [int(x) for x in re.findall(r"-?\d+", text)]


def main():
    if not os.path.isdir(REF):
        print("skipped: /root/reference absent")
        return 0
    bi = g.bi_table()
    # plain table: strip comments, take all integers after the '=' of the array
    src = open(os.path.join(REF, "table/fd_ed25519_ge_bi_precomp.c")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    body = src[src.index("=") + 1:]
    vals = ints(body)
    want = [v for row in bi for fe in row for v in fe]
    assert vals == want, "bi_precomp mismatch"
    # AVX swizzled table: [8][40] = limb-major, lanes [1, y-x, y+x, 2dxy]
    src = open(os.path.join(REF, "table/fd_ed25519_ge_bi_precomp_avx.c")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    body = src[src.index("bi_precomp[8][40]"):]
    body = body[body.index("=") + 1:]
    vals = [int(x) for x in re.findall(r"(\d+)L", body)]
    want = []
    for (ypx, ymx, xy2d) in bi:
        for i in range(10):
            for lane in (1 if i == 0 else 0, ymx[i], ypx[i], xy2d[i]):
                want.append(lane & 0xFFFFFFFF)
    assert vals == want, "bi_precomp_avx mismatch"
    ge = open(os.path.join(REF, "avx/fd_ed25519_ge.c")).read()
    for name, val in (("d", g.D), ("2d", g.D2), ("sqrtm1", g.SQRTM1)):
        limbs = g.limbs(val)
        pat = ", ".join(str(x) for x in limbs)
        flat = re.sub(r"\s+", " ", ge)
        found = pat.replace(", ", ",") in flat.replace(", ", ",").replace(" ,", ",")
        # the AVX file stores some constants as (long)(uint)x lanes; check both
        if not found:
            lane_hits = all(re.search(r"\(uint\)\s*%d\b" % x, ge) for x in limbs)
            assert lane_hits, f"{name} limbs not found in reference"
    print("ok: Bi[8] (plain + AVX lane form), d, 2d, sqrt(-1) match the reference limb for limb")
    return 0


if __name__ == "__main__":
    sys.exit(main())
