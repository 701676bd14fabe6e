#!/bin/bash
# Opcode histogram of k_dsm's main loop (the op-stream loop) for a build.
# usage: tools/isa_loop.sh [extra hipcc -D flags...]
set -e
D=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o $D/k.s \
  "$(dirname $0)/../firedancer_amd/csrc/fd_ed25519_kernels.hip" -I"$(dirname $0)/../firedancer_amd/csrc" "$@" 2>/dev/null
python3 - $D/k.s <<'PY'
import re, sys, collections
s = open(sys.argv[1]).read().split("\n")
# kernel bodies
starts = {}
for i, l in enumerate(s):
    m = re.match(r"^_Z(\d+)(\w+):", l)
    if m:
        starts[m.group(2)[:int(m.group(1))]] = i
for k in ("k_prep", "k_decomp", "k_dsm", "k_dsm4", "k_dsm8"):
    i = starts[k]
    j = next(n for n in range(i, len(s)) if "s_endpgm" in s[n])
    body = s[i:j]
    meta = "\n".join(s[j:j+120])
    vg = re.search(r"; NumVgprs: (\d+)", meta).group(1)
    occ = re.search(r"; Occupancy: (\d+)", meta).group(1)
    occ += " scratch " + re.search(r"; ScratchSize: (\d+)", meta).group(1)
    ins = [l.split()[0] for l in body if l.startswith("\t") and not l.strip().startswith(";") and not l.strip().startswith(".")]
    print("%-9s vgpr %s occ %s  static instrs %d" % (k, vg, occ, len(ins)))
    if k in ("k_dsm", "k_dsm4", "k_dsm8"):
        # largest loop: any label with a backward branch to it, farthest back-edge wins
        labs = {}
        for n in range(len(body)):
            m = re.match(r"^(\.LBB\d+_\d+):", body[n])
            if m: labs[m.group(1)] = n
        best = None
        for m_ in range(len(body)):
            mm = re.search(r"s_(?:c)?branch\w*\s+(\.LBB\d+_\d+)\s*$", body[m_])
            if mm and mm.group(1) in labs and labs[mm.group(1)] < m_:
                n = labs[mm.group(1)]
                if best is None or m_ - n > best[1] - best[0]:
                    best = (n, m_)
        loop = [l.split()[0] for l in body[best[0]:best[1]+1] if l.startswith("\t") and not l.strip().startswith(";")]
        c = collections.Counter(loop)
        heavy = sum(v for k2, v in c.items() if k2.startswith(("v_mad_i64", "v_mad_u64", "v_mul_lo", "v_lshl_add_u64", "v_ashrrev_i64", "v_lshrrev_b64", "v_lshlrev_b64", "v_mul_hi")))
        valu = sum(v for k2, v in c.items() if k2.startswith("v_"))
        print(k + " main loop: %d instrs, %d VALU (%d 64-bit/mul class), %d v_mad_i64_i32" % (len(loop), valu, heavy, c["v_mad_i64_i32"]))
        print("  " + ", ".join("%s %d" % kv for kv in c.most_common(16)))
PY
rm -rf $D
