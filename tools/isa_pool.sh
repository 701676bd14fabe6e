#!/bin/bash
# Opcode histograms of k_dsmp's blocks (the DBL step block, the mixed step block, and the per-step
# bookkeeping outside them) for a build.  usage: tools/isa_pool.sh [extra hipcc -D flags...]
set -e
D=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o $D/k.s \
  "$(dirname $0)/../firedancer_amd/csrc/fd_ed25519_kernels.hip" -I"$(dirname $0)/../firedancer_amd/csrc" "$@" 2>/dev/null
python3 - $D/k.s <<'PY'
import re, sys, collections
s = open(sys.argv[1]).read().split("\n")
i = next(n for n, l in enumerate(s) if re.match(r"^_Z\d+k_dsmp\w*:", l))
j = next(n for n in range(i, len(s)) if "s_endpgm" in s[n])
body = s[i:j + 1]
meta = "\n".join(s[j:j + 200])
print("k_dsmp vgpr %s occ %s lds %s" % (re.search(r"; NumVgprs: (\d+)", meta).group(1),
      re.search(r"; Occupancy: (\d+)", meta).group(1), re.search(r"; LDSByteSize: (\d+)", meta).group(1)))
blocks, cur = {}, "entry"
blocks[cur] = []
for l in body:
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        cur = m.group(1); blocks[cur] = []; continue
    if l.startswith("\t") and not l.strip().startswith(";") and not l.strip().startswith("."):
        blocks[cur].append(l.split()[0])
over = collections.Counter()
for k, ins in blocks.items():
    c = collections.Counter(ins)
    mad = c["v_mad_i64_i32"]
    valu = sum(v for kk, v in c.items() if kk.startswith("v_"))
    if mad in (520, 800):
        print("%s block %s: %d VALU, %d v_mad_i64_i32" % ("DBL" if mad == 520 else "mixed", k, valu, mad))
        print("  " + ", ".join("%s %d" % kv for kv in c.most_common(18)))
    else:
        over.update(c)
print("other blocks (bookkeeping, refill, drain selection, park; not all run every step): %d VALU, %d SALU, %d LDS" % (
    sum(v for k, v in over.items() if k.startswith("v_")), sum(v for k, v in over.items() if k.startswith("s_")),
    sum(v for k, v in over.items() if k.startswith("ds_"))))
PY
rm -rf $D
