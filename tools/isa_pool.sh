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
# issue cost per wave64 VALU instruction from the sustained rates of tools/ubench_valu.hip
# (profiles/r01_ubench_valu.txt): 55.3-56.8 lane-ops/clk/CU for the 64-bit and multiply class,
# 84.6 for v_add_u32; other 32-bit ALU ops are taken at v_add_u32's rate (not measured)
SLOW = ("v_mad_i64_i32", "v_mad_u64_u32", "v_mul_lo_u32", "v_lshl_add_u64", "v_ashrrev_i64", "v_mul_u32_u24",
        "v_mad_i32_i24", "v_lshlrev_b64", "v_lshrrev_b64", "v_add_co_u32", "v_addc_co_u32", "v_mul_hi_u32",
        "v_mul_i32_i24", "v_mad_u32_u24", "v_fma_f64")
def cycles(c):
    slow = sum(v for kk, v in c.items() if kk.startswith("v_") and kk.split("_e32")[0].split("_e64")[0] in SLOW)
    fast = sum(v for kk, v in c.items() if kk.startswith("v_")) - slow
    return slow, fast, slow * 4 * 64 / 55.5 + fast * 4 * 64 / 84.6
over = collections.Counter()
for k, ins in blocks.items():
    c = collections.Counter(ins)
    mad = c["v_mad_i64_i32"]
    valu = sum(v for kk, v in c.items() if kk.startswith("v_"))
    if mad in (520, 800):
        print("%s block %s: %d VALU, %d v_mad_i64_i32" % ("DBL" if mad == 520 else "mixed", k, valu, mad))
        print("  " + ", ".join("%s %d" % kv for kv in c.most_common(18)))
        sl, fa, cy = cycles(c)
        print("  issue cost: %d multiply/64-bit-class VALU x 4.61 + %d 32-bit VALU x 3.03 = %.0f SIMD cycles "
              "(%.2f per VALU; 4.00 if every VALU took 4)" % (sl, fa, cy, cy / max(1, sl + fa)))
    else:
        over.update(c)
print("other blocks (bookkeeping, refill, drain selection, park; not all run every step): %d VALU, %d SALU, %d LDS" % (
    sum(v for k, v in over.items() if k.startswith("v_")), sum(v for k, v in over.items() if k.startswith("s_")),
    sum(v for k, v in over.items() if k.startswith("ds_"))))
PY
rm -rf $D
