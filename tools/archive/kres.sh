#!/bin/bash
# Resource usage (VGPRs, SGPRs, scratch, occupancy, LDS, code size) of the
# engine's kernels for a build: tools/kres.sh [extra hipcc -D flags...]
set -e
D=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o $D/k.s \
  "$(dirname $0)/../firedancer_amd/csrc/fd_ed25519_kernels.hip" -I"$(dirname $0)/../firedancer_amd/csrc" "$@" 2>/dev/null
python3 - $D/k.s <<'PY'
import re, sys
s = open(sys.argv[1]).read()
for m in re.finditer(r"^(_Z\d+(k_\w+?)\w*):", s, re.M):
    seg = s[m.end():]
    j = seg.find("s_endpgm")
    meta = seg[j:j+4000]
    f = lambda k: (re.search(r"; %s: (\d+)" % k, meta) or re.search(r"; %s = (\d+)" % k, meta))
    g = lambda k: f(k).group(1) if f(k) else "?"
    name = re.match(r"_Z(\d+)(\w+)", m.group(1)); name = name.group(2)[:int(name.group(1))]
    print("%-16s vgpr %-4s sgpr %-4s scratch %-5s occ %-2s lds %-6s code %s" % (name, g("NumVgprs"), g("NumSgprs"),
          g("ScratchSize"), g("Occupancy"), (re.search(r"; LDSByteSize: (\d+)", meta) or [0,"?"])[1], g("codeLenInByte")))
PY
rm -rf $D
