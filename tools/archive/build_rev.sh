#!/bin/bash
# Build the engine library of git revision REV into OUT (A/B baselines).
# usage: tools/build_rev.sh REV OUT.so
set -e
REV=$1; OUT=$(realpath -m "$2")
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$(mktemp -d)
git -C "$ROOT" archive "$REV" firedancer_amd/csrc include tools/gen_consts.py firedancer_amd/build.py | tar -x -C "$D"
cd "$D" && python3 - "$OUT" <<'PY'
import sys, os
sys.path.insert(0, os.getcwd())
from firedancer_amd import build
print(build.build_engine(force=True, out=sys.argv[1]))
PY
rm -rf "$D"
