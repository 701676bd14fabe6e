#!/bin/bash
# Regenerate the committed golden fixtures (tests/golden/) from the compiled
# reference and check them byte for byte.  Build container only: needs
# /root/reference and `make -C oracle ref tools` (done by __graft_entry__.build()).
#   tools/regen_golden.sh [outdir]      (default: a temp dir; compare only)
#   tools/regen_golden.sh tests/golden  (rewrite the fixtures in place)
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-$(mktemp -d)}
FIX=/root/reference/src/ballet/txn/fixtures
mkdir -p "$OUT"
oracle/_ref/gen_golden vectors "$OUT/ed25519_vectors.bin" "$FIX" oracle/false_rejects.txt
{ oracle/_ref/gen_golden stream 1234 65536 128 128 0
  oracle/_ref/gen_golden stream 2020 65536 200 200 1
  oracle/_ref/gen_golden stream 4040 32768 64 1232 1; } > "$OUT/ed25519_streams.jsonl"
oracle/_ref/gen_txn_golden "$OUT/txn_mutations.bin" "$FIX/transaction1.bin" "$FIX/transaction2.bin" "$FIX/transaction3.bin"
for f in ed25519_vectors.bin ed25519_streams.jsonl txn_mutations.bin; do
  cmp "$OUT/$f" "tests/golden/$f" && echo "$f: identical to the committed fixture"
done
