#!/usr/bin/env python3
"""Summarise tools/prof_pmc.sh output: per-kernel counter means over dispatches,
plus derived values (HBM bytes with the gfx950 FETCH_SIZE x2 correction of
MI355X_MICROARCH.md s HBM, VALU busy, wait shares)."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
n_sigs = int(sys.argv[2]) if len(sys.argv) > 2 else 262144   # the --sigs of the profiled bench run
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    der = {}
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        der["hbm_bytes_per_launch"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        der["fetch_kb_raw"] = m["FETCH_SIZE"]
        der["write_kb_raw"] = m["WRITE_SIZE"]
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        w = m["SQ_WAVE_CYCLES"]
        der["active_share"] = m.get("SQ_ACTIVE_INST_ANY", 0) / w
        der["wait_inst_share"] = m.get("SQ_WAIT_INST_ANY", 0) / w
        der["wait_any_share"] = m.get("SQ_WAIT_ANY", 0) / w
    if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m and m["SQ_WAVES"]:
        der["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
    out[k] = {"counters": m, "derived": der}
out["_sigs_per_launch"] = n_sigs
json.dump(out, sys.stdout, indent=1, sort_keys=True)
print()
