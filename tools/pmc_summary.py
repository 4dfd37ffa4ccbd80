"""Per-kernel summary of rocprofv3 PMC passes (tools/pmc_ggap_modes.sh): the
counters summed over each kernel's dispatches, divided by the dispatch count,
and the derived shares (wait cycles per wave cycle, VALU per busy cycle).
usage: python tools/pmc_summary.py DIR [DIR ...] > summary.json"""
import collections
import csv
import glob
import json
import os
import sys


def kernel_key(name):
    for k in ("k_gwin_probs", "k_gwin", "k_gband", "k_ggap_plan", "k_ggap<32", "k_ggap<64, false", "k_ggap<64, true"):
        if k in name:
            return k
    return None


out = {}
for d in sys.argv[1:]:
    cfg = os.path.basename(os.path.normpath(d)).rsplit("_pmc", 1)[0]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        tot = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            if k is None:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        for k, c in tot.items():
            e = out.setdefault(cfg, {}).setdefault(k, {"dispatches": len(disp[k])})
            e["dispatches"] = max(e["dispatches"], len(disp[k]))
            for n, v in c.items():
                e[n] = v / len(disp[k])
for cfg, ks in out.items():
    for k, e in ks.items():
        if "SQ_WAIT_ANY" in e and "SQ_WAVE_CYCLES" in e:
            e["wait_any_per_wave_cycle"] = round(e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"], 4)
        if "SQ_INSTS_VALU" in e and "SQ_WAVES" in e:
            e["valu_insts_per_wave"] = round(e["SQ_INSTS_VALU"] / e["SQ_WAVES"], 1)
        if "SQ_INSTS_VALU" in e and "SQ_BUSY_CYCLES" in e:
            e["valu_insts_per_busy_cycle"] = round(e["SQ_INSTS_VALU"] / e["SQ_BUSY_CYCLES"], 3)
print(json.dumps(out, indent=1, sort_keys=True))
