"""Summarise rocprofv3 --pmc csv passes (tools/pmc_attn.sh) per kernel: mean counter value per
dispatch of each prfl kernel.  usage: python tools/pmc_summary.py gpurun_out/pmc_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "*", "pmc_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "at::" in name:
            continue
        if "anonymous namespace)::" in name:
            short = name.split("::")[1].split("((")[0].split("(")[0] if "<" not in name else name.split("::")[1].split(">(")[0] + ">"
        else:                      # a library kernel (hipBLASLt Cijk_...): keep its name head
            short = name[:72]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
for k, cs in acc.items():
    print(f"== {k}  (mean dispatch {sum(dur[k]) / len(dur[k]):.2f} ms)")
    mean = {c: sum(v) / len(v) for c, v in cs.items()}
    for c, v in sorted(mean.items()):
        print(f"   {c:28s} {v:.4g}")
    ms = sum(dur[k]) / len(dur[k])
    if "GRBM_GUI_ACTIVE" in mean:      # MI355X_MICROARCH.md, DVFS give-back: sum over 8 XCDs
        print(f"   -> effective clock {mean['GRBM_GUI_ACTIVE'] / 8 / (ms * 1e-3) / 1e9:.2f} GHz")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            print(f"   -> MFMA busy {mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (mean['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
