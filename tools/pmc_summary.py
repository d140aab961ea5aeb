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
        if "anonymous namespace)::" not in name or "at::" in name:
            continue
        short = name.split("::")[1].split("(")[0]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
for k, cs in acc.items():
    print(f"== {k}  (mean dispatch {sum(dur[k]) / len(dur[k]):.2f} ms)")
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):.4g}")
