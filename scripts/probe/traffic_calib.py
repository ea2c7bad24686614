"""FETCH_SIZE / WRITE_SIZE calibration of k_hess's access patterns from
scripts/probe/traffic_probe (two rocprofv3 --pmc passes). Prints, per probe
kernel, counter bytes / known bytes (the guide's 16-B streaming read: 0.5).
usage: traffic_calib.py DIR  (DIR/fetch, DIR/write: rocprofv3 -d outputs;
DIR/probe.txt: the probe's stdout)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
known = defaultdict(list)
for line in open(os.path.join(d, "probe.txt")):
    name, b = line.split()
    known[name].append(int(b))
out = {}
for ctr, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
    rows = defaultdict(list)
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != ctr:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            rows[k].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]) * 1024.0))
    for k, v in rows.items():
        if "k_flush" in k:
            continue
        name = k if k in known else next((n for n in known if n.split("<")[0] == k.split("<")[0]
                                          and (("<" not in n) or n.split("<")[1] in k)), None)
        if name is None:
            continue
        vals = [x for _, x in sorted(v)]
        ratio = [x / b for x, b in zip(vals, known[name])]
        out.setdefault(name, {})[ctr] = {"bytes_counted": vals, "bytes_known": known[name], "ratio": ratio}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
