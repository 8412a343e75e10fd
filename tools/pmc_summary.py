#!/usr/bin/env python3
"""Mean per-dispatch value of every counter in rocprofv3 --pmc passes
(tools/profile.sh output dirs) for kernels matching a pattern, as JSON:
  python tools/pmc_summary.py <out.json> <kernel substring> <prof dir> [<prof dir>...]
SQ_* wave counters count quad-cycles summed over waves (MI355X_MICROARCH.md)."""
import csv
import glob
import json
import os
import sys


def main():
    out, pat, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = {}
    for d in dirs:
        for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
            acc, disp = {}, set()
            for r in csv.DictReader(open(f)):
                if pat not in r.get("Kernel_Name", ""):
                    continue
                acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
            if disp:
                res["%s/%s" % (os.path.basename(d.rstrip("/")), f.split(os.sep)[-2])] = {
                    k: v / len(disp) for k, v in sorted(acc.items())}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
