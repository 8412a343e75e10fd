#!/usr/bin/env python3
"""HBM bytes per mixed-rate step (bench.py --mixed) from rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE passes over ALL kernels of the run: sum over the
decode-path kernels (everything but the input generator and torch's own
kernels) of 2 x FETCH_SIZE + WRITE_SIZE (KB; gfx950 counts half of wide
reads, MI355X_MICROARCH.md HBM section), divided by the steps run (warmup +
timed).  Writes profiles/traffic.json["mixed_<set>_b<B>_it<I>"].
usage: python tools/mixed_traffic.py <fetch dir> <write dir> <steps run> <key> [out.json]"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SKIP = ("awgn_i8_k", "at::native", "__amd_rocclr")


def total(d, counter):
    tot, n = 0.0, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter or any(s in r.get("Kernel_Name", "") for s in SKIP):
                continue
            tot += float(r["Counter_Value"])
            n.add(r["Dispatch_Id"])
    return tot, len(n)


def main():
    fd, wd, steps, key = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(ROOT, "profiles", "traffic.json")
    fkb, nf = total(fd, "FETCH_SIZE")
    wkb, nw = total(wd, "WRITE_SIZE")
    per_step = (2.0 * fkb + wkb) * 1024.0 / steps
    tr = json.load(open(out)) if os.path.exists(out) else {}
    tr[key] = {"hbm_bytes_per_step": per_step, "fetch_kb_total": fkb, "write_kb_total": wkb, "steps": steps,
               "dispatches": [nf, nw], "source": "%s, %s" % (fd, wd)}
    json.dump(tr, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(tr[key]))


if __name__ == "__main__":
    main()
