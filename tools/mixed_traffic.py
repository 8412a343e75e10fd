#!/usr/bin/env python3
"""HBM bytes per mixed-rate step (bench.py --mixed) from rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE passes over ALL kernels of the run: sum over the
decode-path kernels (everything but the input generator and torch's own
kernels) of 2 x FETCH_SIZE + WRITE_SIZE (KB; gfx950 counts half of wide
reads, MI355X_MICROARCH.md HBM section), divided by the steps run (warmup +
timed).  The workload key, the step count and the source hash of the build
come from the bench JSON line the FETCH pass itself printed, so
profiles/traffic.json["mixed_<set>_b<B>_it<I>"] carries the src_sha16 that
bench.py matches before reporting the number.
usage: python tools/mixed_traffic.py <fetch dir> <write dir> <fetch pass log> [out.json]"""
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


def bench_line(log):
    line = None
    for l in open(log):
        if l.startswith("{") and '"metric"' in l:
            line = json.loads(l)
    if line is None:
        raise SystemExit("mixed_traffic: no bench line in %s" % log)
    return line


def main():
    fd, wd, log = sys.argv[1], sys.argv[2], sys.argv[3]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles", "traffic.json")
    b = bench_line(log)
    cfg = b["config"]
    key = "mixed_%s_b%d_it%d" % (cfg.get("code_set", "configs4"), cfg["batch_per_gpu"], cfg["iters_max"])
    steps = b["steps"] + b["warmup"]
    fkb, nf = total(fd, "FETCH_SIZE")
    wkb, nw = total(wd, "WRITE_SIZE")
    per_step = (2.0 * fkb + wkb) * 1024.0 / steps
    tr = json.load(open(out)) if os.path.exists(out) else {}
    tr[key] = {"hbm_bytes_per_step": per_step, "fetch_kb_total": fkb, "write_kb_total": wkb, "steps": steps,
               "dispatches": [nf, nw], "source": "%s, %s" % (fd, wd),
               "src_sha16": b.get("build", {}).get("src_sha16")}
    json.dump(tr, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(tr[key]))


if __name__ == "__main__":
    main()
