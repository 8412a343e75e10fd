#!/usr/bin/env python3
"""Turn the rocprofv3 output merged back into gpurun_out/prof (tools/profile.sh)
into committed summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (pass 1; every launch, warm-up included)
  profiles/<tag>_kernel_steady.json per kernel from the kernel trace: the bench's warm-up launches
                                    excluded, median / mean / min / max of the rest (the number to
                                    compare with the bench's HIP-event kernel time and ms_per_step)
  profiles/<tag>_bench.json         the bench JSON line printed under pass 1
  profiles/<tag>_pmc.json           per-kernel FETCH_SIZE / WRITE_SIZE per dispatch
  profiles/traffic.json             {workload key: {hbm_bytes_per_launch, ...}} read by bench.py

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes): on gfx950
FETCH_SIZE reports half of the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM section); both counters are summed over the XCDs.
usage: python tools/summarize_profiles.py <tag> [gpurun_out/prof]
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def find(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    return hits[-1] if hits else None


def pmc_per_kernel(path, counter):
    """mean counter value per dispatch, keyed by kernel name."""
    acc = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "?")
            acc.setdefault(name, []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def steady(trace_csv, warmup):
    """Per kernel name: durations in dispatch order, the first `warmup`
    dropped (the bench launches each step kernel once per step)."""
    acc = {}
    with open(trace_csv) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "?")
            acc.setdefault(name, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = {}
    for name, v in acc.items():
        d = [x[1] for x in sorted(v)]
        k = d[warmup:] if len(d) > warmup else d
        k_sorted = sorted(k)
        med = k_sorted[len(k) // 2] if len(k) % 2 else 0.5 * (k_sorted[len(k) // 2 - 1] + k_sorted[len(k) // 2])
        out[name] = dict(calls=len(d), excluded_warmup=len(d) - len(k), measured=len(k), median_ms=med / 1e6,
                         mean_ms=sum(k) / len(k) / 1e6, min_ms=min(k) / 1e6, max_ms=max(k) / 1e6)
    return out


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = find(os.path.join(src, "trace", "**", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats, os.path.join(dst, "%s_kernel_stats.csv" % tag))
    bench = None
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{") and '"metric"' in line:
                bench = json.loads(line)
        if bench:
            json.dump(bench, open(os.path.join(dst, "%s_bench.json" % tag), "w"), indent=1)
    ktrace = find(os.path.join(src, "trace", "**", "*kernel_trace.csv"))
    if ktrace:
        st = steady(ktrace, bench["warmup"] if bench else 0)
        top = sorted(st.items(), key=lambda kv: -kv[1]["median_ms"] * kv[1]["measured"])
        json.dump(dict(top), open(os.path.join(dst, "%s_kernel_steady.json" % tag), "w"), indent=1)
        for name, v in top[:3]:
            print("%-60s median %.4f ms  mean %.4f  (%d measured, %d warm-up excluded)"
                  % (name[:60], v["median_ms"], v["mean_ms"], v["measured"], v["excluded_warmup"]))
    fetch = find(os.path.join(src, "fetch", "**", "*counter_collection.csv"))
    write = find(os.path.join(src, "write", "**", "*counter_collection.csv"))
    pmc = {}
    if fetch and write:
        fk = pmc_per_kernel(fetch, "FETCH_SIZE")
        wk = pmc_per_kernel(write, "WRITE_SIZE")
        for k in fk:
            pmc[k] = dict(fetch_kb=fk[k], write_kb=wk.get(k), hbm_bytes=(2 * fk[k] + (wk.get(k) or 0)) * 1024)
        # other counter passes (sq, tcc, ...): mean per dispatch
        for extra in ("sq", "sq2", "tcc", "tcp"):
            path = find(os.path.join(src, extra, "**", "*counter_collection.csv"))
            if not path:
                continue
            names = sorted({r["Counter_Name"] for r in csv.DictReader(open(path))})
            for cn in names:
                for k, v in pmc_per_kernel(path, cn).items():
                    pmc.setdefault(k, {})[cn] = v
        json.dump(pmc, open(os.path.join(dst, "%s_pmc.json" % tag), "w"), indent=1)
    if bench and pmc:
        cfg = bench["config"]
        key = "%s_b%d_it%d_%s" % (cfg["code"], cfg["batch_per_gpu"], cfg["iters"], cfg["kernel"])
        dec = [v for k, v in pmc.items() if "decode" in k]
        if dec:
            tr_path = os.path.join(dst, "traffic.json")
            tr = json.load(open(tr_path)) if os.path.exists(tr_path) else {}
            # the source hash the bench line reports (the build the passes ran
            # on): bench.py uses the entry only for that build
            tr[key] = dict(hbm_bytes_per_launch=dec[0]["hbm_bytes"], fetch_kb=dec[0]["fetch_kb"],
                           write_kb=dec[0]["write_kb"], source="profiles/%s_pmc.json" % tag,
                           src_sha16=bench.get("build", {}).get("src_sha16"))
            json.dump(tr, open(tr_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(dict(stats=stats, bench=bool(bench), pmc=list(pmc)), indent=1))


if __name__ == "__main__":
    main()
