"""Summarise a tools/profile_round.sh run into profiles/.

* profiles/<tag>_kernel_stats.csv : rocprofv3 --stats kernel summary (copied)
* profiles/<tag>_bench.json       : the bench line measured under the tracer
* profiles/<tag>_pmc.csv          : per-kernel HBM bytes per launch from the
  FETCH_SIZE / WRITE_SIZE passes
* profiles/pmc_traffic.json       : the dominant bench kernel's HBM bytes per
  launch, read by bench.py for roofline.traffic

Unit handling follows /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced streaming reads, so it is doubled.  Our record
streams are 8-B-per-lane loads (not the guide's calibrated 16-B case), so the
doubled value is an estimate; the raw counters are kept next to it.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def counters(path):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            a = agg[name]
            a[0] += 1
            a[1] += float(r["Counter_Value"])
    return agg


def main():
    out, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, "%s_kernel_stats.csv" % tag))
    bench = json.load(open(os.path.join(out, "bench.json")))
    json.dump(bench, open(os.path.join(prof, "%s_bench.json" % tag), "w"), indent=1)
    fetch = counters(os.path.join(out, "pmc_FETCH_SIZE"))
    write = counters(os.path.join(out, "pmc_WRITE_SIZE"))
    rows = []
    for name in sorted(set(fetch) | set(write)):
        nf, f = fetch.get(name, [0, 0.0])
        nw, w = write.get(name, [0, 0.0])
        n = max(nf, nw, 1)
        rows.append({"kernel": name, "launches": n,
                     "fetch_kib_raw_per_launch": f / max(nf, 1),
                     "write_kib_per_launch": w / max(nw, 1),
                     "hbm_bytes_per_launch": (2.0 * f / max(nf, 1) + w / max(nw, 1)) * 1024.0})
    with open(os.path.join(prof, "%s_pmc.csv" % tag), "w", newline="") as fh:
        wr = csv.DictWriter(fh, fieldnames=list(rows[0]))
        wr.writeheader()
        wr.writerows(rows)
    dom = bench["roofline"]["kernel"]
    per = {timer_name(r["kernel"]): r["hbm_bytes_per_launch"] for r in rows}
    # the bench's roofline.traffic source: the headline (C2 consume) workload
    # only; other profiles (C4, C5, queries) go to <tag>_traffic.json
    headline = bench["config"]["workload"].startswith("Countgraph k=21 4x1e+09, consume of 50000000 ")
    traffic_json = os.path.join(prof, "pmc_traffic.json" if headline else "%s_traffic.json" % tag)
    json.dump({"kernel": dom, "config": bench["config"]["workload"],
               "hbm_bytes_per_launch": per.get(dom),
               "kernels": per,
               "note": "HBM bytes per launch (FETCH_SIZE doubled per the gfx950 calibration + WRITE_SIZE), "
                       "keyed by the engine's kernel timer names; tag %s" % tag},
              open(traffic_json, "w"), indent=1)
    print("dominant", dom, per.get(dom))


def timer_name(device_kernel):
    """kh::k_apply_count<1> -> apply_byte, kh::k_scatter_l1<...> -> scatter_l1 (kh_engine.hip TIMED names)."""
    base = device_kernel.split("<")[0].split("::")[-1]
    if base.startswith("k_"):
        base = base[2:]
    if base == "apply_count":
        kind = device_kernel.split("<")[1].split(">")[0].split(",")[0].strip()
        return {"1": "apply_byte", "7": "apply_nibble"}.get(kind, base)
    if base == "apply_bit":
        return "apply_bit"
    # the fixed-capacity partitions time under the same names as the exact ones
    return {"scatter_l1f": "scatter_l1", "scatter_l1p": "scatter_l1", "scatter_l2f": "scatter_l2", "hist_wf": "hist_w", "scatter_wf": "scatter_w",
            "mark_wf": "mark", "median_fixed": "median"}.get(base, base)


if __name__ == "__main__":
    main()
