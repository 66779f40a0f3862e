#!/usr/bin/env python3
"""Turn a tools/collect_profiles.sh output directory into the committed profile set:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary of the bench command (verbatim)
  profiles/<tag>_frame.txt          per-launch durations of one steady-state frame, by position
  profiles/<tag>_pmc.json           per frame position (kernel#k = k-th launch of that kernel in a
                                    frame): mean duration and mean PMC counters over the timed frames;
                                    fetch_bytes = FETCH_SIZE x 2 x 1024 (gfx950 correction,
                                    MI355X_MICROARCH.md §HBM), write_bytes = WRITE_SIZE x 1024
  profiles/<tag>_pmc.txt            the same as a table

    python tools/profile_summary.py gpurun_out/prof_r01 r01 [out_dir (default profiles/)]
"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", name).replace("gs::", "")


def frames_of(rows, key_start="k_cull"):
    """Split dispatches (in order) into frames starting at k_cull; label positions."""
    frames, cur = [], None
    for r in rows:
        n = short(r["Kernel_Name"])
        if n.split("<")[0] == key_start:
            cur = []
            frames.append(cur)
        if cur is not None:
            cur.append(r)
    out = []
    for f in frames:
        seen = defaultdict(int)
        lab = []
        for r in f:
            n = short(r["Kernel_Name"])
            lab.append(("%s#%d" % (n, seen[n]), r))
            seen[n] += 1
        out.append(lab)
    return out


def load_trace(path):
    with open(path) as fh:
        rows = list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(prof, tag + "_kernel_stats.csv"))

    # durations by frame position (skip warm-up: the 20 frames before the last, which is
    # bench.py's untimed one-chunk statistics frame)
    trace = frames_of(load_trace(os.path.join(src, "stats", "run_kernel_trace.csv")))
    timed = trace[-21:-1]
    dur = defaultdict(list)
    for f in timed:
        for lab, r in f:
            dur[lab].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    f = trace[-3]
    lines = ["one steady-state frame (third to last), %d launches" % len(f),
             "(gaps inside the stream are host launch latency under the tracer; untraced frames",
             " keep the queue full: compare span with bench ms_per_step)"]
    prev = None
    for lab, r in f:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        lines.append("  gap %7.2f us  dur %8.2f us  %s" % (gap, (e - s) / 1e3, lab))
        prev = e
    span = (int(f[-1][1]["End_Timestamp"]) - int(f[0][1]["Start_Timestamp"])) / 1e3
    lines.append("span %.1f us" % span)
    open(os.path.join(prof, tag + "_frame.txt"), "w").write("\n".join(lines) + "\n")

    # PMC counters by frame position
    pmc = defaultdict(lambda: defaultdict(list))
    for grp in ("sq1", "sq2", "fetch", "write"):
        p = os.path.join(src, grp, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        with open(p) as fh:
            rows = list(csv.DictReader(fh))
        # one row per (dispatch, counter); rebuild dispatch order from timestamps
        disp = {}
        for r in rows:
            d = disp.setdefault(r["Dispatch_Id"], {"Kernel_Name": r["Kernel_Name"],
                                                   "Start_Timestamp": r["Start_Timestamp"], "c": defaultdict(float)})
            d["c"][r["Counter_Name"]] += float(r["Counter_Value"])
        order = sorted(disp.values(), key=lambda d: int(d["Start_Timestamp"]))
        for fr in frames_of(order)[-6:-1]:
            for lab, d in fr:
                for c, v in d["c"].items():
                    pmc[lab][c].append(v)
    out = {}
    for lab in sorted(set(dur) | set(pmc), key=lambda s: (s.split("#")[0], int(s.split("#")[1]))):
        e = {"calls_per_frame_position": len(dur.get(lab, [])),
             "mean_us": round(sum(dur[lab]) / len(dur[lab]), 3) if dur.get(lab) else None}
        for c, vs in sorted(pmc.get(lab, {}).items()):
            e[c] = sum(vs) / len(vs)
        if "FETCH_SIZE" in e:
            e["fetch_bytes"] = e["FETCH_SIZE"] * 2 * 1024
        if "WRITE_SIZE" in e:
            e["write_bytes"] = e["WRITE_SIZE"] * 1024
        if "fetch_bytes" in e and "write_bytes" in e:
            e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        out[lab] = e
    json.dump(out, open(os.path.join(prof, tag + "_pmc.json"), "w"), indent=1)
    cols = ["mean_us", "fetch_bytes", "write_bytes", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
            "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT"]
    lines = ["%-26s" % "launch" + "".join("%15s" % c.replace("SQ_", "")[:14] for c in cols)]
    for lab, e in out.items():
        lines.append("%-26s" % lab + "".join("%15.4g" % e[c] if e.get(c) is not None else "%15s" % "-" for c in cols))
    open(os.path.join(prof, tag + "_pmc.txt"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
