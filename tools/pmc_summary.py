#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter collected by tools/pmc.sh (rocprofv3 csv output).
FETCH_SIZE is reported as collected and x2 (gfx950 correction, MI355X_MICROARCH.md §HBM);
both sizes are in KB as rocprofv3 reports them."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", name).replace("gs::", "")


def main():
    root = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                vals[k][row["Counter_Name"]].append((row.get("Dispatch_Id"), float(row["Counter_Value"])))
    for k in sorted(vals):
        print(k)
        for c in sorted(vals[k]):
            # one value per dispatch (sum over dimensions already done by rocprofv3 per row)
            per = defaultdict(float)
            for d, v in vals[k][c]:
                per[d] += v
            xs = list(per.values())
            mean = sum(xs) / len(xs)
            extra = ""
            if c == "FETCH_SIZE":
                extra = "  (x2 corrected: %.0f KB)" % (2 * mean)
            print("   %-24s n=%3d mean=%.4g%s" % (c, len(xs), mean, extra))


if __name__ == "__main__":
    main()
