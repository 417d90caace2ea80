#!/usr/bin/env python3
"""Per-kernel average of one rocprofv3 --pmc pass (summed over counter instances): pmc_kernels.py DIR"""
import csv, glob, os, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float))
for path in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            per[(row["Kernel_Name"][:70], row["Counter_Name"])][(path, row.get("Dispatch_Id"))] += float(row["Counter_Value"])
for (k, c), v in sorted(per.items()):
    print(f"{c:12s} {sum(v.values()) / len(v):12.1f} x{len(v):3d}  {k}")
