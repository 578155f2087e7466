#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per dispatch, by kernel-name substring: pmc_by_kernel.py <dir>... -k <substr>"""
import csv
import glob
import sys
from collections import defaultdict

args = sys.argv[1:]
sub = args[args.index("-k") + 1] if "-k" in args else ""
dirs = [a for a in args if a not in ("-k", sub)]
tot, cnt = defaultdict(float), defaultdict(set)
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / max(1, len(cnt[k])):16.4g}  (dispatches {len(cnt[k])})")
