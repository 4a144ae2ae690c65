"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per kernel."""
import csv
import sys
from collections import defaultdict


def load(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


if __name__ == "__main__":
    acc = load(sys.argv[1:])
    for k, cs in sorted(acc.items()):
        if not k.startswith("gsr"):
            continue
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:24s} {sum(v) / len(v):16.1f}   (n={len(v)})")
