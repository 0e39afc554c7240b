"""Sum rocprofv3 counter_collection.csv values of the render kernel(s) in a directory."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rt_book1" in r["Kernel_Name"] or "rt_render" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(d, " ".join(f"{k}={v:.4g}" for k, v in sorted(agg.items())))
