"""Mean per-dispatch counter values per kernel from a rocprofv3 --pmc output directory."""
import collections
import csv
import glob
import sys

KEEP = ("k_lean", "k_decode", "k_fast_merge", "k_big", "k_seq", "k_plan", "k_exec", "k_pack")


def main(d):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"]
        if any(k in name for k in KEEP):
            short = name.split("(")[0].replace("void ", "").replace("ym::", "")
            agg[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"{k:40s} {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
