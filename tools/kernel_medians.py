"""Per-kernel launch counts and median / mean durations from rocprofv3
--kernel-trace CSVs (one or more run directories), grouped by kernel name and
grid size.  usage: python tools/kernel_medians.py DIR [DIR ...] [--match SUBSTR]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    match = None
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        del args[i:i + 2]
    for d in args:
        files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        groups = defaultdict(list)
        for f in files:
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if match and match not in name:
                    continue
                grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
                groups[(name.split("(")[0][:70], grid)].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        print(f"== {d}")
        for (name, grid), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
            v.sort()
            print(f"  {name:70s} grid {grid:>10s} n {len(v):3d} median {v[len(v) // 2]:9.3f} ms "
                  f"mean {sum(v) / len(v):9.3f} ms")


if __name__ == "__main__":
    main()
