"""Sums SQ counters over the decode kernel's dispatches (rocprofv3
counter_collection CSVs, any number of passes) and prints the instruction mix
and wait shares per wave.  usage: sq_summary.py pass1.csv [pass2.csv ...]"""
import csv
import os
import sys
from collections import defaultdict

KERNEL = os.environ.get("SQ_KERNEL", "ctcx_beam_decode")   # substring of the kernel name

tot = defaultdict(float)
disp = defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(tot):
    print("%-24s %18.0f  (%d dispatches)" % (k, tot[k], len(disp[k])))
w = tot.get("SQ_WAVES", 0.0)
cyc = tot.get("SQ_WAVE_CYCLES", 0.0)
if w and cyc:
    print("per wave: %.0f wave-cycles" % (cyc / w))
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
        if k in tot:
            print("  %-18s %12.0f per wave" % (k, tot[k] / w))
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS", "SQ_BUSY_CYCLES"):
        if k in tot:
            print("  %-18s %6.1f%% of wave-cycles" % (k, 100.0 * tot[k] / cyc))
