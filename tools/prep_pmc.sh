#!/bin/bash
# SQ instruction counters of the pre-pass kernels for library variants
# (one counter pass per variant).  usage (on the box):
#   TAG=x CFG=cfg5 SEQ=600 bash tools/prep_pmc.sh label:lib.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${TAG:-prep}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  label=${v%%:*}; lib=${v#*:}
  [ -n "$lib" ] && export CTCEXT_LIB_PATH=$R/$lib || unset CTCEXT_LIB_PATH
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_$label -o run -- python3 $R/bench.py --config ${CFG:-cfg5} --seq-len ${SEQ:-600} --steps 1 --warmup 1 --no-cpu --no-host-io --no-strong > $O/pmc_$label.log 2>&1 || exit 1
  f=$(find $O/pmc_$label -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$label" <<'PY' >> $O/pmc_summary.txt
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "row_" not in n:
        continue
    k = n.split("(")[0][-28:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    w = d["SQ_WAVES"] or 1
    print("%-8s %-28s waves %.0f  per wave: VALU %.0f SALU %.0f LDS %.0f  wave-cycles(quad) %.0f  busy %.0f" % (
        sys.argv[2], k, w, d["SQ_INSTS_VALU"] / w, d["SQ_INSTS_SALU"] / w, d["SQ_INSTS_LDS"] / w,
        d["SQ_WAVE_CYCLES"] / w, d["SQ_BUSY_CYCLES"]))
PY
done
