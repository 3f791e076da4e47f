#!/bin/bash
# Pre-pass kernel times (rocprofv3 kernel-trace stats) of library variants at
# a large-C config, T shortened.  usage (on the box):
#   TAG=x CFG=cfg5 SEQ=600 bash tools/prep_stats.sh label:lib.so ...   (lib "" = in-tree)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${TAG:-prep}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  label=${v%%:*}; lib=${v#*:}
  [ -n "$lib" ] && export CTCEXT_LIB_PATH=$R/$lib || unset CTCEXT_LIB_PATH
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$label -o run -- python3 $R/bench.py --config ${CFG:-cfg5} --seq-len ${SEQ:-600} --steps 2 --warmup 1 --no-cpu --no-host-io --no-strong > $O/$label.log 2>&1 || exit 1
  f=$(find $O/$label -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$label" <<'PY' >> $O/summary.txt
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "row_" in n or "beam_decode" in n:
        print("%-8s %-40s %4s %10.3f ms" % (sys.argv[2], n.split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
