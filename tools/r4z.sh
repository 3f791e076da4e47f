#!/bin/bash
# Round-4 pass: pre-pass test + large-C parity, gather-queue depth A/B (cfg4, cfg5), cfg4 pre-pass stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-r4z}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_prepass.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "prepass or row_facts or large or full or helper or ring" > $O/gputest.log 2>&1
echo "tests rc=$?" >> $O/summary.txt
for c in cfg4 cfg5; do
  echo "== $c" >> $O/summary.txt
  CFG=$c bash tools/abv.sh 2 "q4|||" "q2||ab/libq2.so|" "q1||ab/libq1.so|" >> $O/summary.txt 2>&1 || exit 1
done
TAG=$TAG CFG=cfg4 SEQ=2000 bash tools/prep_stats.sh r4p4:ab/libr4p.so new4: || exit 1
echo done >> $O/summary.txt
