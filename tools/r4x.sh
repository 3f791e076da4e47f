#!/bin/bash
# Round-4 pre-pass / global-state-tier pass: the -m gpu suite, the parity
# sweep, the tier line, pre-pass kernel stats against the round's profiled
# build (ab/libr4p.so) and their SQ counters.  usage (on the box): TAG=r4x bash tools/r4x.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-r4x}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "tests rc=$?" >> $O/summary.txt
timeout -k 10 300 python -u tools/parity_sweep.py ${SWEEP:-400} > $O/parity_sweep.txt 2>&1
echo "sweep rc=$?" >> $O/summary.txt
timeout -k 10 200 python -u tools/tier_bench.py > $O/tier.json 2>&1 || exit 1
TAG=$TAG CFG=cfg5 SEQ=600 bash tools/prep_stats.sh r4p:ab/libr4p.so new: $EXTRA_LIBS || exit 1
TAG=$TAG CFG=cfg4 SEQ=2000 bash tools/prep_stats.sh r4p4:ab/libr4p.so new4: || exit 1
TAG=$TAG CFG=cfg5 SEQ=600 bash tools/prep_pmc.sh r4p:ab/libr4p.so new: || exit 1
if [ "$PHASES" = 1 ]; then
  export CTCEXT_LIB_PATH=$R/tools/libctcext_phases.so
  timeout -k 10 120 python3 -u tools/diag_phases.py 128 400 64 1 1000 > $O/phases_cfg4_hw.txt 2>&1 || exit 1
  CTCEXT_HELPER=0 timeout -k 10 120 python3 -u tools/diag_phases.py 128 400 64 1 1000 > $O/phases_cfg4_onewave.txt 2>&1 || exit 1
  timeout -k 10 180 python3 -u tools/diag_phases.py 256 100 256 1 5000 > $O/phases_cfg5_hw.txt 2>&1 || exit 1
  unset CTCEXT_LIB_PATH
fi
echo done >> $O/summary.txt
