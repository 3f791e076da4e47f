#!/bin/bash
# Round-4 GPU pass: the -m gpu suite, then same-box A/B of the round-3 library
# (ab/libr3.so), the two-wave kernels (default), the two-wave kernel with the
# record ring, and the one-wave kernels of this build (CTCEXT_HELPER=0), at
# cfg3, cfg4 and cfg5.  usage (on the box): TAG=r4b bash tools/r4_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-r4}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
  echo "tests rc=$?" >> $O/summary.txt
fi
for cfg in ${CFGS:-cfg3 cfg4 cfg5}; do
  echo "== $cfg" >> $O/summary.txt
  if [ $cfg = cfg3 ]; then
    CFG=$cfg bash tools/abv.sh ${ROUNDS:-2} "r3||ab/libr3.so|" "hw|||" "hwnoring|||--no-ring" "nohw|CTCEXT_HELPER=0||" >> $O/summary.txt 2>&1 || exit 1
  else
    CFG=$cfg bash tools/abv.sh ${ROUNDS:-2} "r3||ab/libr3.so|" "hw|||" "nohw|CTCEXT_HELPER=0||" >> $O/summary.txt 2>&1 || exit 1
  fi
done
if [ "$PHASES" = 1 ]; then
  CTCEXT_LIB_PATH=$R/tools/libctcext_phases.so timeout -k 10 120 python tools/diag_phases.py 256 300 128 3 > $O/phases_cfg3.txt 2>&1
fi
echo done >> $O/summary.txt
