#!/bin/bash
# One GPU-box pass for a build under test (usage on the box:
#   TAG=r5d TESTS="tests/test_gpu_helper_modes.py" AB="cfg3 cfg4" VARIANTS='...' bash tools/gpu_pass.sh):
#   1. the given pytest files (default: the whole -m gpu suite); a test
#      failure (rc 1) goes on to the timings, anything worse (a crash, a
#      time limit) ends the pass;
#   2. same-box A/B rounds of bench.py per config over VARIANTS (tools/abv.sh
#      syntax: 'label|ENV=VAL|lib.so|bench args', space-separated);
#   3. PHASES=1: the per-phase cycle split (tools/gpu_phases.sh) with the
#      diagnostics build, under each HELPER in $PHASE_HELPERS.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-r5}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
step() { echo "[$(date +%T)] $*" >> $O/steps.log; }
if [ "$SKIP_TESTS" != 1 ]; then
  step tests
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
  rc=$?
  echo "tests rc=$rc" >> $O/summary.txt
  [ $rc -le 1 ] || exit 11
fi
for cfg in $AB; do
  step ab-$cfg
  echo "== $cfg" >> $O/summary.txt
  eval "CFG=$cfg bash tools/abv.sh ${ROUNDS:-2} $VARIANTS" >> $O/summary.txt 2>&1 || exit 12
done
if [ "$PHASES" = 1 ]; then
  for h in ${PHASE_HELPERS:-1}; do
    step phases-$h
    CTCEXT_HELPER=$h bash tools/gpu_phases.sh || exit 13
    for c in cfg3 cfg4 cfg5; do mv gpurun_out/ph_$c.txt $O/ph_${c}_h$h.txt; done
  done
fi
step done
