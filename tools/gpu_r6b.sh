set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-r6b}; mkdir -p $O; cd $R
echo "[$(date +%T)] tests" >> $O/steps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/summary.txt
[ $rc -le 1 ] || exit 11
echo "[$(date +%T)] ab" >> $O/steps.log
for cfg in ${AB_CFGS:-cfg3 cfg2}; do echo "== $cfg" >> $O/summary.txt; eval "CFG=$cfg bash tools/abv.sh ${ROUNDS:-3} $VARIANTS" >> $O/summary.txt 2>&1 || exit 13; done
echo "[$(date +%T)] phases" >> $O/steps.log
if [ -n "$PHASES_LIB" ]; then
PHASES_LIB=$R/$PHASES_LIB bash tools/gpu_phases.sh || exit 14
for c in cfg3 cfg4 cfg5; do mv gpurun_out/ph_$c.txt $O/ph_$c.txt; done
fi
echo "[$(date +%T)] done" >> $O/steps.log
