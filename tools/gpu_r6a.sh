set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/r6a; mkdir -p $O; cd $R
echo "[$(date +%T)] tests" >> $O/steps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/summary.txt
[ $rc -le 1 ] || exit 11
echo "[$(date +%T)] bench" >> $O/steps.log
timeout -k 10 400 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit 12
echo "[$(date +%T)] ab" >> $O/steps.log
for cfg in cfg3 cfg4; do echo "== $cfg" >> $O/summary.txt; CFG=$cfg bash tools/abv.sh 2 'r5||abrun/libr5.so|' 'r6||' >> $O/summary.txt 2>&1 || exit 13; done
echo "[$(date +%T)] done" >> $O/steps.log
echo "[$(date +%T)] phases" >> $O/steps.log
PHASES_LIB=$R/abrun/libctcext_phases.so bash tools/gpu_phases.sh || exit 14
for c in cfg3 cfg4 cfg5; do mv gpurun_out/ph_$c.txt $O/ph_$c.txt; done
echo "[$(date +%T)] done2" >> $O/steps.log
