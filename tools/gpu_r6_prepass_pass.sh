set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-r6g}; mkdir -p $O; cd $R
echo "[$(date +%T)] prepass tests" >> $O/steps.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_prepass.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/focus.log 2>&1 || exit 10
echo "[$(date +%T)] tests" >> $O/steps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/summary.txt
[ $rc -le 1 ] || exit 11
for cfg in cfg4 cfg5; do echo "[$(date +%T)] ab $cfg" >> $O/steps.log; echo "== $cfg" >> $O/summary.txt
  CFG=$cfg bash tools/abv.sh 3 'interp||' 'bisect||abrun/libbisect.so|' >> $O/summary.txt 2>&1 || exit 13; done
echo "[$(date +%T)] done" >> $O/steps.log
