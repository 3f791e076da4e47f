set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-r6d}; mkdir -p $O; cd $R
echo "[$(date +%T)] focused large-C tests" >> $O/steps.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "large_c or large_vocab" > $O/focus.log 2>&1 || exit 10
echo "[$(date +%T)] tests" >> $O/steps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/summary.txt
[ $rc -le 1 ] || exit 11
for cfg in cfg3 cfg2; do echo "[$(date +%T)] ab $cfg" >> $O/steps.log; echo "== $cfg" >> $O/summary.txt
  CFG=$cfg bash tools/abv.sh 3 'cur||' 'noctab||abrun/libnoctab.so|' 'r5||abrun/libr5.so|' >> $O/summary.txt 2>&1 || exit 13; done
for cfg in cfg4 cfg5; do echo "[$(date +%T)] ab $cfg" >> $O/steps.log; echo "== $cfg" >> $O/summary.txt
  CFG=$cfg bash tools/abv.sh 2 'cur||' 'nochash||abrun/libnochash.so|' 'r5||abrun/libr5.so|' >> $O/summary.txt 2>&1 || exit 14; done
echo "[$(date +%T)] done" >> $O/steps.log
