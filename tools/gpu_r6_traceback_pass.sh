set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-r6e}; mkdir -p $O; cd $R
echo "[$(date +%T)] focused traceback tests" >> $O/steps.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "paper or edge or single_class or record_ring or global_state_tier_shapes or full_length_golden or cfg3_full" > $O/focus.log 2>&1 || exit 10
echo "[$(date +%T)] tests" >> $O/steps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/summary.txt
[ $rc -le 1 ] || exit 11
for cfg in cfg3 cfg4 cfg5; do echo "[$(date +%T)] ab $cfg" >> $O/steps.log; echo "== $cfg" >> $O/summary.txt
  CFG=$cfg bash tools/abv.sh 2 'seg||' 'old|CTCEXT_TRACEBACK=0||' >> $O/summary.txt 2>&1 || exit 13; done
echo "[$(date +%T)] ab extbig" >> $O/steps.log; echo "== cfg4 rank extract at large C (extbig: CTCX_EXT_BIG=1; its traceback is the old kernel)" >> $O/summary.txt
CFG=cfg4 bash tools/abv.sh 2 'cur||' 'extbig||abrun/libextbig.so|' >> $O/summary.txt 2>&1 || exit 15
echo "[$(date +%T)] bench" >> $O/steps.log
timeout -k 10 400 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit 14
echo "[$(date +%T)] done" >> $O/steps.log
