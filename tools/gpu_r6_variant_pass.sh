# Round-6 pass for one library variant (abrun/lib$V.so): its parity tests
# (rank extract, bench digests, parity), then same-box A/B against the
# round's final build (abrun/libr6z.so) over $CFGS.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-r6m}; mkdir -p $O; cd $R
echo "[$(date +%T)] tests $V" >> $O/steps.log
CTCEXT_LIB_PATH=$R/abrun/lib$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_rank_extract.py tests/test_gpu_bench_digest.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_$V.log 2>&1 || exit 10
for cfg in ${CFGS:-cfg3 cfg2 cfg4}; do echo "[$(date +%T)] ab $cfg" >> $O/steps.log; echo "== $cfg" >> $O/summary.txt
  CFG=$cfg bash tools/abv.sh ${ROUNDS:-3} 'r6z||abrun/libr6z.so|' "$V||abrun/lib$V.so|" >> $O/summary.txt 2>&1 || exit 13; done
echo "[$(date +%T)] done" >> $O/steps.log
