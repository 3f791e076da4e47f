# Round-6 pass: the fast helper rank and the early first poll (variants in
# abrun/), their rank-extract and bench-digest tests, then same-box A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-r6l}; mkdir -p $O; cd $R
for v in rf16 rf8; do
  echo "[$(date +%T)] tests $v" >> $O/steps.log
  CTCEXT_LIB_PATH=$R/abrun/lib$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_rank_extract.py tests/test_gpu_bench_digest.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || exit 10
done
for cfg in cfg3 cfg2; do echo "[$(date +%T)] ab $cfg" >> $O/steps.log; echo "== $cfg" >> $O/summary.txt
  CFG=$cfg bash tools/abv.sh 3 'r6z||abrun/libr6z.so|' 'rf||abrun/librf.so|' 'rf16||abrun/librf16.so|' 'rf8||abrun/librf8.so|' >> $O/summary.txt 2>&1 || exit 13; done
echo "[$(date +%T)] done" >> $O/steps.log
