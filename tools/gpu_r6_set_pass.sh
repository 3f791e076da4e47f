# Round-6 pass for the set mode (abrun/libsetm.so): parity tests, the
# diagnostics build's set / replay counts, then same-box A/B against r6z.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/${TAG:-r6p}; mkdir -p $O; cd $R
echo "[$(date +%T)] tests" >> $O/steps.log
CTCEXT_LIB_PATH=$R/abrun/libsetm.so timeout -k 10 500 python -u -m pytest tests/test_gpu_rank_extract.py tests/test_gpu_bench_digest.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_setm.log 2>&1 || exit 10
echo "[$(date +%T)] diag" >> $O/steps.log
CTCEXT_LIB_PATH=$R/abrun/libphases.so CTCX_DIAG_SET=1 timeout -k 10 120 python3 -u tools/diag_phases.py 256 300 128 3 > $O/set_cfg3.txt 2>&1 || exit 11
CTCEXT_LIB_PATH=$R/abrun/libphases.so CTCX_DIAG_SET=1 timeout -k 10 120 python3 -u tools/diag_phases.py 32 1000 64 1 > $O/set_cfg2.txt 2>&1 || exit 12
for cfg in cfg3 cfg2; do echo "[$(date +%T)] ab $cfg" >> $O/steps.log; echo "== $cfg" >> $O/summary.txt
  CFG=$cfg bash tools/abv.sh 3 'r6z||abrun/libr6z.so|' 'setm||abrun/libsetm.so|' >> $O/summary.txt 2>&1 || exit 13; done
echo "[$(date +%T)] done" >> $O/steps.log
