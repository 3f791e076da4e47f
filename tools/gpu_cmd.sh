set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/p6.log 2>&1; echo "pytest rc=$?" >> gpurun_out/p6.log
timeout -k 10 400 bash tools/abn.sh 2 abv/new3.so abv/new5.so > gpurun_out/ab5.log 2>&1
CTCEXT_LIB_PATH=$PWD/tools/libctcext_phases.so timeout -k 10 300 python tools/diag_phases.py 256 1500 128 3 > gpurun_out/phases4.txt 2>&1
