set -o pipefail
cd $GRAFT_REPO_ROOT
CTCEXT_LIB_PATH=$PWD/tools/libctcext_phases.so timeout -k 10 300 python tools/diag_phases.py 256 1500 128 3 > gpurun_out/phases7.txt 2>&1
timeout -k 10 400 bash tools/abn.sh 1 abv/new9.so abv/new10.so > gpurun_out/ab10.log 2>&1
