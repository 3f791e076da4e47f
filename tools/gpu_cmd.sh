set -o pipefail
cd $GRAFT_REPO_ROOT
CTCEXT_LIB_PATH=$PWD/tools/libctcext_phases.so timeout -k 10 300 python tools/diag_phases.py 256 1500 128 3 > gpurun_out/phases2.txt 2>&1
