set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/p10.log 2>&1; echo "pytest rc=$?" >> gpurun_out/p10.log
timeout -k 10 400 bash tools/abn.sh 2 abv/base3.so abv/new9.so > gpurun_out/ab9.log 2>&1
