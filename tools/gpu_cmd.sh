set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/p2.log 2>&1; echo "pytest rc=$?" >> gpurun_out/p2.log
