#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2c_pytest.log 2>&1 || exit 21
TAG=r2c bash tools/profile_round.sh
