#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2d_pytest.log 2>&1 || exit 21
QUICK=${QUICK:-0} TAG=r2d bash tools/profile_round.sh
