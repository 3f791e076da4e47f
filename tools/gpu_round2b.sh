#!/bin/bash
# GPU tests, then the profiling pass (tools/profile_round.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/r2b_pytest.log 2>&1 || exit $?
[ "$PROFILE" = 0 ] || bash tools/profile_round.sh
