#!/bin/bash
# One GPU-box pass for a build under test: the -m gpu suite, then kernel-trace
# stats of bench.py at cfg3 / cfg4 / cfg5 (the decode and pre-pass kernels),
# then the global-state-tier line.  Every step under its own time limit; the
# first failure ends the run.  usage (on the box): TAG=r4a bash tools/gpu_check.sh
# SKIP_TESTS=1 skips the suite; CFGS="cfg3 cfg5" picks the configs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-r4}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*" >> $O/steps.log; }
if [ "$SKIP_TESTS" != 1 ]; then
  step tests
  (cd $R && timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1) || exit 11
fi
for cfg in ${CFGS:-cfg3 cfg4 cfg5}; do
  step stats-$cfg
  steps=3; [ $cfg = cfg5 ] && steps=1
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$cfg -o run -- python3 $R/bench.py --config $cfg --steps $steps --warmup 1 --no-cpu --no-host-io --no-strong > $O/bench_$cfg.json 2> $O/bench_$cfg.err) || exit 12
done
if [ "$SKIP_TIER" != 1 ]; then
  step tier
  (cd $R && timeout -k 10 200 python tools/tier_bench.py > $O/tier.json 2> $O/tier.err) || exit 13
fi
step done
