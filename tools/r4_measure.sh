#!/bin/bash
# Round-4 measurement pass on the box: kernel-trace stats of bench.py at cfg3,
# cfg4, cfg5 (rocprofv3 --stats), the tier line, the default bench line.
# usage: TAG=r4i bash tools/r4_measure.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-r4}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for cfg in ${CFGS:-cfg3 cfg4 cfg5}; do
  steps=3; [ $cfg = cfg5 ] && steps=2
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$cfg -o run -- python3 $R/bench.py --config $cfg --steps $steps --warmup 1 --no-cpu --no-host-io --no-strong > $O/bench_$cfg.json 2> $O/bench_$cfg.err) || exit 11
done
(cd $R && timeout -k 10 200 python tools/tier_bench.py > $O/tier.json 2> $O/tier.err) || exit 12
echo done > $O/done.txt
