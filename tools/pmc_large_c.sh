#!/bin/bash
# FETCH_SIZE / WRITE_SIZE counter passes of the decode kernel at cfg4 and cfg5
# (separate passes, each under its own time limit), the calibration passes
# over tools/fetch_calib, and the stamped summaries profiles/pmc_cfg4.json,
# profiles/pmc_cfg5.json.  usage (on the box): TAG=r5p bash tools/pmc_large_c.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-r5p}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
step() { echo "[$(date +%T)] $*" >> $O/steps.log; }
step fetch-calib
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_calib -o run -- $R/tools/fetch_calib > $O/calib.json 2> $O/fetch_calib.log || exit 14
step write-calib
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_calib -o run -- $R/tools/fetch_calib > /dev/null 2> $O/write_calib.log || exit 15
cc() { find $1 -name '*counter_collection.csv' | head -1; }
for cfg in ${CFGS:-cfg4 cfg5}; do
  steps=2; [ $cfg = cfg5 ] && steps=1
  step fetch-$cfg
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$cfg -o run -- python3 $R/bench.py --config $cfg --steps $steps --warmup 1 --no-cpu --no-host-io --no-strong > $O/fetch_$cfg.log 2>&1 || exit 12
  step write-$cfg
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$cfg -o run -- python3 $R/bench.py --config $cfg --steps $steps --warmup 1 --no-cpu --no-host-io --no-strong > $O/write_$cfg.log 2>&1 || exit 13
  T=2000; [ $cfg = cfg5 ] && T=3000
  READ_PATTERN=stream16 REC_BYTES=8 python3 $R/tools/pmc_summary.py $(cc $O/fetch_$cfg) $(cc $O/write_$cfg) $cfg $T $(cc $O/fetch_calib) $(cc $O/write_calib) $O/calib.json > $O/pmc_$cfg.json || exit 16
done
step done
