#!/bin/bash
# One GPU-box pass that produces every judged number of a round:
#   kernel-trace stats of bench.py (cfg3; cfg4 and cfg5 at full T unless QUICK=1),
#   the FETCH_SIZE / WRITE_SIZE passes of cfg3 plus the calibration passes over
#   tools/fetch_calib (same counters, known byte counts), the stamped
#   pmc_cfg3.json, and finally the default bench line (which then reads it).
# usage (on the box): TAG=r2 bash tools/profile_round.sh   -> gpurun_out/$TAG/
# tools/fetch_calib is built beforehand on the CPU side:
#   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${TAG:-r2}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
step() { echo "[$(date +%T)] $*" >> $O/steps.log; }
step stats-cfg3
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_cfg3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-host-io --no-strong > $O/stats_cfg3.log 2>&1 || exit 11
step fetch-cfg3
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_cfg3 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-host-io --no-strong > $O/fetch_cfg3.log 2>&1 || exit 12
step write-cfg3
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_cfg3 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-host-io --no-strong > $O/write_cfg3.log 2>&1 || exit 13
step fetch-calib
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_calib -o run -- $R/tools/fetch_calib > $O/calib.json 2> $O/fetch_calib.log || exit 14
step write-calib
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_calib -o run -- $R/tools/fetch_calib > /dev/null 2> $O/write_calib.log || exit 15
cc() { find $1 -name '*counter_collection.csv' | head -1; }
REC_BYTES=${REC_BYTES:-4} python3 $R/tools/pmc_summary.py $(cc $O/fetch_cfg3) $(cc $O/write_cfg3) cfg3 1500 $(cc $O/fetch_calib) $(cc $O/write_calib) $O/calib.json > $O/pmc_cfg3.json || exit 16
cp $O/pmc_cfg3.json $R/profiles/pmc_cfg3.json
step bench-cfg3
cd $R
timeout -k 10 300 python3 bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit 17
if [ "$QUICK" != 1 ]; then
  cd /tmp
  step stats-cfg4
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_cfg4 -o run -- python3 $R/bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu --no-host-io --no-strong > $O/stats_cfg4.log 2>&1 || exit 18
  step stats-cfg5
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_cfg5 -o run -- python3 $R/bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu --no-host-io --no-strong > $O/stats_cfg5.log 2>&1 || exit 19
fi
step done
