#!/bin/bash
# Kernel-trace stats + HBM counter passes of bench.py (cfg3) on the GPU box.
# usage (on the box): bash tools/profile_round.sh   -> gpurun_out/prof_{stats,fetch,write}/
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/prof_stats.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/prof_fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/prof_write.log 2>&1
