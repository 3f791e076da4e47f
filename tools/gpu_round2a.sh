#!/bin/bash
# Round-2 first GPU pass: host CPU share probe, GPU tests, cfg3 bench, cfg4/cfg5 full-size bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
O=gpurun_out
{ echo "nproc $(nproc)"; python -c "import os;print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; } > $O/r2_cpuinfo.txt
[ "$PYTEST_SEL" = skip ] || timeout -k 10 900 python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/r2_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > $O/r2_bench_cfg3.json 2> $O/r2_bench_cfg3.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu --no-host-io > $O/r2_bench_cfg4.json 2> $O/r2_bench_cfg4.err || exit $?
timeout -k 10 400 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu --no-host-io > $O/r2_bench_cfg5.json 2> $O/r2_bench_cfg5.err || exit $?
