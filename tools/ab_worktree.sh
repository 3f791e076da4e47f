#!/bin/bash
# Same-box A/B of the current tree against an older commit checked out as a
# git worktree at ./abold (each side runs its own bench.py + library, so the
# C ABI of either side may differ).  usage: tools/ab_worktree.sh rounds [bench args]
N=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
for r in $(seq $N); do
  for side in abold .; do
    v=$(cd $R/$side && timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu --no-host-io "$@" 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f %.2f" % (d["value"], d["roofline"]["kernel_ms"]))') || exit 1
    echo "$side $v"
  done
done
