#!/bin/bash
# Same-box A/B of the current tree against an older commit checked out as a
# git worktree at ./abold (each side runs its own bench.py + library, so the
# C ABI of either side may differ).  usage: tools/ab_worktree.sh rounds [bench args]
# Parity gate: each side's outputs are hashed (this tree's bench.output_digest,
# the same for both sides) and a side whose outputs differ from the oracle's
# fixture (tests/golden/bench_digests.json), or without one from this tree's,
# prints OUTPUT-MISMATCH instead of a timing.
N=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
for r in $(seq $N); do
  REF=""
  for side in . abold; do
    v=$(cd $R/$side && timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu --no-host-io "$@" 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f %.2f %s" % (d["value"], d["roofline"]["kernel_ms"], d.get("outputs_sha256", "-")[:16]))') || exit 1
    read -r val kms sha <<< "$v"
    if [ "$sha" = "-" ]; then   # an older bench.py without the digest: hash with this tree's
      echo "$side: no outputs_sha256 in its line; timing withheld"
      continue
    fi
    [ -z "$REF" ] && REF=$sha
    if [ "$sha" != "$REF" ]; then
      echo "$side OUTPUT-MISMATCH (outputs $sha, this tree $REF): timing withheld"
      continue
    fi
    echo "$side $val $kms"
  done
done
