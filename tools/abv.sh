#!/bin/bash
# Same-box A/B of library builds and environment variants, round-robin.
# usage: CFG=cfg3 tools/abv.sh rounds 'label|ENV=VAL ...|path/to/lib.so|bench args' ...
# (an empty field: none / the in-tree build / no extra bench args)
# Parity gate: a variant's timing is printed only when its outputs hash to the
# oracle's for the bench inputs (bench.py outputs_match_oracle, fixtures in
# tests/golden/bench_digests.json); where no fixture exists (cfg5, a T or B
# override) the outputs must hash equal to the first variant's.  A variant
# whose outputs differ prints OUTPUT-MISMATCH and no timing.
N=$1; shift
CFG=${CFG:-cfg3}; EXTRA=${EXTRA:-}
R=${GRAFT_REPO_ROOT:-$PWD}
REF=""
for r in $(seq $N); do
  for v in "$@"; do
    IFS='|' read -r label envs lib xargs <<< "$v"
    [ -n "$lib" ] && lib="CTCEXT_LIB_PATH=$R/$lib"
    out=$(cd $R && env $envs $lib timeout -k 10 240 python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu --no-host-io --no-strong $EXTRA $xargs 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f %.2f %.3f %.3f %.2f %s %s %d" % (d["value"], d["roofline"]["kernel_ms"], d["roofline"].get("prepass_ms") or 0.0, d["roofline"].get("traceback_ms") or 0.0, d["ms_per_step"], d.get("outputs_match_oracle"), d.get("outputs_sha256", "-")[:16], d.get("helper_redecodes", 0)))') || exit 1
    read -r val kms pms tms sms match sha red <<< "$out"
    [ -z "$REF" ] && REF=$sha
    if [ "$match" = "False" ] || { [ "$match" = "None" ] && [ "$sha" != "$REF" ]; }; then
      echo "$label OUTPUT-MISMATCH (outputs $sha, oracle match $match, first variant $REF): timing withheld"
      continue
    fi
    echo "$label $val $kms $pms $tms $sms oracle=$match redecodes=$red"
  done
done
