#!/bin/bash
# Same-box A/B of library builds and environment variants, round-robin.
# usage: CFG=cfg3 tools/abv.sh rounds 'label|ENV=VAL ...|path/to/lib.so|bench args' ...
# (an empty field: none / the in-tree build / no extra bench args)
N=$1; shift
CFG=${CFG:-cfg3}; EXTRA=${EXTRA:-}
R=${GRAFT_REPO_ROOT:-$PWD}
for r in $(seq $N); do
  for v in "$@"; do
    IFS='|' read -r label envs lib xargs <<< "$v"
    [ -n "$lib" ] && lib="CTCEXT_LIB_PATH=$R/$lib"
    out=$(cd $R && env $envs $lib timeout -k 10 240 python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu --no-host-io --no-strong $EXTRA $xargs 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.0f %.2f %.3f %.3f %.2f" % (d["value"], d["roofline"]["kernel_ms"], d["roofline"].get("prepass_ms") or 0.0, d["roofline"].get("traceback_ms") or 0.0, d["ms_per_step"]))') || exit 1
    echo "$label $out"
  done
done
