#!/bin/bash
# A/B/... of several libctcext builds on one box: round-robin bench runs (cfg3 unless $CFG).
# usage: tools/abn.sh rounds libA.so libB.so ...
N=$1; shift; CFG=${CFG:-cfg3}; EXTRA=${EXTRA:-}
for r in $(seq $N); do
  for L in "$@"; do
    v=$(CTCEXT_LIB_PATH=$PWD/$L timeout -k 10 240 python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu $EXTRA 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.0f %.2f" % (d["value"], d["roofline"]["kernel_ms"]))') || exit 1
    echo "$L $v"
  done
done
