#!/bin/bash
# A/B of two libctcext builds on one box: alternate bench runs (cfg3 unless $CFG).
# usage: tools/ab.sh libA.so libB.so [rounds]
A=$1; B=$2; N=${3:-2}; CFG=${CFG:-cfg3}; EXTRA=${EXTRA:-}
for r in $(seq $N); do
  for L in $A $B; do
    v=$(CTCEXT_LIB_PATH=$PWD/$L timeout -k 10 240 python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu $EXTRA | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.0f %.2f" % (d["value"], d["roofline"]["kernel_ms"]))') || exit 1
    echo "$L $v"
  done
done
