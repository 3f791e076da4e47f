#!/bin/bash
# A/B/C... of libctcext builds on one box: tools/ab3.sh rounds lib1.so lib2.so ...
N=$1; shift
for r in $(seq $N); do
  for L in "$@"; do
    v=$(CTCEXT_LIB_PATH=$PWD/$L timeout -k 10 240 python bench.py --config ${CFG:-cfg3} --steps 3 --warmup 1 --no-cpu ${EXTRA:-} | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.0f %.2f" % (d["value"], d["roofline"]["kernel_ms"]))') || exit 1
    echo "$L $v"
  done
done
