"""Calibration of the CPU baseline: the oracle's reference-cost ("faithful")
mode timed on the survey's shapes, one item per fresh process (as bench.py's
cpu_baseline runs it), against the compiled reference's figures the survey
measured on the same container type.

Each process decodes the item twice: the first call is the cold one (fresh
heap: its ~2.4 GB of nodes and vectors page-fault in), the second reuses the
freed heap.  bench.py times cold calls.  Prints one JSON line per shape with
the medians and the port / reference ratios.

    python tools/cpu_calibrate.py [runs]
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (name, T, C, W, P, merge, survey frames/s per core of the compiled reference)
SHAPES = [("cfg3_shape", 1500, 29, 128, 3, True, 189.0),
          ("cfg2_shape", 1000, 29, 64, 1, True, 455.0),
          ("cfg4_shape_T100", 100, 1000, 64, 1, True, 23.8)]
CHILD = r"""
import sys, time, json, numpy as np
sys.path.insert(0, %r)
import oracle
T, C, W, P, merge = %d, %d, %d, %d, %r
x = np.random.default_rng(20251015).standard_normal((T, 1, C), dtype=np.float32)
out = []
for rep in range(2):
    t0 = time.perf_counter()
    oracle.raw_decode(x, np.array([T], np.int32), W, P, merge, 0, -1, mode="faithful")
    out.append(T / (time.perf_counter() - t0))
print(json.dumps(out))
"""


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for name, T, C, W, P, merge, ref in SHAPES:
        cold, warm = [], []
        for _ in range(runs):
            code = CHILD % (os.path.join(ROOT, "oracle"), T, C, W, P, merge)
            r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True)
            c, w = json.loads(r.stdout.strip().splitlines()[-1])
            cold.append(c)
            warm.append(w)
        mc, mw = statistics.median(cold), statistics.median(warm)
        print(json.dumps({"shape": name, "T": T, "C": C, "beam_width": W, "top_paths": P, "runs": runs,
                          "port_cold_fps": [round(v, 1) for v in cold], "port_warm_fps": [round(v, 1) for v in warm],
                          "port_cold_median": round(mc, 1), "port_warm_median": round(mw, 1),
                          "reference_fps_survey": ref, "cold_ratio": round(mc / ref, 3),
                          "warm_ratio": round(mw / ref, 3), "cpu": os.cpu_count()}), flush=True)


if __name__ == "__main__":
    main()
