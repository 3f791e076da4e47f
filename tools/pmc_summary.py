"""Per-launch HBM bytes of the decode kernel from two rocprofv3 counter passes.

usage: python tools/pmc_summary.py FETCH.csv WRITE.csv [config] > profiles/pmc_<config>.json

FETCH.csv / WRITE.csv are the counter_collection.csv files of
  rocprofv3 --pmc FETCH_SIZE --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu
  rocprofv3 --pmc WRITE_SIZE --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu
(separate passes: the two do not fit one TCC pass).  Values are KB per
dispatch; FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950 tallies each
128-B read request at 64 B), WRITE_SIZE is used as read.
"""
import csv
import json
import sys


def per_launch(path, counter):
    vals, name = [], None
    with open(path) as f:
        for row in csv.DictReader(f):
            if "ctcx_beam_decode" in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
                name = row["Kernel_Name"]
    if not vals:
        raise SystemExit("no ctcx_beam_decode %s rows in %s" % (counter, path))
    return sum(vals) / len(vals), len(vals), name


def main():
    fetch, nf, name = per_launch(sys.argv[1], "FETCH_SIZE")
    write, nw, _ = per_launch(sys.argv[2], "WRITE_SIZE")
    cfg = sys.argv[3] if len(sys.argv) > 3 else "cfg3"
    rd = fetch * 1024 * 2
    wr = write * 1024
    out = {
        "config": cfg, "kernel": name, "round": 1,
        "fetch_size_kb_raw": fetch, "write_size_kb": write, "launches": [nf, nw],
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                  "'python3 bench.py --steps 2 --warmup 1 --no-cpu' (MI355X); KB -> bytes; FETCH_SIZE "
                  "doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B read requests at 64 B); WRITE_SIZE as read",
        "note": "writes are the per-(item, frame, beam) 8-byte back-pointer records (256*1500*128*8 B = 393 MB) "
                "that the traceback kernel walks; reads are the logit rows and row normalisers",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
