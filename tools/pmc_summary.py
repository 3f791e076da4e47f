"""Per-launch HBM bytes of the decode kernel from two rocprofv3 counter passes,
stamped with the library build they measured.

usage: python tools/pmc_summary.py FETCH.csv WRITE.csv CONFIG SEQ_LEN CALIB_FETCH.csv CALIB_WRITE.csv CALIB.json
       > profiles/pmc_<CONFIG>.json

FETCH.csv / WRITE.csv are the counter_collection.csv files of
  rocprofv3 --pmc FETCH_SIZE --output-format csv -- python3 bench.py --config CONFIG --steps 2 --warmup 1 --no-cpu
  rocprofv3 --pmc WRITE_SIZE --output-format csv -- python3 bench.py --config CONFIG --steps 2 --warmup 1 --no-cpu
(separate passes: the two do not fit one TCC pass).  Values are KB per dispatch.

Unit correction: MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16 B/lane
streaming reads (it reports 1/2 of the bytes).  The decode kernel reads its
logit rows at 4 B/lane (C*4-byte rows, neighbouring items' rows sharing 128-B
lines on different XCDs) and stores 8 B/lane records, so the factors applied
here come from tools/fetch_calib.hip, which replays exactly those two access
patterns over known byte counts in the same two counter passes
(CALIB_*.csv; CALIB.json is its stdout).  factor = known bytes / counter bytes.
"""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ctc-beam-search-op_amd", "ctcext_amd", "lib", "libctcext.so")


def per_launch(path, counter, kname):
    vals, name = [], None
    with open(path) as f:
        for row in csv.DictReader(f):
            if kname in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
                name = row["Kernel_Name"]
    if not vals:
        raise SystemExit("no %s %s rows in %s" % (kname, counter, path))
    return sum(vals) / len(vals), len(vals), name


def all_kernels(fetch_path, write_path, f_read, f_write):
    """Every kernel of the decode call in the two passes (the pre-pass, the
    decode, the traceback and packing): per-launch corrected bytes and their
    sum over one call (each kernel runs once per call)."""
    acc = {}
    for path, counter in ((fetch_path, "FETCH_SIZE"), (write_path, "WRITE_SIZE")):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != counter:
                    continue
                k = row["Kernel_Name"]
                if "ctcx" not in k:   # (torch's own kernels: input generation, copies)
                    continue
                e = acc.setdefault(k, {"FETCH_SIZE": [], "WRITE_SIZE": []})
                e[counter].append(float(row["Counter_Value"]))
    out, call = {}, 0.0
    for k, e in sorted(acc.items()):
        rd = (sum(e["FETCH_SIZE"]) / len(e["FETCH_SIZE"]) * 1024 * f_read) if e["FETCH_SIZE"] else 0.0
        wr = (sum(e["WRITE_SIZE"]) / len(e["WRITE_SIZE"]) * 1024 * f_write) if e["WRITE_SIZE"] else 0.0
        out[k.split("(")[0]] = {"read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                               "launches": [len(e["FETCH_SIZE"]), len(e["WRITE_SIZE"])]}
        call += rd + wr
    return out, call


def main():
    fetch_csv, write_csv, cfg, seq_len, cf_csv, cw_csv, calib_json = sys.argv[1:8]
    known = json.load(open(calib_json))
    fetch, nf, name = per_launch(fetch_csv, "FETCH_SIZE", "ctcx_beam_decode")
    write, nw, _ = per_launch(write_csv, "WRITE_SIZE", "ctcx_beam_decode")
    c_rows, _, _ = per_launch(cf_csv, "FETCH_SIZE", "calib_rows")
    c_s16, _, _ = per_launch(cf_csv, "FETCH_SIZE", "calib_stream16")
    # the decode kernel's record width: REC_BYTES=4 for the two-wave kernel
    # (stats.record_bytes), else the 8-byte records
    rb = int(os.environ.get("REC_BYTES", "8"))
    cname, kname = ("calib_rec32_store", "calib_rec32_store_write") if rb == 4 else ("calib_rec_store", "calib_rec_store_write")
    c_rec, _, _ = per_launch(cw_csv, "WRITE_SIZE", cname)
    f_rows = known["calib_rows"] / (c_rows * 1024)
    f_s16 = known["calib_stream16"] / (c_s16 * 1024)
    f_rec = known[kname] / (c_rec * 1024)
    # the decode kernel's row reads: 4 B/lane (C <= 64, the default) or, for
    # large C, batches of 16-byte loads (READ_PATTERN=stream16)
    pattern = os.environ.get("READ_PATTERN", "rows4")
    rd = fetch * 1024 * (f_s16 if pattern == "stream16" else f_rows)
    wr = write * 1024 * f_rec
    with open(LIB, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    out = {
        "config": cfg, "seq_len": int(seq_len), "kernel": name, "lib_sha16": sha,
        "fetch_size_kb_raw": fetch, "write_size_kb_raw": write, "launches": [nf, nw],
        "calibration": {"fetch_factor_rows_4B_lane": f_rows, "fetch_factor_stream_16B_lane": f_s16,
                        "write_factor_records": f_rec, "record_bytes": rb, "read_pattern": pattern,
                        "tool": "tools/fetch_calib.hip"},
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                  "'python3 bench.py --config %s --steps 2 --warmup 1 --no-cpu' (MI355X); KB -> bytes; "
                  "each counter scaled by the factor tools/fetch_calib.hip measured for the same access "
                  "pattern over a known byte count in the same pass" % cfg,
    }
    # the whole call: every kernel's bytes (reads at the stream16 factor for
    # the large-C pre-pass and rows, writes at the record factor)
    ak, call = all_kernels(fetch_csv, write_csv, f_s16 if pattern == "stream16" else f_rows, f_rec)
    out["all_kernels"] = ak
    out["hbm_bytes_per_call"] = call
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
