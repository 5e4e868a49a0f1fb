#!/usr/bin/env python3
"""Counter / known-bytes ratios of tools/calib_traffic.hip's kernels.

FETCH_SIZE and WRITE_SIZE are reported by rocprofv3 in KiB (MI355X_MICROARCH.md, HBM section).  For
every calibration kernel: the bytes it reads and writes by construction (its `known.txt` line) and
the counters of its launch; ratio = counter bytes / known bytes.  The guide's statement for 16-B/lane
streaming reads is FETCH ratio 0.5.  usage: python tools/calib_traffic.py gpurun_out/calib [out.json]"""
import csv
import glob
import json
import os
import sys


def counters(root, name):
    out = {}
    for f in glob.glob(os.path.join(root, name, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != name:
                    continue
                k = row.get("Kernel_Name", "").split("(")[0].split()[-1]
                out[k] = out.get(k, 0.0) + float(row["Counter_Value"])
    return out


def main(root, dst=None):
    known = {}
    with open(os.path.join(root, "known.txt")) as fh:
        for ln in fh:
            p = ln.split()
            if len(p) == 3 and p[0].startswith("k_"):
                known[p[0]] = (int(p[1]), int(p[2]))
    fetch, write = counters(root, "FETCH_SIZE"), counters(root, "WRITE_SIZE")
    res = {}
    for k, (rd, wr) in known.items():
        f = fetch.get(k, 0.0) * 1024
        w = write.get(k, 0.0) * 1024
        res[k] = {"known_read_bytes": rd, "known_write_bytes": wr, "FETCH_SIZE_bytes": f, "WRITE_SIZE_bytes": w,
                  "fetch_ratio": f / rd if rd else None, "write_ratio": w / wr if wr else None}
        print(f"{k:18s} read {rd / 1e6:9.1f} MB  FETCH {f / 1e6:9.1f} MB  ratio {res[k]['fetch_ratio'] or 0:6.3f}   "
              f"write {wr / 1e6:9.1f} MB  WRITE {w / 1e6:9.1f} MB  ratio {res[k]['write_ratio'] or 0:6.3f}")
    res["_note"] = ("counter bytes / bytes moved by construction, per calibration kernel "
                    "(tools/calib_traffic.hip); FETCH_SIZE and WRITE_SIZE in KiB x 1024")
    if dst:
        with open(dst, "w") as fh:
            json.dump(res, fh, indent=1)
    return res


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else os.path.join(sys.argv[1], "calib_traffic.json"))
