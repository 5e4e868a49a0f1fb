#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc.sh).

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB and derive from the
L2's memory-side request counters; on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide
coalesced reads, so it is doubled here; WRITE_SIZE is taken as reported.  Infinity-Cache hits are
counted, so this is L2-miss traffic.  Writes a JSON keyed by kernel tag.
usage: python tools/pmc_traffic.py gpurun_out/pmc profiles/r01/pmc_traffic.json
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def per_launch(root: str, counter: str):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                k = short(row.get("Kernel_Name", ""))
                if k.startswith("k_"):
                    acc[k][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in acc.items() if v}


def main(root: str, out: str) -> None:
    fetch, write = per_launch(root, "FETCH_SIZE"), per_launch(root, "WRITE_SIZE")
    sq = {c: per_launch(root, c) for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                                          "SQ_WAVES")}
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f_kib, w_kib = fetch.get(k), write.get(k)
        tb = None if f_kib is None or w_kib is None else 2.0 * f_kib * 1024 + w_kib * 1024
        res[k] = {"fetch_size_kib": f_kib, "write_size_kib": w_kib, "traffic_bytes": tb,
                  "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950, MI355X_MICROARCH.md HBM section; calibrated "
                                "for this build's access widths in profiles/r05/calib/calib_traffic.json: vector loads "
                                "of 1, 4 and 16 B per lane and 8-B gathers count at exactly half, scalar loads exactly, "
                                "stores exactly; a scattered 8-B store costs a 32-B write)"}
        for c, d in sq.items():  # per-launch instruction counts (the issue-side view of the kernel)
            if k in d:
                res[k][c.lower()] = d[k]
    res["_config"] = json.loads(os.environ.get("PMC_CONFIG", "null")) or \
        {"command": "python3 bench.py --steps 3 --warmup 1 --no-cpu", "msgs_per_gpu": 1000000}
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc",
         sys.argv[2] if len(sys.argv) > 2 else "profiles/r01/pmc_traffic.json")
