#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs: mean counter value per dispatch, per kernel."""
import collections
import csv
import glob
import os
import sys


def short(name: str) -> str:
    for key, tag in (("k_step", "k_step"), ("k_ms_classes", "k_pulses<MS>"), ("k_pulses<0, 4,", "k_pulses<MU>"), ("k_pulses<1, 4,", "k_pulses<MS>"),
                     ("k_pulses<1, 2,", "k_pulses<MS,narrow>"), ("k_pulsesILi1ELi2E", "k_pulses<MS,narrow>"),
                     ("k_pulses<0, 64,", "k_pulses<MU,long>"), ("k_pulses<1, 64,", "k_pulses<MS,long>"),
                     ("k_pulsesILi0ELi4E", "k_pulses<MU>"), ("k_pulsesILi1ELi4E", "k_pulses<MS>"),
                     ("k_mc<8", "k_mc<long>"), ("k_mcILi8", "k_mc<long>"), ("k_mc", "k_mc"), ("k_parse_lines", "k_parse_lines"), ("k_sel_count", "k_sel_count"),
                     ("k_sel_write", "k_sel_write"), ("k_mn(", "k_mn"), ("k_parse_rare", "k_parse_rare"), ("k_parse_comp", "k_parse_comp")):
        if key in name:
            return tag
    return name[:40]


def main(root: str) -> None:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if not k.startswith("k_"):
                    continue
                acc[k][(row["Dispatch_Id"], row["Counter_Name"])].append(float(row["Counter_Value"]))
    for k in sorted(acc):
        per = collections.defaultdict(list)
        for (disp, cn), vals in acc[k].items():
            per[cn].append(sum(vals))  # sum over dimensions (SE/XCD instances) within one dispatch
        print(f"== {k}")
        for cn in sorted(per):
            v = per[cn]
            print(f"  {cn:24s} {sum(v) / len(v):16.4e}   ({len(v)} dispatches)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
