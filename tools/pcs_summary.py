#!/usr/bin/env python3
"""Summarise a rocprofv3 PC-sampling CSV (stochastic, cycles): samples per instruction of one
kernel, with the instruction text and the stall reason columns the CSV carries, plus per source
line when the code object has line info.  usage: python tools/pcs_summary.py DIR [kernel-substring] [top]"""
import collections
import csv
import glob
import os
import sys


def main(root, kern="k_pulses<0", top=60):
    files = [f for f in glob.glob(os.path.join(root, "**", "*.csv"), recursive=True) if "pc_sampl" in f.lower()]
    if not files:
        files = glob.glob(os.path.join(root, "**", "*.csv"), recursive=True)
    print("files:", [os.path.relpath(f, root) for f in files])
    for f in files:
        with open(f, newline="") as fh:
            rd = csv.DictReader(fh)
            cols = rd.fieldnames or []
            print(os.path.basename(f), "columns:", cols)
            rows = list(rd)
        if not rows or not any("nstruction" in c for c in cols):
            continue
        kcol = next((c for c in cols if "Kernel" in c or "Dispatch" in c), None)
        icol = next(c for c in cols if c.lower() in ("instruction", "inst"))
        pcol = next((c for c in cols if "Offset" in c or c.lower() in ("pc", "instruction_offset")), None)
        scol = [c for c in cols if "stall" in c.lower() or "reason" in c.lower() or "Issued" in c or "Type" in c]
        sel = [r for r in rows if kern in r.get(kcol, "")] if kcol and any(kern in r.get(kcol, "") for r in rows) else rows
        print(f"{len(sel)} samples of {len(rows)} for '{kern}'")
        cnt = collections.Counter()
        reason = collections.defaultdict(collections.Counter)
        text = {}
        for r in sel:
            key = r.get(pcol, "") if pcol else r[icol]
            cnt[key] += 1
            text[key] = r[icol]
            for c in scol:
                reason[key][f"{c}={r[c]}"] += 1
        tot = sum(cnt.values())
        for key, c in cnt.most_common(int(top)):
            rs = ", ".join(f"{k}:{v}" for k, v in reason[key].most_common(3))
            print(f"{100 * c / tot:6.2f}%  {key:>10}  {text[key][:70]:70s}  {rs}")
        agg = collections.Counter()
        for r in sel:
            for c in scol:
                agg[f"{c}={r[c]}"] += 1
        print("overall:", agg.most_common(20))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:]))
