#!/usr/bin/env python3
"""Stamp a tools/pmc.sh summary (gpurun_out/<run>/pmc_traffic.json) with the commit and the libsdx
source hash it was taken on, and install it as PMC_TRAFFIC.json at the repo root -- the tracked file
bench.py reads for roofline.traffic / issue (it ships to the GPU box; profiles/ does not).

usage: python tools/pmc_commit.py gpurun_out/<run>/pmc_traffic.json [profiles/r06/<dir>]
The tree must be clean at HEAD (the counters were taken on HEAD's sources): the script refuses a dirty
tree of kernel sources, so the recorded commit is the one the counters describe."""
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(src: str, profiles: str = "") -> None:
    from pysignalduino_amd import build as B
    dirty = subprocess.run(["git", "status", "--porcelain", "--", "pysignalduino_amd/csrc", "include"], cwd=REPO,
                           capture_output=True, text=True, check=True).stdout.strip()
    if dirty:
        raise SystemExit(f"kernel sources differ from HEAD; commit first:\n{dirty}")
    head = subprocess.run(["git", "rev-parse", "HEAD"], cwd=REPO, capture_output=True, text=True, check=True).stdout.strip()
    with open(src) as fh:
        tj = json.load(fh)
    tj["_source"] = {"commit": head, "sdx_source_hash": B.source_hash(),
                     "profiles": profiles or None,
                     "note": "counters from tools/pmc.sh (separate rocprofv3 --pmc passes) over the command in "
                             "_config, on the sources of this commit"}
    with open(os.path.join(REPO, "PMC_TRAFFIC.json"), "w") as fh:
        json.dump(tj, fh, indent=1)
    if profiles:
        os.makedirs(os.path.join(REPO, profiles), exist_ok=True)
        shutil.copy(os.path.join(REPO, "PMC_TRAFFIC.json"), os.path.join(REPO, profiles, "pmc_traffic.json"))
    print(f"PMC_TRAFFIC.json <- {src} (commit {head[:12]}, source hash {tj['_source']['sdx_source_hash']})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
