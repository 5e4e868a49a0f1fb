"""Kernel time of the general path (sdx_demod_pulses_general) on the general goldens' MU / MS
messages (multi-digit ids, 4097..25000 pulses), and beside it the CPU oracle (oracle/sd_oracle.py, one
core, the Python restatement: the C oracle has no multi-character pattern ids) on the first
--cpu messages of each kind.  usage: python tools/time_general.py [--cpu N]"""
import gzip
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pysignalduino_amd import packing, runtime
from pysignalduino_amd.sd_protocols import SDProtocols


def main():
    g = json.load(gzip.open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                         "general_golden.json.gz"), "rt"))
    ncpu = int(sys.argv[sys.argv.index("--cpu") + 1]) if "--cpu" in sys.argv else 0
    p = SDProtocols()
    eng = p._ensure()
    for kind in ("MU", "MS"):
        gp = packing.GeneralPacker(kind)
        for c in g[kind.lower()]:
            try:
                gp.add(c["msg"])
            except Exception:
                pass
        arr = gp.arrays()
        gd = eng.to_device_general(arr)
        kd = runtime.KIND_MU if kind == "MU" else runtime.KIND_MS
        eng.run_general(kd, gd)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            eng.run_general(kd, gd)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 3
        n = gd["n"]
        print(f"{kind}: {n} messages, {int(arr['offsets'][-1])} pulses, {dt * 1e3:.1f} ms per run_general "
              f"(incl. read-back) -> {n / dt:.0f} msgs/s", flush=True)
        if ncpu:
            from oracle import sd_oracle as O   # the checker, timed as the CPU baseline only
            ob = O.OracleBank()
            msgs = [c["msg"] for c in g[kind.lower()]][:ncpu]
            t = time.perf_counter()
            for m in msgs:
                try:
                    O.demod(ob, dict(m), kind)
                except Exception:
                    pass
            dc = time.perf_counter() - t
            print(f"  CPU oracle (Python, 1 core): {len(msgs)} messages in {dc:.2f} s -> {len(msgs) / dc:.1f} msgs/s",
                  flush=True)


if __name__ == "__main__":
    main()
