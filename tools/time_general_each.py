"""Per-message time of the general MU path on the general goldens (which messages are slow)."""
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
    p = SDProtocols()
    eng = p._ensure()
    rows = []
    for k, c in enumerate(g["mu"][:80]):
        gp = packing.GeneralPacker("MU")
        try:
            gp.add(c["msg"])
        except Exception:
            continue
        gd = eng.to_device_general(gp.arrays())
        torch.cuda.synchronize()
        t = time.perf_counter()
        eng.run_general(runtime.KIND_MU, gd)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        m = c["msg"]
        ids = [key for key in m if key.startswith("P")]
        rows.append((dt, k, len(m["data"]), len(ids), len(c["exp"].get("results", []))))
        print(f"{k}: {dt * 1e3:.1f} ms, {len(m['data'])} pulses, {len(ids)} patterns {ids}, "
              f"{len(c['exp'].get('results', []))} results", flush=True)
    rows.sort(reverse=True)
    print("slowest:", rows[:5])


if __name__ == "__main__":
    main()
