"""The per-step grouping alone (nothing beside it): sdx_group_pulses of the bench step's MU and MS
batches (333k messages each), timed with HIP events; run under rocprofv3 --kernel-trace --stats for
its kernels' uncontended durations.  usage: python tools/time_group.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pysignalduino_amd import bank as bankmod, runtime, synth


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    P = bk.protocols
    n = 333333
    bds = {"MU": eng.to_device_pulses(synth.mu_corpus(P, n, seed=42)),
           "MS": eng.to_device_pulses(synth.ms_corpus(P, n, seed=43))}
    gb = {k: eng.group_buffers(n) for k in bds}
    kd = {"MU": runtime.KIND_MU, "MS": runtime.KIND_MS}
    for _ in range(3):
        for k in bds:
            eng.group(kd[k], bds[k], bufs=gb[k])
    torch.cuda.synchronize()
    ts = {k: [] for k in ("MU", "MS", "both")}
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        eng.group(kd["MU"], bds["MU"], bufs=gb["MU"])
        ev[1].record()
        eng.group(kd["MS"], bds["MS"], bufs=gb["MS"])
        ev[2].record()
        torch.cuda.synchronize()
        ts["MU"].append(ev[0].elapsed_time(ev[1]))
        ts["MS"].append(ev[1].elapsed_time(ev[2]))
        ts["both"].append(ev[0].elapsed_time(ev[2]))
    print("grouping alone (ms, median): " + ", ".join(f"{k} {np.median(v):.4f}" for k, v in ts.items()), flush=True)


if __name__ == "__main__":
    main()
