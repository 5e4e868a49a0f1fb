"""Each kind's tiles inside k_step (sdx_demod_step with one kind only) against its own kernel
(k_pulses<MU>, k_ms_classes, k_mc): what the fused kernel's shared register allocation and LDS union cost
each body.  Bench corpus (333k messages per kind, grouped order).  usage: python tools/time_step_parts.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pysignalduino_amd import bank as bankmod, runtime, synth


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    eng.use_mrec = set()
    P = bk.protocols
    n = 333333
    bds = {"MU": eng.to_device_pulses(synth.mu_corpus(P, n, seed=42)),
           "MS": eng.to_device_pulses(synth.ms_corpus(P, n, seed=43)),
           "MC": eng.to_device_mc(synth.mc_corpus(P, n + 1, seed=44))}
    caps = {"MU": (12, 320), "MS": (4, 64), "MC": (4, 96)}
    outs = {k: eng.alloc_out(bds[k]["n"], caps[k][0] * bds[k]["n"] + 4096, caps[k][1] * bds[k]["n"] + 65536,
                             eng.pulses_work_bytes(bds[k]["n"]) if k != "MC" else 0) for k in caps}
    order = {}
    for k, kd in (("MU", runtime.KIND_MU), ("MS", runtime.KIND_MS)):
        g = eng.group_buffers(n)
        order[k] = eng.group(kd, bds[k], bufs=g)
    torch.cuda.synchronize()

    def alone(k):
        if k == "MC":
            eng.launch_mc(bds[k], outs[k])
        else:
            eng.launch_pulses(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bds[k], outs[k], sel=order[k],
                              group=False)

    def fused(k):
        if k == "MC":
            eng.launch_step(mc=(bds[k], outs[k], None))
        else:
            eng.launch_step(**{k.lower(): (bds[k], outs[k], order[k], None)})

    res = {}
    for k in ("MU", "MS", "MC"):
        for name, fn in (("alone", alone), ("k_step", fused)):
            ts = []
            for r in range(reps + 2):
                outs[k]["cursor"].zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn(k)
                e1.record()
                torch.cuda.synchronize()
                if r >= 2:
                    ts.append(e0.elapsed_time(e1))
            res[(k, name)] = float(np.median(ts))
    print(" | ".join(f"{k}: alone {res[(k, 'alone')]:.4f} ms, in k_step {res[(k, 'k_step')]:.4f} ms"
                     for k in ("MU", "MS", "MC")), flush=True)


if __name__ == "__main__":
    main()
