"""Experiment: the bench step's MU / MS / MC launches in sequence vs on three streams."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pysignalduino_amd import bank as bankmod, runtime, synth


def main():
    bk = bankmod.Bank()
    P = bk.protocols
    eng = runtime.Engine(bk, 0)
    n3 = 333333
    mu, ms, mc = synth.mu_corpus(P, n3, seed=42), synth.ms_corpus(P, n3, seed=43), synth.mc_corpus(P, n3 + 1, seed=44)
    bmu, bms, bmc = eng.to_device_pulses(mu), eng.to_device_pulses(ms), eng.to_device_mc(mc)
    outs = {"MU": eng.alloc_out(mu.n, 8 * mu.n + 4096, 200 * mu.n + 65536),
            "MS": eng.alloc_out(ms.n, 4 * ms.n + 4096, 64 * ms.n + 65536),
            "MC": eng.alloc_out(mc.n, 4 * mc.n + 4096, 96 * mc.n + 65536)}
    streams = {k: torch.cuda.Stream() for k in outs}
    main_s = torch.cuda.current_stream()

    def launch(k):
        if k == "MC":
            eng.launch_mc(bmc, outs[k])
        else:
            eng.launch_pulses(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bmu if k == "MU" else bms, outs[k])

    def seq(order=("MU", "MS", "MC")):
        for k in outs:
            outs[k]["cursor"].zero_()
        for k in order:
            launch(k)

    def par(order=("MU", "MS", "MC")):
        for k in outs:
            outs[k]["cursor"].zero_()
        ev = torch.cuda.Event()
        ev.record(main_s)
        for k in order:
            s = streams[k]
            s.wait_event(ev)
            with torch.cuda.stream(s):
                launch(k)
        for k in order:
            e = torch.cuda.Event()
            e.record(streams[k])
            main_s.wait_event(e)

    for name, fn in (("seq", seq), ("par", par), ("par MS,MC,MU", lambda: par(("MS", "MC", "MU"))),
                     ("seq", seq), ("par", par)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 10
        print(f"{name:14s} {dt*1e3:.3f} ms/step  {1e6/dt/1e6:.1f}M msgs/s", flush=True)


if __name__ == "__main__":
    main()
