"""Experiment: what the per-step grouping (sdx_group_pulses on the side stream) costs the
demodulation kernels it runs beside.  Times K steps of the three launches (a) with the grouping
of every step on a side stream (bench.py's form) and (b) with the grouped order computed once
before timing (NOT a valid bench: grouping is part of the hot path).  usage: python tools/exp_group_cost.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pysignalduino_amd import bank as bankmod, runtime, synth


def main():
    K = 20
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    P = bk.protocols
    n = 333333
    corp = {"MU": synth.mu_corpus(P, n, seed=42), "MS": synth.ms_corpus(P, n, seed=43), "MC": synth.mc_corpus(P, n + 1, seed=44)}
    bds = {k: (eng.to_device_mc(c) if k == "MC" else eng.to_device_pulses(c)) for k, c in corp.items()}
    caps = {"MU": (12, 320), "MS": (4, 64), "MC": (4, 96)}
    outs = {k: eng.alloc_out(c.n, caps[k][0] * c.n + 4096, caps[k][1] * c.n + 65536,
                             eng.pulses_work_bytes(c.n) if k != "MC" else 0) for k, c in corp.items()}
    gb = {k: eng.group_buffers(corp[k].n) for k in ("MU", "MS")}
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    prio = os.environ.get("PRIO") == "1"
    side = torch.cuda.Stream(priority=lo) if prio else torch.cuda.Stream()
    main_s = torch.cuda.Stream(priority=hi) if prio else torch.cuda.current_stream()
    torch.cuda.set_stream(main_s)
    print("priorities", torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else None,
          "prio" if prio else "default", flush=True)

    def launches():
        for k in ("MU", "MS", "MC"):
            outs[k]["cursor"].zero_()
            if k == "MC":
                eng.launch_mc(bds[k], outs[k])
            else:
                eng.launch_pulses(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bds[k], outs[k],
                                  sel=gb[k][0][:corp[k].n], group=False)

    def group_side():
        with torch.cuda.stream(side):
            for k in ("MU", "MS"):
                eng.group(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bds[k], bufs=gb[k])

    for mode in ("side", "once", "side", "once"):
        group_side()
        torch.cuda.synchronize()
        launches()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            if mode == "side":   # the same buffers: an order race is harmless for timing only
                ev = torch.cuda.Event()
                ev.record(main_s)
                side.wait_event(ev)
                group_side()
            launches()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        print(f"{mode}: {dt * 1e3:.3f} ms/step, {3 * n / dt / 1e6:.1f}M msgs/s", flush=True)
    # the grouping alone
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        for k in ("MU", "MS"):
            eng.group(runtime.KIND_MU if k == "MU" else runtime.KIND_MS, bds[k], bufs=gb[k])
    torch.cuda.synchronize()
    print(f"grouping alone (MU + MS): {(time.perf_counter() - t0) / K * 1e3:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
