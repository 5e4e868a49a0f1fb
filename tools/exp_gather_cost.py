"""Experiment: the cost of the grouped order's gathers.  Times k_pulses (MU, MS) on the grouped
order through sel_dev (the product form) against the same messages physically permuted into that
order (sel_dev = NULL, contiguous per-message fields) -- identical work, different memory access.
usage: python tools/exp_gather_cost.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pysignalduino_amd import bank as bankmod, runtime, synth


def main():
    K = 10
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    P = bk.protocols
    n = 333333
    for kind, gen, seed in (("MU", synth.mu_corpus, 42), ("MS", synth.ms_corpus, 43)):
        kd = runtime.KIND_MU if kind == "MU" else runtime.KIND_MS
        pb = gen(P, n, seed=seed)
        bd = eng.to_device_pulses(pb)
        order = eng.group(kd, bd).clone()
        pbp = pb.subset(order.cpu().numpy())
        bdp = eng.to_device_pulses(pbp)
        out = eng.alloc_out(n, 12 * n + 4096, 320 * n + 65536, eng.pulses_work_bytes(n))
        res = {}
        for name, b_, sel in (("sel", bd, order), ("permuted", bdp, None), ("sel", bd, order), ("permuted", bdp, None)):
            ts = []
            for _ in range(K):
                out["cursor"].zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                eng.launch_pulses(kd, b_, out, sel=sel, group=False)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res.setdefault(name, []).append(sorted(ts)[K // 2])
        print(kind, {k: [round(x, 4) for x in v] for k, v in res.items()}, "ms (median of", K, ")", flush=True)


if __name__ == "__main__":
    main()
