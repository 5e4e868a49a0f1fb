"""Kernel time of k_pulses<MU> / <MS> for the library named by SDX_LIB (variant timing).
usage: SDX_LIB=path/to/libsdx_variant.so python tools/time_mu.py [n] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pysignalduino_amd import bank as bankmod, runtime, synth


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 333333
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    runtime.load_library()
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    res = []
    # SDX_CORPUS: bench (default) | dense (no noise messages) | zipf (templates drawn with Zipf
    # weights, skew 1.2: a capture dominated by a few protocols) -- the A/B corpora of the
    # profile-guided processing order (bank.py MU_COST_KCYC / MS_COST_KCYC)
    corpus = os.environ.get("SDX_CORPUS", "bench")
    kw = {"dense": {"noise_frac": 0.0}, "zipf": {"skew": 1.2}}.get(corpus, {})
    # SDX_KINDS: the kinds to time (default MU,MS,MC; MC times k_mc's short + long launches)
    kinds = os.environ.get("SDX_KINDS", "MU,MS,MC").split(",")
    gens = {"MU": synth.mu_corpus, "MS": synth.ms_corpus, "MC": synth.mc_corpus}
    for kind in kinds:
        if kind == "MC":
            pb = synth.mc_corpus(bk.protocols, n, seed=44)
            bd = eng.to_device_mc(pb)
            out = eng.alloc_out(pb.n, 4 * pb.n + 4096, 96 * pb.n + 65536, 0, wire=bool(os.environ.get("SDX_WIRE")))
        else:
            pb = gens[kind](bk.protocols, n, seed=42, **kw)
            bd = eng.to_device_pulses(pb)
            out = eng.alloc_out(pb.n, 12 * pb.n + 4096, 320 * pb.n + 65536, eng.pulses_work_bytes(pb.n),
                                wire=bool(os.environ.get("SDX_WIRE")))
        k = runtime.KIND_MU if kind == "MU" else runtime.KIND_MS

        def launch():
            if kind == "MC":
                eng.launch_mc(bd, out)
            else:
                eng.launch_pulses(k, bd, out, group=not os.environ.get("SDX_NOGROUP"))
        launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(reps):
            out["cursor"].zero_()
            e0.record()
            launch()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        cur = out["cursor"].cpu().numpy()
        extra = ""
        if kind != "MC" and not os.environ.get("SDX_NOGROUP"):
            # the kernel alone, on the grouped order computed beforehand (the bench groups one step
            # ahead on a side stream)
            sel = eng.group(k, bd).clone()
            torch.cuda.synchronize()
            tk = []
            for _ in range(reps):
                out["cursor"].zero_()
                e0.record()
                eng.launch_pulses(k, bd, out, sel=sel, group=False)
                e1.record()
                torch.cuda.synchronize()
                tk.append(e0.elapsed_time(e1))
            extra = f", kernel alone {min(tk):.3f} ms"
        res.append(f"{kind} {min(ts):.3f} ms (ovf {int(cur[2])}, spill {int(cur[3]) * 112 >> 10} MB{extra})")
    tag = os.path.basename(os.environ.get("SDX_LIB", "libsdx.so")) + (" plain" if os.environ.get("SDX_NOGROUP") else " grouped") + (" order=" + os.environ.get("SDX_MU_ORDER", "lpt")) + " corpus=" + corpus + (" wire" if os.environ.get("SDX_WIRE") else "")
    print(tag, " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
