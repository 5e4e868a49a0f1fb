"""Phase breakdown of k_pulses from the SDX_PROF build (s_memtime cycle counters per wave).
usage: SDX_LIB=pysignalduino_amd/_lib/libsdx_prof.so python tools/prof_phases.py [n]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pysignalduino_amd import bank as bankmod, runtime, synth

NAMES = {0: "stage bitmaps", 1: "MU normalise", 2: "MU pexists(start)", 3: "MU pexists(one/zero/float)",
         4: "MU decode setup", 5: "MU finditer scan", 6: "MU chunk->bits", 7: "MU postDemod",
         8: "MU payload write", 9: "MU format+DFA", 10: "MS decode", 11: "MS finish", 12: "MU decode total",
         13: "flush", 14: "end barrier wait", 15: "kernel total", 16: "MU finish phase (lane = match)",
         17: "  stage: headers + pattern tables", 18: "  stage: id bitmaps", 19: "  stage: pairs + lengths", 20: "#results(MU)", 21: "#survivors(MU)",
         22: "#matches(MU)", 23: "#survivors(MS)", 24: "  finish: tables + sort (to the loop)",
         25: "  finish: match loop", 26: "  finish: end barrier"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 333333
    lib = runtime.load_library()
    lib.sdx_prof_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    lib.sdx_gprof_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    buf = (ctypes.c_ulonglong * 32)()
    for kind, gen in (("MU", synth.mu_corpus), ("MS", synth.ms_corpus)):
        pb = gen(bk.protocols, n, seed=42)
        bd = eng.to_device_pulses(pb)
        out = eng.alloc_out(pb.n, 12 * pb.n + 4096, 320 * pb.n + 65536, eng.pulses_work_bytes(pb.n))
        k = runtime.KIND_MU if kind == "MU" else runtime.KIND_MS
        eng.launch_pulses(k, bd, out)
        torch.cuda.synchronize()
        lib.sdx_prof_read(buf, 1)
        lib.sdx_gprof_read((ctypes.c_ulonglong * 256)(), 1)
        out["cursor"].zero_()
        t = time.perf_counter()
        eng.launch_pulses(k, bd, out)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        lib.sdx_prof_read(buf, 1)
        v = np.array(list(buf), dtype=np.float64)
        gb = (ctypes.c_ulonglong * 256)()
        lib.sdx_gprof_read(gb, 1)
        tot = v[15]
        print(f"== {kind}: {pb.n} msgs, {dt*1e3:.2f} ms wall; wave-cycles total {tot:.3e} "
              f"({tot/pb.n:.0f} per message)")
        for i in sorted(NAMES):
            if v[i] == 0:
                continue
            if 20 <= i < 24:
                print(f"  {NAMES[i]:28s} {v[i]:.0f}  ({v[i]/pb.n:.2f} per message)")
            else:
                print(f"  {NAMES[i]:28s} {v[i]/tot*100:6.2f} %   {v[i]/pb.n:9.0f} wave-cycles/msg")
        g = np.array(list(gb), dtype=np.float64).reshape(2, 128)
        unit = "clock group" if kind == "MU" else "protocol"
        order = np.argsort(-g[0])
        print(f"  per {unit} (processing order index: share of the work-loop cycles, cycles per grab):")
        tot_g = g[0].sum()
        print("   " + " ".join(f"{int(i)}:{g[0, i] / tot_g * 100:.1f}%/{g[0, i] / max(g[1, i], 1):.0f}"
                              for i in order if g[1, i] > 0))
    # k_mc (slots 27-31)
    pb = synth.mc_corpus(bk.protocols, n, seed=44)
    bd = eng.to_device_mc(pb)
    out = eng.alloc_out(pb.n, 4 * pb.n + 4096, 96 * pb.n + 65536, 0)
    for it in range(2):
        out["cursor"].zero_()
        lib.sdx_prof_read(buf, 1)
        lib.sdx_gprof_read((ctypes.c_ulonglong * 256)(), 1)
        t = time.perf_counter()
        eng.launch_mc(bd, out)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    lib.sdx_prof_read(buf, 1)
    v = np.array(list(buf), dtype=np.float64)
    gb = (ctypes.c_ulonglong * 256)()
    lib.sdx_gprof_read(gb, 1)
    g = np.array(list(gb), dtype=np.float64).reshape(2, 128)
    tot = v[31]
    print(f"== MC: {pb.n} frames, {dt*1e3:.2f} ms wall; wave-cycles total {tot:.3e} ({tot/pb.n:.0f} per frame)")
    for i, name in ((27, "stage (hex -> bits)"), (28, "protocol gates + method"), (29, "result staging"),
                    (30, "flush"), (31, "kernel total")):
        print(f"  {name:28s} {v[i]/tot*100:6.2f} %   {v[i]/pb.n:9.0f} wave-cycles/frame")
    print("  per protocol (bank MC index: share of the gates + method cycles, lanes through the gates per frame):")
    print("   " + " ".join(f"{i}:{g[0, i] / max(v[28], 1) * 100:.1f}%/{g[1, i] / pb.n:.3f}"
                          for i in range(32) if g[0, i] > 0))


if __name__ == "__main__":
    main()
