"""Workgroup timeline of k_pulses<MU>/<MS> from the SDX_WGTIME diagnostic build: per-tile start / end
stamps -> tile durations, average concurrency and the tail (time at < 90 % of peak concurrency).
usage: SDX_LIB=pysignalduino_amd/_lib/ab/libsdx_wgt.so python tools/wg_timeline.py [n]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pysignalduino_amd import bank as bankmod, runtime, synth


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 333333
    lib = runtime.load_library()
    lib.sdx_wgtime_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    for kind, gen in (("MU", synth.mu_corpus), ("MS", synth.ms_corpus)):
        pb = gen(bk.protocols, n, seed=42)
        bd = eng.to_device_pulses(pb)
        out = eng.alloc_out(pb.n, 12 * pb.n + 4096, 320 * pb.n + 65536, eng.pulses_work_bytes(pb.n))
        k = runtime.KIND_MU if kind == "MU" else runtime.KIND_MS
        for _ in range(3):
            out["cursor"].zero_()
            eng.launch_pulses(k, bd, out)
        torch.cuda.synchronize()
        nt = (pb.n + 63) // 64
        buf = (ctypes.c_ulonglong * (2 * nt))()
        assert lib.sdx_wgtime_read(buf, nt) == 0
        t = np.array(list(buf), dtype=np.float64).reshape(nt, 2) * 10.0  # 100 MHz ticks -> ns
        t -= t[:, 0].min()
        dur = t[:, 1] - t[:, 0]
        span = t[:, 1].max()
        ev = np.concatenate([np.stack([t[:, 0], np.ones(nt)], 1), np.stack([t[:, 1], -np.ones(nt)], 1)])
        ev = ev[np.argsort(ev[:, 0], kind="stable")]
        conc = np.cumsum(ev[:, 1])
        dt = np.diff(ev[:, 0], append=span)
        peak = conc.max()
        low = dt[conc < 0.9 * peak].sum()
        first_end = t[:, 1].min()
        last_start = t[:, 0].max()
        q = np.percentile(dur, [0, 10, 50, 90, 100]) / 1e3
        print(f"== {kind}: {nt} tiles, span {span/1e3:.1f} us, peak concurrency {peak:.0f}, "
              f"mean {dur.sum()/span:.1f}; ideal (sum dur / peak) {dur.sum()/peak/1e3:.1f} us; "
              f"time below 90% of peak {low/1e3:.1f} us; last start at {last_start/1e3:.1f} us", flush=True)
        print(f"   tile duration us: min {q[0]:.1f} p10 {q[1]:.1f} p50 {q[2]:.1f} p90 {q[3]:.1f} max {q[4]:.1f}; "
              f"first tile ends at {first_end/1e3:.1f} us", flush=True)
        # duration vs start order: do late tiles run faster (less contention)?
        order = np.argsort(t[:, 0])
        for a, b in ((0, 512), (512, 1024), (nt // 2, nt // 2 + 512), (nt - 512, nt)):
            print(f"   tiles started #{a}-{b}: mean duration {dur[order[a:b]].mean()/1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
