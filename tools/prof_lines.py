"""Phase breakdown of k_parse_comp from the SDX_LPROF build (s_memtime cycles per wave: for each
phase the max over the wave's lanes, summed over waves).
usage: SDX_LIB=pysignalduino_amd/_lib/ab/libsdx_lprof.so python tools/prof_lines.py [lines]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pysignalduino_amd import bank as bankmod, frontend, runtime, synth

NAMES = {0: "wave total (scan + parse)", 1: "strip + frame_check", 2: "decompress into the slot",
         3: "fast_payload (slot read back)", 4: "parse_payload (fast path declined)", 5: "finish_fields",
         6: "status stores (global) / payload copy-out (LDS)", 7: "LDS staging of the raw lines", 8: "#lines through parse_payload", 9: "#compressed lines"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    torch.cuda.set_device(0)
    bk = bankmod.Bank()
    eng = runtime.Engine(bk, 0)
    lib = eng.lib
    lib.sdx_lprof_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    lines, _ = synth.line_corpus(bk.protocols, n, seed=45, mix=(1, 1, 1), compress_frac=0.3)
    data, offsets, bad = frontend.pack_lines(lines)
    assert not bad
    lb = frontend.LineBatch(eng, data, offsets)
    buf = (ctypes.c_ulonglong * 16)()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for it in range(4):
        lib.sdx_lprof_read(buf, 1)
        ev[0].record()
        runtime._check(lib, lib.sdx_parse_lines(ctypes.byref(lb.c_lines), ctypes.byref(lb.c_out), eng.stream_ptr()))
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    lib.sdx_lprof_read(buf, 1)
    v = np.array(list(buf), dtype=np.float64)
    tot = v[0]
    print(f"parse (k_parse_lines + k_parse_comp) {min(ts):.3f} ms; {int(v[9])} compressed lines, "
          f"{int(v[8])} through parse_payload")
    for k in range(8):
        if v[k]:
            print(f"  {NAMES.get(k, str(k)):36s} {100 * v[k] / tot:6.2f} %  {v[k] / max(v[9], 1):10.0f} cycles/line")
    tl = v[15]
    print(f"k_parse_lines (per wave: max over its lanes; {n} lines):")
    for k, name in ((10, "strip + header checks"), (11, "fast_payload"), (12, "frame_check + parse_payload (declined)"),
                    (13, "finish_fields"), (14, "D copy by the wave"), (15, "wave total")):
        print(f"  {name:40s} {100 * v[k] / max(tl, 1):6.2f} %  {v[k] / (n / 64):10.0f} cycles/wave")
    # the status array: how many lines the parse marked compressed (decompressed payload length > 0)
    plen = lb.c_out  # noqa: F841 (kept for reference; the counts above are the kernel's own)


if __name__ == "__main__":
    main()
