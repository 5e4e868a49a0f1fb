"""Where the general MU path's time goes (SDX_GPROF variant of sdx_general.hip): cycles per phase
summed over items, and the slowest (message, protocol) items of pass 0.
usage: python tools/build_variant.py gprof --unit sdx_general.hip -DSDX_GPROF
       SDX_LIB=pysignalduino_amd/_lib/ab/libsdx_gprof.so python tools/prof_general.py"""
import ctypes
import gzip
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from pysignalduino_amd import packing, runtime
from pysignalduino_amd.sd_protocols import SDProtocols

PH = {0: "pattern_exists (start + keys)", 1: "finditer: next start / unit", 2: "rep_match", 3: "chunks -> bits",
      4: "finish (postDemod, hex, DFA, emit)", 5: "stage message", 6: "items pass 0", 7: "items pass 1",
      11: "match tables", 8: "#protocols past the key lookups", 9: "#rep_match calls", 10: "#matches",
      12: "#rep_match fallbacks (ambiguous units)"}


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = json.load(gzip.open(os.path.join(root, "tests", "golden", "general_golden.json.gz"), "rt"))
    p = SDProtocols()
    eng = p._ensure()
    lib = eng.lib
    lib.sdx_genprof_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    gp = packing.GeneralPacker("MU")
    msgs = []
    for c in g["mu"]:
        try:
            gp.add(c["msg"])
            msgs.append(c["msg"])
        except Exception:
            pass
    arr = gp.arrays()
    gd = eng.to_device_general(arr)
    kd = runtime.KIND_MU
    n = gd["n"]
    lens = np.asarray(gd["lengths"])
    max_len = int(lens.max(initial=0))
    wb = int(lib.sdx_general_work_bytes(eng.handle, kd, int(gd["total"]), n, max_len, 0))
    work = torch.empty(wb, dtype=torch.uint8, device=eng.dev)
    order = np.argsort(-lens, kind="stable").astype(np.int32)
    sel = torch.from_numpy(order).to(eng.dev)
    buf = (ctypes.c_ulonglong * 16)()
    for rep in range(2):
        out = eng.alloc_out(n, 16 * n + 1024, int(2 * gd["total"] + 256 * n + 65536))
        o = eng._out_struct(out)
        o.work_dev, o.work_cap = work.data_ptr(), int(work.numel())
        b = runtime.SdxGeneralBatch(gd["data"].data_ptr(), gd["offsets"].data_ptr(), gd["npat"].data_ptr(),
                                    gd["pat_ids"].data_ptr(), gd["pat_val"].data_ptr(), gd["cp_slot"].data_ptr(),
                                    gd["ms_ok"].data_ptr(), sel.data_ptr(), n, n, 0, 0, max_len, 0)
        lib.sdx_genprof_read(buf, 1)
        torch.cuda.synchronize()
        t = time.perf_counter()
        assert lib.sdx_demod_pulses_general(eng.handle, kd, ctypes.byref(b), ctypes.byref(o), eng.stream_ptr()) == 0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    lib.sdx_genprof_read(buf, 1)
    v = np.array(list(buf), dtype=np.float64)
    print(f"MU general: {n} messages, {int(lens.sum())} pulses, {dt * 1e3:.1f} ms (one launch sequence)")
    tot = v[6] + v[7]
    for k, name in PH.items():
        if k in (8, 9, 10, 12):
            print(f"  {name:40s} {int(v[k])}")
        else:
            print(f"  {name:40s} {v[k]:.3e} cycles  {100 * v[k] / tot:5.1f} %")
    nprot = len(p._bank.mu_pids)
    raw = work[256:256 + n * nprot * 24].cpu().numpy().view(np.uint32).reshape(n, nprot, 6)
    cyc = raw[:, :, 5].astype(np.float64)
    print(f"  pass-0 item cycles: sum {cyc.sum():.3e}, max {cyc.max():.3e}, "
          f"items > 1e7: {(cyc > 1e7).sum()}, > 1e8: {(cyc > 1e8).sum()}")
    flat = np.argsort(-cyc, axis=None)[:15]
    for f in flat:
        i, pr = divmod(int(f), nprot)
        msg = int(order[i])
        m = msgs[msg]
        ids = [k for k in m if k.startswith("P")]
        print(f"   item (msg {msg}, proto idx {pr}): {cyc[i, pr]:.3e} cycles, {lens[msg]} pulses, "
              f"{len(ids)} patterns, nrec {raw[i, pr, 0]}, raise {raw[i, pr, 4] >> 16}")
    per_msg = cyc.sum(axis=1)
    print(f"  per message: max {per_msg.max():.3e}, mean {per_msg.mean():.3e} cycles")
    per_proto = cyc.sum(axis=0)
    top = np.argsort(-per_proto)[:10]
    print("  per protocol idx (share of pass-0 cycles):",
          " ".join(f"{int(t)}:{100 * per_proto[t] / cyc.sum():.1f}%" for t in top))


if __name__ == "__main__":
    main()
