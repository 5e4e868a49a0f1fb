"""Which engine runs a device -> pinned-host copy, and at what rate: the streaming front end's result
copy (11 MB per 250k-line chunk) ran as a 256-workgroup blit kernel (__amd_rocclr_copyBuffer) that
held a slot on every CU beside the demodulation tiles.  This times hipMemcpyAsync D2H (and H2D) into
host buffers allocated in different ways; run it under rocprofv3 --kernel-trace to see which of them
become kernels.  usage: python tools/d2h_engine_probe.py [MB]"""
import ctypes
import sys
import time

import torch

HIP = ctypes.CDLL("libamdhip64.so")
HIP.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
HIP.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
HIP.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
FLAGS = {"default": 0x0, "portable": 0x1, "mapped": 0x2, "coherent": 0x40000000, "noncoherent": 0x80000000,
         "numa_user": 0x20000000}


def host_malloc(n, flags):
    p = ctypes.c_void_p()
    rc = HIP.hipHostMalloc(ctypes.byref(p), n, flags)
    return p.value if rc == 0 else None


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 11.0
    n = int(mb * 1e6) & ~15
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev.fill_(7)
    s = torch.cuda.current_stream()
    bufs = {"torch_pinned": torch.empty(n, dtype=torch.uint8).pin_memory().data_ptr()}
    for k, f in FLAGS.items():
        p = host_malloc(n, f)
        if p:
            bufs[f"hostmalloc_{k}"] = p
    reg = (ctypes.c_uint8 * (n + 4096))()
    base = (ctypes.addressof(reg) + 4095) & ~4095
    if HIP.hipHostRegister(ctypes.c_void_p(base), n, 0) == 0:
        bufs["registered"] = base
    torch.cuda.synchronize()
    tp = torch.empty(n, dtype=torch.uint8).pin_memory()
    streams = {"null": torch.cuda.default_stream(), "created": torch.cuda.Stream()}
    for sname, s in streams.items():
        for name, hp in list(bufs.items()) + [("torch_copy_", None)]:
            if sname == "null" and name not in ("torch_pinned", "torch_copy_"):
                continue
            for kind, label in ((2, "D2H"), (1, "H2D")):
                ts = []
                for _ in range(4):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    rc = 0
                    if hp is None:
                        with torch.cuda.stream(s):
                            (tp.copy_(dev, non_blocking=True) if kind == 2 else dev.copy_(tp, non_blocking=True))
                    elif kind == 2:
                        rc = HIP.hipMemcpyAsync(ctypes.c_void_p(hp), ctypes.c_void_p(dev.data_ptr()), n, 2, ctypes.c_void_p(s.cuda_stream))
                    else:
                        rc = HIP.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(hp), n, 1, ctypes.c_void_p(s.cuda_stream))
                    e1.record(s)
                    torch.cuda.synchronize()
                    assert rc == 0, rc
                    ts.append(e0.elapsed_time(e1))
                t = sorted(ts)[len(ts) // 2]
                print(f"{sname:8s} {name:24s} {label}: {t * 1e3:8.1f} us  {n / (t * 1e-3) / 1e9:6.1f} GB/s", flush=True)
                torch.cuda.synchronize()
                time.sleep(0.01)   # separates the cases in the kernel trace

if __name__ == "__main__":
    main()
