"""ctypes front end of the plain-C oracle (oracle/sd_oracle_c.c).

*** TEST INFRASTRUCTURE ONLY ***
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use
this module, as the CHECKER or the timed CPU baseline.  The product path never imports it.

The bank handed to C is interpreted here from protocols.json exactly as the reference interprets
each property at its use site (float()/int()/truthiness, sd_protocols/*.py), independently of
the product's bank compiler (pysignalduino_amd/bank.py).  Messages are packed from the reference's
``msg_data`` dicts with the reference's own string operations (message_unsynced.py:28-35,
message_synced.py:21-57).  Inputs outside the C restatement's domain (multi-character pattern
ids, exotic hex literals, unconvertible bank values) raise NotImplementedError.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import sd_oracle as PO

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libsdoracle.so")
SRC = os.path.join(HERE, "sd_oracle_c.c")

MAXS, MAXPAT = 16, 10
PD = ["postDemo_EM", "postDemo_Revolt", "postDemo_FS20", "postDemo_FHT80", "postDemo_FHT80TF",
      "postDemo_WS2000", "postDemo_WS7035", "postDemo_WS7053", "postDemo_lengtnPrefix"]
MC = {"mcBit2Funkbus": 1, "mcBit2Sainlogic": 2, "mcBit2AS": 3, "mcBit2Hideki": 4, "mcBit2Maverick": 4,
      "mcBit2OSV1": 4, "mcBit2OSV2o3": 4, "mcBit2OSPIR": 4, "mcRaw": 5, "mcraw": 6, "mcBit2TFA": 7,
      "mcBit2Grothe": 8, "mcBit2SomfyRTS": 9}
RAISE = {1: IndexError, 2: AttributeError, 3: ValueError, 4: TypeError}


class SoList(C.Structure):
    _fields_ = [("n", C.c_int), ("v", C.c_double * MAXS)]


class SoProto(C.Structure):
    _fields_ = [("mu", C.c_int), ("ms", C.c_int), ("mc", C.c_int), ("active", C.c_int),
                ("mu_clock", C.c_double), ("ms_pclock", C.c_double), ("start_list", C.c_int),
                ("start", SoList), ("one", SoList), ("zero", SoList), ("flt", SoList), ("sync", SoList),
                ("mu_key_err", C.c_int), ("ms_key_err", C.c_int), ("width", C.c_int), ("mu_lmin", C.c_int),
                ("mu_lmax_set", C.c_int), ("mu_lmax", C.c_int), ("ms_lmin", C.c_int), ("lir_min", C.c_int),
                ("lir_max_set", C.c_int), ("lir_max", C.c_long), ("recon", C.c_int), ("pad", C.c_int),
                ("dispatch_bin", C.c_int), ("remove_zero", C.c_int), ("postdemo", C.c_int),
                ("pre", C.c_char * 64), ("pre_len", C.c_int), ("post", C.c_char * 64), ("post_len", C.c_int),
                ("mm", C.c_char * 128), ("cr_lo", C.c_double), ("cr_hi", C.c_double), ("has_cr", C.c_int),
                ("method", C.c_int), ("has_lmin", C.c_int), ("lmin_v", C.c_long), ("has_lmax", C.c_int),
                ("lmax_v", C.c_long), ("lmax_is_str", C.c_int), ("invert", C.c_int), ("pid_num", C.c_int)]


class SoPulses(C.Structure):
    _fields_ = [("data", C.c_void_p), ("offsets", C.c_void_p), ("npat", C.c_void_p), ("pat_id", C.c_void_p),
                ("pat_val", C.c_void_p), ("ms_ok", C.c_void_p), ("cp_slot", C.c_void_p), ("n", C.c_int)]


class SoMc(C.Structure):
    _fields_ = [("hex", C.c_void_p), ("offsets", C.c_void_p), ("clock", C.c_void_p), ("mcbitnum", C.c_void_p),
                ("mtype_lower", C.c_void_p), ("v32", C.c_void_p), ("n", C.c_int)]


RES_DT = np.dtype([("off", "<u4"), ("len", "<u2"), ("proto", "<u2"), ("bitlen", "<u4"), ("msg", "<u4")])


class SoOut(C.Structure):
    _fields_ = [("status", C.c_void_p), ("raise_kind", C.c_void_p), ("rec_begin", C.c_void_p),
                ("n_rec", C.c_void_p), ("rec", C.c_void_p), ("heap", C.c_void_p), ("rec_cap", C.c_uint64),
                ("heap_cap", C.c_uint64), ("rec_total", C.c_uint64), ("heap_total", C.c_uint64)]


def build(force: bool = False) -> str:
    """gcc -O2 -shared: the C restatement into oracle/_build/ (git-ignored, travels to the box)."""
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.run(["gcc", "-O2", "-std=gnu11", "-shared", "-fPIC", "-pthread", "-o", LIB, SRC, "-lm"],
                       check=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.so_bank_set.argtypes = [C.c_void_p, C.c_int]
        L.so_proto_size.restype = C.c_int
        L.so_demod.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.so_rx_supported.argtypes = [C.c_char_p]
        L.so_rx_search.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        if L.so_proto_size() != C.sizeof(SoProto):
            raise RuntimeError("so_proto layout mismatch")
        _lib = L
    return _lib


def _to_int(v, what):
    try:
        return int(v)
    except (ValueError, TypeError):
        raise NotImplementedError(f"{what}: {v!r}")


def _floats(spec):
    try:
        return [float(x) for x in spec], False
    except (ValueError, TypeError):
        return [], True


class CBank:
    """The bank as the reference reads it (sd_protocols.py:25-58,157-160 + use sites)."""

    def __init__(self, protocols: Optional[Dict[str, dict]] = None):
        ob = PO.OracleBank(protocols)
        self.pids: List[str] = list(ob.p.keys())
        arr = (SoProto * max(1, len(self.pids)))()
        for i, pid in enumerate(self.pids):
            self._fill(arr[i], pid, ob.p[pid])
        self.arr = arr
        lib().so_bank_set(C.cast(arr, C.c_void_p), len(self.pids))

    def use(self):
        lib().so_bank_set(C.cast(self.arr, C.c_void_p), len(self.pids))

    @staticmethod
    def _list(dst, vals):
        if len(vals) > MAXS:
            raise NotImplementedError("search list too long")
        dst.n = len(vals)
        for i, v in enumerate(vals):
            dst.v[i] = v

    def _fill(self, r, pid, p):
        r.mu, r.ms, r.mc = int("clockabs" in p), int("sync" in p), int("clockrange" in p)
        r.active = int(bool(p.get("active", True)))
        if r.mu:
            try:
                r.mu_clock = float(p.get("clockabs", 1))          # message_unsynced.py:59
            except (ValueError, TypeError):
                raise NotImplementedError(f"{pid}: clockabs")
            if r.mu_clock == 0:
                raise NotImplementedError(f"{pid}: clockabs 0")
        if r.ms:
            try:
                r.ms_pclock = float(p.get("clockabs", 0))         # message_synced.py:83
            except (ValueError, TypeError):
                raise NotImplementedError(f"{pid}: clockabs")
        sp = p.get("start")
        if sp and isinstance(sp, list):                           # message_unsynced.py:67
            vals, err = _floats(sp)
            if err:
                raise NotImplementedError(f"{pid}: start not numeric")
            r.start_list = 1
            self._list(r.start, vals)
        mu_err = ms_err = False
        for key, fld in (("one", "one"), ("zero", "zero"), ("float", "flt"), ("sync", "sync")):
            spec = p.get(key)
            if not spec:
                continue
            vals, err = _floats(spec)
            if err:
                if key != "sync":
                    mu_err = True
                ms_err = True
                continue
            self._list(getattr(r, fld), vals)
        r.mu_key_err, r.ms_key_err = int(mu_err), int(ms_err)
        lens = {getattr(r, f).n for f in ("one", "zero", "flt") if getattr(r, f).n}
        if r.mu and len(lens) > 1:
            raise NotImplementedError(f"{pid}: one/zero/float lengths differ")
        r.width = len(p["one"]) if p.get("one") else 0
        r.mu_lmin = _to_int(p.get("length_min", 0), f"{pid} length_min") if r.mu else 0
        lm = p.get("length_max", None)
        r.mu_lmax_set = int(bool(lm))
        r.mu_lmax = _to_int(lm, f"{pid} length_max") if lm else 0
        if r.ms:
            r.ms_lmin = _to_int(p.get("length_min", -1), f"{pid} length_min")
        lo = p.get("length_min", -1)                              # helpers.py:144-154
        r.lir_min = _to_int(lo, f"{pid} length_min")
        hi = p.get("length_max")
        r.lir_max_set = 0
        if hi is not None:
            try:
                r.lir_max = int(hi)
                r.lir_max_set = 1
            except (ValueError, TypeError):
                pass
        r.recon = int(bool(p.get("reconstructBit")))
        r.pad = _to_int(p.get("paddingbits", 4), f"{pid} paddingbits")
        if r.pad < 1:
            raise NotImplementedError(f"{pid}: paddingbits < 1")
        r.dispatch_bin = int(_to_int(p.get("dispatchBin", 0), "dispatchBin") == 1)
        r.remove_zero = int(bool(p.get("remove_zero", 0)))
        name = p.get("postDemodulation", None)
        r.postdemo = (PD.index(name.split(".")[-1]) + 1) if name and name.split(".")[-1] in PD else 0
        pre = f"{p.get('preamble', '')}".encode("utf-8")
        post = f"{p.get('postamble', '')}".encode("utf-8")
        if len(pre) > 63 or len(post) > 63:
            raise NotImplementedError(f"{pid}: long preamble/postamble")
        r.pre, r.pre_len, r.post, r.post_len = pre, len(pre), post, len(post)
        mm = p.get("modulematch") or ""
        if mm:
            if len(mm) > 127 or not lib().so_rx_supported(mm.encode()):
                raise NotImplementedError(f"{pid}: modulematch {mm!r} outside the C subset")
            r.mm = mm.encode()
        if r.mc:
            cr = p["clockrange"]
            if cr and len(cr) >= 2:
                r.has_cr, r.cr_lo, r.cr_hi = 1, float(cr[0]), float(cr[1])
            meth = str(p.get("method", "")).split(".")[-1]
            if meth not in MC:
                raise NotImplementedError(f"{pid}: method {meth}")
            r.method = MC[meth]
            if "length_min" in p:
                r.has_lmin, r.lmin_v = 1, _to_int(p["length_min"], "length_min")
            if "length_max" in p:
                r.has_lmax, r.lmax_v = 1, _to_int(p["length_max"], "length_max")
                r.lmax_is_str = int(isinstance(p["length_max"], str))
            r.invert = int(p.get("polarity", "") == "invert")
            try:
                r.pid_num = int(pid)
            except ValueError:
                r.pid_num = -1


# ---------------------------------------------------------------------------------------------
# packing (the reference's own string operations)
# ---------------------------------------------------------------------------------------------
def _data_bytes(s: str) -> bytes:
    """One byte per character (non-ASCII -> 0xFE), so that string indices are preserved."""
    return bytes(ord(c) if ord(c) < 128 else 0xFE for c in s)


def pack_pulses(msgs: Sequence[Dict[str, Any]]):
    n = len(msgs)
    datas, npat = [], np.zeros(n, np.uint8)
    pid = np.zeros((n, MAXPAT), np.uint8)
    pval = np.zeros((n, MAXPAT), np.float64)
    ms_ok, cp_slot = np.zeros(n, np.uint8), np.full(n, -1, np.int8)
    for i, m in enumerate(msgs):
        data = m.get("data", "") or ""
        datas.append(_data_bytes(data))
        pr = PO._patterns(m)                      # message_unsynced.py:28-35
        if len(pr) > MAXPAT:
            raise NotImplementedError("more than 10 patterns")
        for k, (key, v) in enumerate(pr.items()):
            if len(key) != 1:
                raise NotImplementedError("multi-character pattern id")
            pid[i, k] = ord(key)
            pval[i, k] = v
        npat[i] = len(pr)
        cp, sp = m.get("CP", ""), m.get("SP", "")
        ok = bool(data) and data.isdigit() and bool(cp) and cp.isdigit() and bool(sp) and sp.isdigit()
        if "R" in m and not m.get("R", "").isdigit():
            ok = False
        ms_ok[i] = int(ok)                        # message_synced.py:21-47
        if ok:
            cpk = str(int(cp))
            keys = list(pr.keys())
            cp_slot[i] = keys.index(cpk) if cpk in keys else -1
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum([len(d) for d in datas])
    return dict(data=np.frombuffer(b"".join(datas) or b"\0", np.uint8).copy(), offsets=offs, npat=npat,
                pat_id=pid, pat_val=pval, ms_ok=ms_ok, cp_slot=cp_slot, n=n)


def pack_batch(pb) -> dict:
    """A pysignalduino_amd.synth PulseBatch (already in SoA form) for the timed baseline."""
    return dict(data=pb.data, offsets=pb.offsets.astype(np.int64), npat=pb.npat.astype(np.uint8),
                pat_id=pb.pat_id.astype(np.uint8), pat_val=pb.pat_val.astype(np.float64),
                ms_ok=pb.ms_ok.astype(np.uint8), cp_slot=pb.cp_slot.astype(np.int8), n=pb.n)


def pack_mc(frames: Sequence[tuple]) -> dict:
    """frames: (raw_hex, clock, mcbitnum, mtype, version)."""
    n = len(frames)
    hexes = []
    clock, nbit = np.zeros(n, np.int32), np.zeros(n, np.int32)
    low, v32 = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
    for i, (h, c, b, t, v) in enumerate(frames):
        if any(ch not in "0123456789ABCDEFabcdef" for ch in h):
            if any(ch in " _+-xX\t" for ch in h):
                raise NotImplementedError("hex literal syntax beyond plain digits")
        hexes.append(h.encode("latin-1", "replace"))
        clock[i], nbit[i] = int(c), int(b)
        low[i] = int(t == "Mc")
        v32[i] = int(bool(v) and v[:6] == "V 3.2.")
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum([len(h) for h in hexes])
    return dict(hex=np.frombuffer(b"".join(hexes) or b"\0", np.uint8).copy(), offsets=offs, clock=clock,
                mcbitnum=nbit, mtype_lower=low, v32=v32, n=n)


def mc_batch(mb) -> dict:
    """A pysignalduino_amd.synth McBatch for the timed baseline."""
    return dict(hex=mb.hexdata, offsets=mb.offsets.astype(np.int64), clock=mb.clock.astype(np.int32),
                mcbitnum=mb.mcbitnum.astype(np.int32), mtype_lower=mb.mtype.astype(np.uint8),
                v32=mb.v32.astype(np.uint8), n=mb.n)


def _p(a):
    return C.c_void_p(a.ctypes.data)


def run(kind: str, packed: dict, nthreads: int = 1):
    """Demodulate a packed batch: returns (status, raise_kind, rec_begin, n_rec, rec, heap)."""
    L = lib()
    n = packed["n"]
    keep = []
    if kind == "MC":
        s = SoMc(_p(packed["hex"]), _p(packed["offsets"]), _p(packed["clock"]), _p(packed["mcbitnum"]),
                 _p(packed["mtype_lower"]), _p(packed["v32"]), n)
        pin, min_ = None, C.byref(s)
        keep.append(s)
    else:
        s = SoPulses(_p(packed["data"]), _p(packed["offsets"]), _p(packed["npat"]), _p(packed["pat_id"]),
                     _p(packed["pat_val"]), _p(packed["ms_ok"]), _p(packed["cp_slot"]), n)
        pin, min_ = C.byref(s), None
        keep.append(s)
    rec_cap, heap_cap = 16 * n + 1024, 256 * n + 65536
    while True:
        st, rk = np.zeros(max(n, 1), np.uint8), np.zeros(max(n, 1), np.uint8)
        rb, nr = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.uint16)
        rec, heap = np.zeros(rec_cap, RES_DT), np.zeros(heap_cap, np.uint8)
        out = SoOut(_p(st), _p(rk), _p(rb), _p(nr), _p(rec), _p(heap), rec_cap, heap_cap, 0, 0)
        rc = L.so_demod({"MU": 0, "MS": 1, "MC": 2}[kind], pin, min_, C.byref(out), int(nthreads))
        if rc == 0:
            return st[:n], rk[:n], rb[:n], nr[:n], rec[:out.rec_total], heap[:out.heap_total]
        rec_cap, heap_cap = int(out.rec_total) + 16, int(out.heap_total) + 16


def results(bank: CBank, kind: str, packed: dict, nthreads: int = 1) -> List[Any]:
    """Per message: a list of (pid, payload, bit_length) tuples, or the exception class raised."""
    st, rk, rb, nr, rec, heap = run(kind, packed, nthreads)
    out: List[Any] = []
    hb = heap.tobytes()
    for i in range(packed["n"]):
        if st[i]:
            out.append(RAISE[int(rk[i])])
            continue
        lst = []
        for r in rec[int(rb[i]):int(rb[i]) + int(nr[i])]:
            pay = hb[int(r["off"]):int(r["off"]) + int(r["len"])].decode("utf-8")
            lst.append((bank.pids[int(r["proto"])], pay, int(r["bitlen"])))
        out.append(lst)
    return out
