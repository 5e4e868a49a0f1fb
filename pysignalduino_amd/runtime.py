"""ctypes binding of libsdx.so (include/sdx.h) + device-buffer plumbing.

PyTorch is used only for device memory and streams (``torch.cuda``); every
byte of demodulation work runs in the hand-written HIP kernels of
``csrc/sdx_kernels.hip``.  There is NO CPU fallback: when the library or a
GPU is missing, :func:`load_library` / :class:`Engine` raise.
"""
from __future__ import annotations

import ctypes
import os
import struct
from ctypes import POINTER, Structure, c_char_p, c_int, c_int32, c_size_t, c_uint32, c_void_p
from typing import Dict, Optional, Tuple

import numpy as np

from . import bank as bankmod

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_lib", "libsdx.so")
ABI_VERSION = 14   # include/sdx.h SDX_ABI_VERSION

KIND_MU, KIND_MS, KIND_MC = 0, 1, 2
KIND_MN = 3        # host-side tag for Engine.run (sdx_demod_mn)
ST_OK, ST_RAISED, ST_OVF_TILE, ST_OVF_OUT = 0, 1, 2, 3
RAISE_NAMES = {1: IndexError, 2: AttributeError, 3: ValueError, 4: TypeError, 5: ZeroDivisionError}
RAISE_CONTRACT = 6  # SDX_RAISE_CONTRACT: a general-path limit (include/sdx.h), not a reference outcome
SHORT_MAX = 256    # k_pulses<.., 4 words, 64 messages/tile>
LONG_MAX = 4096    # k_pulses<.., 64 words, 4 messages/tile>
MC_HEX_MAX = 128   # MC_MAXW * 16 hex characters
MN_HEX_MAX = 4096  # SDX_MN_HEX_MAX

DESC_DT = np.dtype([("rec_begin", "<u4"), ("n_rec", "<u2"), ("status", "u1"), ("raise_kind", "u1")])
# sdx_msg_rec (include/sdx.h): one message's header fields, written by sdx_group_pulses
MREC_DT = np.dtype([("off", "<i8"), ("len", "<i4"), ("npat", "u1"), ("cp_slot", "i1"), ("ms_ok", "u1"), ("res0", "u1"),
                    ("pat_id", "u1", (10,)), ("res1", "u1", (6,)), ("pat_val", "<f8", (10,)), ("res2", "u1", (16,))])
MREC_BYTES = 128
RES_DT = np.dtype([("payload_off", "<u4"), ("payload_len", "<u2"), ("proto", "<u2"), ("bit_length", "<u4"),
                   ("msg", "<u4")])

EXPORTED = ["sdx_abi_version", "sdx_last_error", "sdx_source_hash", "sdx_layout_size", "sdx_bank_create", "sdx_bank_destroy",
            "sdx_bank_device_ptr", "sdx_demod_pulses", "sdx_demod_pulses_long", "sdx_demod_mc", "sdx_demod_mn",
            "sdx_parse_lines", "sdx_select_lines", "sdx_serialize_json", "sdx_units",
            "sdx_exchange_work_bytes", "sdx_exchange_send_bytes", "sdx_exchange_count", "sdx_exchange_pack", "sdx_exchange_pack_into", "sdx_exchange_unpack_work_bytes",
            "sdx_exchange_unpack", "sdx_pulses_work_bytes", "sdx_group_work_bytes", "sdx_group_pulses",
            "sdx_general_work_bytes", "sdx_demod_pulses_general", "sdx_mc_general_work_bytes", "sdx_demod_mc_general",
            "sdx_lines_general", "sdx_copy_async", "sdx_copy_async_kind", "sdx_copy_async_narrow",
            "sdx_fill_async", "sdx_demod_step", "sdx_group_step"]
GROUP_MIN = int(os.environ.get("SDX_GROUP_MIN", "4096"))   # SDX_GROUP_MIN (the env: A/B of the grouping)


class SdxPulseBatch(Structure):
    _fields_ = [("data_dev", c_void_p), ("offsets_dev", c_void_p), ("npat_dev", c_void_p),
                ("pat_id_dev", c_void_p), ("pat_val_dev", c_void_p), ("cp_slot_dev", c_void_p),
                ("ms_ok_dev", c_void_p), ("len_dev", c_void_p), ("sel_dev", c_void_p), ("n", c_int32),
                ("n_sel", c_int32), ("mrec_dev", c_void_p)]


class SdxGeneralBatch(Structure):
    _fields_ = [("data_dev", c_void_p), ("offsets_dev", c_void_p), ("npat_dev", c_void_p), ("pat_ids_dev", c_void_p),
                ("pat_val_dev", c_void_p), ("cp_slot_dev", c_void_p), ("ms_ok_dev", c_void_p), ("sel_dev", c_void_p),
                ("n", c_int32), ("n_sel", c_int32), ("len_dev", c_void_p), ("work_stride", ctypes.c_int64),
                ("max_len", c_int32), ("res", c_int32)]


class SdxLinesGeneralOut(Structure):
    _fields_ = [(f, c_void_p) for f in ("offsets_dev", "len_dev", "npat_dev", "pat_ids_dev", "pat_val_dev",
                                         "cp_slot_dev", "ms_ok_dev")]


class SdxMcBatch(Structure):
    _fields_ = [("hex_dev", c_void_p), ("offsets_dev", c_void_p), ("clock_dev", c_void_p),
                ("mcbitnum_dev", c_void_p), ("flags_dev", c_void_p), ("len_dev", c_void_p), ("sel_dev", c_void_p),
                ("n", c_int32), ("n_sel", c_int32), ("only_dev", c_void_p), ("max_hex", c_int32), ("res", c_int32)]


class SdxMnBatch(Structure):
    _fields_ = [("hex_dev", c_void_p), ("offsets_dev", c_void_p), ("len_dev", c_void_p), ("sel_dev", c_void_p),
                ("n", c_int32), ("n_sel", c_int32), ("elig", ctypes.c_uint64), ("method", c_int32), ("res", c_int32)]


class SdxJsonIn(Structure):
    _fields_ = [("kind", c_int32), ("first_only", c_int32), ("desc_dev", c_void_p), ("rec_dev", c_void_p),
                ("cursor_dev", c_void_p), ("heap_dev", c_void_p), ("meta_dev", c_void_p), ("pat_val_dev", c_void_p),
                ("cp_slot_dev", c_void_p), ("n", c_int32), ("rec_max", c_int32)]


class SdxJsonOut(Structure):
    _fields_ = [("json_dev", c_void_p), ("off_dev", c_void_p), ("len_dev", c_void_p), ("cursor_dev", c_void_p),
                ("json_cap", c_uint32), ("res", c_uint32)]


class SdxUnitBatch(Structure):
    _fields_ = [("op", c_int32), ("n", c_int32), ("in_dev", c_void_p), ("in_off_dev", c_void_p), ("arg_dev", c_void_p),
                ("val_dev", c_void_p), ("val_off_dev", c_void_p), ("mcrec_dev", c_void_p), ("out_off_dev", c_void_p)]


class SdxXchgPart(Structure):
    _fields_ = [("desc_dev", c_void_p), ("rec_dev", c_void_p), ("heap_dev", c_void_p), ("cursor_dev", c_void_p),
                ("n_msgs", c_uint32), ("rec_cap", c_uint32), ("heap_cap", c_uint32), ("kind", ctypes.c_uint8),
                ("alt", ctypes.c_uint8), ("aux", ctypes.c_uint8), ("res", ctypes.c_uint8),
                ("wire_dev", c_void_p), ("xrec_dev", c_void_p)]


class SdxXchgWire(Structure):
    _fields_ = [("msg_dev", c_void_p), ("rec_dev", c_void_p), ("heap_dev", c_void_p), ("n_msgs", c_uint32),
                ("n_rec", c_uint32), ("n_heap", c_uint32), ("n_payload", c_uint32)]


# the exchange's wire form (include/sdx.h, v3): one word per message, 8 bytes per record, payloads raw or
# as packed hex digits (proto bit 15 = WIRE_NIB: preamble + digits + postamble of the protocol)
WIRE_REC_DT = np.dtype([("proto", "<u2"), ("payload_len", "<u2"), ("bit_length", "<u4")])
WIRE_NIB = 0x8000
XCHG_MAX_RANKS = 32
XCHG_MAX_PARTS = 16
XCHG_COUNTS = 8     # u32 counts per part: messages, records, wire payload bytes, bad, payload bytes, 0, 0, 0
ST_ABSENT = 0xFF    # an exchange overlay's descriptor no re-run wrote
KIND_RAW = 0xFF     # sdx_xchg_part.kind: no affixes (raw payloads only)


class SdxOut(Structure):
    _fields_ = [("desc_dev", c_void_p), ("rec_dev", c_void_p), ("heap_dev", c_void_p), ("cursor_dev", c_void_p),
                ("rec_cap", c_uint32), ("heap_cap", c_uint32), ("work_dev", c_void_p), ("work_cap", ctypes.c_uint64),
                ("wire_dev", c_void_p), ("xrec_dev", c_void_p)]


class SdxStep(Structure):
    _fields_ = [("mu", POINTER(SdxPulseBatch)), ("mu_out", POINTER(SdxOut)), ("ms", POINTER(SdxPulseBatch)),
                ("ms_out", POINTER(SdxOut)), ("mc", POINTER(SdxMcBatch)), ("mc_out", POINTER(SdxOut))]


class SdxGroupJob(Structure):
    _fields_ = [("batch", POINTER(SdxPulseBatch)), ("order_dev", c_void_p), ("mrec_dev", c_void_p),
                ("work_dev", c_void_p), ("work_cap", c_size_t)]


class SdxLines(Structure):
    _fields_ = [("bytes_dev", c_void_p), ("offsets_dev", c_void_p), ("n", c_int32)]


class SdxLinesOut(Structure):
    _fields_ = [(f, c_void_p) for f in ("kind_dev", "status_dev", "slot_dev", "doff_dev", "dlen_dev", "npat_dev",
                                         "pat_id_dev", "pat_val_dev", "cp_slot_dev", "ms_ok_dev", "clock_dev",
                                         "mcbitnum_dev", "mcflags_dev", "meta_dev", "plen_dev")]


# include/sdx.h front-end constants
LINE_NONE, LINE_MU, LINE_MS, LINE_MC, LINE_MN = 0, 1, 2, 3, 4
LS_OK, LS_NOFRAME, LS_NOPARSER, LS_INVALID, LS_NODATA, LS_UNSUPPORTED, LS_RAISES, LS_GENERAL = 0, 1, 2, 3, 4, 5, 6, 7
# (ABI 14: MC lines of <= SDX_MC_SHORT_HEX characters and longer ones are separate classes)
SEL_MU_SHORT, SEL_MU_LONG, SEL_MS_SHORT, SEL_MS_LONG, SEL_MC, SEL_MC_LONG, SEL_MN, SEL_NCLASS = 0, 1, 2, 3, 4, 5, 6, 7
MC_SHORT_HEX = 64   # SDX_MC_SHORT_HEX
SEL_CHUNK = 1024

_LIB = None


def load_library(path: Optional[str] = None):
    """Load libsdx.so (fails loudly -- the product path has no fallback)."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or os.environ.get("SDX_LIB") or LIB_PATH
    # torch bundles its own libamdhip64.so.7: load it FIRST so that libsdx's NEEDED
    # libamdhip64.so.7 resolves to the same runtime (one HIP runtime per process).
    import torch  # noqa: F401
    if not os.path.exists(p):
        raise RuntimeError(f"libsdx.so not built ({p}); run __graft_entry__.build() "
                           "or python -m pysignalduino_amd.build")
    lib = ctypes.CDLL(p)
    lib.sdx_abi_version.restype = c_int
    lib.sdx_last_error.restype = c_char_p
    lib.sdx_source_hash.restype = c_char_p
    lib.sdx_layout_size.argtypes = [c_int]
    lib.sdx_layout_size.restype = c_int
    lib.sdx_copy_async.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p]
    lib.sdx_copy_async.restype = c_int
    lib.sdx_copy_async_kind.argtypes = [c_void_p, c_void_p, c_size_t, c_int, c_void_p]
    lib.sdx_copy_async_kind.restype = c_int
    lib.sdx_copy_async_narrow.argtypes = [c_void_p, c_void_p, c_size_t, c_int, c_void_p]
    lib.sdx_copy_async_narrow.restype = c_int
    lib.sdx_fill_async.argtypes = [c_void_p, c_int, c_size_t, c_void_p]
    lib.sdx_fill_async.restype = c_int
    lib.sdx_bank_create.argtypes = [c_void_p, c_size_t, c_int, POINTER(c_void_p)]
    lib.sdx_bank_create.restype = c_int
    lib.sdx_bank_destroy.argtypes = [c_void_p]
    lib.sdx_bank_destroy.restype = c_int
    lib.sdx_bank_device_ptr.argtypes = [c_void_p]
    lib.sdx_bank_device_ptr.restype = c_void_p
    for fn in ("sdx_demod_pulses", "sdx_demod_pulses_long"):
        f = getattr(lib, fn)
        f.argtypes = [c_void_p, c_int, POINTER(SdxPulseBatch), POINTER(SdxOut), c_void_p]
        f.restype = c_int
    lib.sdx_pulses_work_bytes.argtypes = [c_int]
    lib.sdx_pulses_work_bytes.restype = c_size_t
    lib.sdx_group_work_bytes.argtypes = [c_int]
    lib.sdx_group_work_bytes.restype = c_size_t
    lib.sdx_group_pulses.argtypes = [c_void_p, c_int, POINTER(SdxPulseBatch), c_void_p, c_void_p, c_void_p, c_size_t,
                                     c_void_p]
    lib.sdx_group_pulses.restype = c_int
    lib.sdx_general_work_bytes.argtypes = [c_void_p, c_int, ctypes.c_int64, c_int32, c_int32, ctypes.c_int64]
    lib.sdx_general_work_bytes.restype = ctypes.c_uint64
    lib.sdx_demod_pulses_general.argtypes = [c_void_p, c_int, POINTER(SdxGeneralBatch), POINTER(SdxOut), c_void_p]
    lib.sdx_demod_pulses_general.restype = c_int
    lib.sdx_mc_general_work_bytes.argtypes = [c_int32, c_int32]
    lib.sdx_mc_general_work_bytes.restype = ctypes.c_uint64
    lib.sdx_demod_mc_general.argtypes = [c_void_p, POINTER(SdxMcBatch), c_int32, POINTER(SdxOut), c_void_p]
    lib.sdx_demod_mc_general.restype = c_int
    lib.sdx_lines_general.argtypes = [POINTER(SdxLines), POINTER(SdxLinesOut), c_void_p, c_int32,
                                      POINTER(SdxLinesGeneralOut), c_void_p]
    lib.sdx_lines_general.restype = c_int
    lib.sdx_demod_mc.argtypes = [c_void_p, POINTER(SdxMcBatch), POINTER(SdxOut), c_void_p]
    lib.sdx_group_step.restype = c_int
    lib.sdx_group_step.argtypes = [c_void_p, POINTER(SdxGroupJob), POINTER(SdxGroupJob), c_void_p]
    lib.sdx_demod_step.restype = c_int
    lib.sdx_demod_step.argtypes = [c_void_p, POINTER(SdxStep), c_void_p]
    lib.sdx_demod_mc.restype = c_int
    lib.sdx_demod_mn.argtypes = [c_void_p, POINTER(SdxMnBatch), POINTER(SdxOut), c_void_p]
    lib.sdx_demod_mn.restype = c_int
    lib.sdx_serialize_json.argtypes = [c_void_p, POINTER(SdxJsonIn), POINTER(SdxJsonOut), c_void_p]
    lib.sdx_serialize_json.restype = c_int
    lib.sdx_parse_lines.argtypes = [POINTER(SdxLines), POINTER(SdxLinesOut), c_void_p]
    lib.sdx_parse_lines.restype = c_int
    lib.sdx_select_lines.argtypes = [POINTER(SdxLinesOut), c_int32, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.sdx_select_lines.restype = c_int
    lib.sdx_units.argtypes = [POINTER(SdxUnitBatch), POINTER(SdxOut), c_void_p]
    lib.sdx_units.restype = c_int
    lib.sdx_exchange_work_bytes.argtypes = [c_void_p, c_int]
    lib.sdx_exchange_work_bytes.restype = ctypes.c_uint64
    lib.sdx_exchange_send_bytes.argtypes = [POINTER(SdxXchgPart), c_int]
    lib.sdx_exchange_send_bytes.restype = ctypes.c_uint64
    lib.sdx_exchange_count.argtypes = [c_void_p, POINTER(SdxXchgPart), c_int, c_void_p, ctypes.c_uint64, c_void_p,
                                       c_void_p]
    lib.sdx_exchange_count.restype = c_int
    lib.sdx_exchange_pack.argtypes = [c_void_p, POINTER(SdxXchgPart), c_int, c_void_p, ctypes.c_uint64, c_void_p,
                                      c_void_p, ctypes.c_uint64, c_void_p]
    lib.sdx_exchange_pack.restype = c_int
    lib.sdx_exchange_pack_into.argtypes = [c_void_p, POINTER(SdxXchgPart), c_int, c_void_p, ctypes.c_uint64, c_void_p,
                                           c_void_p, c_void_p, ctypes.c_uint64, c_void_p]
    lib.sdx_exchange_pack_into.restype = c_int
    lib.sdx_exchange_unpack_work_bytes.argtypes = [c_uint32, c_uint32]
    lib.sdx_exchange_unpack_work_bytes.restype = ctypes.c_uint64
    lib.sdx_exchange_unpack.argtypes = [c_void_p, c_int, POINTER(SdxXchgWire), c_int, c_void_p, ctypes.c_uint64,
                                        c_void_p, c_void_p, c_void_p, ctypes.c_uint64, c_void_p]
    lib.sdx_exchange_unpack.restype = c_int
    if lib.sdx_abi_version() != ABI_VERSION:
        raise RuntimeError("libsdx ABI version mismatch")
    check_layout(lib)
    if path is None:
        _LIB = lib
    return lib


def check_layout(lib) -> None:
    """The numpy mirrors of the C structs must match sizeof() on the C side."""
    want = {0: struct.calcsize(bankmod.HDR_FMT), 1: bankmod.PATSPEC.itemsize, 2: bankmod.MU_REC.itemsize, 3: bankmod.MS_REC.itemsize,
            4: bankmod.MC_REC.itemsize, 5: RES_DT.itemsize, 6: DESC_DT.itemsize, 7: bankmod.MU_DESC.itemsize,
            8: bankmod.MN_REC.itemsize, 9: bankmod.JSON_REC.itemsize, 10: bankmod.MU_FILT.itemsize,
            11: bankmod.MS_FILT.itemsize, 12: ctypes.sizeof(SdxXchgPart), 13: ctypes.sizeof(SdxXchgWire),
            14: WIRE_REC_DT.itemsize, 15: MREC_DT.itemsize, 16: ctypes.sizeof(SdxPulseBatch), 17: ctypes.sizeof(SdxOut)}
    for k, v in want.items():
        got = lib.sdx_layout_size(k)
        if got != v:
            raise RuntimeError(f"struct layout mismatch (item {k}): C {got} vs Python {v}")


def _check(lib, rc):
    if rc != 0:
        raise RuntimeError(f"libsdx error {rc}: {lib.sdx_last_error().decode(errors='replace')}")


def _ptr(t) -> Optional[int]:
    return None if t is None else int(t.data_ptr())


def copy_async(dst, src, stream) -> None:
    """dst.copy_(src, non_blocking=True) on ``stream`` through sdx_copy_async: contiguous tensors of
    the same byte size (device or pinned host), one runtime call instead of a framework dispatch."""
    n = src.numel() * src.element_size()
    if n != dst.numel() * dst.element_size() or not (dst.is_contiguous() and src.is_contiguous()):
        raise ValueError("copy_async: contiguous tensors of the same byte size")
    lib = load_library()
    if _COPY_DEFAULT:
        _check(lib, lib.sdx_copy_async(dst.data_ptr(), src.data_ptr(), n, stream.cuda_stream))
        return
    # the direction named explicitly (hipMemcpyKind): with hipMemcpyDefault the runtime ran the
    # device -> pinned-host copies as blit kernels on every CU (__amd_rocclr_copyBuffer, 256 workgroups
    # held for the PCIe transfer), beside the next chunks' demodulation tiles
    kind = (3 if src.is_cuda else 1) if dst.is_cuda else (2 if src.is_cuda else 0)
    _check(lib, lib.sdx_copy_async_kind(dst.data_ptr(), src.data_ptr(), n, kind, stream.cuda_stream))


_COPY_DEFAULT = os.environ.get("SDX_COPY_DEFAULT") == "1"   # A/B: every copy with hipMemcpyDefault
# copy_d2h's workgroups; 0 (default): hipMemcpyAsync.  16 narrow workgroups measured no faster in the
# streaming front end (profiles/r05/stream/r05k_*: 207 vs 212M lines/s, 64: 178M)
D2H_NARROW_WG = int(os.environ.get("SDX_D2H_WG", "0"))


def copy_d2h(dst, src, stream) -> None:
    """A device -> pinned-host copy that occupies few CUs (sdx_copy_async_narrow, D2H_NARROW_WG
    workgroups): for result copies that run beside demodulation kernels."""
    if D2H_NARROW_WG <= 0 or not dst.is_pinned():
        return copy_async(dst, src, stream)
    n = src.numel() * src.element_size()
    if n != dst.numel() * dst.element_size() or not (dst.is_contiguous() and src.is_contiguous()):
        raise ValueError("copy_d2h: contiguous tensors of the same byte size")
    lib = load_library()
    _check(lib, lib.sdx_copy_async_narrow(dst.data_ptr(), src.data_ptr(), n, D2H_NARROW_WG, stream.cuda_stream))


def fill_async(dst, stream, value: int = 0) -> None:
    """dst.fill_(value) bytewise on ``stream`` through sdx_fill_async (contiguous device tensor)."""
    if not dst.is_contiguous():
        raise ValueError("fill_async: contiguous tensor")
    lib = load_library()
    _check(lib, lib.sdx_fill_async(dst.data_ptr(), int(value), dst.numel() * dst.element_size(), stream.cuda_stream))


class Engine:
    """One device + one uploaded bank.  All launches go to the caller's (torch) stream."""

    def __init__(self, bank: "bankmod.Bank", device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("pysignalduino_amd needs a ROCm GPU (MI355X); no CPU fallback exists")
        self.torch = torch
        self.lib = load_library()
        self.bank = bank
        self.device = device
        self.dev = torch.device("cuda", device)
        # message records (sdx_msg_rec): the grouping writes them and k_pulses reads its header
        # fields from them.  Off by default: 18 % / 44 % less HBM traffic for k_pulses<MU> / <MS>,
        # but 3.5 % slower on the bench corpus; SDX_MREC=1 turns them on
        self.use_mrec = os.environ.get("SDX_MREC", "0") == "1"
        h = c_void_p()
        blob = ctypes.create_string_buffer(bank.blob, len(bank.blob))
        with torch.cuda.device(device):
            _check(self.lib, self.lib.sdx_bank_create(ctypes.cast(blob, c_void_p), len(bank.blob), device,
                                                      ctypes.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self.lib.sdx_bank_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- buffers --------------------------------------------------------------------------------
    def to_device_pulses(self, pb) -> Dict[str, "object"]:
        t = self.torch
        d = self.dev
        out = {
            "data": t.from_numpy(np.ascontiguousarray(pb.data) if len(pb.data) else np.zeros(1, np.uint8)).to(d),
            "offsets": t.from_numpy(np.ascontiguousarray(pb.offsets, dtype=np.int64)).to(d),
            "npat": t.from_numpy(np.ascontiguousarray(pb.npat, dtype=np.uint8)).to(d),
            "pat_id": t.from_numpy(np.ascontiguousarray(pb.pat_id, dtype=np.uint8)).to(d),
            "pat_val": t.from_numpy(np.ascontiguousarray(pb.pat_val, dtype=np.float64)).to(d),
            "cp_slot": t.from_numpy(np.ascontiguousarray(pb.cp_slot, dtype=np.int8)).to(d),
            "ms_ok": t.from_numpy(np.ascontiguousarray(pb.ms_ok, dtype=np.uint8)).to(d),
            "n": int(pb.n),
            "lengths": np.diff(pb.offsets),
        }
        return out

    def to_device_mc(self, mb) -> Dict[str, "object"]:
        t = self.torch
        d = self.dev
        flags = (mb.mtype.astype(np.uint8) & 1) | ((mb.v32.astype(np.uint8) & 1) << 1)
        return {
            # 16 bytes of slack: k_mc stages frames with aligned 8-byte loads (include/sdx.h)
            "hex": t.from_numpy(np.concatenate([np.asarray(mb.hexdata, np.uint8), np.zeros(16, np.uint8)])).to(d),
            "offsets": t.from_numpy(np.ascontiguousarray(mb.offsets, dtype=np.int64)).to(d),
            "clock": t.from_numpy(np.ascontiguousarray(mb.clock, dtype=np.int32)).to(d),
            "mcbitnum": t.from_numpy(np.ascontiguousarray(mb.mcbitnum, dtype=np.int32)).to(d),
            "flags": t.from_numpy(np.ascontiguousarray(flags, dtype=np.uint8)).to(d),
            "n": int(mb.n),
            "lengths": np.diff(mb.offsets),
            # every frame's length is known here: sdx_demod_mc skips its long-frame launch when none
            # is longer than SDX_MC_SHORT_HEX (ABI 13)
            "max_hex": int(np.diff(mb.offsets).max(initial=0)),
        }

    def pulses_work_bytes(self, n: int, spill_frac: float = 0.5) -> int:
        """Workspace of an MU/MS launch over n messages: spill room for `spill_frac` of its
        64-message tiles (a grouped order makes tiles of result-heavy messages)."""
        tiles = (n + 63) // 64
        region = int(self.lib.sdx_pulses_work_bytes(1))
        most = (2 ** 32 - 2 * region) // region          # spill offsets are 32-bit (include/sdx.h)
        return int(self.lib.sdx_pulses_work_bytes(int(min(most, max(16, spill_frac * tiles)))))

    def group_buffers(self, n: int, n_batch: Optional[int] = None):
        """(order, work, mrec) device buffers for sdx_group_pulses over n messages of a batch of
        n_batch (default n): mrec holds one 128-byte sdx_msg_rec per batch message."""
        t = self.torch
        nb = n if n_batch is None else n_batch
        mrec = t.empty(max(nb, 1) * MREC_BYTES + 128, dtype=t.uint8, device=self.dev)
        off = (-mrec.data_ptr()) % 128  # 128-byte aligned records
        return (t.empty(max(n, 1), dtype=t.int32, device=self.dev),
                t.empty(max(int(self.lib.sdx_group_work_bytes(int(n))), 1), dtype=t.uint8, device=self.dev),
                mrec[off: off + max(nb, 1) * MREC_BYTES])

    def group(self, kind: int, bd, sel=None, bufs=None):
        """The grouped message order of a batch (or of `sel`) as a device int32 tensor: the sel of
        the launch_pulses that follows (same results, fewer instructions; sdx_group.hip).  `bufs`:
        group_buffers() to use; default: a per-engine cache (one stream at a time).  The grouping
        also writes the batch's message records into bufs[2] (launch_pulses(mrec=...))."""
        n = int(sel.numel()) if sel is not None else bd["n"]
        if bufs is None:
            c = getattr(self, "_gcache", None)
            if c is None or c[0].numel() < n or c[2].numel() < bd["n"] * MREC_BYTES:
                c = self._gcache = self.group_buffers(n, max(n, bd["n"]))
            bufs = c
        order, work, mrec = bufs
        b = self._pulse_batch(bd, sel)
        um = self.use_mrec   # bool, or the set of kinds whose grouping writes message records
        want = um if isinstance(um, bool) else kind in um
        _check(self.lib, self.lib.sdx_group_pulses(self.handle, kind, ctypes.byref(b), _ptr(order),
                                                   _ptr(mrec) if want else None, _ptr(work),
                                                   int(work.numel()), self.stream_ptr()))
        return order[:n]

    def group_step(self, mu_bd, ms_bd, mu_bufs, ms_bufs, mu_sel=None, ms_sel=None):
        """The MU and MS groupings of one mixed step in the same launches (sdx_group_step, ABI 14): the
        orders group(KIND_MU, ...) and group(KIND_MS, ...) return, as (mu_order, ms_order)."""
        um = self.use_mrec
        jobs, keep = [], []
        for kind, bd, bufs, sel in ((KIND_MU, mu_bd, mu_bufs, mu_sel), (KIND_MS, ms_bd, ms_bufs, ms_sel)):
            order, work, mrec = bufs
            b = self._pulse_batch(bd, sel)
            want = um if isinstance(um, bool) else kind in um
            keep.append(b)
            jobs.append(SdxGroupJob(ctypes.pointer(b), _ptr(order), _ptr(mrec) if want else None, _ptr(work),
                                    int(work.numel())))
        _check(self.lib, self.lib.sdx_group_step(self.handle, ctypes.byref(jobs[0]), ctypes.byref(jobs[1]),
                                                 self.stream_ptr()))
        n_mu = int(mu_sel.numel()) if mu_sel is not None else mu_bd["n"]
        n_ms = int(ms_sel.numel()) if ms_sel is not None else ms_bd["n"]
        return mu_bufs[0][:n_mu], ms_bufs[0][:n_ms]

    def alloc_out(self, n: int, rec_cap: int, heap_cap: int, work_bytes: int = 0, wire: bool = False):
        """Output buffers of one launch.  ``wire``: also the exchange's per-message counts and
        per-record classes (sdx_out.wire_dev / xrec_dev, ABI 12), written by the kernels' flushes so
        that sdx_exchange_count / _pack need not re-read the payloads."""
        t = self.torch
        d = self.dev
        return {
            "desc": t.zeros(max(n, 1) * DESC_DT.itemsize, dtype=t.uint8, device=d),
            "rec": t.empty(max(rec_cap, 1) * RES_DT.itemsize, dtype=t.uint8, device=d),
            "heap": t.empty(max(heap_cap, 1), dtype=t.uint8, device=d),
            "cursor": t.zeros(4, dtype=t.int32, device=d),
            "work": t.empty(work_bytes, dtype=t.uint8, device=d) if work_bytes else None,
            "wire": t.zeros(max(n, 1), dtype=t.int64, device=d) if wire else None,
            "xrec": t.empty(max(rec_cap, 1), dtype=t.int32, device=d) if wire else None,
            "rec_cap": rec_cap, "heap_cap": heap_cap, "n": n,
        }

    @staticmethod
    def _out_struct(o) -> SdxOut:
        w = o.get("work")
        return SdxOut(_ptr(o["desc"]), _ptr(o["rec"]), _ptr(o["heap"]), _ptr(o["cursor"]), o["rec_cap"],
                      o["heap_cap"], _ptr(w), 0 if w is None else int(w.numel()), _ptr(o.get("wire")),
                      _ptr(o.get("xrec")))

    def stream_ptr(self):
        return c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    # -- launches -------------------------------------------------------------------------------
    @staticmethod
    def _pulse_batch(bd, sel, mrec=None) -> SdxPulseBatch:
        return SdxPulseBatch(_ptr(bd["data"]), _ptr(bd["offsets"]), _ptr(bd["npat"]), _ptr(bd["pat_id"]),
                             _ptr(bd["pat_val"]), _ptr(bd["cp_slot"]), _ptr(bd["ms_ok"]), _ptr(bd.get("len")),
                             _ptr(sel), bd["n"], 0 if sel is None else int(sel.numel()), _ptr(mrec))

    def launch_pulses(self, kind: int, bd, out, sel=None, long_variant: bool = False, group: bool = True,
                      mrec=None) -> None:
        """MU/MS launch; the short variant runs batches of >= GROUP_MIN messages in the grouped
        order (group()) unless `group` is False (`sel` then runs in its own order).  `mrec`: the
        message records a group() call wrote for this batch (its bufs[2]), read by the short
        variant instead of the scattered SoA fields."""
        n = int(sel.numel()) if sel is not None else bd["n"]
        if group and not long_variant and n >= GROUP_MIN:
            sel = self.group(kind, bd, sel)
            um = self.use_mrec
            mrec = self._gcache[2] if (um if isinstance(um, bool) else kind in um) else None
        b = self._pulse_batch(bd, sel, None if long_variant else mrec)
        o = self._out_struct(out)
        fn = self.lib.sdx_demod_pulses_long if long_variant else self.lib.sdx_demod_pulses
        _check(self.lib, fn(self.handle, kind, ctypes.byref(b), ctypes.byref(o), self.stream_ptr()))

    @staticmethod
    def _mc_batch(bd, sel) -> SdxMcBatch:
        return SdxMcBatch(_ptr(bd["hex"]), _ptr(bd["offsets"]), _ptr(bd["clock"]), _ptr(bd["mcbitnum"]),
                          _ptr(bd["flags"]), _ptr(bd.get("len")), _ptr(sel), bd["n"],
                          0 if sel is None else int(sel.numel()), _ptr(bd.get("only")), int(bd.get("max_hex", 0)), 0)

    def launch_mc(self, bd, out, sel=None) -> None:
        b = self._mc_batch(bd, sel)
        o = self._out_struct(out)
        _check(self.lib, self.lib.sdx_demod_mc(self.handle, ctypes.byref(b), ctypes.byref(o), self.stream_ptr()))

    def launch_step(self, mu=None, ms=None, mc=None) -> None:
        """One mixed step as one kernel (sdx_demod_step, ABI 14): ``mu`` / ``ms`` = (batch, out, sel,
        mrec) and ``mc`` = (batch, out, sel), each optional; the same results as launch_pulses(MU,
        group=False), launch_pulses(MS, group=False) and launch_mc on the current stream.  The caller
        groups (``sel`` = group()'s order): the fused launch takes its kinds' orders as given."""
        keep = []
        st = SdxStep()
        for name, part in (("mu", mu), ("ms", ms)):
            if part is not None:
                bd, out, sel, mrec = part
                b, o = self._pulse_batch(bd, sel, mrec), self._out_struct(out)
                keep += [b, o]
                setattr(st, name, ctypes.pointer(b))
                setattr(st, name + "_out", ctypes.pointer(o))
        if mc is not None:
            bd, out, sel = mc
            b, o = self._mc_batch(bd, sel), self._out_struct(out)
            keep += [b, o]
            st.mc, st.mc_out = ctypes.pointer(b), ctypes.pointer(o)
        _check(self.lib, self.lib.sdx_demod_step(self.handle, ctypes.byref(st), self.stream_ptr()))

    def launch_mc_general(self, bd, out, sel, max_hex: int) -> None:
        """sdx_demod_mc_general over `sel` (frames of any length; its own bit workspace)."""
        wb = int(self.lib.sdx_mc_general_work_bytes(int(sel.numel()), int(max_hex)))
        work = self.torch.empty(max(wb, 1), dtype=self.torch.uint8, device=self.dev)
        b = SdxMcBatch(_ptr(bd["hex"]), _ptr(bd["offsets"]), _ptr(bd["clock"]), _ptr(bd["mcbitnum"]),
                       _ptr(bd["flags"]), _ptr(bd.get("len")), _ptr(sel), bd["n"], int(sel.numel()),
                       _ptr(bd.get("only")))
        o = self._out_struct(out)
        o.work_dev, o.work_cap = _ptr(work), wb
        _check(self.lib, self.lib.sdx_demod_mc_general(self.handle, ctypes.byref(b), int(max_hex), ctypes.byref(o),
                                                       self.stream_ptr()))
        out["_mcg_work"] = work   # alive until the launch has run (the caller's fetch synchronises)

    # -- general path (sdx_demod_pulses_general) --------------------------------------------------
    def to_device_general(self, arrs) -> Dict[str, "object"]:
        t, d = self.torch, self.dev
        data = arrs["data"] if len(arrs["data"]) else np.zeros(1, np.uint8)
        out = {k: t.from_numpy(np.ascontiguousarray(v)).to(d) for k, v in arrs.items() if k != "data"}
        out["data"] = t.from_numpy(np.ascontiguousarray(data)).to(d)
        out["n"] = int(len(arrs["npat"]))
        out["total"] = int(arrs["offsets"][-1])
        out["lengths"] = np.diff(arrs["offsets"])
        return out

    def run_general(self, kind: int, gd, work_stride: int = 0):
        """MU/MS messages on the general path; returns host (desc, rec, heap) like run().
        ``work_stride`` > 0: per-message scratch of that many bytes (gd in slot layout, "len" set)."""
        n = gd["n"]
        rec_cap = 16 * n + 1024
        heap_cap = int(2 * gd["total"] + 256 * n + 65536)
        lens = gd["lens_host"] if "lens_host" in gd else np.asarray(gd["lengths"])
        max_len = int(lens.max(initial=0))
        wb = int(self.lib.sdx_general_work_bytes(self.handle, kind, int(gd["total"]), n, max_len, int(work_stride)))
        work = self.torch.empty(max(wb, 1), dtype=self.torch.uint8, device=self.dev)
        # the longest messages first: the device's work queue then ends on short ones
        order = np.argsort(-lens, kind="stable").astype(np.int32)
        sel = self.torch.from_numpy(order).to(self.dev)
        for attempt in range(6):
            out = self.alloc_out(n, rec_cap, heap_cap)
            o = self._out_struct(out)
            o.work_dev, o.work_cap = _ptr(work), int(work.numel())
            b = SdxGeneralBatch(_ptr(gd["data"]), _ptr(gd["offsets"]), _ptr(gd["npat"]), _ptr(gd["pat_ids"]),
                                _ptr(gd["pat_val"]), _ptr(gd["cp_slot"]), _ptr(gd["ms_ok"]), _ptr(sel), n, n,
                                _ptr(gd.get("len")), int(work_stride), max_len, 0)
            _check(self.lib, self.lib.sdx_demod_pulses_general(self.handle, kind, ctypes.byref(b), ctypes.byref(o),
                                                               self.stream_ptr()))
            desc, rec, heap = self.fetch(out)
            if not (desc["status"] == ST_OVF_OUT).any():
                return desc, rec, heap
            rec_cap, heap_cap = 4 * rec_cap, 4 * heap_cap   # whole-batch re-run with grown outputs
        raise RuntimeError("general path: result capacity overflow persists")

    def general_overlay(self, kind: int, gd, rows: np.ndarray, work_stride: int = 0):
        """The general path over the messages ``rows`` of a general batch ``gd`` that holds every
        message of a launch (placeholders elsewhere), into an exchange overlay indexed like that
        launch (descriptors of the other messages stay ST_ABSENT).  Capacity overflows re-run the
        launch with grown outputs until none is left (host checks; the general path is rare)."""
        rows = np.asarray(rows, np.int32)
        n = gd["n"]
        lens = np.asarray(gd["lengths"])[rows]
        rec_cap = 16 * len(rows) + 1024
        heap_cap = int(2 * int(lens.sum()) + 256 * len(rows) + 65536)
        max_len = int(lens.max(initial=0))
        wb = int(self.lib.sdx_general_work_bytes(self.handle, kind, int(gd["total"]), n, max_len, int(work_stride)))
        work = self.torch.empty(max(wb, 1), dtype=self.torch.uint8, device=self.dev)
        # the longest messages first: the device's work queue then ends on short ones
        order = rows[np.argsort(-lens, kind="stable")].astype(np.int32)
        sel = self.torch.from_numpy(order).to(self.dev)
        for attempt in range(6):
            out = self.overlay_out(n, rec_cap, heap_cap)
            o = self._out_struct(out)
            o.work_dev, o.work_cap = _ptr(work), int(work.numel())
            b = SdxGeneralBatch(_ptr(gd["data"]), _ptr(gd["offsets"]), _ptr(gd["npat"]), _ptr(gd["pat_ids"]),
                                _ptr(gd["pat_val"]), _ptr(gd["cp_slot"]), _ptr(gd["ms_ok"]), _ptr(sel), n,
                                len(order), _ptr(gd.get("len")), int(work_stride), max_len, 0)
            _check(self.lib, self.lib.sdx_demod_pulses_general(self.handle, kind, ctypes.byref(b), ctypes.byref(o),
                                                               self.stream_ptr()))
            self.torch.cuda.current_stream(self.dev).synchronize()
            st = out["desc"][: n * DESC_DT.itemsize].view(-1, DESC_DT.itemsize)[:, 6].cpu().numpy()[rows]
            if not (st == ST_OVF_OUT).any():
                out["_keep"] = (work, sel)
                return out
            rec_cap, heap_cap = 4 * rec_cap, 4 * heap_cap
        raise RuntimeError("general path: result capacity overflow persists")

    def to_device_mn(self, hexes) -> Dict[str, "object"]:
        """MN frames (hex strings / bytes) -> device batch.  Contract: [0-9A-Fa-f]* and at most
        MN_HEX_MAX characters (checked here; ContractError-free callers check before)."""
        t = self.torch
        bs = [h.encode("latin-1") if isinstance(h, str) else bytes(h) for h in hexes]
        lens = np.fromiter((len(b) for b in bs), np.int64, len(bs))
        offsets = np.zeros(len(bs) + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        data = np.concatenate([np.frombuffer(b"".join(bs), np.uint8), np.zeros(16, np.uint8)])  # 8-byte read slack
        return {"hex": t.from_numpy(data).to(self.dev),
                "offsets": t.from_numpy(offsets).to(self.dev), "n": len(bs), "lengths": lens}

    def launch_mn(self, bd, out, elig: int = 0, method: int = -1, sel=None) -> None:
        b = SdxMnBatch(_ptr(bd["hex"]), _ptr(bd["offsets"]), _ptr(bd.get("len")), _ptr(sel), bd["n"],
                       0 if sel is None else int(sel.numel()), elig, method, 0)
        o = self._out_struct(out)
        _check(self.lib, self.lib.sdx_demod_mn(self.handle, ctypes.byref(b), ctypes.byref(o), self.stream_ptr()))

    def launch_json(self, kind: int, demod_out, lines_out, n: int, jout, first_only: bool = True) -> None:
        """sdx_serialize_json over a demodulation launch's device outputs (no host sync).  first_only:
        True / 1 one text per line, 2 the same sparse (only lines with a text are written: launches of
        several kinds share one output), False / 0 one text per record."""
        ji = SdxJsonIn(kind, int(first_only), _ptr(demod_out["desc"]), _ptr(demod_out["rec"]),
                       _ptr(demod_out["cursor"]), _ptr(demod_out["heap"]), _ptr(lines_out["meta"]),
                       _ptr(lines_out.get("pat_val")), _ptr(lines_out.get("cp_slot")), n,
                       0 if first_only else demod_out["rec_cap"])
        jo = SdxJsonOut(_ptr(jout["json"]), _ptr(jout["off"]), _ptr(jout["len"]), _ptr(jout["cursor"]),
                        jout["cap"], 0)
        _check(self.lib, self.lib.sdx_serialize_json(self.handle, ctypes.byref(ji), ctypes.byref(jo),
                                                     self.stream_ptr()))

    def alloc_json(self, items: int, cap: int):
        t, d = self.torch, self.dev
        return {"json": t.empty(max(cap, 8), dtype=t.uint8, device=d), "off": t.empty(max(items, 1), dtype=t.int32, device=d),
                "len": t.empty(max(items, 1), dtype=t.int32, device=d), "cursor": t.zeros(2, dtype=t.int32, device=d),
                "cap": cap, "items": items}

    # -- full run with contract routing and overflow re-runs (all on the GPU) --------------------
    def run(self, kind: int, bd, rec_cap: Optional[int] = None, heap_cap: Optional[int] = None,
            sel_short=None, sel_long=None, mn_elig: int = 0, mn_method: int = -1, workspace: bool = True):
        """Demodulate a device batch; returns host numpy (desc, rec, heap).  The first pass
        (first_pass) then GPU re-runs of overflowed messages (rerun_overlay) merged on the host.

        ``workspace``: MU/MS launches run in the grouped message order with spill regions for
        result-heavy tiles (sdx_group_pulses, sdx_demod_pulses); False runs the messages in batch
        order without a workspace.

        ``sel_short`` / ``sel_long``: device int32 lists of the messages to run with the short /
        long variant (MC: ``sel_short`` only), as sdx_select_lines builds them; the other
        messages keep an empty OK descriptor.  Without them every message runs, routed by length.
        """
        out = self.first_pass(kind, bd, rec_cap, heap_cap, sel_short, sel_long, mn_elig, mn_method, workspace)
        rec_cap, heap_cap = out["rec_cap"], out["heap_cap"]
        desc, rec, heap = self.fetch(out)
        # re-runs on the GPU: grown output buffers / the long variant's larger per-message staging
        for attempt in range(4):
            st = desc["status"]
            redo = np.nonzero((st == ST_OVF_OUT) | (st == ST_OVF_TILE))[0].astype(np.int32)
            if not len(redo):
                break
            if attempt == 3:
                raise RuntimeError("result staging overflow persists (pathological message)")
            rec_cap, heap_cap = 2 * rec_cap + 64 * len(redo), 2 * heap_cap + 8192 * len(redo)
            out2 = self.rerun_overlay(kind, bd, redo, rec_cap, heap_cap, mn_elig=mn_elig, mn_method=mn_method)
            d2, r2, h2 = self.fetch(out2)
            # merge: re-based records appended after the first pass
            base_r, base_h = len(rec), len(heap)
            r2 = r2.copy()
            r2["payload_off"] += base_h
            rec = np.concatenate([rec, r2])
            heap = np.concatenate([heap, h2])
            for i in redo:
                d = d2[i].copy()
                d["rec_begin"] += base_r
                desc[i] = d
        return desc, rec, heap

    def first_pass(self, kind: int, bd, rec_cap: Optional[int] = None, heap_cap: Optional[int] = None,
                   sel_short=None, sel_long=None, mn_elig: int = 0, mn_method: int = -1, workspace: bool = True,
                   wire: bool = False):
        """Output buffers sized for a device batch (default capacities: 8 records and 200 payload
        bytes per message) and the first pass's launches into them (launch_routed), enqueued on the
        current stream; returns the output dict (run() re-runs what overflowed).  ``wire``: the
        kernels also write the exchange's counts (alloc_out), where every message of the launch goes
        to a kernel that writes them (k_pulses, k_mc: not MN, not MC batches with frames for the
        general MC kernel)."""
        n = bd["n"]
        selected = sel_short is not None or sel_long is not None
        if selected:
            n_work = sum(int(s.numel()) for s in (sel_short, sel_long) if s is not None)
        else:
            n_work = n
            lengths = bd["lengths"]
            if kind == KIND_MN:
                if n and int(lengths.max(initial=0)) > MN_HEX_MAX:
                    raise NotImplementedError(f"MN frames longer than {MN_HEX_MAX} hex characters are outside "
                                              "the device contract")
            elif kind == KIND_MC:
                pass   # frames longer than MC_HEX_MAX run on the general MC kernel (below)
            elif n and int(lengths.max(initial=0)) > LONG_MAX:
                raise NotImplementedError(f"messages longer than {LONG_MAX} pulses are outside the device contract")
        rec_cap = rec_cap or (8 * n_work + 1024)
        heap_cap = heap_cap or (200 * n_work + 65536)
        if kind == KIND_MN and not selected:   # parser mode: <= n_mn results of <= preamble + frame bytes
            rec_cap = max(rec_cap, 4 * n_work + 1024)
            heap_cap = max(heap_cap, int(4 * int(np.sum(bd["lengths"])) + 160 * n_work + 65536))
        if wire and (kind == KIND_MN or (kind == KIND_MC and not selected and bool((bd["lengths"] > MC_HEX_MAX).any()))):
            wire = False
        out = self.alloc_out(n, rec_cap, heap_cap,
                             self.pulses_work_bytes(n_work) if workspace and kind in (KIND_MU, KIND_MS) else 0, wire=wire)
        self.launch_routed(kind, bd, out, sel_short=sel_short, sel_long=sel_long, mn_elig=mn_elig, mn_method=mn_method,
                           workspace=workspace)
        return out

    def launch_routed(self, kind: int, bd, out, sel_short=None, sel_long=None, mn_elig: int = 0, mn_method: int = -1,
                      workspace: bool = True) -> None:
        """The first pass of run(): every message (or the given selection lists) to the launch that
        takes it -- MU/MS: the short variant (grouped order, spill regions) for <= SHORT_MAX pulses,
        the long one above; MC: k_mc, frames of more than MC_HEX_MAX characters on the general MC
        kernel; MN: k_mn.  Enqueued on the current stream, no host synchronisation."""
        t = self.torch
        if kind == KIND_MN:
            self.launch_mn(bd, out, elig=mn_elig, method=mn_method, sel=sel_short)
        elif sel_short is not None or sel_long is not None:
            if sel_short is not None and sel_short.numel():
                (self.launch_mc(bd, out, sel=sel_short) if kind == KIND_MC else
                 self.launch_pulses(kind, bd, out, sel=sel_short, group=workspace))
            if sel_long is not None and sel_long.numel():
                self.launch_pulses(kind, bd, out, sel=sel_long, long_variant=True)
        elif kind == KIND_MC:
            lengths = bd["lengths"]
            longf = lengths > MC_HEX_MAX
            if not longf.any():
                self.launch_mc(bd, out)
            else:   # k_mc takes <= MC_HEX_MAX characters; longer frames: sdx_demod_mc_general
                if not longf.all():
                    self.launch_mc(bd, out, sel=t.from_numpy(np.nonzero(~longf)[0].astype(np.int32)).to(self.dev))
                self.launch_mc_general(bd, out, t.from_numpy(np.nonzero(longf)[0].astype(np.int32)).to(self.dev),
                                       int(lengths.max()))
        else:
            lengths = bd["lengths"]
            short = lengths <= SHORT_MAX
            if short.all():
                self.launch_pulses(kind, bd, out, group=workspace)
            else:
                if short.any():
                    self.launch_pulses(kind, bd, out, sel=t.from_numpy(np.nonzero(short)[0].astype(np.int32)).to(self.dev),
                                       group=workspace)
                self.launch_pulses(kind, bd, out, sel=t.from_numpy(np.nonzero(~short)[0].astype(np.int32)).to(self.dev),
                                   long_variant=True)

    def overlay_out(self, n: int, rec_cap: int, heap_cap: int, wire: bool = False):
        """Output buffers of an exchange overlay (include/sdx.h ABI 11): every descriptor at
        ST_ABSENT until a launch writes it."""
        o = self.alloc_out(n, rec_cap, heap_cap, wire=wire)
        o["desc"].fill_(ST_ABSENT)
        return o

    def rerun_overlay(self, kind: int, bd, redo: np.ndarray, rec_cap: int, heap_cap: int, mn_elig: int = 0,
                      mn_method: int = -1):
        """Re-run the messages ``redo`` (host int array of batch indices whose first pass overflowed)
        into a fresh overlay: MU/MS on the long variant (larger per-message staging), MC on k_mc or,
        for frames of more than MC_HEX_MAX characters (k_mc hands them over as ST_OVF_TILE), on
        sdx_demod_mc_general, MN on k_mn; grown output capacities.  Enqueued on the current stream."""
        t = self.torch
        redo = np.asarray(redo, np.int32)
        # MU/MS re-run on the long k_pulses variant, which writes the exchange's counts (ABI 12)
        out2 = self.overlay_out(bd["n"], rec_cap, heap_cap, wire=kind in (KIND_MU, KIND_MS))
        sel = t.from_numpy(redo).to(self.dev)
        if kind == KIND_MN:
            self.launch_mn(bd, out2, elig=mn_elig, method=mn_method, sel=sel)
        elif kind == KIND_MC:
            if "lengths" in bd:
                rl = np.asarray(bd["lengths"])[redo]
            else:                # a line batch: the frames' lengths are on the device
                rl = bd["len"][t.from_numpy(redo.astype(np.int64)).to(self.dev)].cpu().numpy()
            lr = rl > MC_HEX_MAX
            if (~lr).any():
                self.launch_mc(bd, out2, sel=t.from_numpy(redo[~lr]).to(self.dev))
            if lr.any():
                self.launch_mc_general(bd, out2, t.from_numpy(redo[lr]).to(self.dev), int(rl.max()))
        else:
            self.launch_pulses(kind, bd, out2, sel=sel, long_variant=True)
        out2["_sel"] = sel          # alive until the launches have run
        return out2

    def fetch(self, out):
        self.torch.cuda.current_stream(self.dev).synchronize()
        cur = out["cursor"].cpu().numpy().astype(np.uint32)
        n = out["n"]
        desc = out["desc"][: n * DESC_DT.itemsize].cpu().numpy().view(DESC_DT).copy()
        nrec = min(int(cur[0]), out["rec_cap"])
        nheap = min(int(cur[1]), out["heap_cap"])
        rec = out["rec"][: nrec * RES_DT.itemsize].cpu().numpy().view(RES_DT).copy()
        heap = out["heap"][:nheap].cpu().numpy().copy()
        return desc, rec, heap


# ---- unit-level entry (sdx_units) ----------------------------------------------------------------
UNIT_POSTDEMO, UNIT_HEX2BIN, UNIT_BIN2HEX, UNIT_MC2DMC, UNIT_PEXISTS, UNIT_MC_METHOD = 1, 2, 3, 4, 5, 6
UNIT_MC_BITS, UNIT_PX_SEARCH, UNIT_PX_PAT = 512, 32, 16

_UNIT_RUNNERS: Dict[int, "UnitRunner"] = {}


class UnitRunner:
    """sdx_units launches on one device (no bank needed: every input travels with the call)."""

    def __init__(self, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("pysignalduino_amd needs a ROCm GPU (MI355X); no CPU fallback exists")
        self.torch = torch
        self.lib = load_library()
        self.dev = torch.device("cuda", device)

    @staticmethod
    def get(device: int = 0) -> "UnitRunner":
        r = _UNIT_RUNNERS.get(device)
        if r is None:
            r = _UNIT_RUNNERS[device] = UnitRunner(device)
        return r

    def run(self, op: int, ins, caps, args=None, vals=None, mcrecs=None):
        """Run one op over the byte strings ``ins`` (``caps[i]``: payload capacity of item i).
        ``vals``: per-item float64 arrays (UNIT_PEXISTS); ``mcrecs``: numpy MC_REC array (UNIT_MC_METHOD).
        Returns (desc, rec, heap) as host numpy arrays, one desc/rec per item."""
        t, d = self.torch, self.dev
        n = len(ins)
        if n == 0:
            return np.zeros(0, DESC_DT), np.zeros(0, RES_DT), np.zeros(0, np.uint8)
        lens = np.fromiter((len(b) for b in ins), np.int64, n)
        in_off = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=in_off[1:])
        data = np.frombuffer(b"".join(ins) + b"\0" * 8, np.uint8)
        out_off = np.zeros(n + 1, np.int64)
        np.cumsum(np.asarray(caps, np.int64), out=out_off[1:])
        keep = []

        def dev(a):
            a = np.ascontiguousarray(a)
            if not a.flags.writeable:
                a = a.copy()
            x = t.from_numpy(a).to(d)
            keep.append(x)
            return _ptr(x)

        val_p = val_off_p = mc_p = None
        if vals is not None:
            vl = np.fromiter((len(v) for v in vals), np.int64, n)
            val_off = np.zeros(n + 1, np.int64)
            np.cumsum(vl, out=val_off[1:])
            flat = np.concatenate([np.asarray(v, np.float64) for v in vals] + [np.zeros(1)])
            val_p, val_off_p = dev(flat), dev(val_off)
        if mcrecs is not None:
            mc_p = dev(np.frombuffer(np.ascontiguousarray(mcrecs).tobytes(), np.uint8))
        heap_cap = int(out_off[-1])
        out = {"desc": t.zeros(n * DESC_DT.itemsize, dtype=t.uint8, device=d),
               "rec": t.zeros(n * RES_DT.itemsize, dtype=t.uint8, device=d),
               "heap": t.zeros(max(heap_cap, 1), dtype=t.uint8, device=d),
               "cursor": t.zeros(4, dtype=t.int32, device=d)}
        b = SdxUnitBatch(op, n, dev(data), dev(in_off), None if args is None else dev(np.asarray(args, np.int32)),
                         val_p, val_off_p, mc_p, dev(out_off))
        o = SdxOut(_ptr(out["desc"]), _ptr(out["rec"]), _ptr(out["heap"]), _ptr(out["cursor"]), n, max(heap_cap, 1), None, 0)
        _check(self.lib, self.lib.sdx_units(ctypes.byref(b), ctypes.byref(o),
                                            c_void_p(t.cuda.current_stream(d).cuda_stream)))
        t.cuda.current_stream(d).synchronize()
        desc = out["desc"].cpu().numpy().view(DESC_DT).copy()
        rec = out["rec"].cpu().numpy().view(RES_DT).copy()
        heap = out["heap"].cpu().numpy()
        return desc, rec, heap
