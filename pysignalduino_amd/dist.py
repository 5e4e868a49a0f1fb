"""Multi-GPU: contiguous message shards per rank + all-gather of the decoded dmsg buffers.

Messages are independent: each rank demodulates its contiguous shard with no
communication during compute.  The one exchange step gathers every rank's results so that every
rank holds the whole stream's results in global message order (BASELINE config 5).

What travels is the WIRE form of include/sdx.h (v3), per launch and rank, in message order:
  msg  section  u32 per message = n_rec | status << 16 | raise_kind << 24
  rec  section  8 B per record  = proto (| WIRE_NIB), payload_len, bit_length
  heap section  the payloads in record order, zero-padded to 16 bytes; a payload that is its
                protocol's preamble + uppercase hex digits + postamble travels as the digits packed
                two per byte (the receiver has the same bank and rebuilds the affixes)
rec_begin, payload_off and msg are prefix sums and are rebuilt by the receiver
(``sdx_exchange_unpack``).  The wire is canonical: the bytes do not depend on the order in which
tiles wrote their records, so a sharded run and an un-sharded run compare byte for byte.

Overflow re-runs (ABI 11): a launch whose messages overflowed (ST_OVF_TILE / ST_OVF_OUT) is never
exchanged as such.  Its messages are re-run into an OVERLAY (:class:`Part` ``overlays``: outputs over
the same messages, descriptors left at ST_ABSENT where no re-run wrote) and the sender takes each
message from the last overlay that has it.  :class:`Exchange` drives the re-runs itself when the
count exchange reports overflowed messages on any rank (``rerun`` callback, all ranks recount), and
:class:`ShardedDemodulator` is the product entry that shards a batch, demodulates, re-runs and
exchanges.

With the ``nccl`` backend (RCCL over xGMI on ROCm) the buffers stay in HBM and the exchange runs on
its own HIP stream (:class:`Exchange`), overlapped with the next step's kernels:
  step k kernels ─ready_k─▶ [exchange stream] sdx_exchange_count_k ─ all-gather counts_k ─ D2H
  submit(k+1): host waits for counts_k (the GPU runs step k+1 meanwhile), re-runs overflowed
               messages (rare), sizes the sections (max over ranks), enqueues
               sdx_exchange_pack_into_k (this rank's chunk of the receive buffer) ─released_k─
               in-place all-gather data_k, and only then the wait on ready_{k+1} and step k+1's count.
The same protocol runs synchronously on ``gloo`` (CPU tensors: numpy packing; CUDA tensors: the
device kernels, the collective staged through host memory).  ``Exchange(pipeline=True)`` (or
``SDX_XCHG_PIPELINE=1``) runs the pipelined branch above over gloo as well, so the exact code an
RCCL run executes (deferred count, in-place pack, recount after re-runs) is tested at world > 1 on
one GPU; only the transport differs.

Collective-size agreement.  Every count collective carries a fixed-size FRAME (FRAME_INTS int32 per
rank: a header of magic, world size, number of primary launches, phase and flags, then the counts of
up to SDX_XCHG_MAX_PARTS parts), so ranks that disagree on the number of launches can never issue
collectives of different sizes (an RCCL hang, a gloo abort): every rank sees every header and raises
:class:`ExchangeMismatch` together.  The data collective's size T is a function of the gathered counts
alone, hence identical on every rank.  A re-run that fails on one rank is reported through the
frame's flags, so all ranks take part in the recount and raise together.
"""
from __future__ import annotations

import ctypes
import os
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import runtime
from .runtime import DESC_DT, KIND_RAW, RES_DT, ST_ABSENT, WIRE_NIB, WIRE_REC_DT, XCHG_COUNTS

DESC_BYTES = 8
REC_BYTES = 16
WIRE_MSG_BYTES = 4
WIRE_REC_BYTES = 8
RAISE_HOST = 0xFE   # raise_kind of a host overlay row: the host packing raised for this message
OVF = (runtime.ST_OVF_TILE, runtime.ST_OVF_OUT)

# the count collective's fixed-size frame (per rank): header + counts of up to XCHG_MAX_PARTS parts
FRAME_HDR = 8
FRAME_INTS = FRAME_HDR + XCHG_COUNTS * runtime.XCHG_MAX_PARTS
FRAME_MAGIC = 0x53445846         # 'SDXF'
PHASE_COUNT, PHASE_RECOUNT = 1, 2
FLAG_RERUN_FAILED = 1   # this rank's overflow re-run raised
FLAG_LOCAL_ERROR = 2    # this rank failed before its counts (e.g. too many overlays, a bad buffer): no counts
BRANCH_SYNC, BRANCH_PIPELINED = 0, 1   # header word 5: the exchange branch (the collective sequence) of the rank


def _nullctx():
    import contextlib
    return contextlib.nullcontext()


class ExchangeMismatch(RuntimeError):
    """The ranks disagree on an exchange's shape (world size, number of launches, protocol phase) or
    a rank's re-run failed: raised on EVERY rank from the same all-gathered frame headers."""


def check_frames(frames: np.ndarray, world: int, K: int, phase: int) -> Tuple[np.ndarray, np.ndarray]:
    """All-gathered count frames [world * FRAME_INTS] -> (the primary launches' counts S[world, K,
    XCHG_COUNTS], per-rank flags).  Raises ExchangeMismatch, identically on every rank, when a header
    is not this exchange's (magic, world size, K, phase), when the ranks run different exchange branches
    (synchronous / pipelined: their collective sequences are equal only by construction), or when a rank
    flagged a local error (FLAG_LOCAL_ERROR: its frame holds no counts)."""
    f = np.asarray(frames, np.int64).reshape(world, FRAME_INTS)
    hdr = f[:, :FRAME_HDR]
    want = np.array([FRAME_MAGIC, world, K, phase])
    if not (hdr[:, :4] == want).all() or not (hdr[:, 5] == hdr[0, 5]).all():
        rows = {r: dict(magic=hex(int(h[0])), world=int(h[1]), launches=int(h[2]), phase=int(h[3]),
                        branch="pipelined" if h[5] == BRANCH_PIPELINED else "sync")
                for r, h in enumerate(hdr)}
        raise ExchangeMismatch(f"exchange: the ranks' count frames disagree (want world {world}, {K} launches, "
                               f"phase {phase}, one branch): {rows}")
    local = [r for r in range(world) if hdr[r, 4] & FLAG_LOCAL_ERROR]
    if local:
        raise ExchangeMismatch(f"exchange: rank(s) {local} failed before counting (phase {phase})")
    return f[:, FRAME_HDR: FRAME_HDR + K * XCHG_COUNTS].reshape(world, K, XCHG_COUNTS), hdr[:, 4].copy()


def frame_header(world: int, K: int, phase: int, flags: int = 0, branch: int = BRANCH_SYNC) -> np.ndarray:
    h = np.zeros(FRAME_HDR, np.int32)
    h[:6] = (FRAME_MAGIC, world, K, phase, flags, branch)
    return h


def _env_pipeline() -> Optional[bool]:
    v = os.environ.get("SDX_XCHG_PIPELINE")
    return None if v in (None, "") else v not in ("0", "false", "no")


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of ``n`` messages owned by ``rank`` (sizes differ by at most 1)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _r16(x):
    return (x + 15) // 16 * 16


# ---- host (numpy) form of the wire: CPU tensors on gloo, and the checker of the device kernels ----
def _nib_digits(affix, proto: int, p: bytes) -> int:
    """The nibble form's test (sdx_exchange.hip nib_digits): payload == pre + D uppercase hex digits +
    post of the protocol -> D, else -1."""
    if affix is None or proto >= len(affix):
        return -1
    pre, post = affix[proto]
    if len(pre) > 255 or len(p) < len(pre) + len(post) or not p.startswith(pre) or not p.endswith(post):
        return -1   # (a preamble of > 255 bytes does not fit the xrec word: raw)
    mid = p[len(pre): len(p) - len(post)]
    return len(mid) if all(c in b"0123456789ABCDEF" for c in mid) else -1


def _nib_pack(digits: bytes) -> bytes:
    v = [int(chr(c), 16) for c in digits]
    if len(v) % 2:
        v.append(0)
    return bytes((v[i] << 4) | v[i + 1] for i in range(0, len(v), 2))


def _nib_unpack(b: bytes, nd: int) -> bytes:
    out = bytearray()
    for i in range(nd):
        x = (b[i >> 1] >> (0 if i & 1 else 4)) & 15
        out.append(ord("0123456789ABCDEF"[x]))
    return bytes(out)


def resolve_host(levels) -> Tuple[np.ndarray, np.ndarray]:
    """levels: [(desc, ...)] of a launch and its overlays in chain order -> (per message the level
    its results come from, the resolved descriptors): the last level whose descriptor is present."""
    desc = levels[0][0].copy()
    lev = np.zeros(len(desc), np.int64)
    for j, lv in enumerate(levels[1:], 1):
        d = lv[0]
        here = d["status"] != ST_ABSENT
        desc[here] = d[here]
        lev[here] = j
    return lev, desc


def wire_encode(desc: np.ndarray, rec: np.ndarray, heap: np.ndarray, nrec_written: Optional[int] = None,
                nheap_written: Optional[int] = None, affix=None, overlays=()):
    """One launch's host (desc, rec, heap) (plus its overlays: (desc, rec, heap, nrec_written,
    nheap_written) in chain order) -> (msg u32[n], wire records, wire payload bytes, bad count), with
    the validation rules of k_xw_count (a record or payload outside what its launch wrote makes the
    message "bad": shipped with n_rec 0 and status ST_OVF_OUT) and the nibble form where ``affix``
    (Bank.affixes(kind)) is given."""
    def clamp(r, h, nr, nh):
        return (len(r) if nr is None else min(nr, len(r))), (len(h) if nh is None else min(nh, len(h)))

    levels = [(desc, rec, np.asarray(heap, np.uint8), *clamp(rec, heap, nrec_written, nheap_written))]
    for d2, r2, h2, nr2, nh2 in overlays:
        levels.append((d2, r2, np.asarray(h2, np.uint8), *clamp(r2, h2, nr2, nh2)))
    lev, rdesc = resolve_host(levels)
    n = len(desc)
    msg = np.zeros(n, np.uint32)
    recs, pays, bad = [], [], 0
    for m in range(n):
        d = rdesc[m]
        _, rr, hb, nrec_c, nheap_c = levels[int(lev[m])]
        st, nr, rb = int(d["status"]), int(d["n_rec"]), int(d["rec_begin"])
        if st == runtime.ST_RAISED:
            msg[m] = (st << 16) | (int(d["raise_kind"]) << 24)
            continue
        ok = st == runtime.ST_OK and (nr == 0 or rb + nr <= nrec_c)
        if ok:
            rs = rr[rb: rb + nr]
            ok = bool(np.all(rs["msg"] == m)) and bool(np.all(rs["payload_off"].astype(np.int64)
                                                              + rs["payload_len"] <= nheap_c))
        if not ok:
            bad += 1
            msg[m] = (runtime.ST_OVF_OUT << 16) | (int(d["raise_kind"]) << 24)
            continue
        msg[m] = nr | (st << 16) | (int(d["raise_kind"]) << 24)
        for r in rs:
            p = hb[int(r["payload_off"]): int(r["payload_off"]) + int(r["payload_len"])].tobytes()
            pr = int(r["proto"])
            dg = _nib_digits(affix, pr, p)
            if dg >= 0:
                pre = affix[pr][0]
                pays.append(np.frombuffer(_nib_pack(p[len(pre): len(pre) + dg]), np.uint8))
                pr |= WIRE_NIB
            else:
                pays.append(np.frombuffer(p, np.uint8))
            recs.append((pr, int(r["payload_len"]), int(r["bit_length"])))
    wrec = np.array(recs, WIRE_REC_DT) if recs else np.zeros(0, WIRE_REC_DT)
    pay = np.concatenate(pays) if pays else np.zeros(0, np.uint8)
    return msg, wrec, pay.astype(np.uint8), bad


def wire_decode(ranks: Sequence[Tuple[np.ndarray, np.ndarray, np.ndarray]], affix=None):
    """Wire sections of every rank (rank order) -> the whole job's (desc, rec, heap), as
    sdx_exchange_unpack builds them (nibble-form payloads rebuilt with the protocols' affixes)."""
    msg = np.concatenate([np.asarray(m, np.uint32) for m, _, _ in ranks]) if ranks else np.zeros(0, np.uint32)
    wrec = np.concatenate([w for _, w, _ in ranks]) if ranks else np.zeros(0, WIRE_REC_DT)
    wheap = b"".join(np.asarray(p, np.uint8).tobytes() for _, _, p in ranks)
    n = len(msg)
    desc = np.zeros(n, DESC_DT)
    nrec = (msg & 0xFFFF).astype(np.int64)
    desc["n_rec"] = nrec
    desc["status"] = (msg >> 16) & 0xFF
    desc["raise_kind"] = msg >> 24
    desc["rec_begin"] = np.concatenate([[0], np.cumsum(nrec)[:-1]]) if n else np.zeros(0, np.int64)
    rec = np.zeros(len(wrec), RES_DT)
    proto = wrec["proto"].astype(np.int64)
    rec["proto"] = proto & (WIRE_NIB - 1)
    rec["payload_len"] = wrec["payload_len"]
    rec["bit_length"] = wrec["bit_length"]
    pl = wrec["payload_len"].astype(np.int64)
    rec["payload_off"] = np.concatenate([[0], np.cumsum(pl)[:-1]]) if len(pl) else np.zeros(0, np.int64)
    rec["msg"] = np.repeat(np.arange(n, dtype=np.int64), nrec)
    out = bytearray()
    o = 0
    for i in range(len(wrec)):
        ln = int(pl[i])
        if proto[i] & WIRE_NIB:
            pre, post = affix[int(proto[i] & (WIRE_NIB - 1))]
            nd = ln - len(pre) - len(post)
            nb = (nd + 1) // 2
            out += pre + _nib_unpack(wheap[o: o + nb], nd) + post
            o += nb
        else:
            out += wheap[o: o + ln]
            o += ln
    return desc, rec, np.frombuffer(bytes(out), np.uint8).copy()


def canonical(desc: np.ndarray, rec: np.ndarray, heap: np.ndarray):
    """A launch's host outputs in canonical form: records in message order, payloads packed.  The
    exchange delivers exactly this (for the whole job); the tests compare against it."""
    m, w, p, bad = wire_encode(desc, rec, heap)
    if bad:
        raise ValueError(f"{bad} messages overflowed: re-run before comparing")
    return wire_decode([(m, w, p)])


# ---- launches as the exchange sees them ------------------------------------------------------------
class Part:
    """One demodulation launch's outputs as the exchange reads them: byte tensors ``desc`` /
    ``rec`` / ``heap`` of ``n`` messages, the launch's ``cursor`` (records, heap bytes written),
    ``kind`` (runtime.KIND_*: its protocols' affixes for the nibble form; KIND_RAW: raw payloads), the
    ``overlays`` (Parts over the same messages holding re-run / general-path results, in precedence
    order) and ``src`` = (kind, device batch) for re-running its overflowed messages."""

    __slots__ = ("desc", "rec", "heap", "n", "cursor", "kind", "overlays", "src", "keep", "wire", "xrec")

    def __init__(self, desc, rec, heap, n, cursor, kind=KIND_RAW, overlays=(), src=None, keep=None, wire=None,
                 xrec=None):
        self.desc, self.rec, self.heap, self.n, self.cursor = desc, rec, heap, int(n), cursor
        self.kind, self.overlays, self.src, self.keep = kind, list(overlays), src, keep
        self.wire, self.xrec = wire, xrec   # the kernels' exchange counts / record classes (ABI 12), or None

    @staticmethod
    def of(p) -> "Part":
        """A Part, or a (desc, rec, heap, n, cursor[, kind]) tuple."""
        return p if isinstance(p, Part) else Part(*p)

    @staticmethod
    def from_out(out, kind=KIND_RAW, src=None) -> "Part":
        """An Engine.alloc_out dict."""
        return Part(out["desc"], out["rec"], out["heap"], out["n"], out["cursor"], kind, src=src, keep=out,
                    wire=out.get("wire"), xrec=out.get("xrec"))

    def caps(self):
        return self.rec.numel() // REC_BYTES, self.heap.numel()


def _flatten(parts: Sequence[Part]):
    """Primary launches first, then each launch's overlays (chained in order): the sdx_xchg_part
    array with its alt / aux fields, as (Part, alt, aux) triples."""
    flat = [(p, 0, 0) for p in parts]
    for i, p in enumerate(parts):
        prev = i
        for ov in p.overlays:
            flat.append((ov, 0, 1))
            j = len(flat) - 1
            q, _, aux = flat[prev]
            flat[prev] = (q, j + 1, aux)
            prev = j
    if len(flat) > runtime.XCHG_MAX_PARTS:
        raise RuntimeError(f"exchange: {len(flat)} launches + overlays exceed SDX_XCHG_MAX_PARTS")
    return flat


def _nprimary(flat) -> int:
    """The primary launches of a _flatten() array (they come first; overlays follow)."""
    return sum(1 for _, _, aux in flat if not aux)


def _layout(S: np.ndarray):
    """S[world, K, >=3] = (messages, records, wire payload bytes, ...) -> per rank the section offsets
    [world, K, 3] of its send buffer (launch 0, 1, ...: msg, rec, heap sections, each padded to 16
    bytes -- the layout k_xw_pack computes on the device), the section byte counts [world, K, 3]
    and the collective's per-rank size T (the largest rank's buffer)."""
    S = np.asarray(S, np.int64)
    nb = np.stack([S[..., 0] * WIRE_MSG_BYTES, S[..., 1] * WIRE_REC_BYTES, S[..., 2]], axis=-1)
    sizes = _r16(nb).reshape(S.shape[0], -1)                                     # [world, K*3]
    offs = np.concatenate([np.zeros((S.shape[0], 1), np.int64), np.cumsum(sizes, axis=1)[:, :-1]], axis=1)
    T = int(max(16, sizes.sum(axis=1).max()))
    return offs.reshape(S.shape[0], S.shape[1], 3), nb, T


# ---- collectives -------------------------------------------------------------------------------------
def _all_gather_flat(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """all_gather into one contiguous tensor.  The collective is chosen once from the backend:
    RCCL's all_gather_into_tensor on device buffers; gloo's list form on host buffers (CUDA tensors
    are staged through host memory).  Every rank issues the same one."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
        return
    w = dist.get_world_size(group)
    if inp.device.type == "cuda":
        host = torch.empty(out.numel(), dtype=out.dtype)
        dist.all_gather(list(host.chunk(w)), inp.cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather(list(out.chunk(w)), inp, group=group)


class _Pending:
    __slots__ = ("parts", "counts_host", "event", "enc", "cnt", "rerun", "ready")

    def __init__(self, parts, counts_host, event, enc=None, cnt=None, rerun=None, ready=None):
        self.parts, self.counts_host, self.event, self.enc, self.cnt, self.rerun, self.ready = \
            parts, counts_host, event, enc, cnt, rerun, ready


class Exchange:
    """All-gather of the decoded dmsg buffers of K launches per step, pipelined.

    ``submit(parts, stream, rerun)`` is called after the step's kernels are enqueued on ``stream``
    (``parts``: :class:`Part` objects or (desc u8, rec u8, heap u8, n_msgs, cursor[, kind]) tuples;
    cursor[0] = records, cursor[1] = heap bytes, left on the device; the capacities are the buffers'
    sizes).  It first completes the PREVIOUS step's exchange (the data all-gather: its counts arrived
    while this step's kernels were running) and then enqueues this step's count + count all-gather
    behind this step's kernels.  It returns the event after which the PREVIOUS step's output buffers
    may be overwritten (its pack has read them; None on the first call): with the nccl backend a step
    is packed once its counts are on the host, straight into this rank's chunk of the receive buffer,
    and all-gathered in place (no send buffer, no local copy), so double-buffer the outputs.
    ``flush()`` completes the last step and returns the same event for it.  ``gathered()`` gives the
    last completed step's results as per launch (desc, rec, heap) byte tensors of the whole job in
    global message order.

    Overflowed messages (the counts' "bad" column, seen by every rank): each rank whose launch k has
    some calls ``rerun(part)`` -> the Part with one more overlay holding their re-run results, then
    every rank recounts; without a ``rerun`` the completing call raises.  ``engine``: the Engine whose
    bank gives the nibble form's affixes (None: raw payloads)."""

    def __init__(self, group=None, engine=None, defer: bool = False, pipeline: Optional[bool] = None):
        self.group = group
        # defer: a step's count AND pack run only in the NEXT submit, behind its ``after`` event (e.g.
        # the end of the next step's first launch), so the exchange kernels share the GPU with the
        # next step's later launches instead of its first one
        self.defer = defer
        # pipeline: the overlapped branch (exchange stream, in-place pack) for device buffers.  None =
        # with the nccl backend only (the product default); True also over gloo, the collective staged
        # through host memory (tests / rehearsals of the RCCL code path on one GPU; SDX_XCHG_PIPELINE=1)
        self.pipeline = pipeline if pipeline is not None else _env_pipeline()
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.engine = engine
        self.pending: Optional[_Pending] = None
        self.stream = None
        self._bufs = {}
        self.last = None        # (recv, S, offs, nb, T, K, kinds) of the last completed exchange
        self.bytes_sent = []    # per completed step: the collective's bytes per rank (T)
        self.wire_bytes = []    # per completed step: this rank's wire bytes before padding
        self.payload_bytes = []  # per completed step: this rank's payload bytes (before the nibble form)
        self.heap_wire_bytes = []  # per completed step: this rank's payload bytes on the wire (nibble form)
        self.reruns = 0         # launches re-run before exchanging

    @classmethod
    def sender(cls, engine=None) -> "Exchange":
        """The wire serialiser alone (sdx_exchange_count / _pack on one device, no process group): e.g.
        the streaming front end's compact results (stream.LineStream output='wire')."""
        ex = cls.__new__(cls)
        ex.group, ex.world, ex.rank, ex.engine, ex.defer, ex.pipeline = None, 1, 0, engine, False, False
        ex.pending, ex.stream, ex._bufs, ex.last = None, None, {}, None
        ex.bytes_sent, ex.wire_bytes, ex.payload_bytes, ex.heap_wire_bytes, ex.reruns = [], [], [], [], 0
        return ex

    def _bank(self):
        return None if self.engine is None else self.engine.handle

    def _affix(self, kind):
        if self.engine is None or kind == KIND_RAW:
            return None
        c = self.__dict__.setdefault("_affix_cache", {})
        if kind not in c:
            c[kind] = self.engine.bank.affixes(kind)
        return c[kind]

    def _buf(self, name, n, dev, zero=False):
        b = self._bufs.get(name)
        if b is None or b.numel() < n or b.device != dev:
            n2 = max(n, 64) + 256
            b = self._bufs[name] = (torch.zeros if zero else torch.empty)(n2, dtype=torch.uint8, device=dev)
        return b

    # -- device path ----------------------------------------------------------------------------------
    def _xparts(self, flat):
        arr = (runtime.SdxXchgPart * len(flat))()
        for k, (p, alt, aux) in enumerate(flat):
            rcap, hcap = p.caps()
            arr[k] = runtime.SdxXchgPart(p.desc.data_ptr(), p.rec.data_ptr(), p.heap.data_ptr(), p.cursor.data_ptr(),
                                         p.n, rcap, hcap, p.kind if self.engine is not None else KIND_RAW, alt, aux, 0,
                                         runtime._ptr(p.wire), runtime._ptr(p.xrec))
        return arr

    def _work(self, flat, dev):
        """ONE zeroed workspace, grown to the largest layout (the bad counters sit at fixed places in
        its head and the kernels leave them at zero, so any layout may reuse it)."""
        lib = runtime.load_library()
        ns = (ctypes.c_uint32 * len(flat))(*[p.n for p, _, _ in flat])
        wb = int(lib.sdx_exchange_work_bytes(ns, len(flat)))
        w = self._buf("work", wb + 256, dev, zero=True)
        off = (-w.data_ptr()) % 256
        return w[off:], wb

    def _frame(self, dev, K, phase, flags=0, branch=None):
        """A count frame on ``dev`` (FRAME_INTS int32): the header of this exchange (copied from a
        cached pinned host tensor that is never written again, so the copy needs no host sync) and
        room for the counts of up to XCHG_MAX_PARTS parts behind it.  A FLAG_LOCAL_ERROR frame is
        header + zeros (the rank has no counts)."""
        if branch is None:
            branch = BRANCH_PIPELINED if dev.type == "cuda" and self.pipelined else BRANCH_SYNC
        c = self.__dict__.setdefault("_hdr_cache", {})
        key = (K, phase, flags, branch, dev.type)
        if key not in c:
            c[key] = torch.from_numpy(frame_header(self.world, K, phase, flags, branch))
            if dev.type == "cuda":
                c[key] = c[key].pin_memory()
        zero = dev.type != "cuda" or bool(flags & FLAG_LOCAL_ERROR)
        f = (torch.zeros if zero else torch.empty)(FRAME_INTS, dtype=torch.int32, device=dev)
        f[:FRAME_HDR].copy_(c[key], non_blocking=True)
        return f

    def _gather_frame(self, frame):
        """The fixed-size count collective: every rank's frame, [world * FRAME_INTS] on frame's device."""
        allc = torch.empty(self.world * FRAME_INTS, dtype=torch.int32, device=frame.device)
        _all_gather_flat(allc, frame, self.group)
        return allc

    def _count_device(self, flat, stream, frame=None):
        """sdx_exchange_count on `stream`: [len(flat) * XCHG_COUNTS] int32 device counts (the pack
        follows once the host has them: _complete, sdx_exchange_pack_into); written into ``frame``'s
        count area when given."""
        lib = runtime.load_library()
        dev = flat[0][0].desc.device
        work, wb = self._work(flat, dev)
        cnt = self._cnt_out(flat, dev, frame)
        runtime._check(lib, lib.sdx_exchange_count(self._bank(), self._xparts(flat), len(flat),
                                                   ctypes.c_void_p(work.data_ptr()), wb,
                                                   ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(stream.cuda_stream)))
        return cnt

    @staticmethod
    def _cnt_out(flat, dev, frame):
        if frame is None:
            return torch.empty(XCHG_COUNTS * len(flat), dtype=torch.int32, device=dev)
        return frame[FRAME_HDR: FRAME_HDR + XCHG_COUNTS * len(flat)]

    def _count_pack_device(self, flat, stream, frame=None):
        """sdx_exchange_count + sdx_exchange_pack on `stream`: [len(flat) * XCHG_COUNTS] int32 device
        counts (in ``frame`` when given); the wire form of this rank is in the "send" buffer (layout:
        _layout)."""
        lib = runtime.load_library()
        dev = flat[0][0].desc.device
        work, wb = self._work(flat, dev)
        xp = self._xparts(flat)
        cnt = self._cnt_out(flat, dev, frame)
        sp = ctypes.c_void_p(stream.cuda_stream)
        runtime._check(lib, lib.sdx_exchange_count(self._bank(), xp, len(flat), ctypes.c_void_p(work.data_ptr()), wb,
                                                   ctypes.c_void_p(cnt.data_ptr()), sp))
        cap = int(lib.sdx_exchange_send_bytes(xp, len(flat)))
        send = self._buf("send", cap, dev)
        runtime._check(lib, lib.sdx_exchange_pack(self._bank(), xp, len(flat), ctypes.c_void_p(work.data_ptr()), wb,
                                                  ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(send.data_ptr()),
                                                  send.numel(), sp))
        return cnt

    # -- host path (CPU tensors) ------------------------------------------------------------------------
    def _encode_host(self, parts):
        out = []
        for p in parts:
            def arrs(q):
                rcap, _ = q.caps()
                return (q.desc[: q.n * DESC_BYTES].numpy().view(DESC_DT), q.rec[: rcap * REC_BYTES].numpy().view(RES_DT),
                        q.heap.numpy(), int(q.cursor[0]), int(q.cursor[1]))
            d, r, h, nr, nh = arrs(p)
            enc = wire_encode(d, r, h, nr, nh, affix=self._affix(p.kind), overlays=[arrs(o) for o in p.overlays])
            out.append(enc + (int(enc[1]["payload_len"].astype(np.int64).sum()),))
        return out

    def _counts_host(self, enc, K, phase, flags=0, branch=BRANCH_SYNC):
        """The count frame of K primary launches' host encodings (messages, records, wire bytes, bad,
        payload bytes, 0, 0, 0 each)."""
        f = self._frame(torch.device("cpu"), K, phase, flags, branch)
        c = torch.tensor([[len(m), len(w), len(p), b, pb, 0, 0, 0] for m, w, p, b, pb in enc], dtype=torch.int32)
        f[FRAME_HDR: FRAME_HDR + c.numel()] = c.reshape(-1)
        return f

    @property
    def pipelined(self) -> bool:
        """Whether device buffers take the overlapped branch (exchange stream, in-place pack)."""
        if self.pipeline is not None:
            return bool(self.pipeline)
        return dist.get_backend(self.group) == "nccl"

    # -- protocol ----------------------------------------------------------------------------------------
    def submit(self, parts, stream=None, rerun: Optional[Callable[[Part], Part]] = None, after=None):
        parts = [Part.of(p) for p in parts]
        dev = parts[0].desc.device
        overlap = dev.type == "cuda" and self.pipelined
        K = len(parts)
        if not overlap:   # synchronous form: gloo (CPU tensors, or CUDA tensors staged through the host)
            # whatever fails on this rank before its counts are known (the pipelined setting on host
            # buffers, more launches + overlays than a frame holds, the local count / encode) is sent as a
            # FLAG_LOCAL_ERROR frame: the peers are in the same collective and every rank raises together
            err = ValueError("exchange: the pipelined branch needs device buffers") \
                if self.pipeline and dev.type != "cuda" else None
            branch = BRANCH_PIPELINED if self.pipeline else BRANCH_SYNC
            enc = frame = None
            if dev.type == "cuda":
                stream = stream or torch.cuda.current_stream(dev)
                with torch.cuda.stream(stream):
                    try:
                        flat = _flatten(parts)
                        frame = self._frame(dev, K, PHASE_COUNT, branch=branch)
                        self._count_pack_device(flat, stream, frame)
                    except Exception as e:
                        err, frame = e, self._frame(dev, K, PHASE_COUNT, FLAG_LOCAL_ERROR, branch=branch)
                    allc = self._gather_frame(frame).cpu()
            else:
                if err is None:
                    try:
                        _flatten(parts)      # the same launch + overlay limit on every branch
                        enc = self._encode_host(parts)
                        frame = self._counts_host(enc, K, PHASE_COUNT, branch=branch)
                    except Exception as e:
                        err = e
                if err is not None:
                    frame = self._frame(dev, K, PHASE_COUNT, FLAG_LOCAL_ERROR, branch=branch)
                allc = self._gather_frame(frame)
            try:
                check_frames(allc.numpy(), self.world, K, PHASE_COUNT)
            except ExchangeMismatch as m:
                if err is not None:
                    raise ExchangeMismatch(f"{m}: {type(err).__name__}: {err}") from err
                raise
            with torch.cuda.stream(stream) if dev.type == "cuda" else _nullctx():
                self._complete(_Pending(parts, allc, None, enc, rerun=rerun))
            return None
        if self.stream is None:
            # (a low-priority exchange stream measured no different: profiles/r04/s3/xchg_sched_ab.log)
            self.stream = torch.cuda.Stream(dev)
        stream = stream or torch.cuda.current_stream(dev)
        if self.defer:
            return self._submit_deferred(parts, stream, rerun, after)
        # 1. the previous step: its counts are (about to be) on the host -- pack it into its chunk of
        #    the receive buffer and all-gather in place, ahead of anything that waits for this step
        prev, self.pending = self.pending, None
        released = None
        if prev is not None:
            with torch.cuda.stream(self.stream):
                if after is not None:   # the previous step's pack behind this step's ``after`` event
                    self.stream.wait_event(after)
                released = self._complete(prev)
        # 2. this step: count + count all-gather + counts to the host, behind this step's kernels
        ready = torch.cuda.Event()
        ready.record(stream)
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ready)
            host, ev, cnt = self._count_to_host(_flatten(parts), dev, K)
        self.pending = _Pending(parts, host, ev, cnt=cnt, rerun=rerun)
        return released

    def _submit_deferred(self, parts, stream, rerun, after):
        """defer mode: behind ``after`` (default: now on ``stream``) the previous step is counted,
        its counts gathered and brought to the host (this call waits for them), re-run if needed,
        packed into its chunk and all-gathered; this step is only recorded."""
        dev = parts[0].desc.device
        released = None
        prev, self.pending = self.pending, None
        if prev is not None:
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(prev.ready)
                if after is not None:
                    self.stream.wait_event(after)
                prev.counts_host, prev.event, prev.cnt = self._count_to_host(_flatten(prev.parts), dev, len(prev.parts))
                released = self._complete(prev)
        ready = torch.cuda.Event()
        ready.record(stream)
        self.pending = _Pending(parts, None, None, rerun=rerun, ready=ready)
        return released

    def _count_to_host(self, flat, dev, K, phase=PHASE_COUNT, flags=0):
        """count + count-frame all-gather + pinned D2H on the current stream: (host frames, event,
        device counts).  The frame has a fixed size whatever the number of launches and overlays, so
        the collective's size never differs between ranks (check_frames then compares the headers)."""
        frame = self._frame(dev, K, phase, flags)
        cnt = self._count_device(flat, torch.cuda.current_stream(dev), frame)
        allc = self._gather_frame(frame)
        host = torch.empty(allc.numel(), dtype=torch.int32, pin_memory=True)
        host.copy_(allc, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        return host, ev, cnt

    def flush(self):
        """Completes the last submitted step; returns the event after which its output buffers may
        be overwritten (None when nothing was pending)."""
        prev, self.pending = self.pending, None
        if prev is None:
            return None
        with torch.cuda.stream(self.stream):
            if prev.counts_host is None:    # defer mode: not counted yet
                self.stream.wait_event(prev.ready)
                prev.counts_host, prev.event, prev.cnt = self._count_to_host(
                    _flatten(prev.parts), prev.parts[0].desc.device, len(prev.parts))
            return self._complete(prev)

    def _rerun_bad(self, p: _Pending, S: np.ndarray, K: int) -> np.ndarray:
        """Every rank: re-run the launches with overflowed messages on this rank (p.rerun), then
        recount all launches (a collective every rank takes part in) -> the new counts.  A re-run that
        raises on one rank is flagged in that rank's recount frame: every rank still recounts, and all
        raise together (never a rank waiting in a collective that a failed peer left)."""
        for attempt in range(4):
            if not S[:, :K, 3].any():
                return S
            if p.rerun is None:
                bad = {(r, k): int(S[r, k, 3]) for r in range(self.world) for k in range(K) if S[r, k, 3]}
                raise RuntimeError(f"exchange: overflowed messages in (rank, launch) {bad} and no re-run given")
            err = None
            for k in range(K):
                if S[self.rank, k, 3]:
                    try:
                        p.parts[k] = p.rerun(p.parts[k])
                    except Exception as e:   # reported through the recount frame, raised below on all ranks
                        err = e
                        break
                    self.reruns += 1
            flags = FLAG_RERUN_FAILED if err is not None else 0
            dev = p.parts[0].desc.device
            # the local recount preparation (flatten -- at most XCHG_MAX_PARTS launches + overlays --,
            # encode, count) may raise on this rank alone: its frame then carries the failure flag and no
            # counts, and the collective below still runs, so the peers never wait in it
            frame = None
            if err is None:
                try:
                    if dev.type != "cuda":
                        _flatten(p.parts)    # the same launch + overlay limit on every branch
                        p.enc = self._encode_host(p.parts)
                        frame = self._counts_host(p.enc, K, PHASE_RECOUNT, flags)
                    else:
                        flat = _flatten(p.parts)
                        frame = self._frame(dev, K, PHASE_RECOUNT, flags)
                        if p.cnt is None:        # gloo with device tensors: count + pack again
                            self._count_pack_device(flat, torch.cuda.current_stream(dev), frame)
                        else:
                            p.cnt = self._count_device(flat, torch.cuda.current_stream(dev), frame)
                except Exception as e:
                    err, frame = e, None
            if frame is None:
                frame = self._frame(dev, K, PHASE_RECOUNT, FLAG_RERUN_FAILED)
                frame[FRAME_HDR:].zero_()
            allc = self._gather_frame(frame)
            if dev.type == "cuda":
                host = torch.empty(allc.numel(), dtype=torch.int32, pin_memory=True)
                host.copy_(allc, non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
            else:
                host = allc
            S, fl = check_frames(host.numpy(), self.world, K, PHASE_RECOUNT)
            if fl.any():
                failed = [r for r in range(self.world) if fl[r] & FLAG_RERUN_FAILED]
                msg = f"exchange: the overflow re-run failed on rank(s) {failed}"
                if err is not None:
                    raise ExchangeMismatch(f"{msg}: {type(err).__name__}: {err}") from err
                raise ExchangeMismatch(msg)
        raise RuntimeError("exchange: overflow persists after 4 re-runs (pathological message)")

    def _complete(self, p: _Pending):
        """The data collective of a step whose counts are on (or on their way to) the host; device
        buffers: on the current stream.  Pipelined: the step is packed here (sdx_exchange_pack_into)
        into this rank's chunk of the receive buffer and gathered in place; returns the event after
        which the step's output buffers may be overwritten."""
        K = len(p.parts)
        if p.event is not None:
            p.event.synchronize()            # the counts (the GPU has moved on to the next step)
        S, _ = check_frames(p.counts_host.numpy(), self.world, K, PHASE_COUNT)
        S = self._rerun_bad(p, S, K)
        flat = _flatten(p.parts) if p.enc is None else None
        offs, nb, T = _layout(S)             # T: a function of the gathered counts, the same on every rank
        dev = p.parts[0].desc.device
        self.bytes_sent.append(T)
        self.wire_bytes.append(int(nb[self.rank].sum()))
        self.payload_bytes.append(int(S[self.rank, :, 4].sum()))
        self.heap_wire_bytes.append(int(S[self.rank, :, 2].sum()))
        released = None
        if dev.type != "cuda":               # host packing (gloo, CPU tensors)
            send = torch.zeros(T, dtype=torch.uint8)
            sv = send.numpy()
            for k, (m, w, pay, _, _) in enumerate(p.enc):
                o = offs[self.rank, k]
                sv[o[0]: o[0] + 4 * len(m)] = np.asarray(m, np.uint32).view(np.uint8)
                sv[o[1]: o[1] + 8 * len(w)] = w.view(np.uint8)
                sv[o[2]: o[2] + len(pay)] = pay
            recv = torch.empty(self.world * T, dtype=torch.uint8)
        elif p.cnt is not None:              # pipelined: pack into the rank's chunk, all-gather in place
            lib = runtime.load_library()
            recv = self._buf("recv", self.world * T, dev)[: self.world * T]
            send = recv[self.rank * T: (self.rank + 1) * T]
            work, wb = self._work(flat, dev)
            mine = np.zeros((len(flat), XCHG_COUNTS), np.uint32)   # overlay parts: no sections (zeros)
            mine[:K] = S[self.rank, :K]
            mine = mine.reshape(-1)
            runtime._check(lib, lib.sdx_exchange_pack_into(
                self._bank(), self._xparts(flat), len(flat), ctypes.c_void_p(work.data_ptr()), wb,
                ctypes.c_void_p(p.cnt.data_ptr()), mine.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(send.data_ptr()),
                T, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
            released = torch.cuda.Event()
            released.record(torch.cuda.current_stream(dev))   # the launches' buffers have been read
        else:
            # gloo with device buffers: the send buffer was sized from THIS rank's capacities, and T is
            # the largest rank's wire (e.g. a peer that re-ran into bigger overlays): grow it to T,
            # keeping the packed bytes, so every rank hands the collective exactly T bytes
            send = self._bufs["send"]
            if send.numel() < T:
                grown = torch.zeros(T + 256, dtype=torch.uint8, device=dev)
                grown[: send.numel()].copy_(send)
                send = self._bufs["send"] = grown
            send = send[:T]
            recv = self._buf("recv", self.world * T, dev)[: self.world * T]
        if send.numel() != T:
            raise ExchangeMismatch(f"exchange: rank {self.rank} would send {send.numel()} bytes, the collective is {T}")
        _all_gather_flat(recv, send, self.group)
        self.last = (recv, S, offs, nb, T, K, [q.kind for q in p.parts])
        return released

    def gathered(self) -> List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        """Per launch (desc, rec, heap) byte tensors of the last completed exchange: the whole job in
        global message order (canonical form; sdx_exchange_unpack on the device)."""
        recv, S, offs, nb, T, K, kinds = self.last
        out = []
        if recv.device.type != "cuda":
            rv = recv.numpy()
            for k in range(K):
                ranks = []
                for r in range(self.world):
                    o = r * T + offs[r, k]
                    ranks.append((rv[o[0]: o[0] + nb[r, k, 0]].view(np.uint32),
                                  rv[o[1]: o[1] + nb[r, k, 1]].view(WIRE_REC_DT), rv[o[2]: o[2] + nb[r, k, 2]]))
                d, rc, h = wire_decode(ranks, self._affix(kinds[k]))
                out.append(tuple(torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()) for a in (d, rc, h)))
            return out
        if self.stream is not None:
            torch.cuda.current_stream(recv.device).wait_stream(self.stream)
        for k in range(K):
            out.append(unpack_device(recv, S[:, k, :], [r * T + offs[r, k] for r in range(self.world)],
                                     self.engine, kinds[k]))
        return out


def unpack_device(recv: torch.Tensor, S: np.ndarray, offs, engine=None, kind: int = KIND_RAW) -> Tuple[torch.Tensor, ...]:
    """sdx_exchange_unpack of one launch: the wire sections of every rank inside ``recv`` (per rank
    r: offsets offs[r] of its msg / rec / heap sections, counts S[r] = (messages, records, wire bytes,
    bad, payload bytes)) -> (desc, rec, heap) byte tensors of the whole job, on the current stream.
    ``engine`` / ``kind``: the sender's bank and launch kind (the nibble form's affixes)."""
    lib = runtime.load_library()
    dev = recv.device
    world = len(offs)
    S = np.asarray(S, np.int64)
    arr = (runtime.SdxXchgWire * world)()
    base = recv.data_ptr()
    for r in range(world):
        o = [int(x) for x in offs[r]]
        arr[r] = runtime.SdxXchgWire(base + o[0], base + o[1], base + o[2], int(S[r, 0]), int(S[r, 1]),
                                     int(S[r, 2]), int(S[r, 4]) if S.shape[1] > 4 else int(S[r, 2]))
    M, R = int(S[:, 0].sum()), int(S[:, 1].sum())
    H = int(S[:, 4].sum()) if S.shape[1] > 4 else int(S[:, 2].sum())
    desc = torch.empty(max(M, 1) * DESC_BYTES, dtype=torch.uint8, device=dev)
    rec = torch.empty(max(R, 1) * REC_BYTES, dtype=torch.uint8, device=dev)
    heap = torch.empty(_r16(max(H, 1)), dtype=torch.uint8, device=dev)
    wb = int(lib.sdx_exchange_unpack_work_bytes(M, R))
    work = torch.zeros(wb + 64, dtype=torch.uint8, device=dev)
    runtime._check(lib, lib.sdx_exchange_unpack(None if engine is None else engine.handle, kind, arr, world,
                                                ctypes.c_void_p(work.data_ptr()), wb,
                                                ctypes.c_void_p(desc.data_ptr()), ctypes.c_void_p(rec.data_ptr()),
                                                ctypes.c_void_p(heap.data_ptr()), heap.numel(),
                                                ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    torch.cuda.current_stream(dev).synchronize()
    return desc[: M * DESC_BYTES], rec[: R * REC_BYTES], heap[:H]


def allgather_streams(parts: Sequence[Any], group=None, engine=None, rerun=None) -> List[Tuple[torch.Tensor, ...]]:
    """One exchange of several launches (e.g. MU, MS, MC), completed at once: per launch (desc,
    rec, heap) of the whole job in global message order (canonical form)."""
    ex = Exchange(group, engine)
    ex.submit(parts, rerun=rerun)
    ex.flush()
    return ex.gathered()


def allgather_results(desc: torch.Tensor, rec: torch.Tensor, heap: torch.Tensor, n_msgs: int, n_rec: int,
                      n_heap: int, group=None):
    """One launch's (desc[n_msgs], rec[n_rec], heap[n_heap]) of every rank (host-known counts)."""
    cur = torch.tensor([n_rec, n_heap, 0, 0], dtype=torch.int32, device=desc.device)
    return allgather_streams([(desc, rec, heap, n_msgs, cur)], group)[0]


# ---- the product entry -------------------------------------------------------------------------------
class _ShardMeta:
    """meta.rssi / MS meta.clock of the whole job's messages for SDProtocols._decode_pulses (each rank
    packed only its own shard): rssi = msg_data.get('R') (message_unsynced.py:287,
    message_synced.py:238), the MS clock = abs(float(P[CP])) (message_synced.py:66-72) derived with the
    packer's own conversions, only for the messages that have results."""

    def __init__(self, messages, kind):
        self.messages, self.kind = messages, kind
        self.rssi = _Lazy(lambda i: messages[i].get("R"))
        self.clock_abs = _Lazy(self._clock)

    def _clock(self, i):
        from . import packing
        pk = packing.PulsePacker(self.kind)
        try:
            pk.add(self.messages[i])
        except packing.GeneralPathMessage:
            pk = packing.GeneralPacker(self.kind)
            pk.add(self.messages[i])
        return pk.clock_abs[0]


class _Lazy:
    __slots__ = ("f",)

    def __init__(self, f):
        self.f = f

    def __getitem__(self, i):
        return self.f(i)


class ShardedDemodulator:
    """BASELINE config 5 as a product entry: a batch is split into contiguous shards,
    one per rank (one process per GPU); every rank demodulates its shard with the launches and the
    GPU re-runs of ``Engine.run`` (overflowed messages re-run into overlays, never dropped), and one
    all-gather of the decoded dmsg buffers (:class:`Exchange`, RCCL over xGMI with the ``nccl``
    backend) gives every rank the whole job's results in global message order.  The reference runs
    one process over one stream (signalduino/controller.py:252); this entry adds the sharding.

    Batch level (synchronous): ``demodulate_batch(messages, msg_type)`` -- the
    ``SDProtocols.demodulate_batch`` contract (one result list, or the exception instance, per
    message) for the WHOLE batch on every rank, each rank demodulating only its shard.

    Device level (pipelined; the bench's step):  ``part = launch(kind, bd, out)`` for this rank's
    device batch, ``submit(parts, stream)`` per step (re-runs happen inside the exchange when any rank
    reports overflowed messages), ``flush()``, ``gathered()``."""

    def __init__(self, protocols=None, group=None, engine=None, defer: bool = False, nibble: bool = True,
                 pipeline: Optional[bool] = None):
        from .sd_protocols import SDProtocols
        self.protocols = protocols if protocols is not None else SDProtocols(mc_mode="fixed")
        self.group = group
        self.defer = defer      # Exchange(defer=...): count + pack behind the next step's ``after`` event
        self.nibble = nibble    # the wire's nibble form (False: raw payloads)
        self.pipeline = pipeline  # Exchange(pipeline=...): None = the overlapped branch with nccl only
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._eng = engine
        self._ex = None

    @property
    def eng(self):
        return self._eng if self._eng is not None else self.protocols._ensure()

    @property
    def exchange(self) -> Exchange:
        want = self.eng if self.nibble else None
        if self._ex is None or self._ex.engine is not want:
            self._ex = Exchange(self.group, want, defer=self.defer, pipeline=self.pipeline)
        return self._ex

    def shard(self, n: int) -> Tuple[int, int]:
        return shard_bounds(n, self.rank, self.world)

    # -- device level -------------------------------------------------------------------------------------
    def launch(self, kind: int, bd, out=None, mn_elig: int = 0, mn_method: int = -1, grouped_sel=None,
               mrec=None) -> Part:
        """The first pass over this rank's device batch (Engine.launch_routed; ``grouped_sel``: a
        grouping computed ahead, as the bench does) into ``out`` (default: Engine.first_pass's
        capacities); no host synchronisation."""
        eng = self.eng
        if out is None:
            out = eng.first_pass(kind, bd, mn_elig=mn_elig, mn_method=mn_method, wire=True)
        elif grouped_sel is not None:
            eng.launch_pulses(kind, bd, out, sel=grouped_sel, group=False, mrec=mrec)
        else:
            eng.launch_routed(kind, bd, out, mn_elig=mn_elig, mn_method=mn_method)
        return Part.from_out(out, kind, src=(kind, bd, mn_elig, mn_method))

    def rerun(self, part: Part) -> Part:
        """The exchange's re-run callback: this rank's overflowed messages of ``part`` (resolved over
        its overlays) re-run on the GPU into one more overlay (Engine.rerun_overlay: the long MU/MS
        variant, the general MC kernel for long frames, grown capacities)."""
        if part.src is None:
            raise RuntimeError("exchange: a launch with overflowed messages and no source batch to re-run")
        kind, bd, mn_elig, mn_method = part.src
        dev = part.desc.device
        torch.cuda.current_stream(dev).synchronize()
        levels = [part] + part.overlays
        _, rd = resolve_host([(q.desc[: q.n * DESC_BYTES].cpu().numpy().view(DESC_DT),) for q in levels])
        redo = np.nonzero(np.isin(rd["status"], OVF))[0].astype(np.int32)
        if not len(redo):
            return part
        lvl = len(part.overlays)
        rcap = max(4096, 256 * len(redo)) << lvl
        hcap = max(1 << 20, 16384 * len(redo)) << lvl
        out2 = self.eng.rerun_overlay(kind, bd, redo, rcap, hcap, mn_elig=mn_elig, mn_method=mn_method)
        part.overlays.append(Part.from_out(out2, kind))
        return part

    def submit(self, parts: Sequence[Part], stream=None, after=None):
        return self.exchange.submit(parts, stream, rerun=self.rerun, after=after)

    def flush(self):
        return self.exchange.flush()

    def gathered(self):
        return self.exchange.gathered()

    def run_device(self, launches: Sequence[Tuple[int, Any]]) -> List[Tuple[np.ndarray, np.ndarray, np.ndarray]]:
        """[(kind, this rank's device batch)] -> per launch the whole job's host (desc, rec, heap) in
        canonical form (synchronous: launch, exchange with re-runs, unpack)."""
        parts = [self.launch(k, bd) for k, bd in launches]
        return self._exchange_host(parts)

    def _exchange_host(self, parts):
        ex = self.exchange
        ex.submit(parts, rerun=self.rerun)
        ex.flush()
        out = []
        for d, r, h in ex.gathered():
            out.append((d.cpu().numpy().view(DESC_DT).copy(), r.cpu().numpy().view(RES_DT).copy(),
                        h.cpu().numpy().copy()))
        return out

    def _host_overlay(self, n: int, rows, kind: int) -> Part:
        """An overlay that marks ``rows`` as RAISED by the host packing (raise_kind RAISE_HOST): the
        receiving ranks re-derive the exception from the message itself."""
        eng = self.eng
        d = np.zeros(max(n, 1), DESC_DT)
        d["status"] = ST_ABSENT
        rows = np.asarray(sorted(rows), np.int64)
        d["status"][rows] = runtime.ST_RAISED
        d["raise_kind"][rows] = RAISE_HOST
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(eng.dev)  # noqa: E731
        return Part(t(d), torch.zeros(REC_BYTES, dtype=torch.uint8, device=eng.dev),
                    torch.zeros(16, dtype=torch.uint8, device=eng.dev), n,
                    torch.zeros(4, dtype=torch.int32, device=eng.dev), kind)

    # -- batch level ----------------------------------------------------------------------------------------
    def demodulate_batch(self, messages: Sequence[Dict[str, Any]], msg_type: str, raise_errors: bool = False):
        """SDProtocols.demodulate_batch over the whole batch on every rank, each rank demodulating its
        contiguous shard (MU, MS; MC in the 'fixed' chain -- the 'strict' chain reaches no device
        launch and runs unsharded)."""
        P = self.protocols
        messages = list(messages)
        if msg_type == "MC":
            if P.mc_mode == "strict":
                return P.demodulate_batch(messages, "MC", raise_errors=raise_errors)
            return self._demodulate_mc(messages, raise_errors)
        if msg_type not in ("MU", "MS"):
            return P.demodulate_batch(messages, msg_type, raise_errors=raise_errors)
        from . import packing
        eng = self.eng
        kind = runtime.KIND_MU if msg_type == "MU" else runtime.KIND_MS
        lo, hi = self.shard(len(messages))
        mine = messages[lo:hi]
        packer, gen, gen_rows, pack_err = P._pack_pulses(mine, msg_type, raise_errors=False)
        bd = eng.to_device_pulses(packer.batch())
        part = self.launch(kind, bd)
        if gen_rows:   # the general path's results as an overlay indexed like the launch
            genall = packing.GeneralPacker(msg_type)
            gset = set(gen_rows)
            for i, m in enumerate(mine):
                genall.add(m if i in gset else {"data": ""})
            ov = eng.general_overlay(kind, eng.to_device_general(genall.arrays()), np.asarray(gen_rows, np.int32))
            part.overlays.append(Part.from_out(ov, kind))
        if pack_err:
            part.overlays.append(self._host_overlay(len(mine), pack_err.keys(), kind))
        desc, rec, heap = self._exchange_host([part])[0]
        errs = self._host_errors(messages, desc, lambda m: P._pack_error(m, msg_type))
        return P._decode_pulses(msg_type, desc, rec, heap, _ShardMeta(messages, msg_type), errs, raise_errors)

    @staticmethod
    def _host_errors(messages, desc, derive):
        rows = np.nonzero((desc["status"] == runtime.ST_RAISED) & (desc["raise_kind"] == RAISE_HOST))[0]
        return {int(i): derive(messages[int(i)]) for i in rows}

    def _demodulate_mc(self, messages, raise_errors):
        P = self.protocols
        eng = self.eng
        lo, hi = self.shard(len(messages))
        frames, slot_err, only = P._mc_frames(messages[lo:hi], "MC", None, raise_errors=False)
        bd = eng.to_device_mc(packing_mc(frames))
        if any(only):
            bd["only"] = P._mc_only(only, eng)
        part = self.launch(runtime.KIND_MC, bd)
        if slot_err:
            part.overlays.append(self._host_overlay(hi - lo, slot_err.keys(), runtime.KIND_MC))
        desc, rec, heap = self._exchange_host([part])[0]
        errs = self._host_errors(messages, desc, lambda m: P._mc_frame_error(m, "MC"))
        return P._decode_mc(desc, rec, heap, errs, raise_errors)


def packing_mc(frames):
    from . import packing
    return packing.mc_batch_from_frames(frames)
