"""Multi-GPU: contiguous message shards per rank + all-gather of the decoded dmsg buffers.

Messages are independent: each rank demodulates its contiguous shard with no
communication during compute.  The one exchange step gathers every rank's results so that every
rank holds the whole stream's results in global message order (BASELINE config 5).

What travels is the WIRE form of include/sdx.h, per launch and rank, in message order:
  msg  section  u32 per message = n_rec | status << 16 | raise_kind << 24
  rec  section  8 B per record  = proto, payload_len, bit_length
  heap section  the payloads concatenated in record order, zero-padded to 16 bytes
rec_begin, payload_off and msg are prefix sums and are rebuilt by the receiver
(``sdx_exchange_unpack``), so a message costs 4 + 8 * records + payload bytes on the wire instead of
8 + 16 * records + the launch's padded heap.  The wire is also canonical: the bytes do not depend
on the order in which tiles wrote their records, so a sharded run and an un-sharded run compare
byte for byte (tests/test_dist.py).

With the ``nccl`` backend (RCCL over xGMI on ROCm) the buffers stay in HBM and the exchange runs on
its own HIP stream (:class:`Exchange`), overlapped with the next step's kernels:
  step k kernels ─ready_k─▶ [exchange stream] sdx_exchange_count_k ─ all-gather counts_k ─ D2H
  submit(k+1): host waits for counts_k (the GPU runs step k+1 meanwhile), sizes the sections (max
               over ranks), enqueues sdx_exchange_pack_into_k (this rank's chunk of the receive
               buffer) ─released_k─ in-place all-gather data_k, and only then the wait on ready_{k+1}
               and step k+1's count: step k's pack and collective never wait for step k+1's kernels.
The same protocol runs synchronously on ``gloo`` (CPU tensors: numpy packing; CUDA tensors: the
device kernels, the collective staged through host memory).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import runtime
from .runtime import DESC_DT, RES_DT, WIRE_REC_DT

DESC_BYTES = 8
REC_BYTES = 16
WIRE_MSG_BYTES = 4
WIRE_REC_BYTES = 8


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of ``n`` messages owned by ``rank`` (sizes differ by at most 1)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _r16(x):
    return (x + 15) // 16 * 16


# ---- host (numpy) form of the wire: CPU tensors on gloo, and the checker of the device kernels ----
def wire_encode(desc: np.ndarray, rec: np.ndarray, heap: np.ndarray, nrec_written: Optional[int] = None,
                nheap_written: Optional[int] = None):
    """One launch's host (desc, rec, heap) -> (msg u32[n], wire records, payload bytes, bad count),
    with the validation rules of k_xw_count (a record or payload outside what the launch wrote makes
    its message "bad": shipped with n_rec 0 and status ST_OVF_OUT)."""
    nrec_c = len(rec) if nrec_written is None else min(nrec_written, len(rec))
    nheap_c = len(heap) if nheap_written is None else min(nheap_written, len(heap))
    n = len(desc)
    msg = np.zeros(n, np.uint32)
    recs, pays, bad = [], [], 0
    hb = np.asarray(heap, np.uint8)
    for m in range(n):
        d = desc[m]
        st, nr, rb = int(d["status"]), int(d["n_rec"]), int(d["rec_begin"])
        if st == runtime.ST_RAISED:
            msg[m] = (st << 16) | (int(d["raise_kind"]) << 24)
            continue
        ok = st == runtime.ST_OK and (nr == 0 or rb + nr <= nrec_c)
        if ok:
            rs = rec[rb: rb + nr]
            ok = bool(np.all(rs["msg"] == m)) and bool(np.all(rs["payload_off"].astype(np.int64)
                                                              + rs["payload_len"] <= nheap_c))
        if not ok:
            bad += 1
            msg[m] = (runtime.ST_OVF_OUT << 16) | (int(d["raise_kind"]) << 24)
            continue
        msg[m] = nr | (st << 16) | (int(d["raise_kind"]) << 24)
        for r in rs:
            recs.append((int(r["proto"]), int(r["payload_len"]), int(r["bit_length"])))
            pays.append(hb[int(r["payload_off"]): int(r["payload_off"]) + int(r["payload_len"])])
    wrec = np.array(recs, WIRE_REC_DT) if recs else np.zeros(0, WIRE_REC_DT)
    pay = np.concatenate(pays) if pays else np.zeros(0, np.uint8)
    return msg, wrec, pay.astype(np.uint8), bad


def wire_decode(ranks: Sequence[Tuple[np.ndarray, np.ndarray, np.ndarray]]):
    """Wire sections of every rank (rank order) -> the whole job's (desc, rec, heap), as
    sdx_exchange_unpack builds them."""
    msg = np.concatenate([np.asarray(m, np.uint32) for m, _, _ in ranks]) if ranks else np.zeros(0, np.uint32)
    wrec = np.concatenate([w for _, w, _ in ranks]) if ranks else np.zeros(0, WIRE_REC_DT)
    heap = np.concatenate([np.asarray(p, np.uint8) for _, _, p in ranks]) if ranks else np.zeros(0, np.uint8)
    n = len(msg)
    desc = np.zeros(n, DESC_DT)
    nrec = (msg & 0xFFFF).astype(np.int64)
    desc["n_rec"] = nrec
    desc["status"] = (msg >> 16) & 0xFF
    desc["raise_kind"] = msg >> 24
    desc["rec_begin"] = np.concatenate([[0], np.cumsum(nrec)[:-1]]) if n else np.zeros(0, np.int64)
    rec = np.zeros(len(wrec), RES_DT)
    rec["proto"] = wrec["proto"]
    rec["payload_len"] = wrec["payload_len"]
    rec["bit_length"] = wrec["bit_length"]
    pl = wrec["payload_len"].astype(np.int64)
    rec["payload_off"] = np.concatenate([[0], np.cumsum(pl)[:-1]]) if len(pl) else np.zeros(0, np.int64)
    rec["msg"] = np.repeat(np.arange(n, dtype=np.int64), nrec)
    return desc, rec, heap


def canonical(desc: np.ndarray, rec: np.ndarray, heap: np.ndarray):
    """A launch's host outputs in canonical form: records in message order, payloads packed.  The
    exchange delivers exactly this (for the whole job); the tests compare against it."""
    m, w, p, bad = wire_encode(desc, rec, heap)
    if bad:
        raise ValueError(f"{bad} messages overflowed: re-run before comparing")
    return wire_decode([(m, w, p)])


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


def _layout(S: np.ndarray):
    """S[world, K, 4] = (messages, records, payload bytes, bad) -> per rank the section offsets
    [world, K, 3] of its send buffer (launch 0, 1, ...: msg, rec, heap sections, each padded to 16
    bytes -- the layout k_xw_count computes on the device), the section byte counts [world, K, 3]
    and the collective's per-rank size T (the largest rank's buffer)."""
    S = np.asarray(S, np.int64)
    nb = np.stack([S[..., 0] * WIRE_MSG_BYTES, S[..., 1] * WIRE_REC_BYTES, S[..., 2]], axis=-1)
    sizes = _r16(nb).reshape(S.shape[0], -1)                                     # [world, K*3]
    offs = np.concatenate([np.zeros((S.shape[0], 1), np.int64), np.cumsum(sizes, axis=1)[:, :-1]], axis=1)
    T = int(max(16, sizes.sum(axis=1).max()))
    return offs.reshape(S.shape[0], S.shape[1], 3), nb, T


def _part_tuple(p):
    """(desc u8, rec u8, heap u8, n_msgs, cursor) -> the same plus rec_cap / heap_cap from the sizes."""
    desc, rec, heap, n, cur = p
    return desc, rec, heap, int(n), cur, rec.numel() // REC_BYTES, heap.numel()


class _Pending:
    __slots__ = ("parts", "counts_host", "event", "enc", "cnt")

    def __init__(self, parts, counts_host, event, enc=None, cnt=None):
        self.parts, self.counts_host, self.event, self.enc, self.cnt = parts, counts_host, event, enc, cnt


class Exchange:
    """All-gather of the decoded dmsg buffers of K launches per step, pipelined.

    ``submit(parts, stream)`` is called after the step's kernels are enqueued on ``stream``
    (``parts``: per launch (desc u8, rec u8, heap u8, n_msgs, cursor), cursor[0] = records, cursor[1]
    = heap bytes, left on the device; the capacities are the buffers' sizes).  It first completes
    the PREVIOUS step's exchange (the data all-gather: its counts arrived while this step's kernels
    were running) and then enqueues this step's count + pack + count all-gather behind this step's
    kernels.  It returns the event after which the PREVIOUS step's output buffers may be overwritten
    (its pack has read them; None on the first call): with the nccl backend a step is packed once its
    counts are on the host, straight into this rank's chunk of the receive buffer, and all-gathered in
    place (no send buffer, no local copy), so double-buffer the outputs.  ``flush()`` completes the
    last step and returns the same event for it.  ``gathered()`` gives the last completed step's results as
    per launch (desc, rec, heap) byte tensors of the whole job in global message order.

    A launch with overflowed messages (the counts' "bad" column) makes every rank raise in the
    completing call: overflowed results are re-run, never exchanged."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.pending: Optional[_Pending] = None
        self.stream = None
        self._bufs = {}
        self.last = None        # (recv, S, offs, nb, T) of the last completed exchange
        self.bytes_sent = []    # per completed step: the collective's bytes per rank (T)
        self.wire_bytes = []    # per completed step: this rank's wire bytes before padding

    def _buf(self, name, n, dev, zero=False):
        b = self._bufs.get(name)
        if b is None or b.numel() < n or b.device != dev:
            n2 = max(n, 64) + 256
            b = self._bufs[name] = (torch.zeros if zero else torch.empty)(n2, dtype=torch.uint8, device=dev)
        return b

    # -- device path ----------------------------------------------------------------------------------
    @staticmethod
    def _xparts(parts):
        arr = (runtime.SdxXchgPart * len(parts))()
        for k, (desc, rec, heap, n, cur, rcap, hcap) in enumerate(parts):
            arr[k] = runtime.SdxXchgPart(desc.data_ptr(), rec.data_ptr(), heap.data_ptr(), cur.data_ptr(), n, rcap,
                                         hcap, 0)
        return arr

    def _work(self, parts, dev):
        lib = runtime.load_library()
        ns = (ctypes.c_uint32 * len(parts))(*[p[3] for p in parts])
        wb = int(lib.sdx_exchange_work_bytes(ns, len(parts)))
        # one zeroed workspace per launch layout: the kernels keep its counters at zero between uses
        w = self._buf(("work",) + tuple(ns), wb + 256, dev, zero=True)
        off = (-w.data_ptr()) % 256
        return w[off:], wb

    def _count_device(self, parts, stream):
        """sdx_exchange_count on `stream`: [K*4] int32 device counts (the pack follows once the host
        has them: _complete, sdx_exchange_pack_into)."""
        lib = runtime.load_library()
        dev = parts[0][0].device
        work, wb = self._work(parts, dev)
        cnt = torch.empty(4 * len(parts), dtype=torch.int32, device=dev)
        runtime._check(lib, lib.sdx_exchange_count(self._xparts(parts), len(parts), ctypes.c_void_p(work.data_ptr()), wb,
                                                   ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(stream.cuda_stream)))
        return cnt

    def _count_pack_device(self, parts, stream):
        """sdx_exchange_count + sdx_exchange_pack on `stream`: [K*4] int32 device counts; the wire
        form of this rank is in the "send" buffer (layout: _layout)."""
        lib = runtime.load_library()
        dev = parts[0][0].device
        work, wb = self._work(parts, dev)
        xp = self._xparts(parts)
        cnt = torch.empty(4 * len(parts), dtype=torch.int32, device=dev)
        sp = ctypes.c_void_p(stream.cuda_stream)
        runtime._check(lib, lib.sdx_exchange_count(xp, len(parts), ctypes.c_void_p(work.data_ptr()), wb,
                                                   ctypes.c_void_p(cnt.data_ptr()), sp))
        cap = int(lib.sdx_exchange_send_bytes(xp, len(parts)))
        send = self._buf("send", cap, dev)
        runtime._check(lib, lib.sdx_exchange_pack(xp, len(parts), ctypes.c_void_p(work.data_ptr()), wb,
                                                  ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(send.data_ptr()),
                                                  send.numel(), sp))
        return cnt

    # -- host path (CPU tensors) ------------------------------------------------------------------------
    @staticmethod
    def _encode_host(parts):
        out = []
        for desc, rec, heap, n, cur, rcap, hcap in parts:
            d = desc[: n * DESC_BYTES].numpy().view(DESC_DT)
            r = rec[: rcap * REC_BYTES].numpy().view(RES_DT)
            out.append(wire_encode(d, r, heap.numpy(), int(cur[0]), int(cur[1])))
        return out

    # -- protocol ----------------------------------------------------------------------------------------
    def submit(self, parts, stream=None):
        parts = [_part_tuple(p) for p in parts]
        K = len(parts)
        dev = parts[0][0].device
        overlap = dev.type == "cuda" and dist.get_backend(self.group) == "nccl"
        if not overlap:   # synchronous form: gloo (CPU tensors, or CUDA tensors staged through the host)
            if dev.type == "cuda":
                stream = stream or torch.cuda.current_stream(dev)
                with torch.cuda.stream(stream):
                    cnt = self._count_pack_device(parts, stream)
                    allc = torch.empty(self.world * K * 4, dtype=torch.int32, device=dev)
                    _all_gather_flat(allc, cnt, self.group)
                    self._complete(_Pending(parts, allc.cpu(), None))
            else:
                enc = self._encode_host(parts)
                cnt = torch.tensor([[len(m), len(w), len(p), b] for m, w, p, b in enc], dtype=torch.int32).reshape(-1)
                allc = torch.empty(self.world * K * 4, dtype=torch.int32)
                _all_gather_flat(allc, cnt, self.group)
                self._complete(_Pending(parts, allc, None, enc))
            return None
        if self.stream is None:
            self.stream = torch.cuda.Stream(dev)
        stream = stream or torch.cuda.current_stream(dev)
        # 1. the previous step: its counts are (about to be) on the host -- pack it into its chunk of
        #    the receive buffer and all-gather in place, ahead of anything that waits for this step
        prev, self.pending = self.pending, None
        released = None
        if prev is not None:
            with torch.cuda.stream(self.stream):
                released = self._complete(prev)
        # 2. this step: count + count all-gather + counts to the host, behind this step's kernels
        ready = torch.cuda.Event()
        ready.record(stream)
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ready)
            cnt = self._count_device(parts, self.stream)
            allc = torch.empty(self.world * K * 4, dtype=torch.int32, device=dev)
            _all_gather_flat(allc, cnt, self.group)
            host = torch.empty(allc.numel(), dtype=torch.int32, pin_memory=True)
            host.copy_(allc, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.pending = _Pending(parts, host, ev, cnt=cnt)
        return released

    def flush(self):
        """Completes the last submitted step; returns the event after which its output buffers may
        be overwritten (None when nothing was pending)."""
        prev, self.pending = self.pending, None
        if prev is None:
            return None
        with torch.cuda.stream(self.stream):
            return self._complete(prev)

    def _complete(self, p: _Pending):
        """The data collective of a step whose counts are on (or on their way to) the host; device
        buffers: on the current stream.  nccl: the step is packed here (sdx_exchange_pack_into) into
        this rank's chunk of the receive buffer and gathered in place; returns the event after which
        the step's output buffers may be overwritten."""
        K = len(p.parts)
        if p.event is not None:
            p.event.synchronize()            # the counts (the GPU has moved on to the next step)
        S = p.counts_host.numpy().astype(np.int64).reshape(self.world, K, 4)
        if S[..., 3].any():
            bad = {(r, k): int(S[r, k, 3]) for r in range(self.world) for k in range(K) if S[r, k, 3]}
            raise RuntimeError(f"exchange: overflowed messages in (rank, launch) {bad}; re-run them before exchanging")
        offs, nb, T = _layout(S)
        dev = p.parts[0][0].device
        self.bytes_sent.append(T)
        self.wire_bytes.append(int(nb[self.rank].sum()))
        released = None
        if dev.type != "cuda":               # host packing (gloo, CPU tensors)
            send = torch.zeros(T, dtype=torch.uint8)
            sv = send.numpy()
            for k, (m, w, pay, _) in enumerate(p.enc):
                o = offs[self.rank, k]
                sv[o[0]: o[0] + 4 * len(m)] = np.asarray(m, np.uint32).view(np.uint8)
                sv[o[1]: o[1] + 8 * len(w)] = w.view(np.uint8)
                sv[o[2]: o[2] + len(pay)] = pay
            recv = torch.empty(self.world * T, dtype=torch.uint8)
        elif p.cnt is not None:              # nccl: pack into the rank's chunk, all-gather in place
            lib = runtime.load_library()
            recv = self._buf("recv", self.world * T, dev)[: self.world * T]
            send = recv[self.rank * T: (self.rank + 1) * T]
            work, wb = self._work(p.parts, dev)
            mine = np.ascontiguousarray(S[self.rank].reshape(-1).astype(np.uint32))
            runtime._check(lib, lib.sdx_exchange_pack_into(
                self._xparts(p.parts), K, ctypes.c_void_p(work.data_ptr()), wb, ctypes.c_void_p(p.cnt.data_ptr()),
                mine.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(send.data_ptr()), T,
                ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
            released = torch.cuda.Event()
            released.record(torch.cuda.current_stream(dev))   # the launches' buffers have been read
        else:
            send = self._bufs["send"][:T]
            recv = self._buf("recv", self.world * T, dev)[: self.world * T]
        _all_gather_flat(recv, send, self.group)
        self.last = (recv, S, offs, nb, T)
        return released

    def gathered(self) -> List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        """Per launch (desc, rec, heap) byte tensors of the last completed exchange: the whole job in
        global message order (canonical form; sdx_exchange_unpack on the device)."""
        recv, S, offs, nb, T = self.last
        out = []
        if recv.device.type != "cuda":
            rv = recv.numpy()
            for k in range(S.shape[1]):
                ranks = []
                for r in range(self.world):
                    o = r * T + offs[r, k]
                    ranks.append((rv[o[0]: o[0] + nb[r, k, 0]].view(np.uint32),
                                  rv[o[1]: o[1] + nb[r, k, 1]].view(WIRE_REC_DT), rv[o[2]: o[2] + nb[r, k, 2]]))
                d, rc, h = wire_decode(ranks)
                out.append(tuple(torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()) for a in (d, rc, h)))
            return out
        if self.stream is not None:
            torch.cuda.current_stream(recv.device).wait_stream(self.stream)
        for k in range(S.shape[1]):
            out.append(unpack_device(recv, S[:, k, :3], [r * T + offs[r, k] for r in range(self.world)]))
        return out


def unpack_device(recv: torch.Tensor, S: np.ndarray, offs) -> Tuple[torch.Tensor, ...]:
    """sdx_exchange_unpack of one launch: the wire sections of every rank inside ``recv`` (per rank
    r: offsets offs[r] of its msg / rec / heap sections, counts S[r] = (messages, records, bytes))
    -> (desc, rec, heap) byte tensors of the whole job, on the current stream."""
    lib = runtime.load_library()
    dev = recv.device
    world = len(offs)
    arr = (runtime.SdxXchgWire * world)()
    base = recv.data_ptr()
    for r in range(world):
        o = [int(x) for x in offs[r]]
        arr[r] = runtime.SdxXchgWire(base + o[0], base + o[1], base + o[2], int(S[r, 0]), int(S[r, 1]),
                                     int(S[r, 2]), 0)
    M, R, H = (int(S[:, j].sum()) for j in range(3))
    desc = torch.empty(max(M, 1) * DESC_BYTES, dtype=torch.uint8, device=dev)
    rec = torch.empty(max(R, 1) * REC_BYTES, dtype=torch.uint8, device=dev)
    heap = torch.empty(_r16(max(H, 1)), dtype=torch.uint8, device=dev)
    wb = int(lib.sdx_exchange_unpack_work_bytes(M, R))
    work = torch.zeros(wb + 64, dtype=torch.uint8, device=dev)
    runtime._check(lib, lib.sdx_exchange_unpack(arr, world, ctypes.c_void_p(work.data_ptr()), wb,
                                                ctypes.c_void_p(desc.data_ptr()), ctypes.c_void_p(rec.data_ptr()),
                                                ctypes.c_void_p(heap.data_ptr()),
                                                ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
    torch.cuda.current_stream(dev).synchronize()
    return desc[: M * DESC_BYTES], rec[: R * REC_BYTES], heap[:H]


def allgather_streams(parts: Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor, int, torch.Tensor]],
                      group=None) -> List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
    """One exchange of several launches (e.g. MU, MS, MC), completed at once: per launch (desc,
    rec, heap) of the whole job in global message order (canonical form)."""
    ex = Exchange(group)
    ex.submit(parts)
    ex.flush()
    return ex.gathered()


def allgather_results(desc: torch.Tensor, rec: torch.Tensor, heap: torch.Tensor, n_msgs: int, n_rec: int,
                      n_heap: int, group=None):
    """One launch's (desc[n_msgs], rec[n_rec], heap[n_heap]) of every rank (host-known counts)."""
    cur = torch.tensor([n_rec, n_heap, 0, 0], dtype=torch.int32, device=desc.device)
    return allgather_streams([(desc, rec, heap, n_msgs, cur)], group)[0]
