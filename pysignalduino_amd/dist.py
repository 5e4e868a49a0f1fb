"""Multi-GPU: contiguous message shards per rank + all-gather of the decoded dmsg buffers.

Messages are independent: each rank demodulates its contiguous shard with no
communication during compute.  The one exchange step gathers every rank's result buffers
(descriptors, result records, payload heap) so that every rank holds the whole stream's results
in global message order (BASELINE config 5).  With the ``nccl`` backend (RCCL over xGMI on ROCm)
the buffers stay in HBM and the exchange runs on its own HIP stream, overlapped with the next
step's kernels (:class:`Exchange`); the same protocol runs on ``gloo`` with CPU tensors
(tests/test_dist.py).

Per exchange:
  1. one all-gather of every rank's counts (messages, records, heap bytes per launch), read from
     the launches' device cursors on the exchange stream;
  2. the host reads those counts one step later -- while the GPU runs the next step -- and sizes
     the sections (max over ranks, 16-byte aligned);
  3. ``sdx_exchange_pack`` (csrc/sdx_exchange.hip) copies the rank's K launches into one send buffer,
     re-basing rec_begin / payload_off / msg by the counts of the lower ranks;
  4. ONE all-gather moves the packed buffers; receivers only drop the per-rank padding.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

DESC_BYTES = 8
REC_BYTES = 16


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of ``n`` messages owned by ``rank`` (sizes differ by at most 1)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _all_gather_flat(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """all_gather into one contiguous tensor.  The collective is chosen once from the backend:
    RCCL's all_gather_into_tensor, the list form on gloo -- every rank issues the same one."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
    else:
        dist.all_gather(list(out.chunk(dist.get_world_size(group))), inp, group=group)


def _layout(S: np.ndarray, rank: int):
    """S[world, K, 3] = (messages, records, heap bytes) -> section sizes, offsets, bases."""
    nb = S * np.array([DESC_BYTES, REC_BYTES, 1], np.int64)                    # bytes per section
    cap = np.maximum((nb.max(axis=0) + 15) // 16 * 16, 16)                      # [K, 3]
    sec_off = np.concatenate([[0], np.cumsum(cap.reshape(-1))]).astype(np.int64)
    base = S[:rank].sum(axis=0) if rank else np.zeros(S.shape[1:], np.int64)  # lower ranks' counts
    return nb, sec_off, int(sec_off[-1]), base


def _pack_torch(parts, S, rank, sec_off, base, send):
    """The packing step with torch ops (CPU tensors, gloo)."""
    for k, (desc, rec, heap, _, _) in enumerate(parts):
        nm, nr, nh = (int(x) for x in S[rank, k])
        o_d, o_r, o_h = (int(sec_off[3 * k + j]) for j in range(3))
        if nm:
            send[o_d: o_d + nm * DESC_BYTES] = desc[: nm * DESC_BYTES]
            send[o_d: o_d + nm * DESC_BYTES].view(torch.int32).view(nm, 2)[:, 0] += int(base[k, 1])
        if nr:
            send[o_r: o_r + nr * REC_BYTES] = rec[: nr * REC_BYTES]
            rv = send[o_r: o_r + nr * REC_BYTES].view(torch.int32).view(nr, 4)
            rv[:, 0] += int(base[k, 2])
            rv[:, 3] += int(base[k, 0])
        if nh:
            send[o_h: o_h + nh] = heap[:nh]


def _pack_device(parts, S, rank, sec_off, base, send, stream):
    """The packing step on the GPU: one sdx_exchange_pack launch for all K launches."""
    from . import runtime
    lib = runtime.load_library()
    K = len(parts)
    arr = (runtime.SdxXchgPart * K)()
    for k, (desc, rec, heap, _, _) in enumerate(parts):
        nm, nr, nh = (int(x) for x in S[rank, k])
        arr[k] = runtime.SdxXchgPart(desc.data_ptr(), rec.data_ptr(), heap.data_ptr(), nm, nr, nh,
                                     int(base[k, 0]), int(base[k, 1]), int(base[k, 2]),
                                     int(sec_off[3 * k]), int(sec_off[3 * k + 1]), int(sec_off[3 * k + 2]))
    runtime._check(lib, lib.sdx_exchange_pack(arr, K, ctypes.c_void_p(send.data_ptr()),
                                              ctypes.c_void_p(stream.cuda_stream)))


class _Pending:
    __slots__ = ("parts", "counts_host", "event", "S")

    def __init__(self, parts, counts_host, event):
        self.parts, self.counts_host, self.event, self.S = parts, counts_host, event, None


class Exchange:
    """All-gather of the decoded dmsg buffers of K launches per step, pipelined.

    ``submit(parts, stream)`` is called after the step's kernels are enqueued on ``stream``
    (``parts``: per launch (desc u8, rec u8, heap u8, n_msgs, cursor), cursor[0] = records,
    cursor[1] = heap bytes, left on the device).  It enqueues the count all-gather of this step on
    the exchange stream and completes the PREVIOUS step's exchange (pack + data all-gather),
    whose counts arrived while this step's kernels were running.  It returns the event after
    which the previous step's buffers may be overwritten (double-buffer the outputs).  ``flush()``
    completes the last step.  ``gathered()`` gives the last completed step's results as per
    launch (desc, rec, heap) of the whole job in global message order.

    On gloo / CPU tensors every call completes synchronously (same protocol, torch-op packing)."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.pending: Optional[_Pending] = None
        self.stream = None
        self._bufs = {}
        self._ns = {}      # device copies of the launches' message counts
        self.last = None   # (recv, S, nb, sec_off, total) of the last completed exchange

    def _buf(self, name, n, dev):
        b = self._bufs.get(name)
        if b is None or b.numel() < n or b.device != dev:
            b = self._bufs[name] = torch.empty(max(n, 16), dtype=torch.uint8, device=dev)
        return b[:n]

    def _counts(self, parts):
        """(messages, records, heap bytes) per launch, flat, on the device.  The message counts are
        host-known; their device copy is made once per distinct set and cached, because a fresh
        ``torch.tensor(..., device=cuda)`` is a blocking copy on the current (exchange) stream,
        which waits for the step's kernels and stalls the host's enqueue of the next step."""
        dev = parts[0][0].device
        ns = tuple(int(n) for _, _, _, n, _ in parts)
        key = (str(dev), ns)
        nd = self._ns.get(key)
        if nd is None:
            nd = self._ns[key] = torch.tensor(ns, dtype=torch.int64).to(dev)
        cur = torch.stack([c[:2] for _, _, _, _, c in parts]).to(torch.int64)   # [K, 2]
        return torch.cat([nd.view(-1, 1), cur], dim=1).reshape(-1)

    def submit(self, parts, stream=None):
        parts = list(parts)
        K = len(parts)
        dev = parts[0][0].device
        overlap = dev.type == "cuda" and dist.get_backend(self.group) == "nccl"
        if not overlap:
            allc = torch.empty(self.world * K * 3, dtype=torch.int64, device=dev)
            _all_gather_flat(allc, self._counts(parts), self.group)
            self._complete(_Pending(parts, allc.cpu(), None))
            return None
        if self.stream is None:
            self.stream = torch.cuda.Stream(dev)
        stream = stream or torch.cuda.current_stream(dev)
        ready = torch.cuda.Event()
        ready.record(stream)
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ready)
            allc = torch.empty(self.world * K * 3, dtype=torch.int64, device=dev)
            _all_gather_flat(allc, self._counts(parts), self.group)
            host = torch.empty(allc.numel(), dtype=torch.int64, pin_memory=True)
            host.copy_(allc, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        prev, self.pending = self.pending, _Pending(parts, host, ev)
        return self._complete(prev) if prev is not None else None

    def flush(self):
        prev, self.pending = self.pending, None
        return self._complete(prev) if prev is not None else None

    def _complete(self, p: _Pending):
        K = len(p.parts)
        if p.event is not None:
            p.event.synchronize()            # the counts (the GPU has moved on to the next step)
        S = p.counts_host.numpy().reshape(self.world, K, 3).astype(np.int64)
        nb, sec_off, total, base = _layout(S, self.rank)
        dev = p.parts[0][0].device
        if p.event is None:
            send = torch.zeros(total, dtype=torch.uint8, device=dev)
            _pack_torch(p.parts, S, self.rank, sec_off, base, send)
            recv = torch.empty(self.world * total, dtype=torch.uint8, device=dev)
            _all_gather_flat(recv, send, self.group)
            self.last = (recv, S, nb, sec_off, total)
            return None
        with torch.cuda.stream(self.stream):
            send = self._buf("send", total, dev)
            _pack_device(p.parts, S, self.rank, sec_off, base, send, self.stream)
            recv = self._buf("recv", self.world * total, dev)
            _all_gather_flat(recv, send, self.group)
            done = torch.cuda.Event()
            done.record(self.stream)
        self.last = (recv, S, nb, sec_off, total)
        return done

    def gathered(self) -> List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        """Per launch (desc, rec, heap) of the last completed exchange, whole job, global order."""
        recv, S, nb, sec_off, total = self.last
        if self.stream is not None:
            self.stream.synchronize()
        out = []
        for k in range(S.shape[1]):
            secs = []
            for j in range(3):
                o = int(sec_off[3 * k + j])
                secs.append(torch.cat([recv[r * total + o: r * total + o + int(nb[r, k, j])]
                                       for r in range(self.world)]))
            out.append(tuple(secs))
        return out


def allgather_streams(parts: Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor, int, torch.Tensor]],
                      group=None) -> List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
    """One exchange of several launches (e.g. MU, MS, MC), completed at once: per launch (desc,
    rec, heap) of the whole job in global message order, with rec_begin / payload_off / msg
    re-based to the concatenation."""
    ex = Exchange(group)
    ex.submit(parts)
    ex.flush()
    return ex.gathered()


def allgather_results(desc: torch.Tensor, rec: torch.Tensor, heap: torch.Tensor, n_msgs: int, n_rec: int,
                      n_heap: int, group=None):
    """One launch's (desc[n_msgs], rec[n_rec], heap[n_heap]) of every rank (host-known counts)."""
    cur = torch.tensor([n_rec, n_heap, 0, 0], dtype=torch.int32, device=desc.device)
    return allgather_streams([(desc, rec, heap, n_msgs, cur)], group)[0]
