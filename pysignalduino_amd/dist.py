"""Multi-GPU: contiguous message shards per rank + all-gather of the decoded dmsg buffers.

Messages are independent: each rank demodulates its contiguous shard
with no communication, then ONE exchange step gathers every rank's result buffers
(descriptors, result records, payload heap) so that every rank holds the whole stream's
results in global message order.  With the ``nccl`` backend (RCCL over xGMI on ROCm) the
buffers stay in HBM; the same code runs on ``gloo`` with CPU tensors (tests/test_dist.py).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

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
    """all_gather into one contiguous tensor (one collective; list form where the backend lacks it)."""
    try:
        dist.all_gather_into_tensor(out, inp, group=group)
    except (RuntimeError, NotImplementedError, AttributeError):
        dist.all_gather(list(out.chunk(dist.get_world_size(group))), inp, group=group)


def allgather_streams(parts: Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor, int, torch.Tensor]],
                      group=None) -> List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
    """Gather the result buffers of several demodulation launches (e.g. MU, MS, MC) in ONE exchange.

    ``parts``: per launch (desc u8, rec u8, heap u8, n_msgs, cursor) with ``cursor`` the launch's
    device cursor (cursor[0] = records, cursor[1] = heap bytes): the counts stay on the device.
    Steps: one all-gather of every rank's counts (the only host synchronisation), then every rank
    packs its sections into one buffer -- re-basing its own rec_begin / payload_off / msg by the
    counts of the lower ranks while copying -- and ONE all-gather moves all of it; the receivers
    only drop the per-rank padding.  Returns per launch (desc, rec, heap) of the whole job in
    global message order (the contract of :func:`allgather_results`).
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    K = len(parts)
    dev = parts[0][0].device
    counts = torch.stack([torch.stack([torch.tensor(n, dtype=torch.int64, device=dev), cur[0].to(torch.int64),
                                       cur[1].to(torch.int64)]) for _, _, _, n, cur in parts])  # [K, 3]
    allc = torch.empty(world * K * 3, dtype=torch.int64, device=dev)
    _all_gather_flat(allc, counts.reshape(-1), group)
    S = allc.view(world, K, 3).cpu()
    nb = S * torch.tensor([DESC_BYTES, REC_BYTES, 1], dtype=torch.int64)        # section bytes
    cap = ((nb.max(dim=0).values + 15) // 16 * 16).clamp(min=16)                # [K, 3]
    sec_off = torch.cumsum(torch.cat([torch.zeros(1, dtype=torch.int64), cap.reshape(-1)]), 0)
    total = int(sec_off[-1])
    base = S[:rank].sum(dim=0) if rank else torch.zeros(K, 3, dtype=torch.int64)  # (msgs, recs, heap) below
    send = torch.zeros(total, dtype=torch.uint8, device=dev)
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
    recv = torch.empty(world * total, dtype=torch.uint8, device=dev)
    _all_gather_flat(recv, send, group)
    out = []
    for k in range(K):
        secs = []
        for j in range(3):
            o = int(sec_off[3 * k + j])
            secs.append(torch.cat([recv[r * total + o: r * total + o + int(nb[r, k, j])] for r in range(world)]))
        out.append(tuple(secs))
    return out


def allgather_results(desc: torch.Tensor, rec: torch.Tensor, heap: torch.Tensor, n_msgs: int, n_rec: int,
                      n_heap: int, group=None):
    """Gather every rank's (desc[n_msgs], rec[n_rec], heap[n_heap]) byte buffers.

    Returns (desc, rec, heap) uint8 tensors of the whole job in global message order, with
    rec_begin / payload_off / msg re-based to the concatenation.
    """
    world = dist.get_world_size(group)
    dev = desc.device
    sizes = torch.tensor([n_msgs, n_rec, n_heap], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    S = torch.stack(all_sizes).cpu()
    mx = S.max(dim=0).values.clamp(min=1)

    def gather(buf: torch.Tensor, nbytes: int, cap: int):
        padded = torch.zeros(cap, dtype=torch.uint8, device=dev)
        if nbytes:
            padded[:nbytes] = buf[:nbytes]
        parts = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(world)]
        dist.all_gather(parts, padded, group=group)
        return parts

    dparts = gather(desc, n_msgs * DESC_BYTES, int(mx[0]) * DESC_BYTES)
    rparts = gather(rec, n_rec * REC_BYTES, int(mx[1]) * REC_BYTES)
    hparts = gather(heap, n_heap, int(mx[2]))
    out_d, out_r, out_h = [], [], []
    m_base = r_base = h_base = 0
    for k in range(world):
        nm, nr, nh = (int(x) for x in S[k])
        d = dparts[k][: nm * DESC_BYTES].clone().view(torch.int32).view(nm, 2)
        d[:, 0] += r_base
        r = rparts[k][: nr * REC_BYTES].clone().view(torch.int32).view(nr, 4)
        r[:, 0] += h_base
        r[:, 3] += m_base
        out_d.append(d.reshape(-1).view(torch.uint8))
        out_r.append(r.reshape(-1).view(torch.uint8))
        out_h.append(hparts[k][:nh])
        m_base += nm
        r_base += nr
        h_base += nh
    return torch.cat(out_d), torch.cat(out_r), torch.cat(out_h)
