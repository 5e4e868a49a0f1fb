"""Multi-GPU: contiguous message shards per rank + all-gather of the decoded dmsg buffers.

Messages are independent: each rank demodulates its contiguous shard
with no communication, then ONE exchange step gathers every rank's result buffers
(descriptors, result records, payload heap) so that every rank holds the whole stream's
results in global message order.  With the ``nccl`` backend (RCCL over xGMI on ROCm) the
buffers stay in HBM; the same code runs on ``gloo`` with CPU tensors (tests/test_dist.py).
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist

DESC_BYTES = 8
REC_BYTES = 16


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of ``n`` messages owned by ``rank`` (sizes differ by at most 1)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


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
