"""BASELINE configs 2-4 at their stated size (1M messages of one kind) on the GPU,
checked message by message against the plain-C oracle through a size-independent signature: per
message, a hash of its ordered result list (protocol id, bit length, payload bytes) and its
status / raise kind.  The product path is the bench's: grouped order with spill regions (MU/MS)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1_000_000
_P = np.uint64(0x100000001B3)     # FNV-style multipliers (wrapping uint64 arithmetic)
_Q = np.uint64(0x9E3779B97F4A7C15)


def _seg_sum(vals, lens):
    """Wrapping uint64 sums of consecutive segments of the given lengths (0 for empty ones)."""
    out = np.zeros(len(lens), np.uint64)
    nz = lens > 0
    if nz.any():
        starts = (np.cumsum(lens) - lens)[nz]
        out[nz] = np.add.reduceat(vals, starts)
    return out


def _signatures(n, status, raise_kind, begin, count, rec_proto_gid, rec_bitlen, rec_off, rec_len, heap):
    """uint64 per message: status/raise and the ordered (pid, bit_length, payload) of its records."""
    heap = np.asarray(heap, np.uint8)
    lens = np.asarray(rec_len, np.int64)
    with np.errstate(over="ignore"):
        tot = int(lens.sum())
        pos = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(lens) - lens, lens)
        byte = heap[np.repeat(np.asarray(rec_off, np.int64), lens) + pos].astype(np.uint64) + np.uint64(1)
        contrib = byte * ((pos.astype(np.uint64) + np.uint64(1)) * _P) * _Q
        h = _seg_sum(contrib, lens) * _P + np.asarray(rec_proto_gid, np.uint64) * _Q + \
            np.asarray(rec_bitlen, np.uint64) + lens.astype(np.uint64)
        cnt = np.where(status == 0, count, 0).astype(np.int64)
        k = np.arange(int(cnt.sum()), dtype=np.int64) - np.repeat(np.cumsum(cnt) - cnt, cnt)
        rid = np.repeat(np.asarray(begin, np.int64), cnt) + k
        part = h[rid] * (k.astype(np.uint64) + np.uint64(7)) * _Q
        sig = _seg_sum(part, cnt)
        sig = sig + cnt.astype(np.uint64) * _P + np.asarray(status, np.uint64) * np.uint64(1 << 40) + \
            np.where(status == 1, raise_kind, 0).astype(np.uint64) * np.uint64(1 << 48)
    return sig


def _compare_with_c_oracle(kind, bk, batch, desc, rec, heap):
    """Every message's signature from the device outputs (desc, rec, heap) == the C oracle's on the
    same host batch; returns the number of device records."""
    from oracle import c_oracle as CO
    from pysignalduino_amd import runtime
    cb = CO.CBank()
    n = batch.n
    if kind == "MC":
        packed, cls = CO.mc_batch(batch), bk.mc_pids
    else:
        packed, cls = CO.pack_batch(batch), (bk.mu_pids if kind == "MU" else bk.ms_pids)
    st, rk, rb, nr, crec, cheap = CO.run(kind, packed, max(1, min(16, len(os.sched_getaffinity(0)))))
    gid = {p: i for i, p in enumerate(cb.pids)}
    dev_gid = np.array([gid[p] for p in cls], np.int64)
    dstatus = np.where(desc["status"] == runtime.ST_RAISED, 1, np.where(desc["status"] == runtime.ST_OK, 0, 2))
    assert (dstatus != 2).all(), "unresolved overflow status"
    bl = (lambda a: np.zeros_like(a)) if kind == "MC" else (lambda a: a)
    sd = _signatures(n, dstatus, desc["raise_kind"], desc["rec_begin"], desc["n_rec"], dev_gid[rec["proto"].astype(np.int64)],
                     bl(rec["bit_length"]), rec["payload_off"], rec["payload_len"], heap)
    sc = _signatures(n, st.astype(np.int64), rk, rb, np.where(st == 0, nr, 0), crec["proto"].astype(np.int64),
                     bl(crec["bitlen"]), crec["off"], crec["len"], cheap)
    bad = np.nonzero(sd != sc)[0]
    assert len(bad) == 0, f"{kind}: {len(bad)} of {n} messages differ from the C oracle; first: {bad[:5].tolist()}"
    return int(desc["n_rec"][desc["status"] == runtime.ST_OK].sum())


@pytest.mark.parametrize("kind,seed", [("MU", 4242), ("MS", 4343), ("MC", 4444)])
def test_config_size_vs_c_oracle(kind, seed):
    from pysignalduino_amd import bank as B, runtime, synth
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    gen = {"MU": synth.mu_corpus, "MS": synth.ms_corpus, "MC": synth.mc_corpus}[kind]
    batch = gen(bk.protocols, N, seed=seed)
    if kind == "MC":
        desc, rec, heap = eng.run(runtime.KIND_MC, eng.to_device_mc(batch))
    else:
        desc, rec, heap = eng.run(runtime.KIND_MU if kind == "MU" else runtime.KIND_MS, eng.to_device_pulses(batch))
    assert _compare_with_c_oracle(kind, bk, batch, desc, rec, heap) > N // 4   # the corpora decode


@pytest.mark.parametrize("batch", [0, 1, 2])
def test_bench_step_vs_c_oracle(batch):
    """The kernel the bench times, at the bench's exact configuration, against the C oracle (VERDICT r05
    #1): bench.py's corpora (seeds 42/43/44, 333,333 / 333,333 / 333,334 messages, noise 0.15 / 0.1),
    one sdx_group_step for the MU and MS orders, then ONE sdx_demod_step (k_step: MU, MS and MC tiles,
    the MS length classes, MC with its max_hex bound) into the bench's output capacities -- every
    message's status and ordered result list equal to oracle/sd_oracle_c.c's
    (message_unsynced.py:11-296, message_synced.py:10-243, manchester.py:49-144).  batch: each of the
    three corpora bench.py cycles by default (--batches 3: seeds + 100 * batch)."""
    import torch
    from pysignalduino_amd import bank as B, runtime, synth
    bk = B.Bank()
    eng = runtime.Engine(bk, 0)
    P = bk.protocols
    msgs = 1_000_000
    per = {"MU": msgs // 3, "MS": msgs // 3, "MC": msgs - 2 * (msgs // 3)}
    sd = 100 * batch
    corp = {"MU": synth.mu_corpus(P, per["MU"], seed=42 + sd, noise_frac=0.15),
            "MS": synth.ms_corpus(P, per["MS"], seed=43 + sd, noise_frac=0.1),
            "MC": synth.mc_corpus(P, per["MC"], seed=44 + sd)}
    bds = {k: (eng.to_device_mc(c) if k == "MC" else eng.to_device_pulses(c)) for k, c in corp.items()}
    assert 0 < bds["MC"]["max_hex"] <= runtime.MC_HEX_MAX
    caps = {"MU": (12, 320), "MS": (4, 64), "MC": (4, 96)}   # bench.py's capacities
    outs = {k: eng.alloc_out(per[k], caps[k][0] * per[k] + 4096, caps[k][1] * per[k] + 65536,
                             eng.pulses_work_bytes(per[k]) if k != "MC" else 0) for k in corp}
    gb = {k: eng.group_buffers(per[k]) for k in ("MU", "MS")}
    o_mu, o_ms = eng.group_step(bds["MU"], bds["MS"], gb["MU"], gb["MS"])
    eng.launch_step(mu=(bds["MU"], outs["MU"], o_mu, None), ms=(bds["MS"], outs["MS"], o_ms, None),
                    mc=(bds["MC"], outs["MC"], None))
    torch.cuda.synchronize()
    nres = 0
    for k in ("MU", "MS", "MC"):
        assert int(outs[k]["cursor"][2].item()) == 0, f"{k}: overflow in the bench configuration"
        desc, rec, heap = eng.fetch(outs[k])
        assert len(rec) == int(outs[k]["cursor"][0].item())
        nres += _compare_with_c_oracle(k, bk, corp[k], desc, rec, heap)
    assert nres > msgs   # ~1.8 results per message at the bench mix
