"""The streaming front end (pysignalduino_amd/stream.py): LineStream's per-line results
equal the batch API's (SignalParser.parse_lines_json / parse_lines) on mixed lines in many small
chunks -- MU/MS/MC/MN, compressed lines, general-path lines (multi-digit ids), lines outside the
device contract, MC frames of > 128 hex characters (ST_OVF_TILE re-runs) -- in submission order,
with polls interleaved and a drain at the end."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mixed_lines(golden, seed=7):
    from pysignalduino_amd import bank as B, synth
    P = B.Bank().protocols
    rng = np.random.default_rng(seed)
    raw, _ = synth.line_corpus(P, 9000, seed=seed, mix=(1, 1, 1), compress_frac=0.3)
    raw += [synth.frame(synth.mn_payload(*f)) for f in synth.mn_frames(2000, seed=seed + 1)]
    # general-path MU/MS lines (reference-recorded: multi-digit ids, > 4096 pulses) and long MC frames
    raw += [c["line"].encode("latin-1") if isinstance(c["line"], str) else bytes(c["line"])
            for c in golden("lines_general_golden.json.gz")][:200]
    for h, c, L, t, v in synth.general_mc_frames(P, 30, seed=seed + 4):
        c = max(int(c), 1)
        raw.append(synth.frame(("%s;LL=%d;LH=%d;SL=%d;SH=%d;D=%s;C=%d;L=%d;R=10;"
                                % (t, -2 * c, 2 * c, -c, c, h, c, L)).encode("latin-1")))
    raw += [synth.mutate_line(rng, raw[int(rng.integers(0, len(raw)))]) for _ in range(500)]
    idx = rng.permutation(len(raw))
    return [raw[i] for i in idx]


@pytest.mark.parametrize("output", ["json", "wire"])
def test_stream_matches_batch_api(output, golden):
    from pysignalduino_amd import runtime
    from pysignalduino_amd.frontend import SignalParser
    from pysignalduino_amd.sd_protocols import SDProtocols
    lines = _mixed_lines(golden)
    sp = SignalParser(SDProtocols(mc_mode="fixed"))
    ls = sp.stream(chunk_lines=1500, chunk_bytes=1500 * 4200, output=output, lag=3)
    chunks = []
    i = 0
    rng = np.random.default_rng(3)
    while i < len(lines):
        k = int(rng.integers(200, 1501))
        chunks.append(lines[i: i + k])
        i += k
    got = []
    for j, ch in enumerate(chunks):
        ls.submit(ch)
        if j % 2:
            got += [r.detach() for r in ls.poll()]
    got += [r.detach() for r in ls.drain()]
    assert [r.id for r in got] == list(range(len(chunks)))
    bk = sp.protocols._bank
    pid = {"MU": bk.mu_pids, "MS": bk.ms_pids, "MC": bk.mc_pids, "MN": bk.mn_pids}
    lk = {runtime.LINE_MU: "MU", runtime.LINE_MS: "MS", runtime.LINE_MC: "MC", runtime.LINE_MN: "MN"}
    nres = nhost = 0
    for ch, r in zip(chunks, got):
        assert r.n == len(ch)
        nhost += len(r.host)
        if output == "json":
            exp = sp.parse_lines_json(ch)
            for i, (e, g) in enumerate(zip(exp, r.texts())):
                if isinstance(e, Exception):
                    assert isinstance(g, type(e)), (i, e, g)
                else:
                    assert e == g, (i, e, g)
                    nres += e is not None
            continue
        exp = sp.parse_lines(ch)
        dec = {nm: r.decode(j) for j, nm in enumerate(r.names)}
        for i, e in enumerate(exp):
            if i in r.host:
                g = r.host[i]
                if isinstance(e, Exception):
                    assert isinstance(g, type(e))
                else:
                    assert [(m.protocol_id, m.payload, m.metadata) for m in g] == \
                        [(m.protocol_id, m.payload, m.metadata) for m in e]
                continue
            nm = lk.get(int(r.kind[i]))
            if int(r.status[i]) != runtime.LS_OK or nm not in dec:
                assert e == [], (i, e)
                continue
            d, rc, h = dec[nm]
            got_i = [(str(pid[nm][int(x["proto"])]),
                      h[int(x["payload_off"]): int(x["payload_off"]) + int(x["payload_len"])].tobytes().decode("latin-1"))
                     for x in rc[int(d[i]["rec_begin"]): int(d[i]["rec_begin"]) + int(d[i]["n_rec"])]]
            assert got_i == [(m.protocol_id, m.payload) for m in e], (i, got_i, e)
            nres += bool(e)
    assert nres > 3000 and nhost > 50, (nres, nhost)


@pytest.mark.parametrize("output", ["json", "wire"])
def test_stream_chunk_matches_reference_line_goldens(output, golden):
    """LineStream against the REFERENCE's recorded results, not against the batch API:
    the reference-run lines of tests/golden/lines_golden.json.gz (every hot-path test line, synthetic
    and mutated lines, compressed lines) tiled 5x into one chunk -- so that both short classes pass
    GROUP_MIN and the chunk runs the product's sdx_group_step + ONE k_step -- then per line the MQTT
    text the reference publishes (json: controller.py:254-257, mqtt.py:227-245) or its full
    (protocol_id, payload) list (wire: parser/mu.py:75-80, ms.py:51, mc.py:78)."""
    from oracle import json_oracle as J
    from pysignalduino_amd import runtime
    from pysignalduino_amd.frontend import SignalParser
    from pysignalduino_amd.packing import ContractError
    cases = golden("lines_golden.json.gz")
    lines = [c["line"].encode("latin-1") for c in cases] * 5
    exp_all = [c.get("e2e", []) for c in cases] * 5
    sp = SignalParser()                        # the reference's configuration: MC 'strict'
    ls = sp.stream(chunk_lines=len(lines), chunk_bytes=sum(map(len, lines)) + 4096, output=output, lag=2)
    ls.submit(lines)
    got = [r.detach() for r in ls.drain()]
    assert len(got) == 1 and got[0].n == len(lines)
    r = got[0]
    kinds = r.kind
    assert int((kinds == runtime.LINE_MU).sum()) >= runtime.GROUP_MIN and \
        int((kinds == runtime.LINE_MS).sum()) >= runtime.GROUP_MIN
    nres = contract = 0
    if output == "json":
        for i, (e, g) in enumerate(zip(exp_all, r.texts())):
            if isinstance(g, ContractError):
                contract += 1
                continue
            assert g == J.published(e), (i, lines[i][:80], g, e)
            nres += g is not None
    else:
        bk = sp.protocols._bank
        pid = {"MU": bk.mu_pids, "MS": bk.ms_pids, "MC": bk.mc_pids, "MN": bk.mn_pids}
        lk = {runtime.LINE_MU: "MU", runtime.LINE_MS: "MS", runtime.LINE_MC: "MC", runtime.LINE_MN: "MN"}
        dec = {nm: r.decode(j) for j, nm in enumerate(r.names)}
        for i, e in enumerate(exp_all):
            want = [(x[0], x[1]) for x in e]
            if i in r.host:
                g = r.host[i]
                if isinstance(g, Exception):
                    contract += 1
                    continue
                got_i = [(m.protocol_id, m.payload) for m in g]
            else:
                nm = lk.get(int(r.kind[i]))
                if int(r.status[i]) != runtime.LS_OK or nm not in dec:
                    got_i = []
                else:
                    d, rc, h = dec[nm]
                    got_i = [(str(pid[nm][int(x["proto"])]),
                              h[int(x["payload_off"]): int(x["payload_off"]) + int(x["payload_len"])].tobytes()
                              .decode("latin-1"))
                             for x in rc[int(d[i]["rec_begin"]): int(d[i]["rec_begin"]) + int(d[i]["n_rec"])]]
            assert got_i == want, (i, lines[i][:80], got_i, want)
            nres += bool(want)
    assert nres >= 5 * 1200 and contract <= 0.05 * len(lines), (nres, contract)


@pytest.mark.parametrize("output", ["json", "wire"])
def test_stream_mc_class_boundary_64_65(output):
    """the stream promises k_step's MC range frames of <= SDX_MC_SHORT_HEX (64) characters,
    measured by the line classifier (sel_class: dlen <= 64); frames of exactly 63, 64, 65 and 66 hex
    characters in one chunk -- no frame of the fused range is flagged SDX_ST_OVF_TILE (no line goes back
    to the batch API) and every line's results equal the batch API's."""
    from pysignalduino_amd import bank as B, synth
    from pysignalduino_amd.frontend import SignalParser
    from pysignalduino_amd.sd_protocols import SDProtocols
    P = B.Bank().protocols
    rng = np.random.default_rng(64)
    lines = []
    for j, (h, c, L, t, v) in enumerate(synth.mc_planted_frames(P, 800, seed=65, corrupt_frac=0.1)):
        n = (63, 64, 65, 66)[j % 4]
        h = (h + "".join("0123456789ABCDEF"[int(x)] for x in rng.integers(0, 16, 80)))[:n]
        c = max(int(c), 1)
        lines.append(synth.frame(("%s;LL=%d;LH=%d;SL=%d;SH=%d;D=%s;C=%d;L=%d;R=10;"
                                  % (t, -2 * c, 2 * c, -c, c, h, c, 4 * n if j % 3 else L)).encode("latin-1")))
    sp = SignalParser(SDProtocols(mc_mode="fixed"))
    ls = sp.stream(chunk_lines=len(lines), chunk_bytes=sum(map(len, lines)) + 4096, output=output, lag=1)
    ls.submit(lines)
    (r,) = [x.detach() for x in ls.drain()]
    assert not r.host, f"{len(r.host)} lines went back to the batch API (an MC overflow flag)"
    if output == "json":
        exp = sp.parse_lines_json(lines)
        assert r.texts() == exp
        assert sum(e is not None for e in exp) > 0   # (few: extended frames fail most methods' length checks)
        return
    from pysignalduino_amd import runtime
    exp = sp.parse_lines(lines)
    d, rc, h = r.decode(r.names.index("MC"))
    pid = sp.protocols._bank.mc_pids
    n_ok = 0
    for i, e in enumerate(exp):
        assert int(r.kind[i]) == runtime.LINE_MC and int(r.status[i]) == runtime.LS_OK
        got_i = [(str(pid[int(x["proto"])]),
                  h[int(x["payload_off"]): int(x["payload_off"]) + int(x["payload_len"])].tobytes().decode("latin-1"))
                 for x in rc[int(d[i]["rec_begin"]): int(d[i]["rec_begin"]) + int(d[i]["n_rec"])]]
        assert got_i == [(m.protocol_id, m.payload) for m in e], (i, got_i, e)
        n_ok += bool(e)
    assert n_ok > 0


def test_stream_capacity_and_empty_chunk():
    from pysignalduino_amd.frontend import SignalParser
    sp = SignalParser()
    ls = sp.stream(chunk_lines=100, chunk_bytes=100 * 300, output="json", lag=2)
    with pytest.raises(ValueError):
        ls.submit([b"\x02MU;P0=1;D=0;\x03"] * 101)
    ls.submit([])
    out = ls.drain()
    assert len(out) == 1 and out[0].n == 0 and out[0].texts() == []


def test_stream_pinned_submit_matches_batch_api(golden):
    """submit_packed from PINNED torch tensors (uploaded in place, no host copy): the same texts as
    the batch API, fallback lines (general path, contract) taken from the tensor."""
    import torch
    from pysignalduino_amd.frontend import SignalParser, pack_lines
    from pysignalduino_amd.sd_protocols import SDProtocols
    lines = _mixed_lines(golden, seed=11)[:6000]
    sp = SignalParser(SDProtocols(mc_mode="fixed"))
    ls = sp.stream(chunk_lines=2000, chunk_bytes=2000 * 4200, output="json", lag=2)
    chunks, got = [], []
    for i in range(0, len(lines), 2000):
        ch = lines[i: i + 2000]
        data, offs, bad = pack_lines(ch)
        assert not bad
        t = torch.from_numpy(data.copy()).pin_memory()
        chunks.append((ch, t))                      # kept alive until collected
        ls.submit_packed(t, offs)
        got += [r.detach() for r in ls.poll()]
    got += [r.detach() for r in ls.drain()]
    assert len(got) == len(chunks)
    nres = 0
    for (ch, _), r in zip(chunks, got):
        exp = sp.parse_lines_json(ch)
        for i, (e, g) in enumerate(zip(exp, r.texts())):
            if isinstance(e, Exception):
                assert isinstance(g, type(e)), (i, e, g)
            else:
                assert e == g, (i, e, g)
                nres += e is not None
    assert nres > 1000


def test_copy_and_fill_async_on_a_stream():
    """sdx_copy_async / sdx_fill_async (the pipeline's per-chunk transfers and resets): pinned host ->
    device, device -> device, device -> pinned host on a side stream, odd sizes and offsets; a
    zero-byte call is a no-op; mismatched sizes are refused on the host."""
    import torch
    from pysignalduino_amd import runtime
    runtime.load_library()
    st = torch.cuda.Stream()
    rng = np.random.default_rng(3)
    src = torch.from_numpy(rng.integers(0, 256, 100_003, dtype=np.uint8)).pin_memory()
    dev = torch.empty(100_019, dtype=torch.uint8, device="cuda")
    dev2 = torch.empty_like(dev)
    back = torch.zeros(100_003, dtype=torch.uint8).pin_memory()
    with torch.cuda.stream(st):
        runtime.copy_async(dev[5: 5 + 100_003], src, st)
        runtime.copy_async(dev2[:100_003], dev[5: 5 + 100_003], st)
        runtime.fill_async(dev2[7: 7 + 1001], st, 0xAB)
        runtime.copy_async(back, dev2[:100_003], st)
        runtime.copy_async(back[:0], dev2[:0], st)
    st.synchronize()
    want = src.numpy().copy()
    want[7: 7 + 1001] = 0xAB
    assert np.array_equal(back.numpy(), want)
    with pytest.raises(ValueError):
        runtime.copy_async(back[:10], dev[:11], st)


@pytest.mark.parametrize("wg", [1, 16])
def test_narrow_device_to_host_copy(wg):
    """sdx_copy_async_narrow (the few-workgroup device -> pinned-host copy of the streaming output):
    16-byte aligned and unaligned ends, a tail of odd length, and a zero-byte copy."""
    import torch
    from pysignalduino_amd import runtime
    lib = runtime.load_library()
    st = torch.cuda.Stream()
    rng = np.random.default_rng(4)
    src = torch.from_numpy(rng.integers(0, 256, 300_017, dtype=np.uint8)).cuda()
    for a, b, n in ((0, 0, 300_000), (3, 0, 299_990), (0, 5, 123_457), (16, 32, 17)):
        back = torch.zeros(300_064, dtype=torch.uint8).pin_memory()
        runtime._check(lib, lib.sdx_copy_async_narrow(back.data_ptr() + b, src.data_ptr() + a, n, wg, st.cuda_stream))
        st.synchronize()
        h = back.numpy()
        assert np.array_equal(h[b: b + n], src.cpu().numpy()[a: a + n]), (a, b, n)
        assert not h[:b].any() and not h[b + n:].any()
    runtime._check(lib, lib.sdx_copy_async_narrow(back.data_ptr(), src.data_ptr(), 0, wg, st.cuda_stream))
    assert lib.sdx_copy_async_narrow(back.data_ptr(), src.data_ptr(), 8, 0, st.cuda_stream) < 0
