"""The plain-C oracle under AddressSanitizer + UndefinedBehaviorSanitizer.

The C restatement (oracle/sd_oracle_c.c) is the checker of the large GPU parity corpora, so it is
itself run instrumented on the host: oracle/sanitize_driver.c links it into a small executable
(exact-size heap buffers, so any out-of-bounds access is reported), which demodulates the golden
inputs, seeded synthetic corpora and the planted accept-path corpora on 2 threads.  Any sanitizer
report fails the run; the results must also equal the uninstrumented library's, record by
record.  CPU only."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from oracle import c_oracle as CO
from pysignalduino_amd import bank as B, packing, synth

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DRIVER = os.path.join(REPO, "oracle", "sanitize_driver.c")
EXE = os.path.join(REPO, "oracle", "_build", "sdoracle_san")


@pytest.fixture(scope="module")
def exe():
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    subprocess.run(["gcc", "-std=gnu11", "-g", "-O1", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-I", os.path.join(REPO, "oracle"), DRIVER, "-o", EXE, "-lm",
                    "-pthread"], check=True)
    return EXE


def _dump(path, kind, packed, cbank, nthreads=2):
    n = packed["n"]
    arr = bytes(cbank.arr)
    with open(path, "wb") as f:
        f.write(struct.pack("<5i", {"MU": 0, "MS": 1, "MC": 2}[kind], n, len(cbank.pids), CO.C.sizeof(CO.SoProto),
                            nthreads))
        f.write(arr[: len(cbank.pids) * CO.C.sizeof(CO.SoProto)])
        f.write(np.ascontiguousarray(packed["offsets"], np.int64).tobytes())
        if kind == "MC":
            f.write(np.ascontiguousarray(packed["hex"], np.uint8)[: int(packed["offsets"][n])].tobytes())
            for k, dt in (("clock", np.int32), ("mcbitnum", np.int32), ("mtype_lower", np.uint8), ("v32", np.uint8)):
                f.write(np.ascontiguousarray(packed[k], dt).tobytes())
        else:
            f.write(np.ascontiguousarray(packed["data"], np.uint8)[: int(packed["offsets"][n])].tobytes())
            f.write(np.ascontiguousarray(packed["npat"], np.uint8).tobytes())
            f.write(np.ascontiguousarray(packed["pat_id"], np.uint8).reshape(-1).tobytes())
            f.write(np.ascontiguousarray(packed["pat_val"], np.float64).reshape(-1).tobytes())
            f.write(np.ascontiguousarray(packed["ms_ok"], np.uint8).tobytes())
            f.write(np.ascontiguousarray(packed["cp_slot"], np.int8).tobytes())


def _read(path, n):
    b = open(path, "rb").read()
    o = 0
    st = np.frombuffer(b, np.uint8, n, o); o += n
    rk = np.frombuffer(b, np.uint8, n, o); o += n
    rb = np.frombuffer(b, np.uint32, n, o); o += 4 * n
    nr = np.frombuffer(b, np.uint16, n, o); o += 2 * n
    rt, ht = struct.unpack_from("<QQ", b, o); o += 16
    rec = np.frombuffer(b, CO.RES_DT, rt, o); o += rt * CO.RES_DT.itemsize
    heap = np.frombuffer(b, np.uint8, ht, o)
    return st, rk, rb, nr, rec, heap


def _cases(golden):
    P = B.load_protocols()
    out = []
    for kind, fname in (("MU", "mu_golden.json.gz"), ("MS", "ms_golden.json.gz")):
        msgs = []
        for c in golden(fname):
            try:
                CO.pack_pulses([dict(c["msg"])])
            except NotImplementedError:
                continue
            msgs.append(dict(c["msg"]))
        out.append((kind + "-golden", kind, CO.pack_pulses(msgs)))
    out.append(("MU-synth", "MU", CO.pack_batch(synth.mu_corpus(P, 3000, seed=31))))
    out.append(("MS-synth", "MS", CO.pack_batch(synth.ms_corpus(P, 3000, seed=32))))
    out.append(("MU-planted", "MU", CO.pack_pulses(synth.planted_pulse_messages(P, "MU", 2000, seed=33))))
    out.append(("MS-planted", "MS", CO.pack_pulses(synth.planted_pulse_messages(P, "MS", 1000, seed=34))))
    frames = [(f["hex"], f["clock"], f["L"], f["mtype"], f["version"]) for f in golden("mc_golden.json.gz")]
    out.append(("MC-golden", "MC", CO.pack_mc(frames)))
    out.append(("MC-synth", "MC", CO.mc_batch(synth.mc_corpus(P, 3000, seed=35))))
    out.append(("MC-planted", "MC", CO.pack_mc(synth.mc_planted_frames(P, 3000, seed=36))))
    return out


def test_c_oracle_under_asan_ubsan(exe, golden, tmp_path):
    cbank = CO.CBank()
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    for name, kind, packed in _cases(golden):
        fin, fout = str(tmp_path / (name + ".in")), str(tmp_path / (name + ".out"))
        _dump(fin, kind, packed, cbank)
        r = subprocess.run([exe, fin, fout], env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0 and "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, \
            f"{name}: rc={r.returncode}\n{r.stderr[-4000:]}"
        got = _read(fout, packed["n"])
        ref = CO.run(kind, packed, 2)
        for a, b in zip(got[:4], ref[:4]):
            assert np.array_equal(a, b), name
        assert np.array_equal(got[4], ref[4]) and np.array_equal(got[5], ref[5]), name
