"""Build libsdx.so (hand-written HIP for gfx950) in-tree:  python -m pysignalduino_amd.build"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, "csrc", "sdx_kernels.hip"),   # demodulation kernels + bank + C-ABI
        os.path.join(HERE, "csrc", "sdx_lines.hip"),     # wire-line front end (sdx_parse_lines/select)
        os.path.join(HERE, "csrc", "sdx_mn.hip"),        # MN (FSK) engine (sdx_demod_mn)
        os.path.join(HERE, "csrc", "sdx_json.hip"),      # publish-ready JSON (sdx_serialize_json)
        os.path.join(HERE, "csrc", "sdx_units.hip"),     # unit-level helpers (sdx_units)
        os.path.join(HERE, "csrc", "sdx_exchange.hip"),  # multi-GPU exchange packing (sdx_exchange_pack)
        os.path.join(HERE, "csrc", "sdx_group.hip"),     # MU/MS message grouping (k_sig + radix sort)
        os.path.join(HERE, "csrc", "sdx_general.hip")]   # general path: multi-digit ids, long messages/frames
OUT = os.path.join(HERE, "_lib", "libsdx.so")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared"]


DEPS = [*SRCS, os.path.join(HERE, "csrc", "sdx_device.h"), os.path.join(HERE, "csrc", "sdx_lane.h"),
        os.path.join(HERE, "csrc", "sdx_mc.h"),
        os.path.join(os.path.dirname(HERE), "include", "sdx.h"),
        os.path.join(os.path.dirname(HERE), "include", "sdx_bank.h")]


def source_hash() -> str:
    """sha256 (first 16 hex digits) of every source and header libsdx.so is built from, plus the
    flags: compiled into the library (sdx_source_hash()), so a run can prove it loaded a library
    built from the tree it runs in (__graft_entry__.smoke checks it)."""
    import hashlib
    h = hashlib.sha256(" ".join(FLAGS).encode())
    for d in DEPS:
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    deps = DEPS
    hsrc = os.path.join(os.path.dirname(OUT), "obj", "sdx_hash.cpp")
    built_hash = open(hsrc).read() if os.path.exists(hsrc) else ""
    if (not force and os.path.exists(OUT) and source_hash() in built_hash and
            all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps)):
        return OUT
    # one object per translation unit, compiled in parallel, then one link.  A unit is recompiled when
    # its source or any shared header is newer than its object (the headers are few; every unit may
    # include them); the source hash lives in a generated unit of its own, rebuilt every time
    objdir = os.path.join(os.path.dirname(OUT), "obj")
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(src) + ".o") for src in SRCS]
    hdr_t = max(os.path.getmtime(d) for d in DEPS if d not in SRCS)
    stale = [(src, obj) for src, obj in zip(SRCS, objs)
             if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t)]
    cmds = [[HIPCC, *FLAGS[:-1], "-c", src, "-o", obj] for src, obj in stale]
    with open(hsrc, "w") as fh:
        fh.write('extern "C" const char* sdx_source_hash(void) { return "%s"; }\n' % source_hash())
    hobj = hsrc + ".o"
    cmds.append(["g++", "-O2", "-fPIC", "-c", hsrc, "-o", hobj])
    if verbose:
        for c in cmds:
            print(" ".join(c))
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(len(cmds), 8)) as ex:
        for f in [ex.submit(subprocess.run, c, check=True) for c in cmds]:
            f.result()
    cmd = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", *objs, hobj, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
