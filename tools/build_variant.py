"""Build a variant of libsdx.so for A/B timing: sdx_kernels.hip from a given file (default the
working tree) with extra -D flags, linked with the other translation units' objects of the
in-tree build.  usage: python tools/build_variant.py NAME [--unit FILE.hip] [--src FILE] [-DFLAG ...]
-> pysignalduino_amd/_lib/ab/libsdx_NAME.so (time with SDX_LIB=... tools/time_mu.py)"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pysignalduino_amd import build as B  # noqa: E402


def main():
    name = sys.argv[1]
    args = sys.argv[2:]
    unit = "sdx_kernels.hip"
    if "--unit" in args:   # vary another translation unit (e.g. sdx_group.hip)
        i = args.index("--unit")
        unit = args[i + 1]
        del args[i:i + 2]
    src = os.path.join(REPO, "pysignalduino_amd", "csrc", unit)
    if "--src" in args:
        i = args.index("--src")
        src = os.path.abspath(args[i + 1])
        del args[i:i + 2]
    B.build()
    out_dir = os.path.join(REPO, "pysignalduino_amd", "_lib", "ab")
    os.makedirs(out_dir, exist_ok=True)
    obj = os.path.join(out_dir, f"{unit}_{name}.o")
    inc = ["-I", os.path.join(REPO, "pysignalduino_amd", "csrc")]
    subprocess.run([B.HIPCC, *B.FLAGS[:-1], *inc, *args, "-c", src, "-o", obj], check=True)
    others = [os.path.join(REPO, "pysignalduino_amd", "_lib", "obj", os.path.basename(s) + ".o") for s in B.SRCS
              if os.path.basename(s) != unit] + [os.path.join(REPO, "pysignalduino_amd", "_lib", "obj", "sdx_hash.cpp.o")]
    so = os.path.join(out_dir, f"libsdx_{name}.so")
    subprocess.run([B.HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", obj, *others, "-o", so], check=True)
    print(so)


if __name__ == "__main__":
    main()
