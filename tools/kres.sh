#!/bin/bash
# tools/kres.sh OBJ [KERNEL_REGEX]: per-kernel VGPRs / spills / LDS of a hipcc -c object (gfx950)
# (the code object's metadata notes; no recompile with -Rpass-analysis needed)
set -eu -o pipefail
B=/opt/rocm/lib/llvm/bin; t=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$t/f "$1"
$B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$t/f --output=$t/co --unbundle
$B/llvm-readelf --notes $t/co | python3 -c '
import sys, re
pat = re.compile(sys.argv[1])
cur = {}
rows = []
for ln in sys.stdin:
    if re.match(r"\s*- \.agpr_count:", ln):
        if cur: rows.append(cur)
        cur = {}
    m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)", ln)
    if m:
        cur[m.group(1)] = m.group(2)
if cur: rows.append(cur)
for r in rows:
    n = r.get("name", "")
    if n and pat.search(n):
        print(n[:60], "vgpr", r.get("vgpr_count"), "agpr", r.get("agpr_count"), "vspill", r.get("vgpr_spill_count"),
              "sspill", r.get("sgpr_spill_count"), "lds", r.get("group_segment_fixed_size"), "scratch", r.get("private_segment_fixed_size"))
' "${2:-.}"
rm -rf $t
