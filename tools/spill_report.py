#!/usr/bin/env python3
"""Where a kernel's register spills are reloaded: compile a HIP source for gfx950 to assembly and,
per kernel, count the scratch reloads by the loop depth of their basic block (the compiler's
"in Loop: ... Depth=d" annotation; depth 0 = straight-line code).  A reload at the depth of the
innermost (per-task) loop costs every iteration; one at the outer depths costs once per pass.

Usage: python tools/spill_report.py [SOURCE.hip] [-DFLAG ...]   (default csrc/mmq_kstream.hip)
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = next((a for a in sys.argv[1:] if not a.startswith("-")),
           os.path.join(ROOT, "gguf-triton-kernel_amd", "csrc", "mmq_kstream.hip"))
flags = [a for a in sys.argv[1:] if a.startswith("-")]
with tempfile.TemporaryDirectory() as d:
    asm = os.path.join(d, "k.s")
    subprocess.run(["hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "--cuda-device-only", "-S",
                    "-o", asm, os.path.abspath(src), *flags], check=True, cwd=d, stderr=subprocess.DEVNULL)
    text = open(asm).read()
for m in re.finditer(r"\n(\S+):\s*; @\1\n(.*?)\.Lfunc_end", text, re.S):
    name, body = m.group(1), m.group(2)
    meta = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"\n(.*?)\.end_amdhsa_kernel", text, re.S)
    if not meta:
        continue
    vg = re.search(r"\.amdhsa_next_free_vgpr (\d+)", meta.group(1)).group(1)
    scr = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", meta.group(1)).group(1)
    depth, by, stores, maxd = 0, collections.Counter(), 0, 0
    for line in body.split("\n"):
        if line.startswith(".LBB") or line.startswith("; %bb"):
            mm = re.search(r"Depth=(\d+)", line)
            depth = int(mm.group(1)) if mm else 0
            maxd = max(maxd, depth)
        if "scratch_load" in line:
            by[depth] += 1
        if "scratch_store" in line:
            stores += 1
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    print(f"{dem}: next_free_vgpr {vg}, scratch {scr} B/lane, spill stores {stores}, "
          f"reloads by loop depth {dict(sorted(by.items()))} (deepest loop {maxd})")
