"""Lists raw workgroup barriers that an LDS write reaches without an `s_waitcnt lgkmcnt(0)`, per
kernel, from the `make -C gguf-triton-kernel_amd asm` output (or any `-S` output given).

Why: on gfx950 (back-off barrier) the compiler inserts NO wait in front of a raw
`__builtin_amdgcn_s_barrier()`; a `ds_write` issued before it may still be queued in the LDS
when another wave, released by the barrier, reads the same bytes -- that wave can see the old
value.  This was the round-4 row-stream race (`rstream_kernel`: per-wave sums written to LDS,
raw barrier, another wave sums them; non-identical bits between two calls).  Every barrier that
publishes LDS writes must be preceded by `s_waitcnt lgkmcnt(0)` (the kernels' `lds_barrier()`).

The scan is linear over each kernel's instruction text (labels reset nothing), so a write on
one side of a branch is also seen on the other: a flag is a candidate to read, not a proof.
Usage: python tools/check_barriers.py [file.s ...]; exit status 1 if any barrier is flagged.
"""
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ds_ instructions that do not write LDS memory
NOWRITE = ("ds_read", "ds_swizzle", "ds_permute", "ds_bpermute", "ds_consume", "ds_append", "ds_gws", "ds_nop")


def scan(path):
    out = {}
    name, pend = None, None
    for ln in open(path, errors="replace"):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", ln)
        if m:
            name, pend = m.group(1), None
            continue
        if name is None:
            continue
        s = ln.strip()
        if s.startswith("ds_") and not s.startswith(NOWRITE):
            pend = s
        elif s.startswith("s_waitcnt") and re.search(r"lgkmcnt\(0\)", s):
            pend = None
        elif s.startswith("s_barrier") and pend is not None:
            out.setdefault(name, []).append(pend)
        if s.startswith("s_endpgm") or s.startswith(".Lfunc_end"):
            pend = None
    return out


def main():
    files = sys.argv[1:] or sorted(glob.glob(os.path.join(ROOT, "gguf-triton-kernel_amd", "build", "*gfx950*.s")))
    bad = 0
    for f in files:
        for k, writes in scan(f).items():
            bad += 1
            print(f"{os.path.basename(f)}: {k[:100]}: {len(writes)} barrier(s) after an unwaited LDS write "
                  f"(e.g. {writes[0]})")
    print("ok" if not bad else f"{bad} kernel(s) with a barrier after an unwaited LDS write")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
