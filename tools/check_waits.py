"""Lists the vmcnt waits the compiler added (outside the kernels' own inline-asm waits) in
front of LDS reads, per kernel, from the `make -C gguf-triton-kernel_amd asm` output.

The LDS-DMA kernels (stream_decode_kernel, gemm_kernel) count their DMAs with explicit
s_waitcnt vmcnt(N); a compiler-inserted vmcnt wait before a ds_read means the waitcnt pass
could not tell the read from the DMA just issued into another ring slot, and it serializes
the stream with the multiply.  Usage: python tools/check_waits.py [file.s ...]
"""
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def scan(path):
    out = {}
    name, in_asm, pend = None, False, None
    for ln in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", ln)
        if m:
            name, pend = m.group(1), None
            continue
        if name is None:
            continue
        s = ln.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
        elif s.startswith(";;#ASMEND"):
            in_asm = False
        elif s.startswith("s_waitcnt") and "vmcnt" in s and not in_asm:
            pend = s
        elif s.startswith("ds_read") and pend is not None:
            out.setdefault(name, []).append(pend)
            pend = None
        elif s and not s.startswith(";") and not s.startswith("v_") and not s.startswith("s_"):
            pend = None if not s.startswith("ds_") else pend
        if s.startswith("s_endpgm"):
            name = None
    return out


def main():
    files = sys.argv[1:] or glob.glob(os.path.join(ROOT, "gguf-triton-kernel_amd", "build", "mmq_*gfx950.s"))
    bad = 0
    for f in files:
        for k, waits in scan(f).items():
            if "stream_decode_kernel" in k or "gemm_kernel" in k:
                bad += 1
                print(f"{os.path.basename(f)}: {k[:90]}: {len(waits)} compiler vmcnt wait(s) before ds_read: "
                      f"{sorted(set(waits))}")
    print("ok" if not bad else f"{bad} kernel(s) with compiler-added vmcnt waits before LDS reads")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
