"""HBM traffic per launch of each bench config's dominant kernel, from rocprofv3 FETCH_SIZE.

Usage (GPU box):  python tools/pmc_traffic.py [CONFIG ...]
For each config: one `rocprofv3 --pmc FETCH_SIZE --kernel-trace` pass (its own run, nothing
else collected) over `tools/gemm_tune.py --step CONFIG`, then
    hbm_bytes_per_launch = mean FETCH_SIZE (KiB) * 1024 * 2
of the dominant kernel (the step's matmul launch: the one fetching the most), the factor 2
being MI355X_MICROARCH.md's gfx950 correction (FETCH_SIZE counts 64 B per 128-B request of
a wide streaming read).  Writes profiles/pmc_<config>.json, which bench.py reads into
roofline.traffic.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out", "pmc_traffic")


def run(cfg):
    d = os.path.join(OUT, cfg + ("_" + os.path.basename(os.environ["PMC_LIB"]) if os.environ.get("PMC_LIB") else ""))
    os.makedirs(d, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    lib = os.environ.get("PMC_LIB")  # A/B of a diagnostic build: that library, records not written to profiles/
    cmd = ["rocprofv3", "--pmc", "FETCH_SIZE", "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run",
           "--", sys.executable, os.path.join(ROOT, "tools", "gemm_tune.py"), "--step"] + \
          ([f"--lib={os.path.abspath(lib)}"] if lib else []) + [cfg]
    subprocess.run(["timeout", "-k", "10", "120"] + cmd, check=True, cwd="/tmp", env=env,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if "gq::" not in k:
                continue
            vals.setdefault(k, []).append(float(r["Counter_Value"]))
    fmt, M, K, N = bench.CONFIGS[cfg]
    # the dominant kernel: the step's matmul launch (decode, skinny, or either GEMM -- the
    # library routes by type and token count), i.e. the gq kernel that fetches the most
    # (not act_quant, not the split-K reduce)
    main = {k: v for k, v in vals.items() if "act_quant" not in k and "reduce" not in k}
    if not main:
        raise SystemExit(f"{cfg}: no matmul dispatch in the PMC output")
    dom = [max(main, key=lambda k: sum(main[k]) / len(main[k]))]
    v = vals[dom[0]]
    hbm = sum(v) / len(v) * 1024 * 2
    wbytes, alg, _ = bench.model(fmt, M, K, N)
    name = dom[0].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    rec = {"config": cfg, "kernel": name, "dispatches": len(v),
           "fetch_size_kib_mean": sum(v) / len(v), "hbm_bytes_per_launch": hbm,
           "alg_bytes_per_launch": alg, "traffic_over_alg": hbm / alg,
           "method": "rocprofv3 --pmc FETCH_SIZE (own pass), x1024 x2 (gfx950 correction)"}
    if lib:
        rec["lib"] = os.path.basename(lib)
    for dst in ((OUT,) if lib else (os.path.join(ROOT, "profiles"), OUT)):  # profiles/ for bench.py, gpurun_out/ to bring back
        with open(os.path.join(dst, f"pmc_{cfg}{'_' + os.path.basename(lib) if lib else ''}.json"), "w") as fh:
            json.dump(rec, fh, indent=1)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    for c in sys.argv[1:] or list(bench.CONFIGS):
        run(c)
