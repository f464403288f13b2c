"""bench.py's N > 1 line at world 1 on the GPU (`--strong`: RCCL process group of one rank, the
Q6_K 28672x8192 row-sharded step with its all-gather captured in HIP graphs, the rank-agreed
capture decision): the line parses, carries the strong fields, and says how it was timed."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_strong_world1():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--strong", "--steps", "4", "--warmup", "2",
                        "--no-cpu"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["scaling"] == "strong"
    assert line["value"] > 0 and [s["M_tok"] for s in line["strong"]] == [1, 128]
    for s in line["strong"]:
        assert s["compute_ms_per_step"] > 0 and s["e2e_chain_ms_per_step"] > 0 and s["ranks"] == 1
        assert s["timing"].startswith("hipGraph") or s["timing"].startswith("eager"), s["timing"]
