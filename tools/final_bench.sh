#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench_default_end.json 2> gpurun_out/final/bench_default_end.err || { tail -20 gpurun_out/final/bench_default_end.err; exit 2; }
python3 -c "
import json
l=[x for x in open('gpurun_out/final/bench_default_end.json') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['unit'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
