#!/usr/bin/env bash
# GPU session: new-path parity tests, then bench default (per-type sweep + CPU baselines) and
# the strong-scaling headline at N=1.  Each GPU step has its own limit; failures stop here.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -x -v --timeout 300 --timeout-method thread > $OUT/paths_pytest.log 2>&1
rc=$?; tail -4 $OUT/paths_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 100 --warmup 10 > $OUT/bench_default.json 2> $OUT/bench_default.err
rc=$?; tail -c 600 $OUT/bench_default.json; [ $rc -eq 0 ] || { tail -20 $OUT/bench_default.err; exit $rc; }
timeout -k 10 300 python bench.py --strong --steps 50 --warmup 5 --no-cpu > $OUT/bench_strong1.json 2> $OUT/bench_strong1.err
rc=$?; cat $OUT/bench_strong1.json; [ $rc -eq 0 ] || { tail -20 $OUT/bench_strong1.err; exit $rc; }
echo ALL_DONE
