#!/bin/bash
# Interleaved A/B of two builds of libgguf_mmq.so on the same specs (tools/gemm_tune.py), then
# the GPU parity tests of gemm/paths under build B.  Usage: tools/libab.sh LIB_B "spec ..." [R]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=$1; SPECS=$2; R=${3:-2}
for r in $(seq $R); do
  for L in gguf-triton-kernel_amd/lib/libgguf_mmq.so $B; do
    timeout -k 10 300 python tools/gemm_tune.py --lib=$L $SPECS 2>&1 | grep kernel_us | sed "s|^|$(basename $L) |" || exit 1
  done
done | python3 -c "
import sys, collections
d = collections.OrderedDict()
for l in sys.stdin:
    f = l.split(); k = f[0] + ' ' + f[1]; v = float(l.split('kernel_us=')[1].split()[0])
    d.setdefault(k, []).append(v)
for k in sorted(d, key=lambda k: (k.split()[1], k.split()[0])): print(f'{k:70s} min={min(d[k]):7.2f} all={d[k]}')
" > gpurun_out/libab.txt; cat gpurun_out/libab.txt
if [ -n "$TESTS" ]; then
  cp $B gguf-triton-kernel_amd/lib/libgguf_mmq.so
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > gpurun_out/libab_tests.log 2>&1; rc=$?
  tail -3 gpurun_out/libab_tests.log; exit $rc
fi
