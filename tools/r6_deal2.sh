#!/bin/bash
# Round 6 (after the kstream issue priority): per-workgroup stamps of the grouped layer, and the
# deal offset re-measured (30 / 80 against the product's 55) at 8 / 16 / 24 / 32 tokens.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/kstream_layer_stamps.py 16 32 > gpurun_out/r6_klayer7.txt 2>&1
rc=$?; cat gpurun_out/r6_klayer7.txt; [ $rc -eq 0 ] || exit $rc
L=gguf-triton-kernel_amd/lib
for r in 1 2; do
  for v in "" off30 off80; do
    if [ -z "$v" ]; then a=""; n=off55; else a="--lib $L/libgguf_mmq_$v.so"; n=$v; fi
    timeout -k 10 300 python3 tools/layer_time.py 8,16,24,32 --grouped-only $a | sed "s/^/$n /" || exit $?
  done
done 2>&1 | grep points | tee gpurun_out/r6_deal2_layer.txt
