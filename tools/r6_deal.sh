#!/bin/bash
# Round 6: the grouped K-chunked stream's deal weights (per super-block: its bytes - offset; the
# product: 55 -- Q6_K / Q4_K 1.74) against offsets 0 (1.46, bytes), -120 (1.25) and 80 (2.07):
# (after per-workgroup stamps with the summing wave identified) the 7B layer at 8 / 16 / 24 / 32 tokens, interleaved.  (Any deal gives the same bits.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/kstream_layer_stamps.py 16 32 > gpurun_out/r6_klayer5.txt 2>&1
rc=$?; cat gpurun_out/r6_klayer5.txt; [ $rc -eq 0 ] || exit $rc
L=gguf-triton-kernel_amd/lib
for r in 1 2; do
  for v in "" off0 offm120 off80; do
    if [ -z "$v" ]; then a=""; n=off55; else a="--lib $L/libgguf_mmq_$v.so"; n=$v; fi
    timeout -k 10 300 python3 tools/layer_time.py 8,16,24,32 --grouped-only $a | sed "s/^/$n /" || exit $?
  done
done 2>&1 | grep points | tee gpurun_out/r6_deal_layer.txt
