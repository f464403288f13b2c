#!/bin/bash
# Round-4 batch 22: the row-stream GEMM with 16-row groups and a 4-slot ring (GQ_RSTREAM=3: three
# 18 KB stages in flight): parity, steps, the layer with per-call projections.
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
t 300 'python -u -m pytest tests/test_gpu_rgemm.py -q -k rstream --timeout 120 --timeout-method thread' \
steps 300 "python -u $RC --steps-only --rounds 3 --variants def=GQ_RSTREAM:0,rs1=GQ_RSTREAM:1,rs3=GQ_RSTREAM:3 --configs q4_k_22016x4096_m16,q4_k_11008x4096_m16,q4_k_4096x11008_m16,q4_k_4096x4096_m16" \
layer 300 "python -u tools/layer_time.py 8,16 --grouped-only --gemm-min 100 && python -u tools/layer_time.py 8,16 --grouped-only --gemm-min 100 --tune GQ_RSTREAM=3"
