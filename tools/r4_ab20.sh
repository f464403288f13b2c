#!/bin/bash
# Round-4 batch 20: the row-stream GEMM (GQ_RSTREAM=1, Q4_K 5..16 tokens): parity, single-matrix
# steps against the default route, and the layer with per-call prepared projections.
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
t 300 'python -u -m pytest tests/test_gpu_rgemm.py -q -k rstream --timeout 120 --timeout-method thread' \
steps 300 "python -u $RC --steps-only --rounds 3 --variants def=GQ_RSTREAM:0,rs=GQ_RSTREAM:1,rs4=GQ_RSTREAM:2 --configs q4_k_11008x4096_m16,q4_k_4096x11008_m16,q4_k_4096x4096_m16,q4_k_22016x4096_m16,q4_k_11008x4096_m8" \
layer 300 "python -u tools/layer_time.py 8,16 --grouped-only && python -u tools/layer_time.py 8,16 --grouped-only --gemm-min 100 && python -u tools/layer_time.py 8,16 --grouped-only --gemm-min 100 --tune GQ_RSTREAM=1 && python -u tools/layer_time.py 8,16 --grouped-only --gemm-min 100 --tune GQ_RSTREAM=2"
