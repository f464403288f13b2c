#!/bin/bash
# Round-4 batch 21: the row-stream GEMM with fewer, longer streams (GQ_RSTREAM_WPC: workgroups per
# K chunk; default CUs / chunks = 128 at K = 4096): is its time the per-workgroup prologue?
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
steps 300 "python -u $RC --steps-only --rounds 3 --variants def=GQ_RSTREAM:0,w128=GQ_RSTREAM:1,w64=GQ_RSTREAM:1+GQ_RSTREAM_WPC:64,w32=GQ_RSTREAM:1+GQ_RSTREAM_WPC:32,w96=GQ_RSTREAM:1+GQ_RSTREAM_WPC:96 --configs q4_k_22016x4096_m16,q4_k_11008x4096_m16"
