#!/bin/bash
# Round-4 batch 8: the eager call through lib/_gqcall (bench's eager_host_us); Q4_K fragments by
# byte permutes (new) vs the masked pairs (pre) at 16..128 tokens and in the layer; the layer at
# 8/12/16 tokens grouped with stream-K vs the default routes.
PRE=gguf-triton-kernel_amd/lib/libgguf_mmq_pre.so
NEW=gguf-triton-kernel_amd/lib/libgguf_mmq.so
bash tools/gpu_steps.sh \
t 300 'python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_rgemm.py tests/test_gpu_gemm_grouped.py tests/test_abi.py -q --timeout 120 --timeout-method thread' \
eager 200 'python -u tools/eager_probe.py && python -u -c "import bench,torch; print(bench.eager_call_us(torch.device(\"cuda:0\")))"' \
perm 300 "python -u tools/rgemm_check.py --steps-only --configs q4_k_4096x4096_m16,q4_k_11008x4096_m16,q4_k_22016x4096_m16,q4_k_4096x11008_m16,q4_k_4096x4096_m128,q4_k_11008x4096_m64,q4_k_11008x4096_m128 --variants def=GQ_SGEMM:-1 --rounds 3 --libs pre=$PRE,new=$NEW" \
layer 500 "python -u tools/layer_time.py 8,16,128 --grouped-only --lib $PRE && python -u tools/layer_time.py 8,16,128 --grouped-only && python -u tools/layer_time.py 8,12,16 --grouped-only --gemm-min 5 --tune GQ_SGEMM_STREAMK=1 && python -u tools/layer_time.py 8,12,16 --grouped-only --gemm-min 5"
