#!/bin/bash
# Round-4 batch 8: the eager call through lib/_gqcall (bench's eager_host_us), and the layer at
# 8/12/16 tokens grouped with stream-K vs the default routes.
bash tools/gpu_steps.sh \
t 200 'python -u -m pytest tests/test_gpu_paths.py tests/test_abi.py -q --timeout 120 --timeout-method thread' \
eager 200 'python -u tools/eager_probe.py && python -u -c "import bench,torch; print(bench.eager_call_us(torch.device(\"cuda:0\")))"' \
layer 400 'python -u tools/layer_time.py 8,12,16 --grouped-only && python -u tools/layer_time.py 8,12,16 --grouped-only --gemm-min 5 --tune GQ_SGEMM_STREAMK=1 && python -u tools/layer_time.py 8,12,16 --grouped-only --gemm-min 5'
