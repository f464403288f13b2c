#!/bin/bash
# Round-4 batch 5: the GPU suite; PMC passes (one counter group per rocprofv3 run) on the
# streaming and resident GEMMs.
bash tools/gpu_steps.sh \
tests 800 'python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread' \
pmc 600 'PASSES="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_WAIT_INST_LDS|SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_VALU_MFMA_COEXEC_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_BUSY_CYCLES,SQ_INSTS_SALU|GRBM_GUI_ACTIVE,TA_BUSY_avr,TCC_HIT_sum,TCC_MISS_sum|FETCH_SIZE" bash tools/gpu.sh pmc q6_k_28672x8192_m128 q8_0_4096x4096_m128 q4_k_4096x4096_m128'
