cd $GRAFT_REPO_ROOT
A=""
for nb in 8 4 2 1; do for s in 1 2 4 8; do A="$A q8_0_4096x4096_m128:GQ_GEMM_NB=$nb,GQ_GEMM_SPLITS=$s"; done; done
for nb in 8 4 2; do for s in 1 2 4; do A="$A q6_k_28672x8192_m128:GQ_GEMM_NB=$nb,GQ_GEMM_SPLITS=$s"; done; done
for nb in 8 4 2 1; do for s in 1 2 4 8; do A="$A q4_k_4096x4096_m128:GQ_GEMM_NB=$nb,GQ_GEMM_SPLITS=$s"; done; done
timeout -k 10 300 python tools/gemm_tune.py $A > gpurun_out/sweep1.txt 2>&1
