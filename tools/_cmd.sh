cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ktr -o run -- python3 $R/tools/gemm_tune.py --step q8_0_4096x4096_m128 q4_k_11008x4096_m128 > $R/gpurun_out/ktr.txt 2>&1 || exit 1
python3 $R/tools/kstats.py $R/gpurun_out/ktr/run_kernel_stats.csv | grep gq::; grep kernel_us $R/gpurun_out/ktr.txt
