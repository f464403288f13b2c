cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for a in 0 15 31 16; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt$a -o run -- python3 $R/tools/gemm_tune.py --abl q8_0_4096x4096_m128:GQ_ABLATE=$a q6_k_28672x8192_m128:GQ_ABLATE=$a > /dev/null 2>&1 || exit 1
echo "== ABL $a"; python3 $R/tools/kstats.py $R/gpurun_out/kt$a/run_kernel_stats.csv | grep gq::
done
