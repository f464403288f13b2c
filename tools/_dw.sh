set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/dw; mkdir -p $O
for r in 1 2; do for L in gguf-triton-kernel_amd/lib/libgguf_mmq.so gguf-triton-kernel_amd/lib/libgguf_mmq_dw10.so; do
timeout -k 10 200 python -u tools/msweep.py --lib $L --shapes q6_k:28672:8192,q4_k:11008:4096,q8_0:4096:4096,q6_k:4096:4096 --tokens 1,2 >> $O/sweep.log 2>&1 || exit 1
done; done
grep -v amdgpu $O/sweep.log
