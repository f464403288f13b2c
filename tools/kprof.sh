#!/usr/bin/env bash
# rocprofv3 kernel-trace stats of tools/gemm_tune.py runs given as arguments (one process).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/${KPROF_NAME:-kprof}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/tools/gemm_tune.py "$@" > $OUT/tune.txt 2>&1
rc=$?; cat $OUT/tune.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
python3 $R/tools/kstats.py $OUT/run_kernel_stats.csv
