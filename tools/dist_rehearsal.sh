#!/usr/bin/env bash
# Rehearse bench.py's N > 1 path (RowShardedMMQ, weak + strong) with 2 ranks on the one GPU
# of a gpurun box over gloo (RCCL needs one GPU per rank).  Not the product collective.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/dist2_weak.json 2> gpurun_out/dist2_weak.err
rc=$?; cat gpurun_out/dist2_weak.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/dist2_weak.err; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 2 --strong --steps 20 --warmup 3 > gpurun_out/dist2_strong.json 2> gpurun_out/dist2_strong.err
rc=$?; cat gpurun_out/dist2_strong.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/dist2_strong.err; exit $rc; }
# RCCL graph capture of the exchange at world 1 (a real ncclAllGather on one rank)
unset BENCH_BACKEND
export BENCH_FORCE_DIST=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519 \
  bench.py --steps 20 --warmup 3 > gpurun_out/dist1_rccl.json 2> gpurun_out/dist1_rccl.err
rc=$?; cat gpurun_out/dist1_rccl.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/dist1_rccl.err; exit $rc; }
