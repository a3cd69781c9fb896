#!/bin/bash
# Exercise the N>1 code path (RCCL exchange + gather) with two ranks sharing the one GPU of a
# gpurun box.  RCCL may refuse two ranks on one device; the log says which.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export NCCL_DEBUG=WARN
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 tools/multirank_check.py
