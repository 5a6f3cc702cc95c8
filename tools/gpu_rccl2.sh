set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_ranks_check.py > gpurun_out/rccl2.log 2>&1
echo "rccl2 rc=$?" >> gpurun_out/rccl2.log
