set -o pipefail
mkdir -p gpurun_out/ipc
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import torch;print(torch.cuda.get_device_name(0))"
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29601 scripts/ipc_probe.py --flags device --out gpurun_out/ipc/device.jsonl > gpurun_out/ipc/device.log 2>&1
echo "rc_device=$?"
tail -20 gpurun_out/ipc/device.log
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 scripts/ipc_probe.py --flags host --out gpurun_out/ipc/host.jsonl > gpurun_out/ipc/host.log 2>&1
echo "rc_host=$?"
tail -20 gpurun_out/ipc/host.log
