# The driver's multi-GPU launch form at N=1 on a one-GPU box (torch.distributed.run, one rank)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/r4g_torchrun.json 2> gpurun_out/r4g.err
echo rc=$?
