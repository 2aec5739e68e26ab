set -o pipefail
mkdir -p gpurun_out
export SRL_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 8 --warmup 4 > gpurun_out/bench2_gloo.log 2>&1; rc=$?
tail -5 gpurun_out/bench2_gloo.log
exit $rc
