set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c3
SRL_HOST_TIMES=1 timeout -k 10 400 python -u bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r5c3/host.log 2>&1 && tail -2 gpurun_out/r5c3/host.log | cut -c1-200
