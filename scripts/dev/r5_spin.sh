set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dv3_overlap_gpu.py > gpurun_out/r5s/ovt.log 2>&1; tail -3 gpurun_out/r5s/ovt.log
for i in 0 1; do
SRL_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 6 > gpurun_out/r5s/spin$i.log 2>&1 && tail -2 gpurun_out/r5s/spin$i.log | cut -c1-180 &&
SRL_SPIN_WAIT=0 SRL_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 6 > gpurun_out/r5s/block$i.log 2>&1 && tail -2 gpurun_out/r5s/block$i.log | cut -c1-180 || exit 1
done
