set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5st
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_algos_gpu.py tests/test_dreamer_gpu.py tests/test_actor_loss_cont_gpu.py tests/test_imagine_cont_gpu.py tests/test_dv3_step_oracle_gpu.py > gpurun_out/r5st/tests.log 2>&1; tail -2 gpurun_out/r5st/tests.log
grep -E "^FAILED|^E " gpurun_out/r5st/tests.log | head -8
for i in 0 1; do
SRL_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 6 > gpurun_out/r5st/b$i.log 2>&1 && tail -2 gpurun_out/r5st/b$i.log | cut -c1-170 || exit 1
done
timeout -k 10 400 python -u bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r5st/c0.log 2>&1 && tail -1 gpurun_out/r5st/c0.log | cut -c1-150
