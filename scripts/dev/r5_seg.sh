set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5sg
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dreamer_gpu.py tests/test_dp_graphs_gpu.py tests/test_rccl_gpu.py > gpurun_out/r5sg/tests.log 2>&1; tail -1 gpurun_out/r5sg/tests.log
grep -E "^FAILED|^E " gpurun_out/r5sg/tests.log | head -5
for i in 0 1; do
timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 --segmented > gpurun_out/r5sg/seg$i.log 2>&1 && tail -1 gpurun_out/r5sg/seg$i.log | cut -c1-110 &&
timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5sg/single$i.log 2>&1 && tail -1 gpurun_out/r5sg/single$i.log | cut -c1-110 || exit 1
done
bash scripts/rehearse_2rank.sh > gpurun_out/r5sg/r2.log 2>&1; grep -o '"value": [0-9.]*\|"dp_param_spread": [0-9.e-]*\|"final_wm_loss": [0-9.]*' gpurun_out/rehearse2.log
