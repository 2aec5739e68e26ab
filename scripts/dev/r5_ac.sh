# actor phase on a side stream beside the critic phase (dreamer_v3.py overlap_ac): correctness + same-box A/B
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ac
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dv3_step_oracle_gpu.py tests/test_dreamer_gpu.py > gpurun_out/r5ac/tests.log 2>&1 && tail -2 gpurun_out/r5ac/tests.log &&
timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5ac/on0.log 2>&1 && tail -1 gpurun_out/r5ac/on0.log &&
SRL_DV3_AC_OVERLAP=0 timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5ac/off0.log 2>&1 && tail -1 gpurun_out/r5ac/off0.log &&
timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5ac/on1.log 2>&1 && tail -1 gpurun_out/r5ac/on1.log &&
SRL_DV3_AC_OVERLAP=0 timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5ac/off1.log 2>&1 && tail -1 gpurun_out/r5ac/off1.log &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_imagine_cont_gpu.py > gpurun_out/r5ac/tests_cont.log 2>&1 && tail -1 gpurun_out/r5ac/tests_cont.log &&
timeout -k 10 400 python -u bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r5ac/con.log 2>&1 && tail -1 gpurun_out/r5ac/con.log | cut -c1-200 &&
SRL_DV3_AC_OVERLAP=0 timeout -k 10 400 python -u bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r5ac/coff.log 2>&1 && tail -1 gpurun_out/r5ac/coff.log | cut -c1-200
