set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prey
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_dreamer_gpu.py -k "scan" > gpurun_out/prey/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/prey/tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 > gpurun_out/prey/step.log 2>&1; tail -3 gpurun_out/prey/step.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 6 > gpurun_out/prey/bench.log 2>&1 && tail -1 gpurun_out/prey/bench.log | cut -c1-150
hipcc -O3 --offload-arch=gfx950 -o gpurun_out/prey/xcd_handoff scripts/dev/xcd_handoff.hip > /dev/null 2>&1 && timeout -k 10 60 gpurun_out/prey/xcd_handoff 2000 | tee gpurun_out/prey/xcd.txt; rm -f gpurun_out/prey/xcd_handoff
