set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5xl
timeout -k 10 500 python -u bench.py --xl --steps 10 --warmup 4 > gpurun_out/r5xl/on0.log 2>&1 && tail -1 gpurun_out/r5xl/on0.log | cut -c1-120 &&
SRL_DV3_AC_OVERLAP=0 timeout -k 10 500 python -u bench.py --xl --steps 10 --warmup 4 > gpurun_out/r5xl/off0.log 2>&1 && tail -1 gpurun_out/r5xl/off0.log | cut -c1-120 &&
timeout -k 10 500 python -u bench.py --xl --steps 10 --warmup 4 > gpurun_out/r5xl/on1.log 2>&1 && tail -1 gpurun_out/r5xl/on1.log | cut -c1-120 &&
SRL_DV3_AC_OVERLAP=0 timeout -k 10 500 python -u bench.py --xl --steps 10 --warmup 4 > gpurun_out/r5xl/off1.log 2>&1 && tail -1 gpurun_out/r5xl/off1.log | cut -c1-120
