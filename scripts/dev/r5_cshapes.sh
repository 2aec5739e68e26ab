set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5g
SRL_PROFILE_SHAPES=1 timeout -k 10 400 python -u bench.py --continuous --steps 2 --warmup 3 --torch-profile 1 > gpurun_out/r5g/cshapes.log 2>&1 && grep "^GEMM" gpurun_out/r5g/cshapes.log | head -45
