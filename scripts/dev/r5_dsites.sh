set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5d
SRL_PROFILE_SITES=1 SRL_PROFILE_TOP=120 timeout -k 10 400 python -u bench.py --steps 2 --warmup 3 --torch-profile 1 > gpurun_out/r5d/sites.log 2>&1 && grep SITE gpurun_out/r5d/sites.log | head -120
