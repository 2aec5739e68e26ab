set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
SRL_PROFILE_SITES=1 SRL_PROFILE_TOP=90 timeout -k 10 400 python -u bench.py --continuous --steps 2 --warmup 3 --torch-profile 1 > gpurun_out/r5c/sites.log 2>&1 && grep SITE gpurun_out/r5c/sites.log | head -90
