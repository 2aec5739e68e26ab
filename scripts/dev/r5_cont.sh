set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cont
SRL_PROFILE_SITES=1 SRL_PROFILE_TOP=150 timeout -k 10 400 python -u bench.py --continuous --steps 2 --warmup 4 --torch-profile 1 > gpurun_out/cont/sites.log 2>&1; grep SITE gpurun_out/cont/sites.log | head -150
