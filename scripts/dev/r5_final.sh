# End-of-round GPU validation + every bench line at HEAD (one box)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5f
bash scripts/gpu_validate.sh || exit 1
timeout -k 10 400 python -u bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r5f/cont.log 2>&1 && tail -1 gpurun_out/r5f/cont.log > gpurun_out/r5f/cont.json &&
timeout -k 10 400 python -u bench.py --algo sac > gpurun_out/r5f/sac.log 2>&1 && tail -1 gpurun_out/r5f/sac.log > gpurun_out/r5f/sac.json &&
timeout -k 10 600 python -u bench.py --xl --steps 10 --warmup 4 > gpurun_out/r5f/xl.log 2>&1 && tail -1 gpurun_out/r5f/xl.log > gpurun_out/r5f/xl.json &&
timeout -k 10 400 python -u scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 10 > gpurun_out/r5f/prey.log 2>&1 && tail -2 gpurun_out/r5f/prey.log
for f in cont sac xl; do cut -c1-160 gpurun_out/r5f/$f.json; done
