set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/xcd
hipcc -O3 --offload-arch=gfx950 -o gpurun_out/xcd/xcd_handoff scripts/dev/xcd_handoff.hip > /dev/null 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 60 gpurun_out/xcd/xcd_handoff 2000 | tee gpurun_out/xcd/result.txt
rm -f gpurun_out/xcd/xcd_handoff
bash scripts/dev/r5_cont.sh
