#!/bin/bash
set -u
export TMPDIR=/tmp PYTHONPATH=.
for m in use off; do
  echo "tunable=$m"
  python - <<PY
from sheeprl_prey_amd.parallel.gemm_tuning import configure
configure("$m")
import runpy; runpy.run_path("scripts/xl_gemm_probe.py", run_name="__main__")
PY
done 2>&1 | grep -v amdgpu.ids
