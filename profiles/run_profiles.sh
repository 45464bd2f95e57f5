#!/bin/bash
# GPU-box profiling recipe for the round's bench: kernel trace + stats, then two separate PMC
# passes (FETCH_SIZE, WRITE_SIZE) on the env-step kernel (MI355X_MICROARCH.md HBM section: one
# counter group per pass, FETCH_SIZE doubled for wide streaming reads on gfx950).
# Usage (on the GPU box, from the repo root):  bash profiles/run_profiles.sh <tag> [envs]
set -euo pipefail
TAG=${1:-r02}
ENVS=${2:-131072}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 2 --envs $ENVS --seeds 0 --no-cpu-baseline --c2-steps 0 --extra-steps 0 --milestone-seconds 0"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o trace -- python3 $B > "$OUT/trace.log" 2>&1
echo "trace done"
# the passes below count k_env_step alone: the plain sequential step (the overlapped one shares the GPU
# with the field kernels while it runs, so the default trace's k_env_step mean times the sharing).  The
# sequential trace's k_env_step mean is what the bench's live launch_ms (eager, sequential) measures.
export USV_STEP_OVERLAP=0
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o seqtrace -- python3 $B > "$OUT/seqtrace.log" 2>&1
echo "sequential trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_env_step --output-format csv -d "$OUT" -o pmc_fetch -- python3 $B > "$OUT/pmc_fetch.log" 2>&1
echo "fetch done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_env_step --output-format csv -d "$OUT" -o pmc_write -- python3 $B > "$OUT/pmc_write.log" 2>&1
echo "write done"
