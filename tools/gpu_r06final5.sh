#!/bin/bash
# r06final5: the round's evidence on the final tree -- the full GPU suite, smoke(), then the profile round (kernel stats
# overlapped + sequential, PMC FETCH_SIZE / WRITE_SIZE passes on the env step at 4,096 and 131,072 envs) and the
# default bench line
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06final5
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/gpu_profile_round.sh r06final5 > $O/profile_round.log 2>&1 || exit $?
tail -2 $O/profile_round.log
