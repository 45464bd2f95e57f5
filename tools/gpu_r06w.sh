#!/bin/bash
# r06w: per-phase timing of the gradient / reduction / policy / sweep kernels on the final tree (probe build)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06w
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/phase_probe.py > $O/phase_probe_131072.txt 2>&1 || exit $?
cat $O/phase_probe_131072.txt
