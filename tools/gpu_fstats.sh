set -uo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fstats; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_env_gpu.py -x -q --timeout 200 --timeout-method thread -k "field or fixture or philox or replay" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
VARIANTS=base TOP=12 bash tools/gpu_kvariants.sh
