#!/bin/bash
# GPU box: sweep work queue -- env / field GPU tests on the default build, then bench A/B against the round-robin
# build (lib/rr.so) at the default length and late in training (93 epochs), two reps
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05queue; mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_env_gpu.py tests/test_headline_gpu.py tests/test_overlap_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
B="--no-cpu-baseline --c2-steps 0 --extra-steps 0 --milestone-seconds 0"
for rep in 1 2; do
for v in queue:base rr:rr.so; do
  name=${v%%:*}; lib=${v#*:}; [ "$lib" = base ] && lib=""
  for len in 20 90; do
    USV_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps $len --warmup 3 $B > $O/$name.$len.$rep.json 2> $O/$name.$len.$rep.err || { tail -3 $O/$name.$len.$rep.err; exit 1; }
    python3 - $O/$name.$len.$rep.json $name $len $rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
print("%-6s epochs %3s rep %s value %.3fM rollout %.2f ms update %.2f ms device-only rollout %.2f ms" % (
    sys.argv[2], sys.argv[3], sys.argv[4], d["value"] / 1e6, e["rollout_ms"], e["update_ms"], e["device_only"]["rollout_ms"]))
PY
  done
done
done
