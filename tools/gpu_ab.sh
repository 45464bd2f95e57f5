#!/bin/bash
# GPU box: GPU tests, then bench A (default) and bench B (BENCH_B_ARGS) back to back
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1
  rc=$?
  tail -3 $O/pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python3 bench.py --no-cpu-baseline ${BENCH_A_ARGS:-} > $O/a.json 2> $O/a.err || exit $?
timeout -k 10 600 python3 bench.py --no-cpu-baseline ${BENCH_B_ARGS:-} > $O/b.json 2> $O/b.err || exit $?
python3 - <<'PY'
import json, os
for k in "ab":
    d = json.load(open(os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/ab", k + ".json")))
    e = d["extra"]
    print(k, "value %.3gM ms/step %.3f rollout %.3f update %.3f env_kernel %.1f us envonly131k kernel %.1f us" % (
        d["value"] / 1e6, d["ms_per_step"], e.get("rollout_ms", 0), e.get("update_ms", 0),
        d["roofline"]["launch_ms"] * 1e3, e.get("env_step_kernel_ms", 0) * 1e3))
PY
