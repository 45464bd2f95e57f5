set -uo pipefail
mkdir -p gpurun_out/c3
timeout -k 10 600 python3 -u -m pytest tests/test_ppo_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/c3/pytest.log 2>&1; rc=$?; tail -12 gpurun_out/c3/pytest.log; [ $rc -ne 0 ] && exit $rc
for mp in "" "--mixed-precision"; do
  timeout -k 10 300 python3 bench.py --envs 65536 --steps 10 --no-cpu-baseline --c2-steps 0 $mp > gpurun_out/c3/b$mp.json 2> gpurun_out/c3/b$mp.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/c3/b$mp.json'));e=d['extra'];print('$mp', d['value']/1e6, d['ms_per_step'], e['rollout_ms'], e['update_ms'], e['update_us_per_minibatch'], d['roofline_ppo']['launch_ms'], d['wall_clock_to_reward'])"
done
