set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05x; mkdir -p $O
cd $R
for rep in 1 2; do
  for g in 0 192 128 64; do
    USV_POLICY_GRID=$g timeout -k 10 300 python3 bench.py --no-cpu-baseline --c2-steps 0 --extra-steps 0 > $O/g$g.$rep.json 2> $O/g$g.$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$O/g$g.$rep.json'));e=d['extra'];print('grid $g', $rep, 'value %.3fM ms/step %.2f rollout %.2f update %.2f' % (d['value']/1e6, d['ms_per_step'], e['rollout_ms'], e['update_ms']))"
  done
done
