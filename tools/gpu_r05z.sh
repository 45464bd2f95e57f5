set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05z; mkdir -p $O
cd $R
for rep in 1 2; do
  for v in base env stats both; do
    case $v in base) E=0; S=0;; env) E=1; S=0;; stats) E=0; S=1;; both) E=1; S=1;; esac
    USV_ENV_FIRST=$E USV_STATS_FIRST=$S timeout -k 10 300 python3 bench.py --no-cpu-baseline --c2-steps 0 --extra-steps 0 > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail $O/$v.$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$v.$rep.json'));e=d['extra'];print('$v', $rep, 'value %.3fM ms/step %.2f rollout %.2f update %.2f' % (d['value']/1e6, d['ms_per_step'], e['rollout_ms'], e['update_ms']))"
  done
done
