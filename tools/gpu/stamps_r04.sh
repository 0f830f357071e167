# Round 4 phase stamps (FPM_STAMPS=1: shader-clock cycles per LED step, first
# and last wave) of the metric kernel and the shard workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04st}
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
for W in "metric:--patches-total_256" "pt128:--patches-total_128" "pt64:--patches-total_64" "pt32:--patches-total_32" "c2:--config_c2" "c3:--config_c3"; do
  N=${W%%:*}; A=${W#*:}; A=${A//_/ }
  FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gather $A > $O/st_$N.json 2> $O/st_$N.err || { echo "stamps $N rc=$?"; tail -3 $O/st_$N.err; exit 1; }
  echo "== $N $(python3 -c "import json; d=json.load(open('$O/st_$N.json')); print(d['value'], d['led_ms_per_step'], d['config']['kernel'])")"
  grep "fpm stamps" $O/st_$N.err | tail -2
done
