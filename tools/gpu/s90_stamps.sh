set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s90st
mkdir -p $O
FPM_STAMPS=1 timeout -k 10 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/st.json 2> $O/st.err || { echo "rc=$?"; tail -3 $O/st.err; exit 1; }
grep "fpm stamps" $O/st.err | tail -2
