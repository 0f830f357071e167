# phase stamps (FPM_STAMPS=1) of the metric bench for the default build and
# each variant in VARIANTS (lib_var/NAME)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-st}
mkdir -p $O
for v in default ${VARIANTS}; do
  if [ $v = default ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$PWD/fpm-opencv_amd/lib_var/$v/libfpm_hip.so; fi
  FPM_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/s_$v.json 2> $O/s_$v.err || { echo "stamps $v rc=$?"; tail $O/s_$v.err; exit 1; }
  echo "$v: $(grep 'fpm stamps' $O/s_$v.err | tail -1)"
done
