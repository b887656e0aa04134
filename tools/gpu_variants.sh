# One gpurun call: optionally the -m gpu suite (TESTS=1), then tools/time_dec.py
# for the product library and each variant named on the command line
# (entropy_coders_amd/libfsehip_NAME.so, built by tools/variant_build.sh).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && { echo "pytest rc=$rc: stopping"; exit $rc; }
fi
for v in - "$@"; do
  lib=libfsehip.so; [ "$v" != "-" ] && lib=libfsehip_$v.so
  FSEHIP_LIB=$lib timeout -k 10 120 python3 tools/time_dec.py > gpurun_out/td_$v.json 2> gpurun_out/td_$v.err || { echo "variant $v failed rc=$?"; tail -3 gpurun_out/td_$v.err; exit 1; }
  cat gpurun_out/td_$v.json
done
