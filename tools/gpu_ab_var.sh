# A/B of compile-time variants (tools/variant_build.sh NAME ...): the decode
# and encode parity tests on each variant library, then tools/time_dec.py for
# the product and each variant, twice.  Usage: bash tools/gpu_ab_var.sh NAME...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in "$@"; do
  FSEHIP_LIB=libfsehip_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stage.py tests/test_gpu_c3.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/pt_$v.log; [ $rc -ne 0 ] && { echo "pytest $v rc=$rc"; exit $rc; }
done
bash tools/gpu_variants.sh "$@" && bash tools/gpu_variants.sh "$@"
