# A/B of encoder variants: the GPU encode parity tests on the product
# library, then tools/time_dec.py for the product and each variant named on
# the command line (built by tools/variant_build.sh), twice.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_onestate.py tests/test_gpu_fuzz.py tests/test_gpu_edge.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_enc.log 2>&1
rc=$?; tail -2 gpurun_out/pt_enc.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
bash tools/gpu_variants.sh "$@" && bash tools/gpu_variants.sh "$@"
