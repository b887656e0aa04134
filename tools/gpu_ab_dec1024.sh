# A/B: 1024-thread decode workgroups at 32-pair checkpoints (libfsehip_d1024.so)
# against the product at 64- and 32-pair checkpoints, twice.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stage.py tests/test_gpu_c3.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_dec.log 2>&1
rc=$?; tail -2 gpurun_out/pt_dec.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
FSEHIP_LIB=libfsehip_d1024.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stage.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_dec2.log 2>&1
rc=$?; tail -2 gpurun_out/pt_dec2.log; [ $rc -ne 0 ] && { echo "pytest d1024 rc=$rc"; exit $rc; }
for rep in 1 2; do
  for cfg in "libfsehip.so 64" "libfsehip.so 32" "libfsehip_d1024.so 32"; do
    set -- $cfg
    FSEHIP_LIB=$1 CKPT=$2 timeout -k 10 120 python3 tools/time_dec.py > gpurun_out/td_ab.json 2> gpurun_out/td_ab.err || { echo "failed $cfg"; tail -3 gpurun_out/td_ab.err; exit 1; }
    cat gpurun_out/td_ab.json
  done
done
