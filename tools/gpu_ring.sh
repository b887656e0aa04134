set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_onestate.py tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_blocks.py tests/test_gpu_dtables.py tests/test_gpu_stream.py > gpurun_out/t_ring.log 2>&1; rc=$?; tail -3 gpurun_out/t_ring.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/nosidecar_time.py > gpurun_out/ns2.log 2>&1 && cat gpurun_out/ns2.log
NS_STATES=1 timeout -k 10 200 python -u tools/nosidecar_time.py > gpurun_out/ns1.log 2>&1 && cat gpurun_out/ns1.log
NS_BYTES=1073741824 NS_CASES=c2_lut0155 timeout -k 10 200 python -u tools/nosidecar_time.py > gpurun_out/ns_1g.log 2>&1 && cat gpurun_out/ns_1g.log
