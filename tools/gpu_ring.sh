set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_blocks.py tests/test_gpu_edge.py tests/test_gpu_stage.py > gpurun_out/t_ring.log 2>&1 && tail -3 gpurun_out/t_ring.log &&
timeout -k 10 200 python -u tools/nosidecar_time.py > gpurun_out/ns_new.log 2>&1 && cat gpurun_out/ns_new.log &&
NS_BYTES=1073741824 NS_CASES=c2_lut0155 timeout -k 10 200 python -u tools/nosidecar_time.py > gpurun_out/ns_new1g.log 2>&1 && cat gpurun_out/ns_new1g.log &&
NS_BYTES=1073741824 NS_CASES=c2_lut0155 FSEHIP_SERIAL_OLD=1 timeout -k 10 200 python -u tools/nosidecar_time.py > gpurun_out/ns_old1g.log 2>&1 && cat gpurun_out/ns_old1g.log
