# Sidecar-less decode check: the whole -m gpu suite, then tools/nosidecar_time.py
# (2-state and 1-state at 256 MiB, C2 and skewed L=12 at 1 GiB).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1 && tail -3 gpurun_out/t_all.log &&
timeout -k 10 200 python -u tools/nosidecar_time.py > gpurun_out/ns2.log 2>&1 && cat gpurun_out/ns2.log &&
NS_STATES=1 timeout -k 10 200 python -u tools/nosidecar_time.py > gpurun_out/ns1.log 2>&1 && cat gpurun_out/ns1.log &&
NS_BYTES=1073741824 NS_CASES=c2_lut0155,lut077_L12 timeout -k 10 300 python -u tools/nosidecar_time.py > gpurun_out/ns_1g.log 2>&1 && cat gpurun_out/ns_1g.log
