mkdir -p gpurun_out
ST_BYTES=268435456 timeout -k 10 200 python -u tools/stamps.py > gpurun_out/st64.log 2>&1 && FSEHIP_ENC_LANES=32 ST_BYTES=268435456 timeout -k 10 200 python -u tools/stamps.py > gpurun_out/st32.log 2>&1; grep -h "encode:" gpurun_out/st64.log gpurun_out/st32.log
