set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/enc_path.py > gpurun_out/enc_path.log 2>&1
FSEHIP_ENC_PATH=2 FSEHIP_ENC_WARM=64 FSEHIP_ENC_PMAX=256 ST_BYTES=1073741824 timeout -k 10 300 python3 tools/stamps.py > gpurun_out/stamps_p2.log 2>&1
echo ok
