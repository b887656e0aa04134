# A/B timing: the GPU tests, then the bench (no CPU leg, no sweep) once per
# environment setting given as arguments ("NAME=VAL" or "-" for none).
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=10 --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
i=0
for kv in "$@"; do
  i=$((i+1))
  if [ "$kv" = "-" ]; then
    timeout -k 10 300 python3 bench.py --no-cpu --no-sweep > gpurun_out/ab$i.json 2> gpurun_out/ab$i.err
  else
    env "$kv" timeout -k 10 300 python3 bench.py --no-cpu --no-sweep > gpurun_out/ab$i.json 2> gpurun_out/ab$i.err
  fi
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab$i.json')); c=d.get('c3_decode_only',{}); print('$kv', 'value', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'c3', c.get('decode_ms'), c.get('roofline',{}).get('frac'), 'ok', d['verified_roundtrip'])"
done
