# Bench (no CPU leg, no sweep) once per setting: "NAME=VAL[,NAME=VAL]" or "-"
# for the environment; BENCH_ARGS (env) adds bench.py arguments to every run.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
i=0
for kv in "$@"; do
  i=$((i+1))
  envs=""
  [ "$kv" != "-" ] && envs=$(echo "$kv" | tr ',' ' ')
  env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-sweep $BENCH_ARGS > gpurun_out/ab$i.json 2> gpurun_out/ab$i.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab$i.json')); c=d.get('c3_decode_only',{}); print('$kv', '$BENCH_ARGS', 'value', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'c3', c.get('decode_ms'), c.get('roofline',{}).get('frac'), 'ok', d['verified_roundtrip'])"
done
