# One gpurun call: the round-1 tree (_ab/r01, built in this container) and
# HEAD timed back to back on the same box, twice each (encode / decode ms).
# (_ab is listed in .gpurunignore so that ordinary calls do not upload it: take
# that line out for this call.)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
  (cd _ab/r01 && timeout -k 10 200 python3 bench.py --no-cpu --no-sweep --no-c3 > ../../gpurun_out/ab_r01_$i.json 2> ../../gpurun_out/ab_r01_$i.err) || { echo "r01 failed"; tail -3 gpurun_out/ab_r01_$i.err; exit 1; }
  timeout -k 10 200 python3 bench.py --no-cpu --no-sweep --no-c3 --no-serial > gpurun_out/ab_head_$i.json 2> gpurun_out/ab_head_$i.err || { echo "head failed"; tail -3 gpurun_out/ab_head_$i.err; exit 1; }
  python3 -c "
import json
for t in ('r01','head'):
    d=json.load(open('gpurun_out/ab_%s_$i.json'%t)); print(t, d['value'], d['encode_ms'], d['decode_ms'], d.get('verified_roundtrip'))"
done
