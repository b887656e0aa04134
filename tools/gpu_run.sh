#!/bin/bash
# One gpurun call, parameterised: every GPU step the rounds use, each under its
# own time limit, stopping at the first failure (no GPU step runs after one
# fails, times out or faults).  Replaces the per-call gpu_*.sh wrappers of
# rounds 1-5 (their history is in git).
#
#   tools/gpu_run.sh OUT STEP [STEP ...]      (results under gpurun_out/OUT)
#
# STEP:
#   tests[:SEL]        pytest -m gpu over tests/ (or SEL: a file or -k expression)
#   smoke              __graft_entry__.smoke()
#   bench[:ARGS]       python3 bench.py ARGS (commas become spaces) -> bench_N.json
#   prof[:ARGS]        rocprofv3 kernel trace + stats of bench.py --no-sweep --no-cpu
#                      --no-host-calls ARGS, the per-(kernel, grid) table
#                      (tools/kernel_by_grid.py) and the fractions recomputed from
#                      the trace (tools/frac_check.py)
#   pmc:C1,C2,...      one rocprofv3 PMC pass (kernel trace only) over tools/prof_bench.py
#   traffic            FETCH_SIZE and WRITE_SIZE passes (tools/pmc_summary.py)
#   fuzz[:CASES[:SEED]] the randomized oracle sweep (tests/test_gpu_fuzz.py)
#   micro:NAME[:ARGS]  a prebuilt probe under tools/micro/
#   ab:V1,V2,...       encode A/B (tools/enc_ab.py, AB_WIDE from the environment) of library
#                      builds libfsehip_V.so ("product" = libfsehip.so), three alternating
#                      rounds, C2 bytes checked against the first build's digest
#   abdec:V1,V2,...    decode A/B (tools/time_dec.py: C3, C2 encode / decode, exactness),
#                      three alternating rounds
#   abpy:SCRIPT:V1,... any tools/SCRIPT.py timing script, three alternating rounds over the builds
#
# Variant libraries (FSEHIP_LIB=libfsehip_NAME.so) are selected by the caller's
# environment: FSEHIP_LIB=libfsehip_diag.so tools/gpu_run.sh OUT bench ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:?usage: tools/gpu_run.sh OUT STEP...}
shift
mkdir -p "$O"
export TMPDIR=/tmp
nb=0; np=0; nm=0
fail() { echo "step '$1' failed (rc $2): stopping"; tail -30 "$3"; exit "$2"; }
for step in "$@"; do
  name=${step%%:*}
  arg=""; [[ "$step" == *:* ]] && arg=${step#*:}
  case "$name" in
    tests)
      sel=${arg:-tests}
      timeout -k 10 900 python3 -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$O/pytest_gpu.log" 2>&1 || fail "$step" $? "$O/pytest_gpu.log"
      tail -1 "$O/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || fail "$step" $? "$O/smoke.log"
      echo smoke-ok ;;
    bench)
      nb=$((nb + 1))
      timeout -k 10 600 python3 bench.py ${arg//,/ } > "$O/bench_$nb.json" 2> "$O/bench_$nb.err" \
        || fail "$step" $? "$O/bench_$nb.err"
      tail -1 "$O/bench_$nb.json" | python3 tools/bench_brief.py ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench -- \
        python3 bench.py --no-sweep --no-cpu --no-host-calls ${arg//,/ } > "$O/bench_prof.json" 2> "$O/bench_prof.err" \
        || fail "$step" $? "$O/bench_prof.err"
      python3 tools/kernel_by_grid.py "$O/prof/bench_kernel_trace.csv" > "$O/kernel_by_grid.txt"
      python3 tools/frac_check.py "$O/bench_prof.json" "$O/prof/bench_kernel_trace.csv" | tee "$O/frac_check.txt" ;;
    pmc)
      np=$((np + 1))
      timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$O/pmc$np" -o run --pmc ${arg//,/ } -- \
        python3 tools/prof_bench.py > "$O/pmc$np.log" 2>&1 || fail "$step" $? "$O/pmc$np.log"
      echo "pmc pass $np done: $arg" ;;
    traffic)
      timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$O/fetch" -o run --pmc FETCH_SIZE -- \
        python3 tools/prof_bench.py > "$O/fetch.log" 2>&1 || fail "$step" $? "$O/fetch.log"
      timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$O/write" -o run --pmc WRITE_SIZE -- \
        python3 tools/prof_bench.py > "$O/write.log" 2>&1 || fail "$step" $? "$O/write.log"
      echo traffic-done ;;
    fuzz)
      cases=${arg%%:*}; seed=""; [[ "$arg" == *:* ]] && seed=${arg#*:}
      FSEHIP_FUZZ_CASES=${cases:-400} FSEHIP_FUZZ_SEED=${seed:-616000} \
        timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread \
        > "$O/pytest_fuzz.log" 2>&1 || fail "$step" $? "$O/pytest_fuzz.log"
      tail -1 "$O/pytest_fuzz.log" ;;
    micro)
      nm=$((nm + 1))
      prog=${arg%%:*}; margs=""; [[ "$arg" == *:* ]] && margs=${arg#*:}
      timeout -k 10 300 "./tools/micro/$prog" ${margs//,/ } > "$O/${prog}_$nm.txt" 2>&1 || fail "$step" $? "$O/${prog}_$nm.txt"
      echo "$prog ${margs//,/ }"; tail -12 "$O/${prog}_$nm.txt" ;;
    ab)
      for r in 1 2 3; do
        for v in ${arg//,/ }; do
          lib=libfsehip_$v.so; [ "$v" = product ] && lib=libfsehip.so
          FSEHIP_LIB=$lib AB_DIGEST="$O/ab_digest" timeout -k 10 300 python3 tools/enc_ab.py >> "$O/ab.txt" 2>&1 \
            || fail "$step" $? "$O/ab.txt"
        done
      done
      cat "$O/ab.txt" ;;
    abdec)
      for r in 1 2 3; do
        for v in ${arg//,/ }; do
          lib=libfsehip_$v.so; [ "$v" = product ] && lib=libfsehip.so
          FSEHIP_LIB=$lib timeout -k 10 300 python3 tools/time_dec.py >> "$O/abdec.txt" 2>&1 || fail "$step" $? "$O/abdec.txt"
        done
      done
      grep '^{' "$O/abdec.txt" ;;
    abpy)
      script=${arg%%:*}; vs=${arg#*:}
      for r in 1 2 3; do
        for v in ${vs//,/ }; do
          lib=libfsehip_$v.so; [ "$v" = product ] && lib=libfsehip.so
          FSEHIP_LIB=$lib timeout -k 10 300 python3 "tools/$script.py" >> "$O/$script.txt" 2>&1 || fail "$step" $? "$O/$script.txt"
        done
      done
      grep -v amdgpu.ids "$O/$script.txt" ;;
    *)
      echo "unknown step '$step'"; exit 2 ;;
  esac
done
echo all-steps-ok
