#!/bin/bash
# Round-6 traffic evidence per bench mode: rocprofv3 FETCH_SIZE and WRITE_SIZE
# passes (each its own profiled process, under its own limit) of the mode's
# bench line, summarised per converge / per launch by scripts/pmc_converge.py.
# MODES: any of ujson node treg tlog.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06pmc}
pass() {  # name counter args...
  local n=$1 c=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_${n}_${c}_$TAG -o run --output-format csv -- \
    python3 bench.py "$@" --no-cpu-baseline > gpurun_out/pmc_${n}_${c}_$TAG.log 2>&1 || { tail -5 gpurun_out/pmc_${n}_${c}_$TAG.log; return 1; }
  echo "pmc $n $c ok"
}
both() { pass "$1" FETCH_SIZE "${@:2}" && pass "$1" WRITE_SIZE "${@:2}"; }
sum() {  # name first skip count keep
  python3 scripts/pmc_converge.py gpurun_out/pmc_${1}_$TAG.json gpurun_out/pmc_${1}_FETCH_SIZE_$TAG \
    gpurun_out/pmc_${1}_WRITE_SIZE_$TAG "$2" "$3" "$4" "$5"
}
for m in ${MODES:-ujson node treg tlog}; do
  case $m in
    ujson) both ujson --type ujson --steps 4 --warmup 6 && sum ujson k_uj_items 7 4 "k_uj_,jydscan::" || exit 1 ;;
    node)  both node --type treg --node --steps 4 --warmup 2 && sum node k_nd_maxlen 3 4 "k_nd,k_key,k_treg,jydscan::" || exit 1 ;;
    treg)  both treg --type treg --steps 4 --warmup 2 --batches 2 && sum treg k_treg_lww 3 4 "k_treg_lww" \
             && python3 scripts/pmc_converge.py gpurun_out/pmc_treg_keyed_$TAG.json gpurun_out/pmc_treg_FETCH_SIZE_$TAG \
                gpurun_out/pmc_treg_WRITE_SIZE_$TAG k_treg_lww 9 4 "k_treg_lww" || exit 1 ;;
    tlog)  both tlog --type tlog --steps 4 --warmup 2 && sum tlog k_tlog_prep 3 4 "k_tlog_,jydscan::" || exit 1 ;;
  esac
done
echo "pmc done"
