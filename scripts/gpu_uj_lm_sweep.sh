set -u
cd "$(dirname "$0")" 2>/dev/null || true
for lm in 32 64 512 0; do
  JY_UJ_LONG_MIN=$lm timeout -k 10 300 python3 bench.py --type ujson --steps 8 --warmup 6 --no-cpu-baseline > gpurun_out/lm_$lm.log 2>&1 || exit 1
  echo "lm=$lm $(grep -h '^{' gpurun_out/lm_$lm.log | grep -o '"converge_ms_avg[^,]*\|"touched_el[^,]*\|"inplace_docs[^,]*\|"promoted[^,]*\|"demoted[^,]*' | tr '\n' ' ')"
done
